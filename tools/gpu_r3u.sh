#!/bin/bash
# Round-3 session u: the whole GPU suite and the driver's bench command on the build with the
# carrier chain run ahead on the GPU (gss_run e2e legs: configs[1..4]).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3u}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log \
    2> gpurun_out/bench_$TAG.err || exit $?
tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json
