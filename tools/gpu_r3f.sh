#!/bin/bash
# Round-3 session f: the driver's bench command with its live rocprofv3 passes kept
# (GSS_PROF_SAVE), then tools/pmc_traffic.py's record from them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3f}
export TMPDIR=/tmp
GSS_PROF_SAVE=$(pwd)/gpurun_out/prof_$TAG timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 \
    > gpurun_out/bench_$TAG.log 2> gpurun_out/bench_$TAG.err || exit $?
tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json
