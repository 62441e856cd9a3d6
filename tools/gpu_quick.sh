#!/bin/bash
# Quick GPU check after a kernel change: the fast-path and parity GPU tests, then a short bench.
# Each step has its own time limit; the first failure ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/quick_pytest_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_EXTRA} \
    > gpurun_out/quick_bench_$TAG.log 2>&1
