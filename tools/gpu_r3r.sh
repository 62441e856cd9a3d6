#!/bin/bash
# Round-3 session r: the fast-path GPU tests on the current build, then the interleaved A/B of
# the current build against _var/* (20 steps after 5 warm-up).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3r}
timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_lin_$TAG.log 2>&1 || exit $?
ROUNDS=${ROUNDS:-3} STEPS=20 WARMUP=5 bash tools/gpu_ablate.sh $TAG
