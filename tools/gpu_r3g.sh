#!/bin/bash
# Round-3 session g: fast-path parity tests on the scalar-window build (_var/sw), then the
# interleaved A/B of the in-tree build against _var/ builds (20 steps after 5 warm-up).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3g}
GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=_var/sw/libgpssim_amd.so timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_lin.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_sw_$TAG.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-3} STEPS=20 WARMUP=5 bash tools/gpu_ablate.sh $TAG
