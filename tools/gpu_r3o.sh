#!/bin/bash
# Round-3 session o: windows by vector buffer loads from the static window table (_var/sw2,
# LIN_SWIN 2): fast-path parity on that build, then the interleaved A/B (20 steps, 5 warm-up).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3o}
GSS_TEST_VARIANT=1 GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=_var/sw2/libgpssim_amd.so timeout -k 10 600 \
    python -u -m pytest tests/test_gpu_lin.py -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_sw2_$TAG.log 2>&1 || exit $?
ROUNDS=${ROUNDS:-3} STEPS=20 WARMUP=5 bash tools/gpu_ablate.sh $TAG
