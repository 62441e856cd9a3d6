#!/bin/bash
# Round-3 session i: the fast-path tests on the scalar-window build (_var/sw), the interleaved
# A/B (20 steps after 5 warm-up), then bench's e2e legs on the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3i}
export TMPDIR=/tmp
GSS_TEST_VARIANT=1 GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=_var/sw/libgpssim_amd.so timeout -k 10 600 \
    python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_parity.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "not cli and not integration" \
    > gpurun_out/pytest_sw_$TAG.log 2>&1 || exit $?
ROUNDS=${ROUNDS:-3} STEPS=20 WARMUP=5 bash tools/gpu_ablate.sh $TAG || exit $?
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact --no-pmc \
    > gpurun_out/bench_e2e_$TAG.log 2> gpurun_out/bench_e2e_$TAG.err || exit $?
