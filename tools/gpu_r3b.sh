#!/bin/bash
# Round-3 session: the 16x16x32 MFMA probe, the NUMA D2H probe, the fast-path and parity GPU
# tests on the in-tree build (LIN_MFMA 2), then the interleaved A/B timing against _var/ builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3b}
timeout -k 10 60 tools/ubench/mfma16_probe > gpurun_out/mfma16_probe_$TAG.log 2>&1 || exit $?
timeout -k 10 180 python tools/numa_d2h_probe.py > gpurun_out/numa_d2h_$TAG.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_parity.py -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} bash tools/gpu_ablate.sh $TAG
