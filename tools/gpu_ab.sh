#!/bin/bash
# One GPU session for a kernel change: the -m gpu suite on the in-tree build, then the
# interleaved A/B timing of the in-tree build against the _var/ builds (tools/gpu_ablate.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}
mkdir -p gpurun_out
if [ -x tools/ubench/mfma_probe ]; then
    timeout -k 10 60 ./tools/ubench/mfma_probe > gpurun_out/mfma_probe_$TAG.log 2>&1 || exit $?
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
ROUNDS=${ROUNDS:-2} bash tools/gpu_ablate.sh $TAG
