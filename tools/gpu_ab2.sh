#!/bin/bash
# The -m gpu suite on the in-tree build, then A/B against _var/ builds at -b 16 and -b 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || exit $?
FMT=16 ROUNDS=2 bash tools/gpu_ab_fmt.sh $TAG && FMT=8 ROUNDS=2 bash tools/gpu_ab_fmt.sh $TAG
