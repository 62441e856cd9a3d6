#!/bin/bash
# Round-3 session l: the whole GPU suite (nav rows and C/A table now built on the device inside
# gss_run), then the per-config gss_run traces and bench's e2e legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3l}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit $?
bash tools/gpu_r3k.sh $TAG
