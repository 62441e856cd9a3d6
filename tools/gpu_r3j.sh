#!/bin/bash
# Round-3 session j: interleaved A/B of the MFMA modes with and without the bias-as-C peel
# (in-tree = LIN_MFMA 2 + LIN_C0 1), 20 steps after 5 warm-up.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3} STEPS=20 WARMUP=5 bash tools/gpu_ablate.sh ${1:-r3j}
