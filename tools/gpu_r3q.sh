#!/bin/bash
# Round-3 session q: interleaved A/B of step-loop ablations (_var/*: VOP2 sign shift, readlane windows, no sign
# bank conflicts, both), 20 steps after 5 warm-up, three rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3} STEPS=20 WARMUP=5 bash tools/gpu_ablate.sh ${1:-r3q}
