#!/bin/bash
# Round-3 session m: gss_run end to end (bench e2e entry) for the in-tree build against
# GSS_RUN_DEPTH=2 and NCOPY=2 builds, three alternating rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
E2E=1 ROUNDS=${ROUNDS:-3} bash tools/gpu_ablate.sh ${1:-r3m}
