#!/bin/bash
# Round-3 session e: how the fast-path kernel's time evolves over 100 back-to-back launches
# (kernel trace), and the shader clock per launch (GRBM_GUI_ACTIVE cycles / duration, own pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3e}
export TMPDIR=/tmp
R=$(pwd)
CHILD="bench.py --steps 100 --warmup 5 --fmt 16 --window 300 --threads 16 --no-cpu-baseline --no-exact --no-configs --no-e2e --no-pmc"
(cd /tmp && timeout -k 10 240 python3 $(which rocprofv3) --kernel-trace -d $R/gpurun_out/ramp_kt_$TAG -o kt -f csv -- python3 $R/$CHILD > $R/gpurun_out/ramp_kt_$TAG.log 2>&1) || exit $?
(cd /tmp && timeout -s KILL 240 python3 $(which rocprofv3) --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/ramp_pmc_$TAG -o pmc -f csv -- python3 $R/$CHILD > $R/gpurun_out/ramp_pmc_$TAG.log 2>&1) || exit $?
