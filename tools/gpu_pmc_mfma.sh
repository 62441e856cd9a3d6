#!/bin/bash
# One PMC pass on the fast kernel for the matrix-core counters (MFMA instructions, MFMA busy
# cycles) beside the VALU ones; its own run, kernel trace only (MI355X_MICROARCH.md).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_mfma
mkdir -p $OUT
BA="--steps 3 --warmup 1 --no-exact --no-configs --no-e2e --no-cpu-baseline --no-pmc"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
    SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc_mfma -o pmc_mfma -f csv \
    -- python3 bench.py $BA > $OUT/pmc_mfma.log 2>&1
