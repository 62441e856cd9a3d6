#!/bin/bash
# Clock and cycle counts of measurement builds: per library (the current build and _var/<names>),
# a kernel-trace pass and one PMC pass (GRBM_GUI_ACTIVE, SQ busy/wave cycles, LDS waits) over the
# bench's 20 timed launches after 5 warm-up; summaries via tools/prof_summary.py.
# Usage: bash tools/gpu_clk.sh tag name...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
BA="--steps 20 --warmup 5 --no-exact --no-configs --no-e2e --no-cpu-baseline --no-pmc"
for name in cur "$@"; do
    lib=gps-sdr-sim_amd/lib/libgpssim_amd.so
    [ "$name" != cur ] && lib=_var/$name/libgpssim_amd.so
    OUT=gpurun_out/clk_${TAG}_$name
    mkdir -p $OUT
    GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        -d $OUT/kt -o kt -f csv -- python3 bench.py $BA > $OUT/kt.log 2>&1 || exit $?
    GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE \
        SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
        SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d $OUT/pmc_clk -o pmc_clk -f csv -- \
        python3 bench.py $BA > $OUT/pmc.log 2>&1 || exit $?
    python3 tools/prof_summary.py $OUT 20 5 > $OUT/summary.json || exit $?
done
