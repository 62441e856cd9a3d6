#!/bin/bash
# Profiling session for the per-window GPU pipeline (bench.py's window leg with device_window:
# gss_spec_kernel + gss_spec_rec_kernel + gss_proof_kernel + the render): kernel trace + stats,
# then one PMC pass per counter group (never combined with other trace domains).
# Usage: bash tools/profile_window.sh [tag]   -> gpurun_out/profw_<tag>/ (summary.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-w}
OUT=gpurun_out/profw_$TAG
mkdir -p $OUT
BA="--steps ${STEPS:-10} --warmup ${WARMUP:-3} --no-exact --no-configs --no-e2e --no-cpu-baseline --no-pmc --no-sustained"
run() {  # name, rocprofv3 args...
    local name=$1; shift
    timeout -k 10 400 rocprofv3 "$@" -d $OUT/$name -o $name -f csv -- python3 bench.py $BA \
        > $OUT/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc" >> $OUT/session.log; return $rc
}
run kt --kernel-trace --stats || exit $?
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR --kernel-trace || exit $?
run pmc_mem --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace || exit $?
python3 tools/prof_summary.py $OUT ${STEPS:-10} ${WARMUP:-3} > $OUT/summary.json || exit $?
find $OUT -name '*.csv' -size +4M -delete
echo done >> $OUT/session.log
