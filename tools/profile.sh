#!/bin/bash
# Profiling session on the GPU box (rocprofv3): kernel trace + stats, then one PMC pass per
# counter group (never combined with other trace domains).  Outputs under gpurun_out/prof_<tag>/.
# Usage: bash tools/profile.sh [tag]   (bench args via PROF_BENCH_ARGS; never the CPU baseline
# or the live PMC passes: a profiled process has the GPU initialised, so it must start no programs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BA="${PROF_BENCH_ARGS:---steps 3 --warmup 1 --no-exact --no-configs --no-e2e} --no-cpu-baseline --no-pmc --no-window"
# the counter passes only need the headline kernel: without the per-config and e2e legs
PA="$BA --no-configs --no-e2e"
run() {  # name, rocprofv3 args...
    local name=$1; shift
    local args="$PA"
    [ "$name" = kt ] && args="$BA"
    timeout -k 10 400 rocprofv3 "$@" -d $OUT/$name -o $name -f csv -- python3 bench.py $args \
        > $OUT/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc" >> $OUT/session.log; return $rc
}
run kt --kernel-trace --stats || exit $?
run pmc_write --pmc WRITE_SIZE --kernel-trace || exit $?
run pmc_fetch --pmc FETCH_SIZE --kernel-trace || exit $?
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR --kernel-trace || exit $?
run pmc_lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace || exit $?
[ -n "$PMC_STALL" ] && { run pmc_stall --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES --kernel-trace || exit $?; }
# summarised here, then the per-dispatch traces dropped (gpurun copies back at most 64 MiB)
steps=$(echo "$BA" | sed -n 's/.*--steps \([0-9]*\).*/\1/p'); warm=$(echo "$BA" | sed -n 's/.*--warmup \([0-9]*\).*/\1/p')
python3 tools/prof_summary.py $OUT ${steps:-0} ${warm:-0} > $OUT/summary.json || exit $?
find $OUT -name '*.csv' -size +4M -delete
echo done >> $OUT/session.log
