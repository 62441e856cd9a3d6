#!/bin/bash
# Profile HEAD (tools/profile.sh) after one driver-style bench run, then the clock of a
# measurement build without output stores (_var/nost, LIN_ABLATE=1: wrong output, timing only):
# GRBM_GUI_ACTIVE over the kernel's duration gives its average shader clock.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2s5}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
bash tools/profile.sh $TAG || exit $?
for v in nost; do
    lib=_var/$v/libgpssim_amd.so
    [ -f $lib ] || continue
    OUT=gpurun_out/prof_${TAG}_$v
    mkdir -p $OUT
    GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        -d $OUT/kt -o kt -f csv -- python3 bench.py --steps 3 --warmup 1 --no-exact --no-configs \
        --no-e2e --no-cpu-baseline --no-pmc > $OUT/kt.log 2>&1 || exit $?
    GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE \
        SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES --kernel-trace -d $OUT/pmc_sq -o pmc_sq \
        -f csv -- python3 bench.py --steps 3 --warmup 1 --no-exact --no-configs --no-e2e \
        --no-cpu-baseline --no-pmc > $OUT/pmc_sq.log 2>&1 || exit $?
done
