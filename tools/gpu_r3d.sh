#!/bin/bash
# Round-3 session d: the GPU test suite on the in-tree build, the rocprofv3 slowdown study (the
# bench's profiling child run bare, under --kernel-trace alone and under --kernel-trace --stats,
# same steps / warm-up as the driver's bench), then the interleaved A/B against _var/ builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3d}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
CHILD="bench.py --steps 20 --warmup 5 --fmt 16 --window 300 --threads 8 --no-cpu-baseline --no-exact --no-configs --no-e2e --no-pmc"
out=gpurun_out/profslow_$TAG.log
: > $out
R=$(pwd)
for i in 1 2; do
    timeout -k 10 200 python $CHILD > gpurun_out/ps_bare$i.log 2>&1 || exit $?
    echo "bare$i $(tail -1 gpurun_out/ps_bare$i.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["stages_ms"]["fast_path"], d["ms_per_step"])')" >> $out
    (cd /tmp && timeout -k 10 200 python3 $(which rocprofv3) --kernel-trace -d $R/gpurun_out/ps_kt$i -o kt -f csv -- python3 $R/$CHILD > $R/gpurun_out/ps_kt$i.log 2>&1) || exit $?
    echo "kt$i $(grep '^{' gpurun_out/ps_kt$i.log | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["stages_ms"]["fast_path"], d["ms_per_step"])')" >> $out
    (cd /tmp && timeout -k 10 200 python3 $(which rocprofv3) --kernel-trace --stats -d $R/gpurun_out/ps_kts$i -o kts -f csv -- python3 $R/$CHILD > $R/gpurun_out/ps_kts$i.log 2>&1) || exit $?
    echo "kts$i $(grep '^{' gpurun_out/ps_kts$i.log | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["stages_ms"]["fast_path"], d["ms_per_step"])')" >> $out
done
ROUNDS=${ROUNDS:-2} bash tools/gpu_ablate.sh $TAG
