#!/bin/bash
# Round-3 session c: the e2e planner-thread sweep (cgroup CPU throttling check), then the
# interleaved A/B timing of the in-tree build against the _var/ ablation builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3c}
out=gpurun_out/e2e_threads_$TAG.log
: > $out
for th in 4 8 12 16; do
    before=$(cat /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
    r=$(timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-exact \
        --no-configs --no-pmc --threads $th 2>/dev/null | tail -1) || exit $?
    after=$(cat /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
    echo "threads $th $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin)["e2e"]; print(d["value"], d["d2h_GBps"], d["steady_d2h_GBps"], d["d2h_ceiling_GBps"], d["wall_s"])')" >> $out
    echo "  cpu.stat before: $before" >> $out
    echo "  cpu.stat after:  $after" >> $out
done
ROUNDS=${ROUNDS:-2} bash tools/gpu_ablate.sh $TAG
