#!/bin/bash
# Round-3 session k: gss_run traces of the per-config e2e legs (configs[2], [3], a 3600 s slice
# of [4]) and of the headline, summarised per slot.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3k}
for a in "2 300" "3 450" "4 3600"; do
    set -- $a
    GSS_RUN_TRACE=1 timeout -k 10 200 python tools/e2e_cfg_probe.py $1 $2 \
        > gpurun_out/e2e_cfg$1_$TAG.out 2> gpurun_out/e2e_cfg$1_$TAG.err || exit $?
    python3 tools/e2e_trace_sum.py gpurun_out/e2e_cfg$1_$TAG.err >> gpurun_out/e2e_cfg$1_$TAG.out
done
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact --no-pmc \
    > gpurun_out/bench_e2e_$TAG.log 2> gpurun_out/bench_e2e_$TAG.err || exit $?
