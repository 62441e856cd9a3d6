#!/bin/bash
# Round-3 session af: what slows the bench's headline e2e leg with the rows thread on: without
# the per-config legs before it, without the prover thread, with the rows thread on the
# planner's pool.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3af}
run() {
    local name=$1; shift
    env "$@" timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc \
        --no-exact $EXTRA > gpurun_out/bench_${name}_$TAG.log 2> gpurun_out/bench_${name}_$TAG.err || exit $?
    python -c "
import json; b=json.loads(open('gpurun_out/bench_${name}_$TAG.log').read().strip().splitlines()[-1])
print('$name', 'e2e', b['e2e']['value'], b['e2e']['frac_of_d2h_ceiling'], b['e2e'].get('steady_d2h_GBps'), [(p['config'], p['e2e']['value']) for p in (b['per_config'] or [])])"
}
EXTRA=--no-configs run noconf GSS_RUN_ROWS_AHEAD=1
EXTRA= run noprover GSS_RUN_PROVER=0
EXTRA= run sharedpool GSS_RUN_ROWS_POOL=0
EXTRA= run trace GSS_RUN_TRACE=1
