#!/bin/bash
# Round-3 session ae: the bench's e2e legs in one process with the rows/prover threads on and off
# (the headline e2e runs after configs[4]'s in the same process).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3ae}
for a in 1 0 1; do
    GSS_RUN_ROWS_AHEAD=$a timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
        --no-pmc --no-exact > gpurun_out/bench_a${a}_$TAG.log 2> gpurun_out/bench_a${a}_$TAG.err || exit $?
    python -c "
import json,sys; b=json.loads(open('gpurun_out/bench_a${a}_$TAG.log').read().strip().splitlines()[-1])
print('ahead=$a', 'e2e', b['e2e']['value'], b['e2e']['frac_of_d2h_ceiling'], [ (p['config'], p['e2e']['value'], p['e2e']['wall_s']) for p in b['per_config']])"
done
