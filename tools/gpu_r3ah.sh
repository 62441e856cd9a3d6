#!/bin/bash
# Round-3 session ah: is the bench process's slower configs[4] e2e leg (1.74 s against 1.35 s in a
# fresh process) the torch CPU thread pool?  The per-config legs with OMP_NUM_THREADS 16 and 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in 16 1; do
    OMP_NUM_THREADS=$t timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
        --no-pmc --no-exact > gpurun_out/bench_omp${t}_r3ah.log 2> gpurun_out/bench_omp${t}_r3ah.err || exit $?
    python -c "
import json; b=json.loads(open('gpurun_out/bench_omp${t}_r3ah.log').read().strip().splitlines()[-1])
print('omp $t', 'e2e', b['e2e']['value'], [(p['config'], p['e2e']['value'], p['e2e']['wall_s']) for p in b['per_config']])"
done
