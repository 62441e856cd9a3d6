#!/bin/bash
# Round-3 session ag: does a gss_run with the rows/prover threads slow a later run's downloads?
# (configs[4] whole day, then static -b 16 1800 s, in one process; GSS_RUN_ROWS_AHEAD per leg)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "1 0" "0 1" "1 1" "0 0"; do
    set -- $v
    timeout -k 10 200 python tools/e2e_order_probe.py $1 $2 2> gpurun_out/order_$1$2_r3ag.err || exit $?
done
