#!/bin/bash
# Round-3 session y: the rows thread on its own worker pool (GSS_RUN_ROWS_POOL) -- gss_run's GPU
# tests, then configs[4] whole day and configs[2] with the rows thread on its own pool, sharing
# the planner's, and without the rows thread.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3y}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider \
    -k "chain_modes or sink_error or streaming_run or two_ranks" --timeout 100 \
    --timeout-method thread > gpurun_out/pytest_rows_$TAG.log 2>&1 || exit $?
for v in "1 1" "1 0" "0 1" "1 1"; do
    set -- $v
    GSS_RUN_ROWS_AHEAD=$1 GSS_RUN_ROWS_POOL=$2 GSS_RUN_TRACE=1 timeout -k 10 120 \
        python tools/e2e_cfg_probe.py 4 > gpurun_out/e2e_cfg4day_a$1p$2_$TAG.out \
        2> gpurun_out/e2e_cfg4day_a$1p$2_$TAG.err || exit $?
    GSS_RUN_ROWS_AHEAD=$1 GSS_RUN_ROWS_POOL=$2 GSS_RUN_TRACE=1 timeout -k 10 120 \
        python tools/e2e_cfg_probe.py 2 > gpurun_out/e2e_cfg2_a$1p$2_$TAG.out \
        2> gpurun_out/e2e_cfg2_a$1p$2_$TAG.err || exit $?
    cat gpurun_out/e2e_cfg4day_a$1p$2_$TAG.out gpurun_out/e2e_cfg2_a$1p$2_$TAG.out
done
for f in gpurun_out/e2e_*_$TAG.err; do python tools/e2e_trace_sum.py $f > ${f%.err}.sum 2>&1 || true; done
