#!/bin/bash
# Round-3 session ad: per-batch walk events with two batches in flight --
# suite, then configs[4] whole day with and without the prover thread, configs[3], configs[2],
# static -b 16 1800 s, with the run's trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3ad}
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || exit $?
for v in 1 0 1; do
    GSS_RUN_PROVER=$v GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 4 \
        > gpurun_out/e2e_cfg4day_p${v}_$TAG.out 2> gpurun_out/e2e_cfg4day_p${v}_$TAG.err || exit $?
    cat gpurun_out/e2e_cfg4day_p${v}_$TAG.out
done
GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 3 \
    > gpurun_out/e2e_cfg3_$TAG.out 2> gpurun_out/e2e_cfg3_$TAG.err || exit $?
GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 2 \
    > gpurun_out/e2e_cfg2_$TAG.out 2> gpurun_out/e2e_cfg2_$TAG.err || exit $?
GSS_PROBE_BATCH=128 GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_probe.py 600 1800 \
    > gpurun_out/e2e_b16_$TAG.out 2> gpurun_out/e2e_b16_$TAG.err || exit $?
for f in gpurun_out/e2e_*_$TAG.err; do python tools/e2e_trace_sum.py $f > ${f%.err}.sum 2>&1 || true; done
