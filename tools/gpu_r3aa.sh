#!/bin/bash
# Round-3 session aa: segment guesses made by the walkers on the GPU (gss_carr_chain_starts) --
# the whole GPU suite, then end-to-end probes with the run's trace: configs[4]
# whole day and first hour, configs[3], configs[2], static -b 16 1800 s.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3aa}
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || exit $?
GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 4 \
    > gpurun_out/e2e_cfg4day_$TAG.out 2> gpurun_out/e2e_cfg4day_$TAG.err || exit $?
GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 4 \
    > gpurun_out/e2e_cfg4day2_$TAG.out 2> gpurun_out/e2e_cfg4day2_$TAG.err || exit $?
GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 3 \
    > gpurun_out/e2e_cfg3_$TAG.out 2> gpurun_out/e2e_cfg3_$TAG.err || exit $?
GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 2 \
    > gpurun_out/e2e_cfg2_$TAG.out 2> gpurun_out/e2e_cfg2_$TAG.err || exit $?
GSS_PROBE_BATCH=128 GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_probe.py 600 1800 \
    > gpurun_out/e2e_b16_$TAG.out 2> gpurun_out/e2e_b16_$TAG.err || exit $?
for f in gpurun_out/e2e_*_$TAG.err; do python tools/e2e_trace_sum.py $f > ${f%.err}.sum 2>&1 || true; done
