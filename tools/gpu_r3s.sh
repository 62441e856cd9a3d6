#!/bin/bash
# Round-3 session s: the carrier chain run ahead on the GPU (gss_spec_device) -- its GPU tests and
# the gss_run ones, then end-to-end probes with the chain on the host (GSS_RUN_SPEC=0) and on the
# GPU: configs[4] (-b 1) first hour, configs[2] (circle -b 8), static -b 16 1800 s.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3s}
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider \
    -k "spec_walks or chain_modes or streaming_run or producers or two_ranks" --timeout 100 \
    --timeout-method thread > gpurun_out/pytest_spec_$TAG.log 2>&1 || exit $?
for spec in ${SPECS:-0 1}; do
    GSS_RUN_SPEC=$spec GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 4 3600 \
        > gpurun_out/e2e_cfg4_spec${spec}_$TAG.out 2> gpurun_out/e2e_cfg4_spec${spec}_$TAG.err || exit $?
    GSS_RUN_SPEC=$spec GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 2 \
        > gpurun_out/e2e_cfg2_spec${spec}_$TAG.out 2> gpurun_out/e2e_cfg2_spec${spec}_$TAG.err || exit $?
    GSS_PROBE_BATCH=128 GSS_RUN_SPEC=$spec GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_probe.py 600 1800 \
        > gpurun_out/e2e_b16_spec${spec}_$TAG.out 2> gpurun_out/e2e_b16_spec${spec}_$TAG.err || exit $?
done
