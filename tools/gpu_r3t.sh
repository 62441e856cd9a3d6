#!/bin/bash
# Round-3 session t: the carrier chain run ahead -- GPU walk latency per batch (GSS_RUN_TRACE) for
# configs[4] / configs[2] / static -b 16, the chain on the GPU (default) and on the host.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3t}
for spec in 1 0; do
    GSS_RUN_SPEC=$spec GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 4 3600 \
        > gpurun_out/e2e_cfg4_spec${spec}_$TAG.out 2> gpurun_out/e2e_cfg4_spec${spec}_$TAG.err || exit $?
    GSS_RUN_SPEC=$spec GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_cfg_probe.py 2 \
        > gpurun_out/e2e_cfg2_spec${spec}_$TAG.out 2> gpurun_out/e2e_cfg2_spec${spec}_$TAG.err || exit $?
    GSS_PROBE_BATCH=128 GSS_RUN_SPEC=$spec GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_probe.py 600 1800 \
        > gpurun_out/e2e_b16_spec${spec}_$TAG.out 2> gpurun_out/e2e_b16_spec${spec}_$TAG.err || exit $?
done
