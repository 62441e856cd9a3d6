#!/bin/bash
# gss_run per-slot trace (GSS_RUN_TRACE=1) at three batch sizes and the D2H copy probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python tools/d2h_probe.py > gpurun_out/d2h_probe.log 2>&1 || exit $?
for b in 64 128 256; do
    GSS_PROBE_BATCH=$b GSS_RUN_TRACE=1 timeout -k 10 120 python tools/e2e_probe.py 600 1800 \
        > gpurun_out/e2e_tr_$b.out 2> gpurun_out/e2e_tr_$b.err || exit $?
done
