#!/bin/bash
# Time the fast-path kernel of each measurement build in _var/ (tools/ablate.sh) with bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ablate_${1:-x}.log
: > $out
for lib in gps-sdr-sim_amd/lib/libgpssim_amd.so _var/*/libgpssim_amd.so; do
    r=$(GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 \
        --no-cpu-baseline --no-exact 2>/dev/null | tail -1) || exit $?
    echo "$lib $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["stages_ms"]["fast_path"], d["value"])')" >> $out
done
