#!/bin/bash
# Time the fast-path kernel of each measurement build in _var/ (tools/ablate.sh) with bench.py;
# with E2E=1 the gss_run end-to-end rate instead (bench.py's e2e entry).  ROUNDS (default 2)
# passes over all builds, alternating, so that the box's clock drift spreads over every build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ablate_${1:-x}.log
: > $out
for round in $(seq ${ROUNDS:-2}); do
for lib in gps-sdr-sim_amd/lib/libgpssim_amd.so _var/*/libgpssim_amd.so; do
    if [ -n "$E2E" ]; then
        r=$(GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 1 --warmup 0 \
            --no-cpu-baseline --no-exact --no-configs --no-pmc 2>/dev/null | tail -1) || exit $?
        echo "$lib $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin)["e2e"]; print(d["value"], d["d2h_GBps"], d["wall_s"], d.get("d2h_ceiling_GBps"))')" >> $out
        continue
    fi
    r=$(GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-2} --no-configs --no-e2e \
        --no-cpu-baseline --no-exact --no-pmc 2>/dev/null | tail -1) || exit $?
    echo "$lib $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["stages_ms"]["fast_path"], d["value"])')" >> $out
done
done
