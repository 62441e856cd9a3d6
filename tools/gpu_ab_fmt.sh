#!/bin/bash
# A/B of the in-tree library against each _var/ build at one output format (FMT, default 16):
# fast-path kernel time from bench.py, ROUNDS passes alternating builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ablate_${1:-x}_b${FMT:-16}.log
for r in $(seq ${ROUNDS:-3}); do for lib in gps-sdr-sim_amd/lib/libgpssim_amd.so _var/*/libgpssim_amd.so; do
  x=$(GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python bench.py --fmt ${FMT:-16} --steps 10 --warmup 2 --no-configs --no-e2e --no-cpu-baseline --no-exact --no-pmc 2>/dev/null | tail -1) || exit $?
  echo "$lib $(echo "$x" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["stages_ms"]["fast_path"], d["value"])')" >> $out
done; done
