#!/bin/bash
# End-to-end CLI rate (host plane + H2D + GPU + D2H, output to /dev/null): the PCIe-inclusive
# number DESIGN.md reports next to bench.py's HBM-resident value.  Usage: cli_rate.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-s}
mkdir -p gpurun_out
BIN=gps-sdr-sim_amd/bin/gps-sdr-sim
NAV=tests/golden/data/brdc3540.14n
for d in 30 300 3000; do
  t0=$(date +%s.%N)
  timeout -k 10 300 $BIN -e $NAV -l 30.286502,120.032669,100 -d $d -b 16 -o /dev/null \
      > gpurun_out/cli_${TAG}_$d.log 2>&1 || exit $?
  t1=$(date +%s.%N)
  python3 - "$d" "$t0" "$t1" >> gpurun_out/cli_rate_$TAG.json <<'PY'
import json, sys
d, t0, t1 = float(sys.argv[1]), float(sys.argv[2]), float(sys.argv[3])
blocks = int(d * 10) - 1
ms = blocks * 260000 / (t1 - t0) / 1e6
print(json.dumps({"cli": f"-d {d:g} -b 16 -o /dev/null", "wall_s": round(t1 - t0, 3),
                  "msps": round(ms, 1), "x_realtime": round(ms / 2.6, 1)}))
PY
done
