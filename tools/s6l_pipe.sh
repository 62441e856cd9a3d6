#!/bin/bash
# device_pipeline A/B: the planning stream at the highest priority (-1, gss_run's) against normal (0),
# interleaved on one box; bench.py without the configs / e2e / PMC legs
set -e
o=gpurun_out/s6l
mkdir -p $o
for r in 1 2; do
  for p in -1 0; do
    GSS_BENCH_PIPE_PRIO=$p timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs \
      --no-e2e --no-cpu-baseline --no-pmc --no-sustained > $o/pipe_p${p}_r$r.json 2> $o/pipe_p${p}_r$r.err
    python - $o/pipe_p${p}_r$r.json <<'PY'
import json, sys
w = json.load(open(sys.argv[1]))["window"]
print(sys.argv[1], w["device_window"]["device_ms"], w["device_pipeline"])
PY
  done
done
