#!/bin/bash
# device_pipeline A/B: three stages on three streams against walks + proofs on one (GSS_BENCH_PIPE_STAGES),
# interleaved on one box (s6l: priority -1 against 0); bench.py without the configs / e2e / PMC legs
set -e
o=gpurun_out/${TAG:-s6m}
mkdir -p $o
for r in 1 2; do
  for p in 3 2; do   # s6m
    GSS_BENCH_PIPE_STAGES=$p timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs \
      --no-e2e --no-cpu-baseline --no-pmc --no-sustained > $o/pipe_st${p}_r$r.json 2> $o/pipe_st${p}_r$r.err
    python - $o/pipe_st${p}_r$r.json <<'PY'
import json, sys
w = json.load(open(sys.argv[1]))["window"]
print(sys.argv[1], w["device_window"]["device_ms"], w["device_pipeline"])
PY
  done
done
