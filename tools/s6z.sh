# GSS_SPEC_K 16 / 32 / 64 with the row-shared walk cache: window legs, configs[4] end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6z; mkdir -p $O
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for r in 1 2; do
for K in 16 32 64; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $K != 16 ] && lib=_var/k$K/libgpssim_amd.so
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > $O/bench_k${K}_$r.json 2> $O/bench_k${K}_$r.err || exit 1
  python - $O/bench_k${K}_$r.json k$K <<'PY'
import json, sys
w = json.load(open(sys.argv[1]))["window"]
d, p = w["device_window"], w["device_pipeline"]
print(sys.argv[2], "spec", d["spec_ms"], "proof", d["proof_ms"], "render", d["render_ms"], "dev", d["device_ms"], d["roofline"]["frac"], "pipe", p["ms_per_window"], p["roofline"]["frac"], p["output_identical"])
PY
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python tools/e2e_cfg_probe.py 4 > $O/e2e4_k${K}_$r.log 2>&1 || exit 1
  tail -1 $O/e2e4_k${K}_$r.log | cut -c1-300
done
done
