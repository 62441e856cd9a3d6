# GSS_SPEC_K 32 (_var/k32) against the in-tree 16 with the row-shared walk cache: the window legs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6y; mkdir -p $O
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for r in 1 2; do
for v in k16 k32; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; K=16; [ $v = k32 ] && { lib=_var/k32/libgpssim_amd.so; K=32; }
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
  python - $O/bench_${v}_$r.json $v <<'PY'
import json, sys
w = json.load(open(sys.argv[1]))["window"]
d, p = w["device_window"], w["device_pipeline"]
print(sys.argv[2], "spec", d["spec_ms"], "proof", d["proof_ms"], "render", d["render_ms"], "dev", d["device_ms"], d["roofline"]["frac"], "pipe", p["ms_per_window"], p["roofline"]["frac"], p["output_identical"])
PY
done
done
# the proof's two halves alone (measurement builds _var/skipc: no carrier part, _var/skipz: no code
# part; their rows are not the host's), tools/proof_bench.py over the headline window's blocks
for v in cur skipc skipz cur; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != cur ] && lib=_var/$v/libgpssim_amd.so
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python tools/proof_bench.py 16 2999 5 2.6e6 2>/dev/null | tail -1 | sed "s/^/$v /" >> $O/proof_halves.txt || exit 1
done
cat $O/proof_halves.txt
