# the cycle-cached walks with a register copy of the last cycle's entry (in-tree) against the build
# before (_var/prevmru): proof_bench over the headline window, then the window legs; GPU suite first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6aj; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
for v in cur prevmru; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != cur ] && lib=_var/$v/libgpssim_amd.so
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python tools/proof_bench.py 16 2999 7 2.6e6 2>/dev/null | tail -1 > $O/pb_${v}_$r.json || exit 1
  python - $O/pb_${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
a = sorted(d["anch_device_ms"]); b = sorted(d["device_ms"])
print(sys.argv[2], "proof anchored median", a[len(a) // 2], "no anchors median", b[len(b) // 2], "host 16 thr", d.get("anch_host_ms_16"), "same", d["same"])
PY
done
done
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for r in 1 2; do
for v in cur prevmru; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != cur ] && lib=_var/$v/libgpssim_amd.so
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
  python - $O/bench_${v}_$r.json $v <<'PY'
import json, sys
w = json.load(open(sys.argv[1]))["window"]
d, p = w["device_window"], w["device_pipeline"]
print(sys.argv[2], "spec", d["spec_ms"], "proof", d["proof_ms"], "render", d["render_ms"], "dev", d["device_ms"], d["roofline"]["frac"], "pipe", p["ms_per_window"], p["roofline"]["frac"], p["output_identical"])
PY
done
done
