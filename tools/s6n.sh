# the speculative walks from a row-shared cycle cache (in-tree, 64 entries per row) against the plain
# per-lane walk (_var/plain, GSS_SPEC_SHARED=0) and 32 entries (_var/sc32): the GPU's spec tests,
# then the window legs interleaved (VARS: variants, _var/<name>; ROUNDS; SKIPTEST=1: no tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-s6n}; mkdir -p $O
[ -n "$SKIPTEST" ] || timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "spec or chain or streaming_run_chain" > $O/pytest_spec.log 2>&1 || { tail -30 $O/pytest_spec.log; exit 1; }
[ -n "$SKIPTEST" ] || tail -3 $O/pytest_spec.log
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for r in ${ROUNDS:-1 2}; do
for v in ${VARS:-shared plain sc32}; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != shared ] && lib=_var/$v/libgpssim_amd.so
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
  python - $O/bench_${v}_$r.json $v <<'PY'
import json, sys
w = json.load(open(sys.argv[1]))["window"]
d, p = w["device_window"], w["device_pipeline"]
print(sys.argv[2], "spec", d["spec_ms"], "proof", d["proof_ms"], "render", d["render_ms"], "dev", d["device_ms"], d["roofline"]["frac"], "pipe", p["ms_per_window"], p["roofline"]["frac"], p["output_identical"])
PY
done
done
