# the proof kernel: per-lane cycle cache entries (GSS_CC_N 4 / 8 against 16) and its register
# budget (5 waves per SIMD against 4 and 6), proof_bench over the headline window, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6am; mkdir -p $O
for r in 1 2; do
for v in cur cc8 cc4 pw6 pw4; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != cur ] && lib=_var/$v/libgpssim_amd.so
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python tools/proof_bench.py 16 2999 9 2.6e6 2>/dev/null | tail -1 > $O/pb_${v}_$r.json || exit 1
  python - $O/pb_${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
a = sorted(d["anch_device_ms"]); b = sorted(d["device_ms"])
print(sys.argv[2], "proof anchored median", a[len(a) // 2], "no anchors median", b[len(b) // 2], "same", d["same"])
PY
done
done
