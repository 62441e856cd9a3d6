# GSS_SPEC_K 16 (in-tree) against 8 (_var/k8): the GPU suite, then end to end (configs[4] -b 1
# with GPU proofs and anchors uploaded per slot; the headline's e2e leg), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for r in 1 2; do
for v in k16 k8; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; K=16; [ $v = k8 ] && { lib=_var/k8/libgpssim_amd.so; K=8; }
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python tools/e2e_cfg_probe.py 4 > $O/e2e4_${v}_$r.log 2>&1 || exit 1
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-configs --no-pmc --no-cpu-baseline --no-exact --no-sustained > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
done
done
