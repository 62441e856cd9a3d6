# GSS_SPEC_K 32 (_var/k32) against the in-tree 16: device window legs and configs[4] end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6i; mkdir -p $O
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for r in 1 2; do
for v in k16 k32; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; K=16; [ $v = k32 ] && { lib=_var/k32/libgpssim_amd.so; K=32; }
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python tools/e2e_cfg_probe.py 4 > $O/e2e4_${v}_$r.log 2>&1 || exit 1
done
done
for v in k16 k32; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; K=16; [ $v = k32 ] && { lib=_var/k32/libgpssim_amd.so; K=32; }
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python tools/proof_bench.py 16 449 5 2e7 2>/dev/null | tail -1 | sed "s/^/$v 20M /" >> $O/proof.txt || exit 1
done
