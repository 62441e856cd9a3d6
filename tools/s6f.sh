set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for v in cur prev spec16 cur prev spec16; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != cur ] && lib=_var/$v/libgpssim_amd.so
  K=8; [ $v = spec16 ] && K=16
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  tail -1 $O/bench_$v.json | sed "s/^/$v /" >> $O/all.txt
done
for v in cur spec16; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != cur ] && lib=_var/$v/libgpssim_amd.so
  K=8; [ $v = spec16 ] && K=16
  GSS_SPEC_K=$K GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python tools/proof_bench.py 16 449 5 2e7 2>/dev/null | tail -1 | sed "s/^/$v 20M /" >> $O/proof.txt || exit 1
done
