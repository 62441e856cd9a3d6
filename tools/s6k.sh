# the device gss_jump in f64 (in-tree) against the committed round-6 build (_var/jprev)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_proof.py tests/test_gpu_lin.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for r in 1 2; do
for v in cur jprev; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != cur ] && lib=_var/$v/libgpssim_amd.so
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || exit 1
done
done
for v in cur jprev; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != cur ] && lib=_var/$v/libgpssim_amd.so
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python tools/proof_bench.py 16 449 5 2e7 2>/dev/null | tail -1 | sed "s/^/$v 20M /" >> $O/proof.txt || exit 1
done
