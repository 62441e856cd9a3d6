set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_proof.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "spec or proof or streaming_run_mixed or linearize" > $O/pytest.log 2>&1 || exit 1
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for v in cur nocc cur nocc; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v = nocc ] && lib=_var/nocc/libgpssim_amd.so
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  tail -1 $O/bench_$v.json | sed "s/^/$v /" >> $O/all.txt
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python tools/proof_bench.py 16 449 5 2e7 2>/dev/null | tail -1 | sed "s/^/$v 20M /" >> $O/proof.txt || exit 1
done
