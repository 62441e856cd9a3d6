set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s6c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_proof.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "proof or spec_records" > $O/pytest.log 2>&1 || exit 1
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for v in cur nocc cur nocc scr; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v = nocc ] && lib=_var/nocc/libgpssim_amd.so
  if [ $v = scr ]; then export HSA_SCRATCH_SINGLE_LIMIT=4294967296; fi
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  tail -1 $O/bench_$v.json | sed "s/^/$v /" >> $O/all.txt
done
