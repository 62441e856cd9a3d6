set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s6b
BA="--steps 10 --warmup 3 --no-configs --no-e2e --no-pmc --no-cpu-baseline --no-exact --no-sustained"
for v in cur nocc cur nocc; do
  lib=gps-sdr-sim_amd/lib/libgpssim_amd.so; [ $v != cur ] && lib=_var/$v/libgpssim_amd.so
  GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 240 python bench.py $BA > gpurun_out/s6b/bench_$v.json 2> gpurun_out/s6b/bench_$v.err || exit 1
  tail -1 gpurun_out/s6b/bench_$v.json >> gpurun_out/s6b/all.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s6b/kt -o kt -f csv -- python3 $GRAFT_REPO_ROOT/bench.py $BA > $GRAFT_REPO_ROOT/gpurun_out/s6b/kt.log 2>&1
