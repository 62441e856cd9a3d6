# gss_run's ramped first slots (GSS_RUN_RAMP=1, the default) against whole batches from the start:
# the GPU suite, then bench.py's e2e workloads in one process each, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-s6af}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ${TESTSEL:-} > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
for ramp in 1 0; do
  GSS_RUN_RAMP=$ramp timeout -k 10 300 python tools/e2e_seq_probe.py h c2 c2 c3 c4 h > $O/seq_ramp${ramp}_$r.txt 2>&1 || exit 1
  grep -v amdgpu.ids $O/seq_ramp${ramp}_$r.txt | sed "s/^/ramp=$ramp /"
done
done
