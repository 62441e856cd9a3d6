# gss_run's output buffers pinned lazily (slots after the first by the planner) against all in the
# set-up (GSS_RUN_LAZY_OUT=0): bench.py's e2e workloads, a fresh process each, interleaved; the GPU
# suite first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-s6ao}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2 3; do
for lz in 1 0; do
  GSS_RUN_LAZY_OUT=$lz timeout -k 10 300 python tools/e2e_seq_probe.py h c2 h > $O/seq_lazy${lz}_$r.txt 2>&1 || exit 1
  grep -v amdgpu.ids $O/seq_lazy${lz}_$r.txt | sed "s/^/lazy=$lz /"
done
done
