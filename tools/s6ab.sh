# configs[2] end to end: slot sizes, three runs per process (the first cold, then warm)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-s6ab}; mkdir -p $O
for b in 256 64 128 256 512 64 128; do
  E2E_REPEAT=3 timeout -k 10 200 python tools/e2e_cfg_probe.py 2 300 16 $b > $O/e2e2_b$b.log 2>&1 || exit 1
  grep "run [12] " $O/e2e2_b$b.log
done
