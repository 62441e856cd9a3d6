set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "b8 or fmt or circle or synthetic" > gpurun_out/q_b8.log 2>&1 || exit $?
for r in 1 2 3; do for lib in gps-sdr-sim_amd/lib/libgpssim_amd.so _var/nosaddr/libgpssim_amd.so; do
  x=$(GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python bench.py --fmt 8 --steps 10 --warmup 2 --no-configs --no-e2e --no-cpu-baseline --no-exact --no-pmc 2>/dev/null | tail -1) || exit $?
  echo "$lib $(echo "$x" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["stages_ms"]["fast_path"], d["value"])')" >> gpurun_out/ablate_b8.log
done; done
