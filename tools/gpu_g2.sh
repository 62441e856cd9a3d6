set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/tput_ubench > gpurun_out/tput2.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_serial.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --pipeline > gpurun_out/b_pipe.log 2>&1 &&
timeout -k 10 300 python -m pytest tests/test_gpu_long.py -q -x --timeout 200 > gpurun_out/long.log 2>&1
