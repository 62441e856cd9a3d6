#!/bin/bash
# Round-3 closing session: the whole GPU suite, the driver's bench command with its live
# rocprofv3 passes kept (GSS_PROF_SAVE), the PMC counter passes (tools/profile.sh: SQ and LDS
# groups, 20 steps after 5 warm-up), and a four-rank torchrun rehearsal on this one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3z}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit $?
GSS_PROF_SAVE=$(pwd)/gpurun_out/prof_$TAG timeout -k 10 900 python bench.py --gpus 1 --steps 20 \
    --warmup 5 > gpurun_out/bench_$TAG.log 2> gpurun_out/bench_$TAG.err || exit $?
tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json
PROF_BENCH_ARGS="--steps 20 --warmup 5 --no-exact --no-configs --no-e2e" bash tools/profile.sh ${TAG}_pmc || exit $?
GSS_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 5 --warmup 2 --no-pmc \
    > gpurun_out/rehearse4_$TAG.log 2> gpurun_out/rehearse4_$TAG.err || exit $?
