#!/bin/bash
# Round-3 session n: gss_run e2e A/B (GSS_RUN_DEPTH / NCOPY builds), then a two-rank rehearsal
# of the driver's torchrun bench on this one-GPU box (GSS_BENCH_REHEARSE: both ranks on GPU 0,
# gloo collectives; the plan-once baton, timing and the JSON line are the driver's path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r3n}
E2E=1 ROUNDS=${ROUNDS:-3} bash tools/gpu_ablate.sh $TAG || exit $?
GSS_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-pmc \
    > gpurun_out/rehearse2_$TAG.log 2> gpurun_out/rehearse2_$TAG.err || exit $?
