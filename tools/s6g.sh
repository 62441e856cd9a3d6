# round-6 closing measurements: the driver's bench command (kernel, PMC traffic, CPU baseline,
# per-config and e2e legs, window + device_window), then the headline profile and the window
# pipeline's profile, all on the committed library
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-s6g}
O=gpurun_out/$T; mkdir -p $O
GSS_PROF_SAVE=$GRAFT_REPO_ROOT/$O/live timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
PROF_BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 900 bash tools/profile.sh $T || exit 1
STEPS=10 WARMUP=3 timeout -k 10 900 bash tools/profile_window.sh $T || exit 1
