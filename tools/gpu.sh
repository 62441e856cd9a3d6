#!/bin/bash
# One GPU-box session (gpurun), built from steps given on the command line, run in order.  Every
# GPU step has its own time limit; the first step that fails ends the session (no retries), and
# everything goes under gpurun_out/<tag>/.
#
#   bash tools/gpu.sh TAG step [step ...]
#
# steps:
#   tests            pytest -m gpu (whole suite)          quick   the fast-path + parity GPU tests
#   smoke            __graft_entry__.smoke()              bench   bench.py as the driver runs it
#   ablate:V1,V2,..  kernel time of the current build and _var/<Vi> (tools/ablate.sh builds),
#                    interleaved ROUNDS (default 2) times, bench.py --no-* legs off
#   clock:V1,V2,..   in-kernel clock stamps of _var/<Vi> (LIN_STAMP builds), interleaved ROUNDS
#   prof             rocprofv3 kernel trace + stats, then one PMC pass per counter group
#                    (tools/profile.sh: traffic, SQ, LDS), never combined with other domains
#   e2e:N            tools/e2e_cfg_probe.py N (gss_run over configs[N] end to end, traced)
#   e2eab:V1,V2,..   bench.py's e2e leg of the current build and _var/<Vi>, interleaved ROUNDS
#   rehearse:N[:T]   the driver's torchrun bench as N ranks on this one GPU (GSS_BENCH_REHEARSE:
#                    gloo collectives, every rank on GPU 0), args REHEARSE_ARGS, output tag T
#   pmcclk:V1,V2,..  per-dispatch clock and cycles from PMC (GRBM_GUI_ACTIVE, SQ busy/wave
#                    cycles) of the current build and _var/<Vi>, one rocprofv3 pass each
#   env:K=V          export K=V for the steps after it (e.g. env:BENCH_ARGS='--steps 20')
#   cmd:'...'        any other command, under a 300 s limit
# env: BENCH_ARGS (bench step), STEPS/WARMUP (ablate), ROUNDS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
log=$OUT/session.log
echo "== $(date) $*" >> $log
step() {  # name, exit status
    echo "$1 rc=$2" >> $log
    [ "$2" -eq 0 ] || { echo "session stopped at $1 (rc=$2)" >> $log; exit "$2"; }
}
for s in "$@"; do
    case "$s" in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
            --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
        step tests $? ;;
    quick)
        timeout -k 10 600 python -u -m pytest tests/test_gpu_lin.py tests/test_gpu_parity.py -x -q \
            -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_quick.log 2>&1
        step quick $? ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
        step smoke $? ;;
    bench)
        timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
        step bench $? ;;
    ablate:*)
        vs=${s#ablate:}
        for r in $(seq ${ROUNDS:-2}); do
            for v in cur ${vs//,/ }; do
                lib=gps-sdr-sim_amd/lib/libgpssim_amd.so
                [ "$v" != cur ] && lib=_var/$v/libgpssim_amd.so
                line=$(GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python bench.py \
                    --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-configs --no-e2e \
                    --no-cpu-baseline --no-exact --no-pmc --no-sustained --no-window 2>>$OUT/ablate.err | tail -1)
                step "ablate $v" $?
                echo "$v $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["stages_ms"]["fast_path"], d["value"])')" >> $OUT/ablate.log
            done
        done ;;
    clock:*)
        vs=${s#clock:}
        for r in $(seq ${ROUNDS:-2}); do
            for v in ${vs//,/ }; do
                GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=_var/$v/libgpssim_amd.so timeout -k 10 200 \
                    python tools/clock_stamp.py --label $v >> $OUT/clock.jsonl 2>>$OUT/clock.err
                step "clock $v" $?
            done
        done ;;
    prof)
        bash tools/profile.sh $TAG/prof
        step prof $? ;;
    e2eab:*)
        vs=${s#e2eab:}
        for r in $(seq ${ROUNDS:-2}); do
            for v in cur ${vs//,/ }; do
                lib=gps-sdr-sim_amd/lib/libgpssim_amd.so
                [ "$v" != cur ] && lib=_var/$v/libgpssim_amd.so
                line=$(GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 200 python bench.py \
                    --steps 1 --warmup 0 --no-cpu-baseline --no-exact --no-configs --no-pmc \
                    --no-sustained 2>>$OUT/e2eab.err | tail -1)
                step "e2eab $v" $?
                echo "$v $(echo "$line" | python3 -c 'import json,sys; d=json.load(sys.stdin)["e2e"]; print(d["value"], d["d2h_GBps"], d["frac_of_d2h_ceiling"], d.get("steady_frac_of_d2h_ceiling"))')" >> $OUT/e2eab.log
            done
        done ;;
    rehearse:*)
        a=${s#rehearse:}; n=${a%%:*}; t=""; [ "$a" != "$n" ] && t=_${a#*:}
        GSS_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
            --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $n \
            ${REHEARSE_ARGS:---steps 3 --warmup 1 --no-pmc} > $OUT/rehearse$n$t.json \
            2> $OUT/rehearse$n$t.err
        step "rehearse $n$t" $? ;;
    pmcclk:*)
        vs=${s#pmcclk:}
        BA="--steps 20 --warmup 5 --no-exact --no-configs --no-e2e --no-cpu-baseline --no-pmc --no-window"
        for v in cur ${vs//,/ }; do
            lib=gps-sdr-sim_amd/lib/libgpssim_amd.so
            [ "$v" != cur ] && lib=_var/$v/libgpssim_amd.so
            d=$OUT/pmcclk_$v
            mkdir -p $d
            GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace \
                --stats -d $d/kt -o kt -f csv -- python3 bench.py $BA > $d/kt.log 2>&1
            step "pmcclk kt $v" $?
            GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc \
                GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY \
                SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d $d/pmc -o pmc \
                -f csv -- python3 bench.py $BA > $d/pmc.log 2>&1
            step "pmcclk pmc $v" $?
            python3 tools/prof_summary.py $d 20 5 > $d/summary.json
        done ;;
    e2e:*)
        n=${s#e2e:}
        GSS_RUN_TRACE=1 timeout -k 10 200 python tools/e2e_cfg_probe.py $n > $OUT/e2e_cfg$n.out \
            2> $OUT/e2e_cfg$n.err
        step "e2e $n" $? ;;
    env:*)
        export "${s#env:}"
        step "env ${s#env:}" 0 ;;
    cmd:*)
        timeout -k 10 300 bash -c "${s#cmd:}" >> $OUT/cmd.log 2>&1
        step "cmd" $? ;;
    *)
        step "unknown step $s" 2 ;;
    esac
done
echo done >> $log
