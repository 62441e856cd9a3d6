#!/bin/bash
# The host side under the sanitizers (CPU only), once with -fsanitize=thread and
# once with -fsanitize=address,undefined; any sanitizer report, row or byte mismatch fails.
#  * gss_run itself (gps-sdr-sim_amd/csrc/hip/gss_run.hip, unchanged: its planner, rows and
#    prover threads, slot state machine, buffer pool, uploads, streams and events) built against
#    the CPU stand-in of the HIP runtime (tests/helpers/fake_hip) and the CPU fakes of its device
#    functions (tests/helpers/fake_dev.cpp), driven through every mode of the run by
#    tests/helpers/run_fake.cpp, which checks every byte the sink gets against independently
#    produced rows;
#  * the host plane alone (scenario, chains, proofs, worker pools, the CLI parser) in
#    tests/helpers/run_harness.c's arrangement of the same threads.
# Logs go to $OUT (default profiles/round5/sanitize).  FAKE_ARGS: the run_fake argument sets
# (";"-separated "seconds batch fmt"), SECS: run_harness's long run, HARNESS_ARGS its second.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-profiles/round5/sanitize}
SECS=${SECS:-300}
mkdir -p $OUT /tmp/gss_san
SRC="gps-sdr-sim_amd/csrc/host/*.c gps-sdr-sim_amd/csrc/cli/cli_args.c tests/helpers/run_harness.c"
CF="-O1 -g -fno-omit-frame-pointer -ffp-contract=off -fno-fast-math -D_FILE_OFFSET_BITS=64 -Iinclude"
NAV=tests/golden/data/brdc3540.14n
rc=0
FK="tests/helpers/fake_hip/fake_hip.cpp tests/helpers/fake_dev.cpp tests/helpers/run_fake.cpp"
# one object per source, built in parallel (each a background job, every status checked)
build() {  # san dir
    local san=$1 d=$2 pids=() f
    for f in gps-sdr-sim_amd/csrc/host/*.c gps-sdr-sim_amd/csrc/cli/cli_args.c \
             tests/helpers/run_harness.c; do
        gcc $CF -fsanitize=$san -c $f -o $d/$(basename ${f%.c}).o & pids+=($!)
    done
    g++ -std=c++17 $CF -Itests/helpers -Itests/helpers/fake_hip -fsanitize=$san -x c++ \
        -c gps-sdr-sim_amd/csrc/hip/gss_run.hip -o $d/gss_run.o & pids+=($!)
    for f in $FK; do
        g++ -std=c++17 $CF -Itests/helpers -Itests/helpers/fake_hip -fsanitize=$san -c $f \
            -o $d/$(basename ${f%.cpp}).o & pids+=($!)
    done
    local bad=0
    for p in "${pids[@]}"; do wait $p || bad=1; done
    return $bad
}
for san in thread address,undefined; do
    tag=${san%%,*}
    # gss_run on the fake device: C host sources by gcc, the C++ ones by g++
    d=/tmp/gss_san/fake_$tag
    rm -rf $d
    mkdir -p $d
    build $san $d || exit 1
    host_objs=$(ls $d/*.o | grep -v -e '/gss_run.o$' -e '/fake_hip.o$' -e '/fake_dev.o$' \
                -e '/run_fake.o$' -e '/run_harness.o$')
    g++ -fsanitize=$san -o $d/run_fake $host_objs $d/gss_run.o $d/fake_hip.o $d/fake_dev.o \
        $d/run_fake.o -lm -lpthread || exit 1
    IFS=';' read -ra fargs <<< "${FAKE_ARGS:-70 64 1;40 16 8;300 512 1}"
    for args in "${fargs[@]}"; do
        log=$OUT/gss_run_${tag}_$(echo $args | tr ' ' _).log
        echo "== -fsanitize=$san, gss_run on the fake device: run_fake $args" > $log
        TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" \
        ASAN_OPTIONS="detect_leaks=1 halt_on_error=1" UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1" \
            timeout -k 10 1800 $d/run_fake $NAV $args >> $log 2>&1
        r=$?
        echo "exit $r" >> $log
        grep -c "WARNING: ThreadSanitizer\|ERROR: AddressSanitizer\|runtime error\|LeakSanitizer" $log \
            | sed 's/^/sanitizer reports: /' >> $log
        tail -3 $log
        [ $r -eq 0 ] || rc=1
    done
    exe=/tmp/gss_san/run_harness_$tag
    gcc -fsanitize=$san -o $exe $host_objs $d/run_harness.o -lm -lpthread || exit 1
    for args in "$SECS 512 1" "${HARNESS_ARGS:-60 64 16}"; do
        log=$OUT/${tag}_$(echo $args | tr ' ' _).log
        echo "== gcc -fsanitize=$san, run_harness $args" > $log
        TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" \
        ASAN_OPTIONS="detect_leaks=1 halt_on_error=1" UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1" \
            timeout -k 10 1200 $exe $NAV $args >> $log 2>&1
        r=$?
        echo "exit $r" >> $log
        grep -c "WARNING: ThreadSanitizer\|ERROR: AddressSanitizer\|runtime error\|LeakSanitizer" $log \
            | sed 's/^/sanitizer reports: /' >> $log
        tail -3 $log
        [ $r -eq 0 ] || rc=1
    done
done
exit $rc
