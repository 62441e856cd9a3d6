#!/bin/bash
# The host plane under the sanitizers (CPU only): the C sources of
# gps-sdr-sim_amd/csrc/host (scenario, chains, proofs, worker pools) and the CLI parser, linked
# with tests/helpers/run_harness.c -- gss_run's rows / planner / prover threads on their own
# pools, walks by gss_spec_host -- once with -fsanitize=thread and once with
# -fsanitize=address,undefined.  Any sanitizer report or row mismatch fails.  Logs go to $OUT
# (default profiles/round4/sanitize).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-profiles/round4/sanitize}
SECS=${SECS:-300}
mkdir -p $OUT /tmp/gss_san
SRC="gps-sdr-sim_amd/csrc/host/*.c gps-sdr-sim_amd/csrc/cli/cli_args.c tests/helpers/run_harness.c"
CF="-O1 -g -fno-omit-frame-pointer -ffp-contract=off -fno-fast-math -D_FILE_OFFSET_BITS=64 -Iinclude"
NAV=tests/golden/data/brdc3540.14n
rc=0
for san in thread address,undefined; do
    tag=${san%%,*}
    exe=/tmp/gss_san/run_harness_$tag
    gcc $CF -fsanitize=$san $SRC -o $exe -lm -lpthread || exit 1
    for args in "$SECS 512 1" "60 64 16"; do
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
