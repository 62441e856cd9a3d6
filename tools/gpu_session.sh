#!/bin/bash
# GPU session: parity tests -> smoke -> bench -> rocprofv3 profile.  Each GPU step is time-
# limited; anything but a clean pass/ordinary test failure ends the session (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-s}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
log=gpurun_out/session_$TAG.log
echo "== $(date)" > $log
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -x -p no:cacheprovider ${PYTEST_ARGS} \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $log; ok $rc || exit $rc
[ -n "$SKIP_SMOKE" ] || { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $log; ok $rc || exit $rc; }
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 5 --warmup 1} > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc" >> $log; ok $rc || exit $rc
if [ -n "$CLI_RATE" ]; then bash tools/cli_rate.sh $TAG; rc=$?; echo "cli_rate rc=$rc" >> $log; ok $rc || exit $rc; fi
if [ -n "$PROFILE" ]; then bash tools/profile.sh $TAG; rc=$?; echo "profile rc=$rc" >> $log; fi
exit $rc
