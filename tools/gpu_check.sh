#!/bin/bash
# GPU box check: the -m gpu suite, then (only if pytest ended normally: all passed or some tests
# failed) one default bench run.  Usage: tools/gpu_check.sh [pytest selection args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/gpu_tests.log
tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc2=$?
tail -3 gpurun_out/bench.log
exit $rc2
