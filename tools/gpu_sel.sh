#!/bin/bash
# GPU box: a selection of the -m gpu tests (args: pytest selection), log in gpurun_out/gpu_sel.log
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_sel.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_sel.log
exit $rc
