#!/bin/bash
# C4 (Cornell + 1M-triangle sphere): k_trace's LDS top treelet size sweep (YAFARAY_AMD_LDS_TOP)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for top in ${TOPS:-0 21 5 85}; do
  YAFARAY_AMD_LDS_TOP=$top timeout -k 10 240 python -u bench.py --scene sphere --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/c4_top$top.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c4_top$top.log').read().strip().splitlines()[-1]); print('top', $top, d['value'], d['ms_per_step'], d['kernels']['k_trace']['ms'])"
done
