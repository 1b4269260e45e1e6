#!/bin/bash
# One GPU: the C2 frame with K device-group members on the one device (each member its own host
# thread and HIP stream over a band of rows): does stream concurrency overlap the VALU-bound
# traversal with the memory-bound shading?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for k in ${KS:-1 2 3 4}; do
  timeout -k 10 240 python -u bench.py --members-per-gpu $k --steps 3 --warmup 1 --no-cpu-baseline --no-parity $BARGS > gpurun_out/members_$k.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/members_$k.log').read().strip().splitlines()[-1]); print('members', $k, d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
