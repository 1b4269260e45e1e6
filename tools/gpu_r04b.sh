#!/bin/bash
# round 4: NEE request word packing — the multi-light / walk tests, then C2 A/B (8-B vs 16-B word)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multi_light.py tests/test_gather_walk.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1
rc=$?; tail -4 gpurun_out/sel_tests.log; [ $rc -eq 0 ] || exit $rc
for v in def pm16 def pm16; do
  if [ $v = pm16 ]; then E="YAFARAY_AMD_NEE_PM16=1"; else E="YAFARAY_AMD_X=0"; fi
  env $E timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --steps 5 --warmup 1 > gpurun_out/c2_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/c2_$v.log').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', d['value'], d['ms_per_step'], k['k_shade']['ms'], k['k_nee']['ms'], k['k_trace']['ms'])"
done
