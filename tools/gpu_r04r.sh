#!/bin/bash
# round 4: C2 segment-count sweep (YAFARAY_AMD_SHADE_GRID: queue segments = k_shade / k_nee workgroups;
# the default is the resident grid, 3 x 256 CUs)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
ab() {   # tag env bench-args...
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --warmup 1 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -3 gpurun_out/ab_$tag.log; return 1; }
  python3 - gpurun_out/ab_$tag.log $tag <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k = d['kernels']
print(sys.argv[2], d['value'], d['ms_per_step'], {n: k[n]['ms'] for n in k if k[n]['ms'] > 0.5})
P
}
ab g768 X=0 --steps 5 && ab g512 YAFARAY_AMD_SHADE_GRID=512 --steps 5 && ab g1024 YAFARAY_AMD_SHADE_GRID=1024 --steps 5 &&
ab g1536 YAFARAY_AMD_SHADE_GRID=1536 --steps 5 && ab g768b X=0 --steps 5 && ab g1024b YAFARAY_AMD_SHADE_GRID=1024 --steps 5
