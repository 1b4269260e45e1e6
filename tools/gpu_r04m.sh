#!/bin/bash
# round 4: C4 traversal cost by the device BVH build's PLOC search radius (16 default, 32, 64)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
ab() {   # tag lib bench-args...
  local tag=$1 lib=$2; shift 2
  YAFARAY_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --warmup 1 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -3 gpurun_out/ab_$tag.log; return 1; }
  python3 - gpurun_out/ab_$tag.log $tag <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k = d['kernels']; tr = d.get('roofline', {}).get('traversal', {})
print(sys.argv[2], d['value'], d['ms_per_step'], {n: k[n]['ms'] for n in k if k[n]['ms'] > 5}, tr.get('node_visits_per_ray'), tr.get('tri_tests_per_ray'), d.get('build', {}).get('extra') if isinstance(d.get('build'), dict) else '')
P
}
V=libyafaray_amd/variants; C=libyafaray_amd/libyafaray4.so
ab r16 $C --scene sphere --steps 2 && ab r32 $V/ploc32.so --scene sphere --steps 2 && ab r64 $V/ploc64.so --scene sphere --steps 2 &&
ab r16b $C --scene sphere --steps 2 && ab r32b $V/ploc32.so --scene sphere --steps 2 && ab r64b $V/ploc64.so --scene sphere --steps 2
