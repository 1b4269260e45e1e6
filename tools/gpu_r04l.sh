#!/bin/bash
# round 4: C4 traversal cost by BVH builder — the device PLOC build (default for >= 64 K triangles)
# against the host binned-SAH build with several leaf sizes / node costs (frame time excludes the build)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
ab() {   # tag env bench-args...
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --warmup 1 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -3 gpurun_out/ab_$tag.log; return 1; }
  python3 - gpurun_out/ab_$tag.log $tag <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k = d['kernels']; tr = d.get('roofline', {}).get('traversal', {})
print(sys.argv[2], d['value'], d['ms_per_step'], {n: k[n]['ms'] for n in k if k[n]['ms'] > 5}, tr.get('node_visits_per_ray'), tr.get('tri_tests_per_ray'))
P
}
ab c4_gpu X=0 --scene sphere --steps 2 && ab c4_host YAFARAY_AMD_BVH_BUILD=host --scene sphere --steps 2 &&
ab c4_host_l2 "YAFARAY_AMD_BVH_BUILD=host YAFARAY_AMD_BVH_LEAF=2" --scene sphere --steps 2 &&
ab c4_host_l4 "YAFARAY_AMD_BVH_BUILD=host YAFARAY_AMD_BVH_LEAF=4" --scene sphere --steps 2 &&
ab c4_gpu2 X=0 --scene sphere --steps 2
