#!/bin/bash
# round 4: C2 occupancy A/B — k_shade / k_nee at 5 waves per SIMD (variants/s5.so, n5.so) against the default 4
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
ab() {   # tag lib bench-args...
  local tag=$1 lib=$2; shift 2
  YAFARAY_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --warmup 1 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -3 gpurun_out/ab_$tag.log; return 1; }
  python3 - gpurun_out/ab_$tag.log $tag <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k = d['kernels']
print(sys.argv[2], d['value'], d['ms_per_step'], {n: k[n]['ms'] for n in k if k[n]['ms'] > 0.5})
P
}
V=libyafaray_amd/variants; C=libyafaray_amd/libyafaray4.so
ab c2_def $C --steps 5 && ab c2_s5 $V/s5.so --steps 5 && ab c2_n5 $V/n5.so --steps 5 &&
ab c2_def2 $C --steps 5 && ab c2_s52 $V/s5.so --steps 5 && ab c2_n52 $V/n5.so --steps 5
