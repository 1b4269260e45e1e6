#!/bin/bash
# round 4: k_shade load hoisting A/B (previous commit / no NEE prefetch / default), then the final
# checks on the current sources: the -m gpu suite, the default bench line, C2 PMC and kernel stats
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
H=libyafaray_amd/variants/head.so; N=libyafaray_amd/variants/nopref.so; C=libyafaray_amd/libyafaray4.so
ab c2_head $H --steps 5 && ab c2_nopref $N --steps 5 && ab c2_pref $C --steps 5 &&
ab c2_head2 $H --steps 5 && ab c2_pref2 $C --steps 5 &&
ab c4_head $H --scene sphere --steps 2 && ab c4_pref $C --scene sphere --steps 2 || exit 1
bash tools/gpu_r04_final1.sh
