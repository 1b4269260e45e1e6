#!/bin/bash
# round 4: C4 / C2 A/B of non-temporal ray streams in k_trace (variants/ntload.so, -DYAF_NT_RAYLOAD=1)
# and a C4 chunk-size sweep (smaller chunks: less streaming traffic per launch beside the BVH in L2 / MALL)
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
N=libyafaray_amd/variants/ntload.so; C=libyafaray_amd/libyafaray4.so
ab c4_def $C --scene sphere --steps 2 && ab c4_nt $N --scene sphere --steps 2 && ab c4_def2 $C --scene sphere --steps 2 && ab c4_nt2 $N --scene sphere --steps 2 &&
ab c2_def $C --steps 5 && ab c2_nt $N --steps 5 &&
ab c4_ch24 $C --scene sphere --steps 2 --chunk 16777216 && ab c4_ch22 $C --scene sphere --steps 2 --chunk 4194304
