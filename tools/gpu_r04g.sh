#!/bin/bash
# round 4: k_level_partition items per thread (4 / 8 / 16) on C5; C4 LDS top treelet 21 vs 85 nodes
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pkd_gpu.py tests/test_photon.py tests/test_gather_walk.py tests/test_final_gather.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sel_tests.log; [ $rc -eq 0 ] || exit $rc
ab() {   # tag lib env bench-args...
  local tag=$1 lib=$2 env=$3; shift 3
  env $env YAFARAY_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --warmup 1 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -3 gpurun_out/ab_$tag.log; return 1; }
  python3 - gpurun_out/ab_$tag.log $tag <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k = d['kernels']
print(sys.argv[2], d['value'], d['ms_per_step'], {n: k[n]['ms'] for n in k if k[n]['ms'] > 0.5})
P
}
V=libyafaray_amd/variants; C=libyafaray_amd/libyafaray4.so
ab c5_head libyafaray_amd/variants/head.so X=0 --scene photon --steps 4 && ab c5_p8 $C X=0 --scene photon --steps 4 && ab c5_p4 $V/p4.so X=0 --scene photon --steps 4 && ab c5_p16 $V/p16.so X=0 --scene photon --steps 4 &&
ab c5_headb libyafaray_amd/variants/head.so X=0 --scene photon --steps 4 && ab c5_p8b $C X=0 --scene photon --steps 4 && ab c5_p4b $V/p4.so X=0 --scene photon --steps 4 && ab c5_p16b $V/p16.so X=0 --scene photon --steps 4 &&
ab c4_t21 $C YAFARAY_AMD_LDS_TOP=21 --scene sphere --steps 2 && ab c4_t85 $C YAFARAY_AMD_LDS_TOP=85 --scene sphere --steps 2 && ab c4_t5 $C YAFARAY_AMD_LDS_TOP=5 --scene sphere --steps 2
