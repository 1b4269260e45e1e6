#!/bin/bash
# round 4: closest-ray queue as 12-B records — the -m gpu suite, then C2 / C4 A/B against the
# previous library (libyafaray_amd/variants/head.so, built from the previous commit)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
ab() {   # tag lib bench-args...
  local tag=$1 lib=$2; shift 2
  YAFARAY_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --warmup 1 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -3 gpurun_out/ab_$tag.log; return 1; }
  python3 - gpurun_out/ab_$tag.log $tag <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k = d['kernels']
print(sys.argv[2], d['value'], d['ms_per_step'], {n: k[n]['ms'] for n in k if k[n]['ms'] > 0.5})
P
}
H=libyafaray_amd/variants/head.so; C=libyafaray_amd/libyafaray4.so
ab c2_head $H --steps 5 && ab c2_new $C --steps 5 && ab c2_head2 $H --steps 5 && ab c2_new2 $C --steps 5 &&
ab c4_head $H --scene sphere --steps 2 && ab c4_new $C --scene sphere --steps 2
