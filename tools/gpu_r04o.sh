#!/bin/bash
# round 4: k_shade's record loads in one round trip — tests, then C2 / C4 A/B: previous commit
# (variants/head.so), hoisted loads without (variants/nopref.so) and with the NEE-slot prefetch (default)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_specular.py tests/test_caustics.py tests/test_multi_light.py tests/test_transparent_shadows.py tests/test_materials_ext.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1
rc=$?; tail -2 gpurun_out/sel_tests.log; [ $rc -eq 0 ] || exit $rc
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
ab c2_head2 $H --steps 5 && ab c2_nopref2 $N --steps 5 && ab c2_pref2 $C --steps 5 &&
ab c4_head $H --scene sphere --steps 2 && ab c4_pref $C --scene sphere --steps 2
