#!/bin/bash
# round 4: camera rays with the default clip planes write no per-ray (tmin, tmax) — tests that
# exercise the camera queue, then C2 A/B against the previous commit's library (variants/head.so)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_specular.py tests/test_crop.py tests/test_film_io.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1
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
H=libyafaray_amd/variants/head.so; C=libyafaray_amd/libyafaray4.so
ab c2_head $H --steps 5 && ab c2_new $C --steps 5 && ab c2_head2 $H --steps 5 && ab c2_new2 $C --steps 5 && ab c2_head3 $H --steps 5 && ab c2_new3 $C --steps 5
