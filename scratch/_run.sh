cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_textures.py tests/test_cancel.py -m gpu -q -k "photon or cancel" --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1
rc=$?; echo "pytest $rc" >> gpurun_out/t3.log; tail -6 gpurun_out/t3.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --scene photon --no-cpu-baseline --no-parity > gpurun_out/bench_c5.log 2>&1; echo "bench $?"; tail -c 2500 gpurun_out/bench_c5.log
