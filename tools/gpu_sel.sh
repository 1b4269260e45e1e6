cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_multi_light.py tests/test_bench_group.py tests/test_device_group.py tests/test_photon_files.py tests/test_cabi.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_sel.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_sel.log
exit $rc
