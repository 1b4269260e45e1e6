cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/refresh_profiles.sh stats || exit $?
timeout -k 10 300 python -u bench.py --scene sphere --steps 3 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --scene photon --steps 5 > gpurun_out/bench_c5.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --scene photon --fg 32 --steps 5 --no-cpu-baseline > gpurun_out/bench_c5fg.log 2>&1 || exit $?
