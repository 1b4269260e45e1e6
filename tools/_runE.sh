cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/_runA.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/prof_stats.sh c2 --steps 3 | tail -3 || exit $?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u bench.py --members-per-gpu 8 --steps 3 --no-cpu-baseline > gpurun_out/bench_members8.log 2>&1 || exit $?
tail -c 200 gpurun_out/bench_members8.log
exit $rc
