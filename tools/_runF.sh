# round-end refresh after tools/_runB.sh (PMC): rocprof stats + bench lines, multi-light, 8 members,
# meshlight, then the GPU suite and the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/_runC.sh || exit $?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
AB_TIMEOUT=300 bash tools/ab.sh 'ml2||--lights 2 --steps 5' 'ml2hash|YAFARAY_AMD_LIGHT_PICK=hash|--lights 2 --steps 5' 'ml2count|YAFARAY_AMD_LIGHT_PICK=count|--lights 2 --steps 5' 'ml3||--lights 3 --steps 5' 'ml3hash|YAFARAY_AMD_LIGHT_PICK=hash|--lights 3 --steps 5' 'ml3count|YAFARAY_AMD_LIGHT_PICK=count|--lights 3 --steps 5' || exit $?
timeout -k 10 300 python -u bench.py --members-per-gpu 8 --steps 3 --no-cpu-baseline > gpurun_out/bench_members8.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --scene meshlight --steps 3 --no-cpu-baseline > gpurun_out/bench_meshlight.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/pkd_member_probe.py > gpurun_out/pkd_members.md 2>&1 || exit $?
cat gpurun_out/pkd_members.md
bash tools/_runA.sh
