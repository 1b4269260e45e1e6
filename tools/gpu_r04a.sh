cd ${GRAFT_REPO_ROOT:-/root/repo} && bash tools/pmc_probe.sh > gpurun_out/pmc_probe_run.log 2>&1; rc=$?; tail -60 gpurun_out/pmc_probe_run.log; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_all.sh photon --scene photon
