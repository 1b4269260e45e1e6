#!/bin/bash
# GPU box: refresh the committed profiles after a kernel-source change (bench.py only uses PMC
# traffic keyed to the current kernel source).  Usage: tools/refresh_profiles.sh pmc|stats
#   pmc   -> gpurun_out/pmc_<key>.json for C2, C4 and C5 (copy to profiles/)
#   stats -> gpurun_out/prof_{c2,c4,c5,c5fg}/ rocprofv3 kernel stats (summaries copied to profiles/)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
set -o pipefail
case "$1" in
pmc)
	bash tools/pmc_all.sh cornell && bash tools/pmc_all.sh sphere --scene sphere && bash tools/pmc_all.sh photon --scene photon
	;;
stats)
	bash tools/prof_stats.sh c2 --steps 3 && bash tools/prof_stats.sh c4 --scene sphere --steps 2 &&
		bash tools/prof_stats.sh c5 --scene photon --steps 3 && bash tools/prof_stats.sh c5fg --scene photon --fg 32 --steps 2
	;;
esac
