#!/bin/bash
# GPU box, round 4: PMC calibration probes, then the A/B of this round's opt-in switches, then the
# rocprofv3 kernel stats of C2 / C4 / C5 / C5+FG.  Every GPU step has its own time limit; the script
# stops at the first failing step.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
set -o pipefail
bench1() {   # tag envs... -- bench args
	local tag=$1; shift
	local envs=()
	while [ "$1" != "--" ]; do envs+=("$1"); shift; done
	shift
	env "${envs[@]}" timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-parity --warmup 1 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -3 gpurun_out/ab_$tag.log; return 1; }
	python3 - gpurun_out/ab_$tag.log $tag <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d['kernels']
print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], {n: k[n]['ms'] for n in ('k_trace', 'k_shade', 'k_nee', 'k_gather', 'k_gather_walk', 'pkd_build') if n in k})
P
}
bash tools/pmc_probe.sh > gpurun_out/pmc_probe_run.log 2>&1 || { echo "pmc probe failed"; tail -5 gpurun_out/pmc_probe_run.log; exit 1; }
tail -40 gpurun_out/pmc_probe_run.log
bench1 c4_top0 YAFARAY_AMD_LDS_TOP=0 -- --scene sphere --steps 3 &&
bench1 c4_top21 YAFARAY_AMD_LDS_TOP=21 -- --scene sphere --steps 3 &&
bench1 c4_def -- --scene sphere --steps 3 &&
bench1 c5_photonorder_exact YAFARAY_AMD_PKD_ORDER=photon YAFARAY_AMD_GATHER_WALK=exact -- --scene photon --steps 3 &&
bench1 c5_exact YAFARAY_AMD_GATHER_WALK=exact -- --scene photon --steps 3 &&
bench1 c5_def -- --scene photon --steps 3 || exit 1
bash tools/refresh_profiles.sh stats
