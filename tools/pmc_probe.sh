#!/bin/bash
# GPU box: FETCH_SIZE of each calibration kernel of tools/pmc_probe.hip (one rocprofv3 --pmc run per
# kernel, counters only), then tools/pmc_calib.py -> gpurun_out/pmc_calibration.json
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
dirs=""
for k in k_stream16 k_node128 k_log8 k_scatter16 k_scatter16x3 k_node16; do
	timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcprobe_$k -o run -- $R/tools/pmc_probe $k \
		> $R/gpurun_out/pmcprobe_$k.log 2>&1 || { echo "probe $k failed ($?)"; tail -3 $R/gpurun_out/pmcprobe_$k.log; exit 1; }
	dirs="$dirs $R/gpurun_out/pmcprobe_$k"
done
cd $R && python3 tools/pmc_calib.py gpurun_out/pmc_calibration.json $dirs
