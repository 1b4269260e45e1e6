#!/bin/bash
# GPU box: what the L2's read counters report for each calibration kernel of tools/pmc_probe.hip, against
# byte counts known by construction.  Two rocprofv3 --pmc runs per kernel (counters only): FETCH_SIZE,
# then the fabric read requests by size (TCC_EA0_RDREQ_32B / _64B / _128B); tools/pmc_calib.py ->
# gpurun_out/pmc_calibration.json (copied to profiles/).
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
dirs=""
for k in k_stream16 k_node128 k_log8 k_scatter16 k_scatter16x3 k_node16; do
	timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcprobe_$k -o run -- $R/tools/pmc_probe $k \
		> $R/gpurun_out/pmcprobe_$k.log 2>&1 || { echo "probe $k failed ($?)"; tail -3 $R/gpurun_out/pmcprobe_$k.log; exit 1; }
	timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv \
		-d $R/gpurun_out/pmcprobe_$k/req -o run -- $R/tools/pmc_probe $k \
		> $R/gpurun_out/pmcprobe_${k}_req.log 2>&1 || { echo "probe $k (requests) failed ($?)"; tail -3 $R/gpurun_out/pmcprobe_${k}_req.log; exit 1; }
	dirs="$dirs $R/gpurun_out/pmcprobe_$k"
done
cd $R && python3 tools/pmc_calib.py gpurun_out/pmc_calibration.json $dirs
