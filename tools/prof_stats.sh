#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats of one bench configuration.
#   tools/prof_stats.sh TAG [bench args...]   -> gpurun_out/prof_TAG/run_kernel_stats.csv + .log
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
	python3 $R/bench.py --no-cpu-baseline --no-parity "$@" > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?
tail -2 $R/gpurun_out/prof_$TAG.log
[ -f $R/gpurun_out/prof_$TAG/run_kernel_stats.csv ] && python3 $R/tools/prof_summary.py $R/gpurun_out/prof_$TAG/run_kernel_stats.csv 
exit $rc
