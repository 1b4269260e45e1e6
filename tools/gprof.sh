# GPU box: kernel-trace stats of the bench command, then the PMC passes (one counter group per run,
# no trace domains) for k_trace's HBM traffic, then the bench line with that traffic.  TAG names outputs.
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --steps 3 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $B > $R/gpurun_out/prof_$TAG.log 2>&1
P="$R/bench.py --no-cpu-baseline --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcF_$TAG -o run -- python3 $P > $R/gpurun_out/pmcF_$TAG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcW_$TAG -o run -- python3 $P > $R/gpurun_out/pmcW_$TAG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/pmcV_$TAG -o run -- python3 $P > $R/gpurun_out/pmcV_$TAG.log 2>&1
cd $R
python3 tools/pmc_traffic.py gpurun_out/pmcF_$TAG/run_counter_collection.csv gpurun_out/pmcW_$TAG/run_counter_collection.csv \
	cornell-1920x1080x64-b8-rr1-chunk67108864 gpurun_out/trace_hbm_bytes_per_launch.json gpurun_out/pmcV_$TAG/run_counter_collection.csv
cp gpurun_out/trace_hbm_bytes_per_launch.json profiles/
timeout -k 10 240 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
