# Profiles for profiles/: kernel stats of the bench command + HBM traffic of k_trace (PMC passes)
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/prof_$TAG.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcF_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $R/gpurun_out/pmcF_$TAG.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcW_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $R/gpurun_out/pmcW_$TAG.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/pmcV_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $R/gpurun_out/pmcV_$TAG.log 2>&1
python3 $R/tools/pmc_traffic.py $R/gpurun_out/pmcF_$TAG/run_counter_collection.csv $R/gpurun_out/pmcW_$TAG/run_counter_collection.csv cornell-1920x1080x64-b8-rr1-chunk33554432 $R/gpurun_out/trace_hbm_bytes_per_launch.json $R/gpurun_out/pmcV_$TAG/run_counter_collection.csv
