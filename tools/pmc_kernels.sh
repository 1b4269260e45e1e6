# PMC passes (counters only, no trace domains) over a short bench; TAG names the output dirs.
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
shift || true
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/pmcA_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > $R/gpurun_out/pmcA_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmcB_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > $R/gpurun_out/pmcB_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/pmcC_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > $R/gpurun_out/pmcC_$TAG.log 2>&1
