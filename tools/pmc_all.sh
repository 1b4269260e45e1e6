#!/bin/bash
# GPU box: per-kernel PMC of one bench frame (each counter group in its own rocprofv3 run, counters
# only — no trace domains), aggregated into profiles/pmc_<CONFIG>.json for bench.py's per-kernel
# roofline.   tools/pmc_all.sh CONFIG [bench args...]
R=${GRAFT_REPO_ROOT:-/root/repo}
CFG=$1; shift
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-parity --steps 1 --warmup 0 $*"
dirs=""
run() {   # name counters...
	local name=$1; shift
	timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmc_${CFG}_$name -o run -- $B \
		> $R/gpurun_out/pmc_${CFG}_$name.log 2>&1 || { echo "pass $name failed ($?)"; tail -3 $R/gpurun_out/pmc_${CFG}_$name.log; exit 1; }
	dirs="$dirs $R/gpurun_out/pmc_${CFG}_$name"
}
run F FETCH_SIZE
run W WRITE_SIZE
run R TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
run A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run B SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS
run D TCC_HIT_sum TCC_MISS_sum
run C SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT
# key the file the way bench.py's load_pmc() looks it up (workload + kernel source)
KEY=$(cd $R && python3 -c "import sys; sys.argv=['bench.py']+sys.argv[1:]; import bench; a=bench.parse(); a.spp=a.spp or (1 if a.scene=='photon' else 64); print(bench.pmc_config(a, a.width, a.height))" "$@")
cd $R && python3 tools/pmc_aggregate.py $KEY gpurun_out/pmc_$KEY.json $dirs > /dev/null && echo "wrote gpurun_out/pmc_$KEY.json (copy to profiles/)"
