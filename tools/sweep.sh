# Run the bench once per variant (GPU box).  Usage: bash tools/sweep.sh TAG spec1 spec2 ...
#   spec = <variant .so name>[:VAR=value[:VAR=value...]]   (env overrides, e.g. YAFARAY_AMD_TRACE_GRID)
set -e
R=$GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p $R/gpurun_out
for spec in "$@"; do
	IFS=: read -r v rest <<< "$spec"
	echo "== $spec" >> $R/gpurun_out/sweep_$TAG.log
	envs=()
	if [ -n "$rest" ]; then IFS=: read -ra envs <<< "$rest"; fi
	env "${envs[@]}" YAFARAY_AMD_LIB=$R/libyafaray_amd/variants/$v.so timeout -k 10 ${BENCH_TIMEOUT:-150} python $R/bench.py --no-cpu-baseline --no-parity --steps 2 --warmup 1 ${BENCH_ARGS} >> $R/gpurun_out/sweep_$TAG.log 2>&1
done
