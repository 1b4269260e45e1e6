# GPU box: parity suite, then one bench line per scene.  Usage: bash tools/gbench.sh [scene ...]
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/p.log 2>&1
for scene in "${@:-cornell}"; do
	timeout -k 10 ${BENCH_TIMEOUT:-200} python bench.py --no-cpu-baseline --scene $scene --steps 2 --warmup 1 ${BENCH_ARGS} > gpurun_out/bench_$scene.log 2>&1
done
