# GPU box: parity suite on the default build, then an occupancy sweep (k_shade / k_nee min waves) and C4.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p_def.log 2>&1
bash tools/sweep.sh occ base s4 n4 sn4 base s4 sn4
BENCH_ARGS="--scene sphere" BENCH_TIMEOUT=200 bash tools/sweep.sh occ_sphere base s4
