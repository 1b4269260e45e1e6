set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t3.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/b3.log 2>&1
