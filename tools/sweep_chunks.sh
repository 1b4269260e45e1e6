set -e
R=$GRAFT_REPO_ROOT
for c in ${CHUNKS:-4194304 8388608 16777216 33554432}; do
  echo "== chunk $c" >> $R/gpurun_out/sweep_${TAG:-c2}.log
  YAFARAY_AMD_LIB=$R/libyafaray_amd/variants/base.so timeout -k 10 300 python $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --chunk $c >> $R/gpurun_out/sweep_${TAG:-c2}.log 2>&1
done
