# BVH4 vs BVH2 on the GPU box: parity suite (all BVH variants), then bench both widths on C2 and C4.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/bvh4_pytest.log 2>&1
for spec in "cornell:4" "cornell:2" "sphere:4" "sphere:2" ${EXTRA_SPECS}; do
	IFS=: read -r scene w lds <<< "$spec"
	echo "== $spec" >> gpurun_out/bvh4_bench.log
	YAFARAY_AMD_LDS_STACK=${lds:-} YAFARAY_AMD_BVH_WIDTH=$w timeout -k 10 200 python bench.py --no-cpu-baseline --scene $scene --steps 2 --warmup 1 >> gpurun_out/bvh4_bench.log 2>&1
done
