# GPU box: exhaustive reciprocal check, parity suite on the fast-rcp + box-FMA variant, bench sweep.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 120 ./tools/rcp_check > gpurun_out/rcp_check.log 2>&1
YAFARAY_AMD_LIB=$R/libyafaray_amd/variants/both.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p_both.log 2>&1
bash tools/sweep.sh rcp base rcp boxfma both base both
