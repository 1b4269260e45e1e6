# GPU box: new-feature parity tests (specular, textures), the full parity suite, the default bench.
# Test failures (pytest exit 1) do not stop the script; anything else (crash, timeout) does.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_specular.py tests/test_textures.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/new.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "new tests ended with $rc"; exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect tests/test_textures.py --deselect tests/test_specular.py > gpurun_out/p.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "parity suite ended with $rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
