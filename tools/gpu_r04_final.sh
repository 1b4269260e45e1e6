#!/bin/bash
# round 4 final sources: PMC of C2 / C5 / C4 (bench.py's per-kernel traffic, keyed to these sources),
# the -m gpu suite, C2 kernel statistics and the default bench line
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
bash tools/pmc_all.sh cornell || exit 1
bash tools/pmc_all.sh photon --scene photon || exit 1
bash tools/pmc_all.sh sphere --scene sphere || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_stats.sh c2 --steps 3 > /dev/null || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
