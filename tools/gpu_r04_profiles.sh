#!/bin/bash
# round 4 final profiles: rocprofv3 kernel stats (C2 / C4 / C5 / C5+FG) and the per-kernel PMC passes
# (C2 / C4 / C5, incl. the sized read-request pass), all on the committed kernel sources
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
bash tools/refresh_profiles.sh stats > gpurun_out/r04_stats.log 2>&1 || { echo "stats failed"; tail -5 gpurun_out/r04_stats.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r04_stats.log | grep -v '^{' | head -40
bash tools/refresh_profiles.sh pmc > gpurun_out/r04_pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/r04_pmc.log; exit 1; }
tail -5 gpurun_out/r04_pmc.log
