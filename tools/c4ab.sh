cd "${GRAFT_REPO_ROOT:-/root/repo}"
export BENCH_ARGS="--scene sphere --steps 3"
export BENCH_TIMEOUT=200
bash tools/sweep.sh c4ab r03 cur:YAFARAY_AMD_LDS_TOP=0 cur:YAFARAY_AMD_LDS_TOP=21 r03 cur:YAFARAY_AMD_LDS_TOP=21 cur:YAFARAY_AMD_LDS_TOP=13 || exit $?
python3 - <<'P'
import json
for l in open('gpurun_out/sweep_c4ab.log'):
    if l.startswith('=='): print(l.strip(), end=' ')
    elif l.startswith('{'):
        d=json.loads(l); print(d['value'], d['kernels']['k_trace']['ms'])
P
