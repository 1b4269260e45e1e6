cd "${GRAFT_REPO_ROOT:-/root/repo}"
# C5 frame with the photon maps' records in kd order (default) against photon order
export BENCH_ARGS="--scene photon --steps 3"
export BENCH_TIMEOUT=200
bash tools/sweep.sh c5ab cur:YAFARAY_AMD_PKD_ORDER=photon:YAFARAY_AMD_GATHER_WALK=exact cur:YAFARAY_AMD_GATHER_WALK=exact cur cur:YAFARAY_AMD_GATHER_WALK=exact cur || exit $?
python3 - <<'P'
import json
for l in open('gpurun_out/sweep_c5ab.log'):
    if l.startswith('=='): print(l.strip(), end=' ')
    elif l.startswith('{'):
        d=json.loads(l); k=d['kernels']; print(d['ms_per_step'], {n: k[n]['ms'] for n in ('k_gather','k_gather_walk','pkd_build') if n in k})
P
