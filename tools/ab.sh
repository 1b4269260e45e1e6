#!/bin/bash
# GPU box: a list of bench.py runs, one summary line each (Msamples/s, ms per frame, kernel ms).
#
#   bash tools/ab.sh 'tag|ENV=v ENV2=w|bench args' ['tag2||bench args' ...]
#
# Each run has its own time limit (AB_TIMEOUT, default 240 s) and writes gpurun_out/ab_<tag>.log;
# the script stops at the first failing run (no retries).  Summaries are appended to
# gpurun_out/ab_summary.txt.  This replaces the per-attempt scripts of earlier rounds: the
# commands behind a number in DESIGN.md are the ab.sh argument lists quoted next to it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
set -o pipefail
for spec in "$@"; do
	IFS='|' read -r tag envs args <<< "$spec"
	# shellcheck disable=SC2086
	env $envs timeout -k 10 "${AB_TIMEOUT:-240}" python -u bench.py --no-cpu-baseline --no-parity --warmup 1 $args > "gpurun_out/ab_$tag.log" 2>&1 ||
		{ echo "run $tag failed (rc $?)"; tail -5 "gpurun_out/ab_$tag.log"; exit 1; }
	python3 - "gpurun_out/ab_$tag.log" "$tag" <<'P' | tee -a gpurun_out/ab_summary.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], d["value"], d["unit"], d["ms_per_step"], {n: k[n]["ms"] for n in k if k[n]["ms"] > 0.3})
P
done
