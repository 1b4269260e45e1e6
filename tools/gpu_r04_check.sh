#!/bin/bash
# round 4 end: smoke() and the default bench line on the committed tree
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
python3 - <<'P'
import json
d = json.loads([l for l in open('gpurun_out/bench_default.log') if l.startswith('{"metric"')][-1])
r = d['roofline']
print(d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['traffic'], d['parity']['rr_off_bitexact']['bit_identical'], d['parity']['band']['pass'])
P
