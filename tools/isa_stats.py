"""Instruction mix per kernel from a gfx950 assembly listing: python tools/isa_stats.py file.s"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
parts = re.split(r'\n(_Z[\w]+):\s*(?:;[^\n]*)?\n', s)
for i in range(1, len(parts), 2):
    name, body = parts[i], parts[i + 1].split('.Lfunc_end')[0]
    ins = [l.strip().split()[0] for l in body.splitlines() if l.startswith('\t') and l.strip() and not l.strip().startswith(('.', ';'))]
    c = collections.Counter(ins)
    if len(ins) < 100:
        continue
    f = lambda pred: sum(v for k, v in c.items() if pred(k))
    print(f"{name[:44]:44s} n={len(ins):6d} f64={f(lambda k: 'f64' in k):5d} barrier={c['s_barrier']:3d} "
          f"div={f(lambda k: 'div_scale' in k) // 2:4d} lane={f(lambda k: 'lane_b32' in k):5d} "
          f"gload={f(lambda k: k.startswith('global_load')):4d} gstore={f(lambda k: k.startswith('global_store')):4d} "
          f"swap/call={f(lambda k: 's_swappc' in k or 's_setpc' in k):3d}")
