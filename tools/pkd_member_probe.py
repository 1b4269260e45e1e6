"""GPU box: the distributed point kd-tree build's per-member device time (yafaray_amd_buildPhotonTreeMember)
at C5 map size — every member of a W-member group runs its own share; here each share is run alone on one GPU,
so the time is what each member of a W-GPU group spends building (the exchange of the subtrees' ranges
comes on top: xGMI peer copies / RCCL broadcasts of 68 B per photon received).

    python tools/pkd_member_probe.py [n [members ...]] > gpurun_out/pkd_members.md"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import libyafaray_amd as Y  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 19_600_000
rng = np.random.default_rng(3)
pos = (rng.random((n, 3), dtype=np.float32) * np.float32(4) - np.float32(2))
print(f"# distributed point kd-tree build, {n} photons (uniform in a cube), device ms per member (second of two builds)\n")
print("| members | split level | member ms (each) | max | whole build / max |")
print("|---|---|---|---|---|")
whole = None
for w in [int(a) for a in sys.argv[2:]] or (1, 2, 4, 8):
    ms, lvl = [], 0
    for r in range(w):
        _, _, _, lvl, t = Y.build_photon_tree_member(pos, r, w)
        ms.append(t)
    if w == 1:
        whole = ms[0]
    print(f"| {w} | {lvl} | {', '.join(f'{t:.2f}' for t in ms)} | {max(ms):.2f} | {(f'{whole / max(ms):.2f}' if whole else '-')} |", flush=True)
