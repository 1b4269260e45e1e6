"""Phase breakdown of k_shade (or, with YAFARAY_AMD_PATH=mega, k_path) — diagnostic build with -DYAF_PHASE_TIMING.

    YAFARAY_AMD_LIB=libyafaray_amd/variants/phase.so python tools/phase_probe.py [W H SPP]
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libyafaray_amd as Y  # noqa: E402
from libyafaray_amd import scenes  # noqa: E402

W, H, SPP = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (1920, 1080, 64)))
L = Y.lib()
L.yafaray_amd_getPhaseCycles.restype = C.c_int
L.yafaray_amd_getPhaseCycles.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()
spec = scenes.cornell(W, H, spp=SPP, bounces=8, rr=True)
Y.render_spec(spec)                      # warm-up
L.yafaray_amd_getPhaseCycles(buf, 16, 1)
_, _, st = Y.render_spec(spec)
n = L.yafaray_amd_getPhaseCycles(buf, 16, 1)
names = (["refill+camera", "trace", "connect+hit", "next-seg", "finalize+keep", "nee"] if os.environ.get("YAFARAY_AMD_PATH") == "mega"
         else ["load", "connect", "hit", "next-seg", "compact+write", "nee"])   # k_path / k_shade phases
tot = sum(buf[k] for k in range(6))
print(f"render {st['render_seconds'] * 1e3:.1f} ms; phase counters: {n}")
for k, nm in enumerate(names):
    print(f"  {nm:14s} {buf[k] / max(tot, 1) * 100:6.2f} %  ({buf[k]:.3e} wave-cycles)")
