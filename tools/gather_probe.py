"""C5 gather probe: per-request walk statistics and kernel times of the one-pass and two-pass
diffuse gather (YAFARAY_AMD_GATHER=single | walk; YAFARAY_AMD_GATHER_WALK=exact | bound).  python tools/gather_probe.py [photons] [W H]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libyafaray_amd as Y  # noqa: E402
from libyafaray_amd import scenes  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
spec = scenes.cornell_photon(W, H, spp=1, photons=n)
for mode, walk, cap in (("single", "-", 512), ("walk", "exact", 512), ("walk", "bound", 512), ("walk", "exact", 512), ("walk", "bound", 512)):
    os.environ["YAFARAY_AMD_GATHER"] = mode
    os.environ["YAFARAY_AMD_GATHER_WALK"] = walk
    os.environ["YAFARAY_AMD_GATHER_LOG"] = str(cap)
    _, _, st = Y.render_spec(spec, profile=True)
    q = max(1, st["gather_queries"])
    kt = st["kernel_times"]
    print(f"{mode:6s} {walk:5s} cap {cap:5d} queries {q} visits/q {st['gather_visits'] / q:.1f} accepts/q {st['gather_accepts'] / q:.1f} "
          f"photons/q {st['gather_photons'] / q:.1f} overflows {st['gather_overflows']} | "
          + " ".join(f"{k} {v['ms']:.2f}" for k, v in kt.items() if k.startswith("k_gather")), flush=True)
