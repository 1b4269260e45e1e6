"""GPU probe: diffuse-gather statistics of the C5 frame (accepted photons per request and log
overflows) for walk logs of 512 / 256 / 128 entries (k_gather split heap)."""
import os, sys
sys.path.insert(0, os.getcwd())
import libyafaray_amd as Y
from libyafaray_amd import scenes
spec = scenes.cornell_photon(1920, 1080, spp=1, photons=10_000_000)
for cap in ("512", "256", "128"):
    os.environ["YAFARAY_AMD_GATHER_LOG"] = cap
    _, _, st = Y.render_spec(spec)
    print(cap, {k: st[k] for k in st if k.startswith("gather")}, flush=True)
