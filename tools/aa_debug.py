"""Debug: diagonal forward splats in adaptive passes (run on the GPU box)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import libyafaray_amd as product
from libyafaray_amd import scenes
from oracle import oracle

for name, spec in {
    "thr0": scenes.cornell(48, 40, spp=5, bounces=2, rr=False).with_render(aa_passes=2, aa_threshold=0.0, aa_inc_samples=2),
    "thr0.01": scenes.cornell(48, 40, spp=5, bounces=2, rr=False).with_render(aa_passes=2, aa_threshold=0.01, aa_inc_samples=2),
    "thr0-gauss": scenes.cornell(48, 40, spp=5, bounces=2, rr=False, filter_type="gauss", pixelwidth=1.5).with_render(aa_passes=2, aa_threshold=0.0, aa_inc_samples=2),
}.items():
    rgba, w, st = product.render_spec(spec, chunk_slots=1 << 20)
    orgba, ow, _ = oracle.OracleScene(spec, threads=8).render()
    bad = np.argwhere(w != ow)
    print(name, "samples", st["samples"], "mismatch", len(bad), [(int(y), int(x), float(w[y, x]), float(ow[y, x])) for y, x in bad[:6]])
