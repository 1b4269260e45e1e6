"""k_trace with and without per-visit statistics (yafaray_amd_setTraceStats; bench.py renders its
timed frames without them).  The STATS = false variants skip the node / triangle counters but still
count the rays they trace (per wave, by ballot): the image is bit-identical and the closest / shadow
ray counts equal the counting variant's.  Covered for the LDS-resident BVH4 scene (C2's variant),
BVH2, the Cornell box kept in global memory, and the C4 sphere mesh (the refill loop's counters)."""
import numpy as np
import pytest

from libyafaray_amd import scenes

pytestmark = pytest.mark.gpu

VARIANTS = {
    "lds-bvh4": ({"YAFARAY_AMD_TRACE": "bvh"}, lambda: scenes.cornell(64, 48, spp=4, bounces=4)),
    "lds-bvh2": ({"YAFARAY_AMD_TRACE": "bvh", "YAFARAY_AMD_BVH_WIDTH": "2"}, lambda: scenes.cornell(64, 48, spp=4, bounces=4)),
    "global-bvh4": ({"YAFARAY_AMD_TRACE": "bvh", "YAFARAY_AMD_SCENE_LDS": "0"}, lambda: scenes.cornell(64, 48, spp=4, bounces=4)),
    "sphere-mesh": ({"YAFARAY_AMD_TRACE": "bvh"}, lambda: scenes.cornell_sphere(width=64, height=48, spp=2, bounces=4)),
}


def render(product, spec, stats_on):
    yi = product.Interface()
    scenes.apply(spec, yi)
    yi.L.yafaray_amd_setTraceStats(yi.h, 1 if stats_on else 0)
    yi.render()
    rgba, w = yi.film()
    st = yi.stats()
    yi.close()
    return rgba, w, st


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_trace_without_stats_counts_the_same_rays(product, variant, monkeypatch):
    env, make = VARIANTS[variant]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    spec = make()
    a, wa, sa = render(product, spec, True)
    b, wb, sb = render(product, spec, False)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(wa, wb)
    assert sa["closest_rays"] == sb["closest_rays"] > 0
    assert sa["shadow_rays"] == sb["shadow_rays"] > 0
    assert sa["node_visits"] > 0
