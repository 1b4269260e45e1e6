"""Render callbacks through the Python binding (libyafaray_amd.Interface.render): the library keeps the
registered pointers between renders (as the reference's yafaray_setRender*Callback do), so a render that
passes no callback after one that did must not call the previous render's (released) ctypes thunk."""
import numpy as np
import pytest

import libyafaray_amd as Y
from libyafaray_amd import scenes


@pytest.mark.gpu
def test_render_without_callbacks_after_one_with_them(product):
    spec = scenes.cornell(64, 48, spp=1)
    yi = Y.Interface()
    scenes.apply(spec, yi)
    flushed, areas = [], []
    yi.render(flush=lambda: flushed.append(1), flush_area=lambda *a: areas.append(a))
    assert flushed and areas
    n_flush, n_areas = len(flushed), len(areas)
    yi.render()                                     # no callbacks: nothing may be called
    assert len(flushed) == n_flush and len(areas) == n_areas
    yi.render(flush=lambda: flushed.append(2))      # a new one is called
    assert flushed[-1] == 2
    rgba, w = yi.film()
    assert np.isfinite(rgba).all() and (w > 0).all()
    yi.close()
