"""Cropped films ("xstart" / "ystart", imagefilm.cc:66, 129-132): the film covers the camera pixels
[xstart, xstart + width) x [ystart, ystart + height).  renderTile's loops run in camera coordinates
(imagesplitter.cc:43-46, integrator_tiled.cc:288-342: pixel offsets, sample positions and camera rays
of the camera pixel), addSample clips the splat footprint at the film's borders (imagefilm.cc:684-687)
and the callbacks report areas in camera coordinates (:462-467, :533) and pixels in film coordinates
(:527).

Checked: the oracle's crop equals the full render away from the crop's top / left border (whose
pixels miss the splats of the rows / columns outside the film); the GPU's crop equals the oracle's
(<= 4 ULP, weights equal), on one GPU and in a device group, and its callbacks carry camera-space
areas."""
import numpy as np
import pytest

from libyafaray_amd import scenes


def _crop(spec, w, h, x0, y0):
    return spec.with_render(width=w, height=h, xstart=x0, ystart=y0)


def _ulp(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7fffffff), a)
    b = np.where(b < 0, -(b & 0x7fffffff), b)
    return np.abs(a - b)


@pytest.mark.parametrize("filt", [("box", 1.0), ("gauss", 1.5)])
def test_oracle_crop_interior_equals_full_render(oracle_built, filt):
    full = scenes.cornell(96, 70, spp=2, bounces=3, rr=False, filter_type=filt[0], pixelwidth=filt[1])
    x0, y0, w, h = 20, 15, 40, 30
    a, wa, _ = oracle_built.OracleScene(full, threads=4).render()
    b, wb, _ = oracle_built.OracleScene(_crop(full, w, h, x0, y0), threads=4).render()
    assert b.shape == (h, w, 4)
    # forward-only footprints reach at most 1 px: rows / columns >= 1 of the crop get every splat
    sub, cut = a[y0 + 1:y0 + h, x0 + 1:x0 + w], b[1:, 1:]
    if filt[0] == "box":
        assert np.array_equal(sub.view(np.uint32), cut.view(np.uint32))
        assert np.array_equal(wa[y0 + 1:y0 + h, x0 + 1:x0 + w], wb[1:, 1:])
    else:
        # the crop's tiles start at its origin, so a pixel's splats arrive in another tile order: the
        # sums agree up to their order (the reference's own tile-order effect)
        assert _ulp(sub, cut).max() <= 8
        assert _ulp(wa[y0 + 1:y0 + h, x0 + 1:x0 + w], wb[1:, 1:]).max() <= 8
    if filt[0] == "gauss":
        # the gauss footprint always reaches the next pixel: the crop's first row / column lacks splats
        assert (wb[0, 1:] < wa[y0, x0 + 1:x0 + w]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["pt-box", "pt-gauss-rr-multipass", "dl-dof"])
@pytest.mark.parametrize("members", [None, 3])
def test_crop_matches_oracle(product, oracle_built, case, members):
    if case == "pt-box":
        spec = _crop(scenes.cornell(96, 70, spp=4, bounces=4, rr=False), 50, 37, 23, 11)
    elif case == "pt-gauss-rr-multipass":
        spec = _crop(scenes.cornell(80, 64, spp=2, bounces=3, rr=False, filter_type="gauss", pixelwidth=1.5), 44, 30, 9, 17).with_render(
            aa_passes=3, aa_inc_samples=2, aa_threshold=0.02)
    else:
        spec = _crop(scenes.test01(72, 72, spp=2), 40, 33, 16, 30).with_camera(aperture=0.12, dof_distance=3.8)
    rgba, w, _ = product.render_spec(spec, members=members, chunk_slots=4096)
    orgba, ow, _ = oracle_built.OracleScene(spec, threads=8).render()
    assert np.array_equal(w.view(np.uint32), ow.view(np.uint32))
    d = _ulp(rgba, orgba)
    assert d.max() <= 4, f"{(d > 4).sum()} values > 4 ULP"


@pytest.mark.gpu
def test_crop_callbacks_use_camera_areas(product):
    spec = _crop(scenes.cornell(96, 70, spp=1, bounces=2), 40, 30, 20, 15)
    spec.render.tile_size = 16
    spec.render.tiles_order = "linear"
    yi = product.Interface()
    scenes.apply(spec, yi)
    areas, px = [], set()
    yi.render(flush_area=lambda aid, x0, y0, x1, y1: areas.append((x0, y0, x1, y1)),
              put_pixel=lambda x, y, r, g, b, a: px.add((x, y)))
    yi.close()
    expect = [(20 + tx, 15 + ty, 20 + min(40, tx + 16), 15 + min(30, ty + 16)) for ty in range(0, 30, 16) for tx in range(0, 40, 16)]
    assert areas == expect
    assert px == {(x, y) for x in range(40) for y in range(30)}
