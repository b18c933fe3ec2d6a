"""The primary-ray cull of the CPU-preset kernel (k_cull_ps / k_render_ps).

k_render_ps traces camera rays only against the triangles its pixel rectangle can
hit.  The cull is sound if no camera ray of the rectangle hits a culled triangle
under the reference's exact test (Ray::closest_intersection, CPU/rays/ray.cpp:14-28,
restated in oracle/).  CPU: the host build of the same cull (rt_rect_candidates)
against the oracle's primary hits.  GPU: the kernel's masks equal the host's.
"""
import ctypes

import numpy as np
import pytest

CAM = (0.0, 0.0, -3.0, 1.0)


def _scene(rtmi_mod, kind):
    if kind == "cornell":
        return rtmi_mod.cornell_geometry(0), CAM
    from conftest import MODELS
    import os
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, kind + ".obj"), kind)
    return g, rtmi_mod.CAMERAS[kind]


@pytest.mark.parametrize("kind,rule,yaw,size,rects", [
    ("cornell", 0, 0.0, 64, [(16, 1), (16, 4), (1, 1)]),
    ("cornell", 1, 0.0, 64, [(16, 1), (16, 4)]),
    ("cornell", 0, 0.3, 48, [(16, 1), (16, 4)]),
    ("archway", 0, 0.0, 48, [(16, 1), (16, 4)]),
    ("complex_light_room", 1, -0.2, 40, [(16, 4)]),
])
def test_cull_keeps_every_primary_hit(rtmi_mod, oracle_mod, kind, rule, yaw, size, rects):
    geom, cam_pos = _scene(rtmi_mod, kind)
    tri = geom.all_triangles()
    filt = rtmi_mod.filter_records(tri)
    p = rtmi_mod.default_params(0, width=size, height=size, spp=8, hit_rule=rule)
    cam = rtmi_mod.camera(cam_pos, yaw_y=yaw)
    ocam = oracle_mod.camera(cam_pos, yaw_y=yaw)
    op = oracle_mod.params_from(p)
    hits = oracle_mod.primary_hits(tri, geom.n_surf, geom.n_light, ocam, op, (0, 0, size, size), 0, 8)
    n_tri = tri.shape[0]
    for (rw, rh) in rects:
        kept = []
        for y0 in range(0, size, rh):
            for x0 in range(0, size, rw):
                x1, y1 = min(x0 + rw, size) - 1, min(y0 + rh, size) - 1
                m = rtmi_mod.rect_candidates(filt, cam, p, x0, y0, x1, y1)
                h = hits[y0:y1 + 1, x0:x1 + 1].ravel()
                h = h[h >= 0]
                assert m[h].all(), f"rect ({x0},{y0})-({x1},{y1}) culls a triangle a camera ray hits"
                kept.append(m.sum())
        # the cull must also cull: a camera ray sees a few triangles, not the scene
        assert np.mean(kept) < 0.6 * n_tri, (rw, rh, np.mean(kept), n_tri)


def test_cull_single_pixels_are_tight(rtmi_mod, oracle_mod):
    """At one pixel per wave (the bench's spp_split 64) the candidates are few."""
    geom, _ = _scene(rtmi_mod, "cornell")
    filt = rtmi_mod.filter_records(geom.all_triangles())
    p = rtmi_mod.default_params(0, width=512, height=512, spp=4)
    cam = rtmi_mod.camera(CAM)
    rng = np.random.default_rng(1)
    counts = [rtmi_mod.rect_candidates(filt, cam, p, x, y, x, y).sum()
              for x, y in rng.integers(0, 512, size=(200, 2))]
    assert np.mean(counts) <= 6.0, np.mean(counts)


@pytest.mark.gpu
@pytest.mark.parametrize("split,yaw,rule", [(1, 0.0, 0), (4, 0.2, 0), (64, 0.0, 1), (8, -0.1, 0)])
def test_device_cull_equals_host(rtmi_mod, gpu_ctx, split, yaw, rule):
    geom = rtmi_mod.cornell_geometry(0)
    filt = rtmi_mod.filter_records(geom.all_triangles())
    W = H = 48
    p = rtmi_mod.default_params(0, width=W, height=H, spp=64, spp_split=split, hit_rule=rule)
    cam = rtmi_mod.camera(CAM, yaw_y=yaw)
    rect = (0, 0, 40, 33)  # clipped 16x16 blocks
    nb = ((rect[2] + 15) // 16) * ((rect[3] + 15) // 16)
    n = nb * split * 4 * 4
    out = np.zeros(n, np.uint64)
    nw = ctypes.c_int64(n)
    with rtmi_mod.Scene(gpu_ctx, geom) as sc:
        rtmi_mod.api.check(rtmi_mod.lib().rt_cull_masks_device(
            gpu_ctx.handle, sc.handle, ctypes.byref(cam), ctypes.byref(p), *rect,
            out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), ctypes.byref(nw)))
    assert nw.value == n
    out = out.reshape(nb, split, 4, 4)
    lg = split.bit_length() - 1
    bi = 0
    for by in range(0, rect[3], 16):
        for bx in range(0, rect[2], 16):
            for part in range(split):
                for w in range(4):
                    q = (part << (8 - lg)) + ((np.arange(64) + 64 * w) >> lg)
                    px, py = bx + (q & 15), by + (q >> 4)
                    ok = (px < rect[2]) & (py < rect[3])
                    got = out[bi, part, w]
                    if not ok.any():
                        assert not got.any()
                        continue
                    m = rtmi_mod.rect_candidates(filt, cam, p, px[ok].min(), py[ok].min(), px[ok].max(),
                                                 py[ok].max())
                    # all 256 bits: the kept triangles and nothing past the scene
                    want = np.zeros(256, bool)
                    want[:m.size] = m
                    bits = np.unpackbits(got.view(np.uint8), bitorder="little").astype(bool)
                    assert np.array_equal(bits, want), (bx, by, part, w)
            bi += 1
