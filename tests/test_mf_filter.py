"""The matrix-core filter of the bounce casts (rt_trace.hpp closest_hit_mf, k_render_ps).

It may only skip a triangle the exact test must reject, so its hits are the reference's
bit for bit: checked here through rt_intersect_method(RT_ISECT_MFMA) against the CPU
restatement on rays from surface points (what k_render_ps casts), rays aimed at triangle
edges and vertices (the pairs nearest the filter's margins), random rays, and rays it
must hand to the exact test whole (non-finite, origin outside the scene's box + 1).
The render parity of k_render_ps itself is in test_gpu_parity.py / test_cull.py.
"""
import os

import numpy as np
import pytest

from conftest import MODELS

pytestmark = pytest.mark.gpu

SCENES = ["cornell_cpu", "door_room", "archway", "complex_light_room"]


def _geom(rtmi, kind):
    if kind == "cornell_cpu":
        return rtmi.cornell_geometry(0)
    return rtmi.obj_geometry(os.path.join(MODELS, f"{kind}.obj"), kind)


def _unit(v):
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def surface_rays(tri, n, seed):
    """Origins on random triangles (+1e-5 along the direction, like the bounce loop),
    directions uniform on the sphere."""
    rng = np.random.default_rng(seed)
    t = tri.reshape(-1, 3, 3).astype(np.float32)
    i = rng.integers(0, t.shape[0], n)
    u = rng.random(n, dtype=np.float32)
    v = rng.random(n, dtype=np.float32)
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    p = t[i, 0] + u[:, None] * (t[i, 1] - t[i, 0]) + v[:, None] * (t[i, 2] - t[i, 0])
    d = _unit(rng.normal(size=(n, 3)))
    o = (p + np.float32(1e-5) * d).astype(np.float32)
    return o, d


def edge_rays(tri, n, seed):
    """From surface points towards points on other triangles' edges and vertices."""
    rng = np.random.default_rng(seed)
    t = tri.reshape(-1, 3, 3).astype(np.float32)
    o, _ = surface_rays(tri, n, seed + 1)
    j = rng.integers(0, t.shape[0], n)
    k = rng.integers(0, 3, n)
    s = rng.random(n).astype(np.float32)
    s[::4] = 0.0  # vertices
    a, b = t[j, k], t[j, (k + 1) % 3]
    target = a + s[:, None] * (b - a)
    d = target - o
    ok = np.linalg.norm(d, axis=1) > 1e-6
    return o[ok], _unit(d[ok])


def _check(rtmi, oracle, ctx, geom, o, d, rule, t_scale=512.0):
    with rtmi.Scene(ctx, geom) as sc:
        t, h, c = rtmi.intersect_method(ctx, sc, o, d, t_scale, rule, rtmi.ISECT_MFMA, count=True)
        ts, hs = rtmi.intersect_method(ctx, sc, o, d, t_scale, rule, rtmi.ISECT_SCAN)
    tc, hc = oracle.intersect(geom.all_triangles(), geom.n_surf, geom.n_light, geom.light_group, o, d,
                              t_scale, rule)
    bad = np.nonzero(h != hc)[0]
    assert bad.size == 0, f"{bad.size} hit mismatches vs the restatement, first {bad[:5]}"
    assert np.array_equal(t.view(np.uint32), tc.view(np.uint32)), "t not bit-exact"
    assert np.array_equal(h, hs) and np.array_equal(t.view(np.uint32), ts.view(np.uint32))
    return h, c


@pytest.mark.parametrize("kind", SCENES)
@pytest.mark.parametrize("rule", [0, 1])
def test_surface_rays_bit_exact(rtmi_mod, oracle_mod, gpu_ctx, kind, rule):
    geom = _geom(rtmi_mod, kind)
    tri = geom.all_triangles()
    n = 400_000 if kind == "cornell_cpu" else 100_000
    o, d = surface_rays(tri, n, seed=21 + rule)
    h, c = _check(rtmi_mod, oracle_mod, gpu_ctx, geom, o, d, rule)
    hit = h != rtmi_mod.RT_HIT_NONE
    # every hit triangle was a candidate; the filter keeps few of the scene's triangles
    assert np.all(c[hit] >= 1)
    n_tri = tri.reshape(-1, 9).shape[0]
    assert c.mean() < 0.25 * n_tri, (c.mean(), n_tri)


@pytest.mark.parametrize("kind", SCENES)
def test_edge_and_vertex_rays_bit_exact(rtmi_mod, oracle_mod, gpu_ctx, kind):
    geom = _geom(rtmi_mod, kind)
    o, d = edge_rays(geom.all_triangles(), 100_000, seed=31)
    for rule in (0, 1):
        _check(rtmi_mod, oracle_mod, gpu_ctx, geom, o, d, rule)


def test_random_rays_and_t_scales(rtmi_mod, oracle_mod, gpu_ctx):
    geom = _geom(rtmi_mod, "cornell_cpu")
    rng = np.random.default_rng(41)
    o = rng.uniform(-1.9, 1.9, size=(200_000, 3)).astype(np.float32)
    d = _unit(rng.normal(size=(200_000, 3)))
    for t_scale in (1.0, 512.0, 16384.0):
        for rule in (0, 1):
            _check(rtmi_mod, oracle_mod, gpu_ctx, geom, o, d, rule, t_scale)


def test_rays_outside_the_bounds_keep_every_triangle(rtmi_mod, oracle_mod, gpu_ctx):
    """Non-finite components and origins beyond the scene's box + 1 take every triangle
    to the exact test (same bits as the scan); ray count not a multiple of the wave."""
    geom = _geom(rtmi_mod, "cornell_cpu")
    n_tri = geom.all_triangles().reshape(-1, 9).shape[0]
    rng = np.random.default_rng(43)
    n = 333
    o = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    d = _unit(rng.normal(size=(n, 3)))
    o[0:8, 0] = np.nan
    d[8:16, 1] = np.nan
    o[16:24, 2] = np.inf
    d[24:32, 0] = -np.inf
    o[32:40] = np.array([0.0, 0.0, -3.0], np.float32)  # the Cornell camera: outside the box + 1
    o[40:48] *= np.float32(1e30)
    d[48:56] = 0.0
    for rule in (0, 1):
        _, c = _check(rtmi_mod, oracle_mod, gpu_ctx, geom, o, d, rule)
        assert np.all(c[:48] == n_tri)
