"""The exact BVH path for large scenes (rt_bvh.cpp, rt_trace.hpp closest_hit_bvh).

SURVEY.md §8(f) item 4: the reference scans every triangle per ray (CPU/rays/ray.cpp:14-28,
GPU/rays/ray.cu:16-141); Models/bunny.obj (4,968 triangles) and Medieval_House.obj (2,663)
make that scan the whole cost.  The BVH path must return the scan's hit bit for bit under
both hit rules, so it is checked against the exact scan (RT_ISECT_SCAN, itself bit-exact
against the CPU restatement in test_gpu_parity.py) and against the restatement directly:
random rays, rays from surface points, rays aimed at edges and vertices, rays lying in a
triangle's plane (the grazing pairs a box test cannot see), and whole renders of the bunny in the Cornell box with both presets.
"""
import os

import numpy as np
import pytest

from conftest import MODELS

pytestmark = pytest.mark.gpu


def _unit(v):
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def bunny_cornell(rtmi, preset):
    """Models/bunny.obj (GPU-engine loader) scaled into the reference's Cornell box."""
    box = rtmi.cornell_geometry(preset)
    b = rtmi.obj_geometry(os.path.join(MODELS, "bunny.obj"), "generic")
    t = b.tri.reshape(-1, 3, 3).astype(np.float64)
    c = 0.5 * (t.reshape(-1, 3).min(0) + t.reshape(-1, 3).max(0))
    t = ((t - c) * 2.5 + np.array([0.1, 0.35, 0.1])).astype(np.float32)
    tri = np.concatenate([box.tri, t.reshape(-1, 9)], 0)
    alb = np.concatenate([box.albedo, np.full((t.shape[0], 3), 0.75, np.float32)], 0)
    return rtmi.Geometry(tri, alb, box.light, box.emission, box.light_group)


def house(rtmi):
    return rtmi.obj_geometry(os.path.join(MODELS, "Medieval_House.obj"), "generic")


def surface_rays(tri, n, seed, hemisphere=False):
    """Origins on random triangles + 1e-5 along the direction (the bounce loop's offset),
    and the triangle of each origin."""
    rng = np.random.default_rng(seed)
    t = tri.reshape(-1, 3, 3).astype(np.float32)
    i = rng.integers(0, t.shape[0], n)
    u = rng.random(n, dtype=np.float32)
    v = rng.random(n, dtype=np.float32)
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    p = t[i, 0] + u[:, None] * (t[i, 1] - t[i, 0]) + v[:, None] * (t[i, 2] - t[i, 0])
    d = _unit(rng.normal(size=(n, 3)))
    if hemisphere:
        nrm = np.cross(t[i, 2] - t[i, 0], t[i, 1] - t[i, 0])
        d = np.where((np.sum(d * nrm, 1) < 0)[:, None], -d, d).astype(np.float32)
    o = (p + np.float32(1e-5) * d).astype(np.float32)
    return o, d, i.astype(np.int32)


def in_plane_rays(tri, n, seed):
    """Rays in (or within a few ulps of) a triangle's plane, from points of that plane:
    the pairs whose exact test can pass far from the triangle."""
    rng = np.random.default_rng(seed)
    t = tri.reshape(-1, 3, 3).astype(np.float64)
    i = rng.integers(0, t.shape[0], n)
    e1, e2 = t[i, 1] - t[i, 0], t[i, 2] - t[i, 0]
    a = rng.uniform(-2, 3, n)[:, None]
    b = rng.uniform(-2, 3, n)[:, None]
    p = t[i, 0] + a * e1 + b * e2
    nrm = np.cross(e1, e2)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    d = rng.normal(size=(n, 3))
    d -= np.sum(d * nrm, 1)[:, None] * nrm
    d += nrm * rng.choice([0.0, 1e-7, -1e-7, 1e-6, 1e-4], n)[:, None]
    p += nrm * rng.choice([0.0, 1e-7, 1e-6, 1e-5], n)[:, None]
    ok = np.all(np.abs(p) < 1.5, axis=1)
    return p[ok].astype(np.float32), _unit(d[ok]), i[ok].astype(np.int32)


def edge_rays(tri, n, seed):
    rng = np.random.default_rng(seed)
    t = tri.reshape(-1, 3, 3).astype(np.float32)
    o, _, reg = surface_rays(tri, n, seed + 1)
    j = rng.integers(0, t.shape[0], n)
    k = rng.integers(0, 3, n)
    s = rng.random(n).astype(np.float32)
    s[::4] = 0.0
    target = t[j, k] + s[:, None] * (t[j, (k + 1) % 3] - t[j, k])
    d = target - o
    ok = np.linalg.norm(d, axis=1) > 1e-6
    return o[ok], _unit(d[ok]), reg[ok]


def _scan(rtmi, ctx, sc, o, d, ts, rule):
    return rtmi.intersect_method(ctx, sc, o, d, ts, rule, rtmi.ISECT_SCAN)


def _bvh(rtmi, ctx, sc, o, d, ts, rule):
    return rtmi.intersect_method(ctx, sc, o, d, ts, rule, rtmi.ISECT_BVH)


def _same(a, b):
    ta, ha = a
    tb, hb = b
    assert np.array_equal(ha, hb), f"{np.count_nonzero(ha != hb)} hits differ"
    assert np.array_equal(ta.view(np.uint32), tb.view(np.uint32)), "t differs"


@pytest.mark.parametrize("rule", [0, 1])
def test_bvh_built_for_large_scene(rtmi_mod, gpu_ctx, rule):
    g = bunny_cornell(rtmi_mod, 0)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        info = sc.accel_info()
        assert info["nodes"] > g.n_tri // 4 and 0 < info["depth"] < 24
        assert info["plane_nodes"] >= g.n_tri // 4


@pytest.mark.parametrize("rule", [0, 1])
def test_bvh_matches_scan_surface_rays(rtmi_mod, gpu_ctx, rule):
    g = bunny_cornell(rtmi_mod, rule)
    ts = 512.0 if rule == 0 else 720.0
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        for seed, hemi in ((1, False), (2, True)):
            o, d, reg = surface_rays(g.all_triangles(), 200_000, seed, hemi)
            ref = _scan(rtmi_mod, gpu_ctx, sc, o, d, ts, rule)
            _same(_bvh(rtmi_mod, gpu_ctx, sc, o, d, ts, rule), ref)


@pytest.mark.parametrize("rule", [0, 1])
def test_bvh_matches_scan_hard_rays(rtmi_mod, gpu_ctx, rule):
    g = bunny_cornell(rtmi_mod, rule)
    ts = 512.0 if rule == 0 else 720.0
    rng = np.random.default_rng(7)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        o, d, reg = edge_rays(g.all_triangles(), 100_000, 3)
        _same(_bvh(rtmi_mod, gpu_ctx, sc, o, d, ts, rule), _scan(rtmi_mod, gpu_ctx, sc, o, d, ts, rule))
        o, d, reg = in_plane_rays(g.all_triangles(), 100_000, 4)
        _same(_bvh(rtmi_mod, gpu_ctx, sc, o, d, ts, rule), _scan(rtmi_mod, gpu_ctx, sc, o, d, ts, rule))
        # random rays inside and outside the box, and rays the BVH must hand to the scan
        o = rng.uniform(-3, 3, (50_000, 3)).astype(np.float32)
        d = _unit(rng.normal(size=(50_000, 3)))
        d[:10] = np.nan
        o[10:20] = 100.0
        d[20:30] = np.array([1.0, 0.0, 0.0], np.float32)
        _same(_bvh(rtmi_mod, gpu_ctx, sc, o, d, ts, rule), _scan(rtmi_mod, gpu_ctx, sc, o, d, ts, rule))


@pytest.mark.parametrize("rule", [0, 1])
def test_bvh_matches_oracle(rtmi_mod, oracle_mod, gpu_ctx, rule):
    g = bunny_cornell(rtmi_mod, rule)
    ts = 512.0 if rule == 0 else 720.0
    o, d, reg = surface_rays(g.all_triangles(), 20_000, 11, True)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        got = rtmi_mod.intersect(gpu_ctx, sc, o, d, ts, rule)  # the scene's default: the BVH
    ref = oracle_mod.intersect(g.all_triangles(), g.n_surf, g.n_light, g.light_group, o, d, ts, rule)
    _same(got, ref)


def test_bvh_house_matches_scan(rtmi_mod, gpu_ctx):
    """Medieval_House.obj: 2,663 triangles over coordinates of several hundred units."""
    g = house(rtmi_mod)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        assert sc.accel_info()["nodes"] > 0
        for rule in (0, 1):
            o, d, reg = surface_rays(g.all_triangles(), 50_000, 5 + rule, True)
            _same(_bvh(rtmi_mod, gpu_ctx, sc, o, d, 720.0, rule),
                  _scan(rtmi_mod, gpu_ctx, sc, o, d, 720.0, rule))


@pytest.mark.parametrize("preset", [0, 1])
def test_bvh_render_matches_oracle(rtmi_mod, oracle_mod, gpu_ctx, preset):
    """The renders of the bunny in the Cornell box: the BVH path is the scan bit for bit."""
    g = bunny_cornell(rtmi_mod, preset)
    cam_pos = rtmi_mod.CAMERAS["cornell"]
    p = rtmi_mod.default_params(preset, width=96, height=96, spp=4, spp_split=2)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        img, casts = rtmi_mod.render(gpu_ctx, sc, rtmi_mod.camera(cam_pos), p, (32, 40, 24, 24))
        sc.set_accel(rtmi_mod.ACCEL_SCAN)
        img_s, casts_s = rtmi_mod.render(gpu_ctx, sc, rtmi_mod.camera(cam_pos), p, (32, 40, 24, 24))
    assert casts == casts_s
    assert np.array_equal(img.view(np.uint32), img_s.view(np.uint32))
    ref, ref_casts = oracle_mod.render(g, oracle_mod.camera(cam_pos), oracle_mod.params_from(p), (32, 40, 24, 24))
    assert casts == ref_casts
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("preset", [0, 1])
def test_bvh_render_frame_equals_scan(rtmi_mod, gpu_ctx, preset):
    g = bunny_cornell(rtmi_mod, preset)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["cornell"], yaw_y=0.1)
    p = rtmi_mod.default_params(preset, width=128, height=128, spp=8, spp_split=4)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        img, casts = rtmi_mod.render(gpu_ctx, sc, cam, p)
        sc.set_accel(rtmi_mod.ACCEL_SCAN)
        img_s, casts_s = rtmi_mod.render(gpu_ctx, sc, cam, p)
    assert casts == casts_s
    assert np.array_equal(img.view(np.uint32), img_s.view(np.uint32))


def test_bvh_small_scene_forced(rtmi_mod, gpu_ctx):
    """ACCEL_BVH on the 168-triangle complex_light_room equals its filter path."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "complex_light_room.obj"), "complex_light_room")
    p = rtmi_mod.default_params(1, width=64, height=64, spp=8, spp_split=8)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["complex_light_room"])
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        img, casts = rtmi_mod.render(gpu_ctx, sc, cam, p)
        sc.set_accel(rtmi_mod.ACCEL_BVH)
        img_b, casts_b = rtmi_mod.render(gpu_ctx, sc, cam, p)
    assert casts == casts_b
    assert np.array_equal(img.view(np.uint32), img_b.view(np.uint32))


@pytest.mark.parametrize("hit_rule,td_mode", [(1, "frame"), (0, "frame"), (1, "inframe")])
def test_bvh_sarsa_render_equals_scan(rtmi_mod, gpu_ctx, hit_rule, td_mode):
    """The SARSA sampler's trace on the BVH (k_sarsa_render_pq<.., BVH>) is the scan bit for bit:
    two frames of the bunny in the Cornell box, the second sampling the map the first trained;
    both hit rules, and the in-frame TD rule (k_sarsa_render_pq<.., TD = 1, BVH>) on a launch
    with one active lane (a 1 x 1 image, one chunk), whose events then run in sample order."""
    g = bunny_cornell(rtmi_mod, rtmi_mod.RT_PRESET_GPU)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["cornell"])
    if td_mode == "frame":
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=96, height=96, spp=8, spp_split=4,
                                    hit_rule=hit_rule)
    else:
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=1, height=1, spp=64, spp_split=1,
                                    hit_rule=hit_rule)
    out = {}
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        for accel in (None, rtmi_mod.ACCEL_SCAN):
            if accel is not None:
                sc.set_accel(accel)
            with rtmi_mod.sarsa.RadianceMap(gpu_ctx, sc, 1984) as m:
                if td_mode == "inframe":
                    m.set_td_mode(rtmi_mod.sarsa.TD_INFRAME)
                out[accel] = [m.render(cam, p, 1) for _ in range(2)] + [m.read()]
        Q, Qs = out[None].pop(), out[rtmi_mod.ACCEL_SCAN].pop()
    for a, b in zip(Q, Qs):
        assert np.array_equal(a, b)
    for (a, ca), (b, cb) in zip(out[None], out[rtmi_mod.ACCEL_SCAN]):
        assert ca == cb
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    if td_mode == "frame":
        assert out[None][1][0].mean() > 0


@pytest.mark.parametrize("hit_rule", [1, 0])
def test_bvh_dqn_render_equals_scan(rtmi_mod, gpu_ctx, hit_rule):
    """The DQN sampler's casts on the BVH (dqn_trace<-1>) are the scan's bit for bit (synthetic
    weights over the box's vertices as the network's inputs).  The DQN renderer implements the
    GPU engine (pre_trained_pathtracer.cu): the CPU object's hit rule is refused, BVH or scan."""
    g = bunny_cornell(rtmi_mod, rtmi_mod.RT_PRESET_GPU)
    box = rtmi_mod.cornell_geometry(rtmi_mod.RT_PRESET_GPU)
    nn = np.unique(box.tri.reshape(-1, 3), axis=0).astype(np.float32).ravel()
    W, b = rtmi_mod.dqn.synthetic_weights(nn.size)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["cornell"])
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=96, height=96, spp=4, hit_rule=hit_rule)
    out = []
    with rtmi_mod.Scene(gpu_ctx, g) as sc, rtmi_mod.dqn.Dqn(gpu_ctx, nn, W, b) as net:
        if hit_rule == 0:
            for accel in (None, rtmi_mod.ACCEL_SCAN):
                if accel is not None:
                    sc.set_accel(accel)
                with pytest.raises(rtmi_mod.RtError):
                    rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p)
            return
        out.append(rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p))
        sc.set_accel(rtmi_mod.ACCEL_SCAN)
        out.append(rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p))
    (a, ca), (b_, cb) = out
    assert ca == cb and a.mean() > 0
    assert np.array_equal(a.view(np.uint32), b_.view(np.uint32))


def test_bvh_neuralq_frame_equals_scan(rtmi_mod, gpu_ctx):
    """The Neural-Q trainer's casts on the BVH (k_nq_trace<true>) are the scan's: the same
    frame, per-sample statistics and trained parameters, bit for bit."""
    g = bunny_cornell(rtmi_mod, rtmi_mod.RT_PRESET_GPU)
    box = rtmi_mod.cornell_geometry(rtmi_mod.RT_PRESET_GPU)
    nn = np.unique(box.tri.reshape(-1, 3), axis=0).astype(np.float32).ravel()
    W, b = rtmi_mod.dqn.synthetic_weights(nn.size)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["cornell"])
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=32, height=24, spp=2)
    out = []
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        for accel in (None, rtmi_mod.ACCEL_SCAN):
            if accel is not None:
                sc.set_accel(accel)
            with rtmi_mod.dqn.DqnTrainer(gpu_ctx, nn, W, b) as tr, \
                    rtmi_mod.dqn.NeuralQ(gpu_ctx, sc, tr, batch_size=256) as nq:
                img, stats, casts = nq.render_frame(cam, p)
                out.append((img, stats, casts, tr.params()))
    (i1, s1, c1, (W1, _)), (i2, s2, c2, (W2, _)) = out
    assert c1 == c2 and np.array_equal(i1, i2) and np.array_equal(s1, s2)
    assert all(np.array_equal(x, y) for x, y in zip(W1, W2))
