"""The bounce-ray candidate table (rt_ctab.cpp): k_render_ps's bounce casts (the CPU engine's
hit rule) and the DQN renderer's (the GPU engine's) take their candidates from it.

The table is sound if every triangle that passes the reference's exact test for a bounce ray
(Triangle::intersects, CPU/rays/ray.cpp:14-28 / GPU/rays/ray.cu:63-64, restated in oracle/:
orc_pass_masks) is among the ray's candidates.  CPU: the host lookup
(rt_ctab_candidates, the kernel's operations) against the oracle's pass sets on rays from
the scenes' surfaces -- sampled as the kernel samples them, aimed at vertices and edges, and
nearly parallel to some triangle's plane -- at every t_scale the table serves.  GPU: the
renders that use it are bit-exact against the oracle (test_gpu_parity.py, test_dqn.py and the
bench line's whole-frame check).
"""
import os

import numpy as np
import pytest

from conftest import MODELS


def _scene(rtmi_mod, kind):
    if kind == "cornell_cpu":
        g = rtmi_mod.cornell_geometry(0)
    elif kind == "cornell_gpu":
        g = rtmi_mod.cornell_geometry(1)
    elif kind == "bunny":
        g = rtmi_mod.obj_geometry(os.path.join(MODELS, "bunny.obj"), "generic")
    else:
        g = rtmi_mod.obj_geometry(os.path.join(MODELS, kind + ".obj"), kind)
    return np.ascontiguousarray(g.all_triangles(), np.float32), g.n_surf


def _frame(n):
    t = np.array([n[2], 0.0, -n[0]]) if abs(n[0]) > abs(n[1]) else np.array([0.0, -n[2], n[1]])
    t = t / np.linalg.norm(t)
    return t, np.cross(n, t)


def bounce_rays(tri, n_surf, n, seed):
    """(surf, origin, direction, kind) of n rays leaving random surface points as the kernel
    forms them: o = pos + 1e-5 sd, d = sd / |sd| in float32 (kind 0: uniform hemisphere, 1: at
    a vertex of the scene, 2: nearly parallel to some triangle's plane, 3: nearly parallel to
    the origin's own plane)"""
    rng = np.random.default_rng(seed)
    v = tri[:n_surf].reshape(-1, 3, 3).astype(np.float64)
    N = np.cross(v[:, 2] - v[:, 0], v[:, 1] - v[:, 0])
    area = 0.5 * np.linalg.norm(N, axis=1)
    N /= np.linalg.norm(N, axis=1, keepdims=True)
    j = rng.choice(n_surf, n, p=area / area.sum())
    a, b = rng.random(n), rng.random(n)
    f = a + b > 1
    a[f], b[f] = 1 - a[f], 1 - b[f]
    pos = (v[j, 0] + a[:, None] * (v[j, 1] - v[j, 0]) + b[:, None] * (v[j, 2] - v[j, 0])).astype(np.float32)
    allv = tri.reshape(-1, 3).astype(np.float64)
    kind = rng.integers(0, 4, n)
    sd = np.zeros((n, 3))
    for i in range(n):
        nn = N[j[i]]
        if kind[i] == 0:
            T, B = _frame(nn)
            r1, r2 = rng.random(), rng.random()
            st = np.sqrt(max(0.0, 1 - r1 * r1))
            s = st * np.cos(2 * np.pi * r2) * B + r1 * nn + st * np.sin(2 * np.pi * r2) * T
        elif kind[i] == 1:
            s = allv[rng.integers(0, len(allv))] - pos[i] + rng.normal(size=3) * 10.0 ** rng.uniform(-7, -3)
        else:
            k = rng.integers(0, len(tri)) if kind[i] == 2 else j[i]
            vk = tri[k].reshape(3, 3).astype(np.float64)
            nk = np.cross(vk[1] - vk[0], vk[2] - vk[0])
            nk /= np.linalg.norm(nk)
            T, B = _frame(nk)
            ph = 2 * np.pi * rng.random()
            s = np.cos(ph) * T + np.sin(ph) * B + nk * abs(rng.normal()) * 10.0 ** rng.uniform(-7, -1.5)
        if np.dot(s, nn) < 0:
            s = -s
        sd[i] = s / np.linalg.norm(s)
    sd = sd.astype(np.float32)
    o = (pos + np.float32(1e-5) * sd).astype(np.float32)
    ln = np.sqrt((sd[:, 0] * sd[:, 0] + sd[:, 1] * sd[:, 1]) + sd[:, 2] * sd[:, 2]).astype(np.float32)
    d = (sd / ln[:, None]).astype(np.float32)
    return j.astype(np.int32), o, d, kind


def _popcount(m):
    return np.array([bin(int(x)).count("1") for x in m])


@pytest.mark.parametrize("kind,rule", [("cornell_cpu", 0), ("cornell_gpu", 0), ("door_room", 0),
                                       ("cornell_gpu", 1), ("door_room", 1), ("archway", 1),
                                       ("complex_light_room", 1)])
def test_ctab_keeps_every_pass(rtmi_mod, oracle_mod, kind, rule):
    tri, n_surf = _scene(rtmi_mod, kind)
    surf, o, d, rk = bounce_rays(tri, n_surf, 8000, seed=7 + rule)
    cand, stats = rtmi_mod.ctab_candidates(tri, n_surf, surf, o, d, hit_rule=rule)
    assert stats[0] > 0 and stats[2] > 0
    assert cand.shape == (o.shape[0], (tri.shape[0] + 63) // 64)
    # rule 0: the t_scale the table serves (>= 256); rule 1: any -- up to kFiltMaxTScale (16384),
    # the largest the launchers serve it at, where ET (rt_bounds.hpp) is sized
    for ts in ((256.0, 512.0, 720.0, 4096.0, 16384.0) if rule == 0 else (0.01, 1.0, 256.0, 720.0, 1024.0, 16384.0)):
        passes = oracle_mod.pass_masks(tri, o, d, ts, rule)
        missed = passes & ~cand
        bad = np.nonzero(missed.any(axis=1))[0]
        assert bad.size == 0, (f"t_scale {ts}: {bad.size} rays miss a passing triangle, e.g. ray {bad[0]} "
                               f"(surface {surf[bad[0]]}, kind {rk[bad[0]]}) words {[hex(int(x)) for x in missed[bad[0]]]}")
    # and the table culls: a bounce ray keeps a few of the scene's triangles
    pc = sum(_popcount(cand[rk == 0, w]) for w in range(cand.shape[1]))
    assert pc.mean() < (0.2 if rule == 0 else 0.3) * tri.shape[0], pc.mean()


def test_ctab_keeps_every_triangle_outside_its_domain(rtmi_mod):
    tri, n_surf = _scene(rtmi_mod, "cornell_cpu")
    surf, o, d, _ = bounce_rays(tri, n_surf, 8, seed=3)
    allbits = (1 << tri.shape[0]) - 1
    # an origin off its surface's plane, a surface index out of range, a non-unit direction,
    # a non-finite origin
    o2 = o.copy()
    o2[0] += np.float32(1e-3) * np.asarray([1.0, 1.0, 1.0], np.float32)
    s2 = surf.copy()
    s2[1] = -1
    s2[2] = n_surf
    d2 = d.copy()
    d2[3] *= np.float32(1.01)
    o2[4, 0] = np.nan
    cand, _ = rtmi_mod.ctab_candidates(tri, n_surf, s2, o2, d2)
    for r in range(5):
        assert int(cand[r, 0]) == allbits, r
    assert all(int(c) != allbits for c in cand[5:, 0])


def test_ctab_refuses_large_scenes(rtmi_mod):
    tri, n_surf = _scene(rtmi_mod, "bunny")
    assert tri.shape[0] > 256
    with pytest.raises(rtmi_mod.RtError):
        rtmi_mod.ctab_candidates(tri, n_surf, np.zeros(1, np.int32), np.zeros((1, 3), np.float32),
                                 np.asarray([[0.0, 0.0, 1.0]], np.float32), hit_rule=1)


# ---------------------------------------------------------------- GPU ----------

def _cornell_frame(rtmi_mod, ctx, sc, preset, yaw_x=0.0):
    # (t_scale = the height: rule 0's table serves t_scale >= 256)
    p = rtmi_mod.default_params(preset, width=64, height=256, spp=8, spp_split=4)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["cornell"])
    cam.yaw_x = yaw_x
    return rtmi_mod.render(ctx, sc, cam, p)


@pytest.mark.gpu
def test_gpu_table_upload_failure_keeps_the_image(rtmi_mod, gpu_ctx, monkeypatch):
    """A table that cannot be uploaded (device memory short: forced by RT_CTAB_TEST_FAIL) is
    skipped, not an error: the render goes on with the matrix-core image's masks -- the same
    image and casts bit for bit -- and the scene reports no table."""
    g = rtmi_mod.cornell_geometry(rtmi_mod.RT_PRESET_CPU)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        ref = _cornell_frame(rtmi_mod, gpu_ctx, sc, rtmi_mod.RT_PRESET_CPU)
        info = sc.ctab_info(rtmi_mod.RT_HIT_RULE_CPU)
        assert info["built"] and info["bytes"] > 0 and info["build_s"] > 0, info
    monkeypatch.setenv("RT_CTAB_TEST_FAIL", "1")
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        img, casts = _cornell_frame(rtmi_mod, gpu_ctx, sc, rtmi_mod.RT_PRESET_CPU)
        assert not sc.ctab_info(rtmi_mod.RT_HIT_RULE_CPU)["built"]
        assert casts == ref[1] and np.array_equal(img, ref[0])
        img2, casts2 = _cornell_frame(rtmi_mod, gpu_ctx, sc, rtmi_mod.RT_PRESET_CPU)  # later calls too
        assert casts2 == ref[1] and np.array_equal(img2, ref[0])


@pytest.mark.gpu
def test_gpu_table_built_only_for_a_launch_that_takes_it(rtmi_mod, gpu_ctx):
    """The GPU preset's table route needs the camera inside the image's bound and pitch 0;
    Cornell's camera (z = -3) is outside, so no render builds a rule-1 table for it."""
    g = rtmi_mod.cornell_geometry(rtmi_mod.RT_PRESET_GPU)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        _cornell_frame(rtmi_mod, gpu_ctx, sc, rtmi_mod.RT_PRESET_GPU)
        assert not sc.ctab_info(rtmi_mod.RT_HIT_RULE_GPU)["built"]
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "door_room.obj"), "door_room")
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=32, height=32, spp=4, spp_split=4)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        cam.yaw_x = 0.1  # pitched: k_render_pq's camera rays cannot take the rectangle cull
        rtmi_mod.render(gpu_ctx, sc, cam, p)
        assert not sc.ctab_info(rtmi_mod.RT_HIT_RULE_GPU)["built"]
        cam.yaw_x = 0.0
        rtmi_mod.render(gpu_ctx, sc, cam, p)
        assert sc.ctab_info(rtmi_mod.RT_HIT_RULE_GPU)["built"]
