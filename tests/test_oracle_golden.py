"""Pin the oracle (and the product's host-side builders) to everything the
reference holds for this path: known-answer vectors, the constants of the
prebuilt hit predicate, the archway loader dump, analytic intersections.
CPU only."""
import json
import math
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN, MODELS

CORNELL_CAM = (0.0, 0.0, -3.0, 1.0)


def code(kind, idx):
    """packed hit code (type << 30) | index as the int32 the ABI returns"""
    return int(np.array([(kind << 30) | idx], np.uint32).view(np.int32)[0])


def f32(word_hex):
    return struct.unpack("<f", struct.pack("<I", int(word_hex, 16)))[0]


# --- RNG ---------------------------------------------------------------------

# Random123 kat_vectors for philox4x32_10 (Salmon et al. SC'11)
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_kat(oracle_mod, ctr, key, want):
    assert tuple(int(x) for x in oracle_mod.philox(ctr, key)) == want


def test_sincos_turn_accuracy(oracle_mod):
    rs = np.linspace(0, 1, 20001, endpoint=False, dtype=np.float32)
    err = 0.0
    for r in rs[::7]:
        s, c = oracle_mod.sincos_turn(float(r))
        err = max(err, abs(s - math.sin(2 * math.pi * float(r))), abs(c - math.cos(2 * math.pi * float(r))))
        assert s * s + c * c == pytest.approx(1.0, abs=4e-7)
    assert err < 2e-7
    # exact quadrant points
    assert oracle_mod.sincos_turn(0.0) == (0.0, 1.0)
    assert oracle_mod.sincos_turn(0.25) == (1.0, -0.0)
    assert oracle_mod.sincos_turn(0.5) == (-0.0, -1.0)


# --- hit predicate -------------------------------------------------------------

def test_predicate_constants_pinned_to_prebuilt_object():
    """The constants the oracle and the kernels use are the words the prebuilt
    Triangle::intersects loads (tests/golden/triangle_o_pin.json)."""
    pin = json.load(open(os.path.join(GOLDEN, "triangle_o_pin.json")))
    assert f32(pin["t_scale_word"]) == 512.0        # SCREEN_HEIGHT of the CPU engine
    assert f32(pin["eps_word"]) == np.float32(1e-5)  # kEps / EPS
    assert f32(pin["one_word"]) == 1.0
    assert pin["accept_order"][-2:] == ["t < dist + eps", "t > eps"]


def _tri(*vs):
    return np.array([np.concatenate(vs)], np.float32)


def test_intersect_analytic(oracle_mod):
    tri = _tri([0, 0, 1], [1, 0, 1], [0, 1, 1])
    o = np.array([[0.1, 0.2, 0.0], [0.9, 0.9, 0.0], [0.1, 0.2, 2.0]], np.float32)
    d = np.array([[0, 0, 1], [0, 0, 1], [0, 0, 1]], np.float32)
    for rule in (0, 1):
        t, h = oracle_mod.intersect(tri, 1, 0, np.zeros(0, np.int32), o, d, 512.0, rule)
        assert t[0] == pytest.approx(1.0 / 512.0, rel=1e-6)
        assert h[0] == code(2, 0)
        assert h[1] == -1 and math.isinf(t[1])   # u + v > 1
        assert h[2] == -1                         # behind the origin


def test_intersect_tie_and_eps_rules(oracle_mod):
    # two coincident triangles: CPU rule (t < dist + eps) -> the LATER wins;
    # GPU rule (t < dist) -> the earlier wins
    a = np.concatenate([[0, 0, 1], [1, 0, 1], [0, 1, 1]])
    tri = np.array([a, a], np.float32)
    o = np.array([[0.1, 0.2, 0.0]], np.float32)
    d = np.array([[0, 0, 1]], np.float32)
    _, h0 = oracle_mod.intersect(tri, 2, 0, np.zeros(0, np.int32), o, d, 512.0, 0)
    _, h1 = oracle_mod.intersect(tri, 2, 0, np.zeros(0, np.int32), o, d, 512.0, 1)
    assert h0[0] == code(2, 1)
    assert h1[0] == code(2, 0)
    # origin on the triangle: t = 0 fails the CPU guard t > 1e-5, passes t >= 0
    o2 = np.array([[0.1, 0.2, 1.0]], np.float32)
    _, g0 = oracle_mod.intersect(tri[:1], 1, 0, np.zeros(0, np.int32), o2, d, 512.0, 0)
    _, g1 = oracle_mod.intersect(tri[:1], 1, 0, np.zeros(0, np.int32), o2, d, 512.0, 1)
    assert g0[0] == -1 and g1[0] == code(2, 0)


def test_light_index_rules(oracle_mod):
    g = oracle_mod.cornell(0)
    tri = np.concatenate([g["tri"], g["light"]])
    # straight up through the ceiling light's second fan triangle (K, J, L)
    lv = g["light"][1].reshape(3, 3)
    target = lv.mean(axis=0)
    o = np.array([[target[0], 0.0, target[2]]], np.float32)
    d = np.array([[0.0, -1.0, 0.0]], np.float32)  # -y is up in the Cornell box
    _, h_cpu = oracle_mod.intersect(tri, 36, 2, g["light_group"], o, d, 512.0, 0)
    _, h_gpu = oracle_mod.intersect(tri, 36, 2, np.array([0, 1], np.int32), o, d, 512.0, 1)
    assert h_cpu[0] == code(1, 0)   # plane index
    assert h_gpu[0] == code(1, 1)   # light-triangle index


# --- scene builders ---------------------------------------------------------------

@pytest.mark.parametrize("variant", [0, 1])
def test_cornell_product_equals_oracle(rtmi_mod, oracle_mod, variant):
    g = rtmi_mod.cornell_geometry(variant)
    o = oracle_mod.cornell(variant)
    for k in ("tri", "albedo", "light", "emission", "light_group"):
        assert np.array_equal(getattr(g, k), o[k]), k
    assert g.n_surf == 36 and g.n_light == 2
    # box spans [-1, 1]^3 after v*(2/l) - 1 and the x/y flip
    allv = g.all_triangles().reshape(-1, 3)
    assert allv.min() == -1.0 and allv.max() == 1.0


def test_cornell_normals_axis_aligned(oracle_mod):
    g = oracle_mod.cornell(0)
    n = oracle_mod.normals(np.concatenate([g["tri"], g["light"]]))
    assert np.allclose(np.linalg.norm(n, axis=1), 1.0, atol=1e-6)
    # room walls: two triangles per wall share a normal
    for i in range(0, 6, 2):
        assert np.array_equal(n[i], n[i + 1])


def test_archway_loader_matches_reference_dump(rtmi_mod):
    """Radiance_Map_Data/vertices.txt = the GPU engine's archway scene as loaded
    (6 significant digits)."""
    gold = np.loadtxt(os.path.join(GOLDEN, "archway_vertices.txt"), dtype=np.float64)
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "archway.obj"), "archway")
    mine = g.all_triangles().astype(np.float64)
    assert mine.shape == gold.shape == (102, 9)
    assert np.all(np.abs(mine - gold) <= 5e-6 * np.maximum(np.abs(gold), 1.0))


@pytest.mark.parametrize("kind,ns,nl,nn", [("door_room", 36, 2, 342), ("archway", 96, 6, 918),
                                           ("complex_light_room", 144, 24, 1512)])
def test_obj_scene_counts(rtmi_mod, kind, ns, nl, nn):
    """Triangle / light / DQN-input counts of the thesis scenes."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, f"{kind}.obj"), kind)
    assert (g.n_surf, g.n_light, g.nn_vertices.size) == (ns, nl, nn)
    assert np.all(g.emission == (12.0 if kind == "complex_light_room" else 8.0))


# --- frame buffer -----------------------------------------------------------------

def test_pack_argb_product_equals_oracle(rtmi_mod, oracle_mod):
    rng = np.random.default_rng(7)
    rgb = rng.uniform(-0.5, 1.5, size=(257, 3)).astype(np.float32)
    rgb[:10] = np.array([0, 1, 1 / 255], np.float32)
    rgb[10:20] = np.array([254.999 / 255, 255.0 / 255, 2.0], np.float32)
    a = rtmi_mod.pack_argb(rgb)
    b = oracle_mod.pack_argb(rgb)
    assert np.array_equal(a, b)
    assert np.all((a >> 24) == 128)
    assert a[0] == (128 << 24) | (0 << 16) | (255 << 8) | 1  # (0, 1, 1/255f): 255*(1/255f) rounds to 1
    assert a[10] == (128 << 24) | (254 << 16) | (255 << 8) | 255  # truncation, clamp


def test_oracle_render_deterministic_and_split_consistent(rtmi_mod, oracle_mod):
    p = rtmi_mod.default_params(0, width=32, height=32, spp=8)
    g = oracle_mod.cornell(0)
    cam = oracle_mod.camera(CORNELL_CAM)
    a, ca = oracle_mod.render(g, cam, oracle_mod.params_from(p))
    b, cb = oracle_mod.render(g, cam, oracle_mod.params_from(p))
    assert np.array_equal(a, b) and ca == cb
    p.spp_split = 4
    c, cc = oracle_mod.render(g, cam, oracle_mod.params_from(p))
    assert cc == ca  # same paths, only the summation order differs
    assert np.max(np.abs(c - a)) <= 1e-6 * max(1.0, float(np.abs(a).max()))
    # rectangle renders are crops of the full frame
    r, _ = oracle_mod.render(g, cam, oracle_mod.params_from(p), rect=(5, 7, 11, 9))
    assert np.array_equal(r, c[7:16, 5:16])


# --- reference_sequential mode (parity gate 3) ---------------

def mean_z(a, b):
    """per-channel z score of the mean per-pixel difference of two independent
    unbiased renders of the same frame (0 expected; |z| < 3 is the gate)"""
    d = (np.asarray(a, np.float64) - np.asarray(b, np.float64)).reshape(-1, 3)
    return d.mean(0) / (d.std(0) / math.sqrt(d.shape[0]))


def test_glibc_rand_kat(oracle_mod):
    # glibc's rand() after srand(1) (= the reference's never-seeded stream)
    assert list(oracle_mod.glibc_rand(1, 4)) == [1804289383, 846930886, 1681692777, 1714636915]


def test_reference_sequential_deterministic_and_guarded(rtmi_mod, oracle_mod):
    g = oracle_mod.cornell(0)
    cam = oracle_mod.camera(CORNELL_CAM)
    p = rtmi_mod.default_params(0, width=24, height=16, spp=4)
    a, ca = oracle_mod.render_sequential(g, cam, oracle_mod.params_from(p))
    b, cb = oracle_mod.render_sequential(g, cam, oracle_mod.params_from(p))
    assert np.array_equal(a, b) and ca == cb and ca >= 24 * 16 * 4
    p.seed = 7  # srand(seed): another stream
    c, _ = oracle_mod.render_sequential(g, cam, oracle_mod.params_from(p))
    assert not np.array_equal(a, c)
    p.sampler = 1
    with pytest.raises(ValueError):
        oracle_mod.render_sequential(g, cam, oracle_mod.params_from(p))


@pytest.mark.parametrize("width,spp", [(128, 16), (64, 128)])
def test_reference_sequential_statistical(rtmi_mod, oracle_mod, width, spp):
    """Gate 3: the Philox renders (this oracle = the GPU kernel, bit for bit) agree
    with the reference's own rand() stream and loop order in the image mean."""
    g = oracle_mod.cornell(0)
    cam = oracle_mod.camera(CORNELL_CAM)
    p = rtmi_mod.default_params(0, width=width, height=width, spp=spp)
    a, ca = oracle_mod.render_sequential(g, cam, oracle_mod.params_from(p))
    b, cb = oracle_mod.render(g, cam, oracle_mod.params_from(p))
    z = mean_z(a, b)
    assert np.all(np.abs(z) < 3.0), z
    assert abs(ca - cb) <= 0.01 * cb  # ray casts per sample: same path-length law
