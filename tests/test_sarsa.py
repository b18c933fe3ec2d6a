"""Expected-SARSA radiance-volume path (BASELINE config 3).

Parity levels:
  * volume placement, KD array, nearest-volume queries: bit-exact with the oracle
  * render + Q-table learning: bit-exact with the oracle (frame-synchronous TD with
    integer fixed-point sums is order-free, so GPU and CPU agree to the last bit:
    image, casts, Q, CDF, visits, irradiance)
  * reference pin (statistical): first-frame average path length per scene vs the
    reference's own training logs (Radiance_Map_Data/sarsa_*.txt -> golden
    sarsa_ref_stats.json): the reference logs floor(mean over pixels of
    floor(per-pixel mean)), i.e. about half a bounce below the true mean.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, MODELS

SCENES = ("cornell", "door_room", "archway", "complex_light_room")


def geometry(rtmi_mod, scene):
    if scene == "cornell":
        return rtmi_mod.cornell_geometry(rtmi_mod.RT_PRESET_GPU)
    return rtmi_mod.obj_geometry(os.path.join(MODELS, scene + ".obj"), scene)


def area_counts(tri, area_per_sample=0.001):
    """floor(area / AREA_PER_SAMPLE) per triangle, Triangle::compute_area's arithmetic (numpy float32)"""
    v = tri.reshape(-1, 3, 3).astype(np.float32)
    a, b = v[:, 1] - v[:, 0], v[:, 2] - v[:, 0]
    dot = lambda x, y: (x[:, 0] * y[:, 0] + x[:, 1] * y[:, 1]) + x[:, 2] * y[:, 2]
    e = np.sqrt(dot(a, a)) * np.sqrt(dot(b, b))
    c = dot(a, b) / e
    s = np.sqrt(1.0 - c.astype(np.float64) ** 2).astype(np.float32)
    area = np.float32(0.5) * e * s
    return np.floor(area / np.float32(area_per_sample)).astype(np.int64)


# sizeof(RadianceVolume) of the reference (GPU/radiance_volumes/radiance_volume.cuh:40-49):
# vec4 position 16 + radiance_grid, radiance_distribution, visits 3 x 144 x 4 + irradiance_accum 4
# + surface_index 4 + vec3 normal 12 + mat4 transformation_matrix 64 + int index 4
RADIANCE_VOLUME_BYTES = 16 + 3 * 144 * 4 + 4 + 4 + 12 + 64 + 4
# Q-table memory the reference's authors record, MB: the thesis's table
# (Descriptions/write_up/chapters/4_critical_evaluation.tex:217-232: Cornell Box 44, Door Room 66,
# Complex Pillars 300) and the archway SARSA render's file name (Images/archway/sarsa_128spp_3avg_272Mb.png)
THESIS_QTABLE_MB = {"cornell": 44, "door_room": 66, "complex_light_room": 300, "archway": 272}


def leaves_under(kd, i, out):
    stack = [i]
    while stack:
        j = stack.pop()
        if kd["leaf"][j]:
            out.append(int(kd["vol"][j]))
        else:
            stack += [int(kd["left"][j]), int(kd["right"][j])]
    return out


# ---------------------------------------------------------------- CPU ----------

def test_stats_line_format(rtmi_mod):
    """GPU/main.cu:330-339: `avg << " " << 0.0 << " " << zero` with avg = total / pixels in
    integer arithmetic, stored in a float: the reference's own lines read "41 0 266689"."""
    f = rtmi_mod.sarsa.stats_line
    assert f(41 * 720 * 720 + 719, 266689, 720 * 720) == "41 0 266689\n"
    assert f(0, 0, 4) == "0 0 0\n"


def test_oracle_stats_bound_casts(rtmi_mod, oracle_mod):
    """per-pixel floors sum to at most casts / spp and more than casts / spp - pixels"""
    g = geometry(rtmi_mod, "cornell")
    m = oracle_mod.Sarsa(g, 1984)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=24, height=16, spp=4)
    _, casts = m.render(oracle_mod.camera(rtmi_mod.CAMERAS["cornell"]), oracle_mod.params_from(p), 1)
    paths, zero = m.stats()
    assert casts // 4 - 24 * 16 < paths <= casts // 4
    assert 0 <= zero <= 24 * 16 * 4

@pytest.mark.parametrize("scene", SCENES)
def test_oracle_volume_placement(rtmi_mod, oracle_mod, scene):
    g = geometry(rtmi_mod, scene)
    m = oracle_mod.Sarsa(g, 1984)
    cnt = area_counts(g.tri)
    assert m.n_volumes == int(cnt.sum()) > 0
    pos, nrm, surf, kd = m.volumes()
    assert np.array_equal(np.bincount(surf, minlength=g.n_surf), cnt)
    assert np.all(np.diff(surf) >= 0)                       # surfaces in order
    # on their triangle (barycentric a1 + a2 <= 1, both >= 0) with its normal
    normals = oracle_mod.normals(g.all_triangles())
    assert np.array_equal(nrm, normals[surf])
    v = g.tri.reshape(-1, 3, 3)[surf].astype(np.float64)
    e1, e2, d = v[:, 1] - v[:, 0], v[:, 2] - v[:, 0], pos - v[:, 0]
    G = np.stack([e1, e2], 2)
    ab = np.einsum("nij,nj->ni", np.linalg.pinv(G), d)
    assert np.all(ab > -1e-4) and np.all(ab.sum(1) < 1 + 1e-4)


@pytest.mark.parametrize("scene", SCENES)
def test_volume_count_matches_reference_qtable_memory(rtmi_mod, oracle_mod, scene):
    """The volume count at the reference's AREA_PER_SAMPLE 0.001 times sizeof(RadianceVolume)
    is the Q-table memory its thesis reports for the scene (floor to the MB): the density the
    reference ran those scenes at is the default one."""
    m = oracle_mod.Sarsa(geometry(rtmi_mod, scene), 1984)
    assert int(m.n_volumes * RADIANCE_VOLUME_BYTES // 10**6) == THESIS_QTABLE_MB[scene], m.n_volumes


def test_oracle_volume_density(rtmi_mod, oracle_mod):
    """AREA_PER_SAMPLE as an argument: 0.1 gives the door room the 344 volumes of the reference's
    Images/door_room/sarsa_128_344_volumes.bmp and sarsa_12_344_volumes.png, 0.001 the 36,028 of
    vor_36028.png; placement follows the same per-surface rule."""
    g = geometry(rtmi_mod, "door_room")
    assert oracle_mod.Sarsa(g, 1984, 0.001).n_volumes == 36028
    m = oracle_mod.Sarsa(g, 1984, 0.1)
    assert m.n_volumes == 344 == int(area_counts(g.tri, 0.1).sum())
    pos, nrm, surf, kd = m.volumes()
    assert np.array_equal(np.bincount(surf, minlength=g.n_surf), area_counts(g.tri, 0.1))
    assert m.n_nodes == 2 * 344 - 1
    # the first volumes are the default map's first volumes (same Philox stream per volume index)
    pd, _, sd, _ = oracle_mod.Sarsa(g, 1984, 0.001).volumes()
    k = int(area_counts(g.tri, 0.1)[0])
    assert np.array_equal(pos[:k], pd[:k]) and np.array_equal(surf[:k], sd[:k])


@pytest.mark.parametrize("scene", ("door_room", "archway"))
def test_oracle_kd_array(rtmi_mod, oracle_mod, scene):
    """RadianceTree::convert_to_array form: children appended as pairs, every volume one
    leaf, medians separate the subtrees on their dimension (x, y, z cycling)."""
    m = oracle_mod.Sarsa(geometry(rtmi_mod, scene), 1984)
    pos, _, _, kd = m.volumes()
    n = m.n_volumes
    assert m.n_nodes == 2 * n - 1
    leaf = kd["leaf"].astype(bool)
    assert np.array_equal(np.sort(kd["vol"][leaf]), np.arange(n))
    assert np.array_equal(kd["data"][leaf], kd["vol"][leaf].astype(np.float32))
    inner = np.nonzero(~leaf)[0]
    assert np.all(kd["right"][inner] == kd["left"][inner] + 1)
    assert np.array_equal(np.sort(kd["left"][inner]), np.arange(1, 2 * n - 1, 2))
    assert kd["dim"][0] == 0 and kd["px"][0] == 0 and kd["py"][0] == 0 and kd["pz"][0] == 0
    rng = np.random.default_rng(0)
    for i in rng.choice(inner, 64, replace=False):
        d, med = int(kd["dim"][i]), kd["data"][i]
        L = leaves_under(kd, int(kd["left"][i]), [])
        R = leaves_under(kd, int(kd["right"][i]), [])
        assert pos[L, d].max() <= med <= pos[R, d].min()
        assert 0 <= len(L) - len(R) <= 1                       # left takes the median
        for c in (int(kd["left"][i]), int(kd["right"][i])):
            assert kd["dim"][c] == (d + 1) % 3


def test_oracle_nearest_self(rtmi_mod, oracle_mod):
    m = oracle_mod.Sarsa(geometry(rtmi_mod, "door_room"), 1984)
    pos, nrm, _, _ = m.volumes()
    idx = np.random.default_rng(1).choice(m.n_volumes, 4000, replace=False)
    got = m.nearest(pos[idx], nrm[idx])
    assert np.array_equal(pos[got], pos[idx]) and np.array_equal(nrm[got], nrm[idx])


def test_oracle_initial_state(rtmi_mod, oracle_mod):
    m = oracle_mod.Sarsa(geometry(rtmi_mod, "door_room"), 1984)
    q, cdf, vis, acc = m.read()
    assert np.all(q == np.float32(np.float32(1 / np.float32(144)) * np.float32(100)))
    k = np.arange(144, dtype=np.float32)
    assert np.array_equal(cdf, np.broadcast_to(k * np.float32(1 / np.float32(144)), cdf.shape))
    assert not vis.any()
    assert np.all(acc > 0)


@pytest.mark.parametrize("scene", SCENES)
def test_oracle_first_frame_path_length_matches_reference(rtmi_mod, oracle_mod, scene):
    """Statistical pin: frame 0 (initial CDF) average path length vs the reference's log."""
    ref = json.load(open(os.path.join(GOLDEN, "sarsa_ref_stats.json")))[scene]["avg_path_length"][0]
    g = geometry(rtmi_mod, scene)
    m = oracle_mod.Sarsa(g, 1984)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=48, height=48, spp=8)
    _, casts = m.render(oracle_mod.camera(rtmi_mod.CAMERAS[scene]), oracle_mod.params_from(p), 1)
    mean = casts / (48 * 48 * 8)
    assert ref - 0.5 <= mean <= ref + 2.5, (scene, mean, ref)


def test_oracle_learning_shortens_paths(rtmi_mod, oracle_mod):
    m = oracle_mod.Sarsa(geometry(rtmi_mod, "door_room"), 1984)
    p = oracle_mod.params_from(rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=64, height=64, spp=8))
    cam = oracle_mod.camera(rtmi_mod.CAMERAS["door_room"])
    lens = [m.render(cam, p, 1)[1] / (64 * 64 * 8) for _ in range(4)]
    assert lens[3] < lens[0] * 0.8, lens
    q, cdf, vis, _ = m.read()
    assert vis.sum() > 0 and np.all(q >= np.float32(1 / np.float32(144)) * np.float32(0.8))
    assert np.all(np.diff(cdf, axis=1) >= 0) and np.all(np.abs(cdf[:, -1] - 1) < 1e-4)


def test_oracle_threads_and_split_do_not_change_learning(rtmi_mod, oracle_mod):
    """Integer TD sums: the Q-table is independent of thread count and spp_split."""
    g = geometry(rtmi_mod, "door_room")
    cam = oracle_mod.camera(rtmi_mod.CAMERAS["door_room"])
    res = []
    n0 = oracle_mod.num_threads()
    try:
        for threads, split in ((1, 1), (n0, 1), (n0, 4)):
            oracle_mod.set_threads(threads)
            m = oracle_mod.Sarsa(g, 1984)
            p = oracle_mod.params_from(rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=24, height=24,
                                                               spp=8, spp_split=split))
            img, casts = m.render(cam, p, 2)
            res.append((img, casts) + m.read())
    finally:
        oracle_mod.set_threads(n0)
    for r in res[1:]:
        assert r[1] == res[0][1]
        for a, b in zip(r[2:], res[0][2:]):
            assert np.array_equal(a, b)
    assert np.array_equal(res[1][0], res[0][0])


def test_selected_volume_format_reads_reference_fixture(rtmi_mod):
    """The reference's selected_sarsa.txt (write_volume_to_file) parses with the reader
    used for this build's own dumps: position, normal, 144-sector distribution."""
    pos, nrm, dist = rtmi_mod.sarsa.read_selected_file(os.path.join(GOLDEN, "selected_sarsa_ref.txt"))
    q = np.loadtxt(os.path.join(GOLDEN, "to_select.txt"), ndmin=2).astype(np.float32)
    assert pos.shape == (3, 3) and nrm.shape == (3, 3) and dist.shape == (3, 144)
    assert np.array_equal(nrm, q[:, 3:6])                          # same-normal volumes
    assert np.all(np.abs(pos[:, 1] - q[:, 1]) < 1e-6)              # on the queried plane
    assert np.all(np.linalg.norm(pos - q[:, :3], axis=1) < 0.5)   # the pruned KD walk is approximate
    assert np.all(np.abs(dist.sum(axis=1) - 1) < 1e-5) and np.all(dist > 0)


# ---------------------------------------------------------------- GPU ----------

def _both(rtmi_mod, oracle_mod, gpu_ctx, scene, seed=1984):
    g = geometry(rtmi_mod, scene)
    sc = rtmi_mod.Scene(gpu_ctx, g)
    return g, sc, rtmi_mod.sarsa.RadianceMap(gpu_ctx, sc, seed), oracle_mod.Sarsa(g, seed)


@pytest.mark.gpu
@pytest.mark.parametrize("scene", SCENES)
def test_gpu_map_build_equals_oracle(rtmi_mod, oracle_mod, gpu_ctx, scene):
    g, sc, rm, om = _both(rtmi_mod, oracle_mod, gpu_ctx, scene)
    try:
        assert (rm.n_volumes, rm.n_nodes) == (om.n_volumes, om.n_nodes)
        for a, b in zip(rm.volumes(), om.volumes()):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
        for a, b in zip(rm.read(), om.read()):
            assert np.array_equal(a, b)
    finally:
        rm.close()
        sc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ("door_room", "complex_light_room"))
def test_gpu_nearest_equals_oracle(rtmi_mod, oracle_mod, gpu_ctx, scene):
    g, sc, rm, om = _both(rtmi_mod, oracle_mod, gpu_ctx, scene)
    try:
        pos, nrm, _, _ = om.volumes()
        rng = np.random.default_rng(5)
        n = 200_000
        i = rng.integers(0, om.n_volumes, n)
        q = pos[i] + rng.normal(0, 0.02, (n, 3)).astype(np.float32)   # near the surfaces
        qn = nrm[i].copy()
        qn[: n // 10] = nrm[rng.integers(0, om.n_volumes, n // 10)]   # mismatched normals
        a = rm.nearest(q, qn)
        b = om.nearest(q, qn)
        assert np.array_equal(a, b)
    finally:
        rm.close()
        sc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ("door_room", "complex_light_room", "archway"))
def test_gpu_nearest_grid_equals_kd(rtmi_mod, oracle_mod, gpu_ctx, scene):
    """The grid fast path returns the KD walk's volume for every query, including
    engineered ties (midpoints of same-normal volume pairs), volume positions, queries
    far from any volume (KD fallback), mismatched and signed-zero normals."""
    g, sc, rm, om = _both(rtmi_mod, oracle_mod, gpu_ctx, scene)
    S = rtmi_mod.sarsa
    try:
        pos, nrm, _, _ = om.volumes()
        rng = np.random.default_rng(11)
        n = 100_000
        i = rng.integers(0, om.n_volumes, n)
        j = rng.integers(0, om.n_volumes, n)
        near = pos[i] + rng.normal(0, 0.03, (n, 3)).astype(np.float32)
        same = (nrm[i] == nrm[j]).all(axis=1)
        mid = ((pos[i] + pos[j]) * np.float32(0.5)).astype(np.float32)[same]
        far = rng.uniform(-3, 3, (n // 10, 3)).astype(np.float32)
        q = np.concatenate([near, mid, pos[i[: n // 10]], far]).astype(np.float32)
        qn = np.concatenate([nrm[i], nrm[i][same], nrm[i[: n // 10]], nrm[j[: n // 10]]]).astype(np.float32)
        qn[::97] = nrm[rng.integers(0, om.n_volumes, len(qn[::97]))]
        qn[::89] = np.where(qn[::89] == 0, np.float32(-0.0), qn[::89])   # -0 components
        rm.set_search(S.SEARCH_KD)
        a = rm.nearest(q, qn)
        rm.set_search(S.SEARCH_GRID)
        st0 = rm.search_stats()
        b = rm.nearest(q, qn)
        st1 = rm.search_stats()
        assert st0["mode"] == S.SEARCH_GRID and st0["grid_cells"] > 0
        assert np.array_equal(a, b)
        assert np.array_equal(b, om.nearest(q, qn))
        fb = st1["kd_fallbacks"] - st0["kd_fallbacks"]
        assert fb < 0.25 * len(q), (fb, len(q))
        # queries close to a volume of their own normal almost never need the KD walk
        st0 = rm.search_stats()
        rm.nearest(pos[i] + rng.normal(0, 0.005, (n, 3)).astype(np.float32), nrm[i])
        assert rm.search_stats()["kd_fallbacks"] - st0["kd_fallbacks"] < 0.01 * n
    finally:
        rm.close()
        sc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ("door_room", "complex_light_room"))
def test_gpu_render_grid_equals_kd(rtmi_mod, gpu_ctx, scene):
    g = geometry(rtmi_mod, scene)
    sc = rtmi_mod.Scene(gpu_ctx, g)
    maps = [rtmi_mod.sarsa.RadianceMap(gpu_ctx, sc, 1984) for _ in range(2)]
    try:
        maps[0].set_search(rtmi_mod.sarsa.SEARCH_KD)
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=128, height=96, spp=16, spp_split=4)
        cam = rtmi_mod.camera(rtmi_mod.CAMERAS[scene])
        for _ in range(2):
            (ia, ca), (ib, cb) = [m.render(cam, p, 1) for m in maps]
            assert ca == cb and np.array_equal(ia, ib)
            for a, b in zip(maps[0].read(), maps[1].read()):
                assert np.array_equal(a, b)
    finally:
        for m in maps:
            m.close()
        sc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scene,split,hit_rule,spp", [("door_room", 1, 1, 8), ("door_room", 4, 1, 8),
                                                       ("cornell", 2, 1, 8), ("archway", 1, 0, 8),
                                                       ("door_room", 64, 1, 256)])  # the bench's split
def test_gpu_render_and_learning_equal_oracle(rtmi_mod, oracle_mod, gpu_ctx, scene, split, hit_rule, spp):
    g, sc, rm, om = _both(rtmi_mod, oracle_mod, gpu_ctx, scene)
    try:
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=48, height=40, spp=spp, spp_split=split,
                                    hit_rule=hit_rule)
        cam = rtmi_mod.camera(rtmi_mod.CAMERAS[scene])
        for frames in (1, 2):
            img_g, casts_g = rm.render(cam, p, frames)
            img_o, casts_o = om.render(oracle_mod.camera(rtmi_mod.CAMERAS[scene]), oracle_mod.params_from(p),
                                       frames)
            assert casts_g == casts_o
            assert np.array_equal(img_g, img_o)
            for a, b in zip(rm.read(), om.read()):
                assert np.array_equal(a, b)
            assert rm.frame_stats() == om.stats()  # the last frame's training statistics
        assert rm.frames == 3
    finally:
        rm.close()
        sc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scene,area", [("door_room", 0.1), ("door_room", 0.0045), ("cornell", 0.01)])
def test_gpu_volume_density_equals_oracle(rtmi_mod, oracle_mod, gpu_ctx, scene, area):
    """rt_sarsa_create_density: placement, KD array, initial state and two learned frames
    bit-exact with the restatement at another AREA_PER_SAMPLE (sparse maps: most queries
    leave the grid's acceptance radius and walk the KD array)."""
    g = geometry(rtmi_mod, scene)
    sc = rtmi_mod.Scene(gpu_ctx, g)
    rm = rtmi_mod.sarsa.RadianceMap(gpu_ctx, sc, 1984, area_per_sample=area)
    om = oracle_mod.Sarsa(g, 1984, area)
    try:
        assert rm.n_volumes == om.n_volumes == int(area_counts(g.tri, area).sum())
        for a, b in zip(rm.volumes(), om.volumes()):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=48, height=40, spp=8, spp_split=4)
        for _ in range(2):
            img_g, casts_g = rm.render(rtmi_mod.camera(rtmi_mod.CAMERAS[scene]), p, 1)
            img_o, casts_o = om.render(oracle_mod.camera(rtmi_mod.CAMERAS[scene]), oracle_mod.params_from(p), 1)
            assert casts_g == casts_o and np.array_equal(img_g, img_o)
            for a, b in zip(rm.read(), om.read()):
                assert np.array_equal(a, b)
            assert rm.frame_stats() == om.stats()
    finally:
        rm.close()
        sc.close()


@pytest.mark.gpu
def test_gpu_inframe_lanes_cap(rtmi_mod, gpu_ctx):
    """rt_sarsa_set_inframe_lanes caps the persistent render's workgroups: under the
    frame-synchronous rule (order-free integer TD sums) a capped launch renders and learns
    bit for bit what the whole-device launch does; a negative count is refused."""
    g = geometry(rtmi_mod, "door_room")
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        maps = [rtmi_mod.sarsa.RadianceMap(gpu_ctx, sc, 1984) for _ in range(2)]
        try:
            with pytest.raises(rtmi_mod.RtError):
                maps[0].set_inframe_lanes(-1)
            maps[1].set_inframe_lanes(300)  # two workgroups
            p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=96, height=64, spp=8, spp_split=4)
            cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
            for _ in range(2):
                (ia, ca), (ib, cb) = [m.render(cam, p, 1) for m in maps]
                assert ca == cb and np.array_equal(ia, ib)
                for a, b in zip(maps[0].read(), maps[1].read()):
                    assert np.array_equal(a, b)
                assert maps[0].frame_stats() == maps[1].frame_stats()
        finally:
            for m in maps:
                m.close()


def test_density_argument_refused(rtmi_mod):
    """area_per_sample must be finite and > 0 (checked before any device work)."""
    import ctypes
    h = ctypes.c_void_p()
    for bad in (0.0, -0.001, float("inf"), float("nan")):
        rc = rtmi_mod.lib().rt_sarsa_create_density(ctypes.c_void_p(1), ctypes.c_void_p(1), 1984, bad,
                                                    ctypes.byref(h))
        assert rc == rtmi_mod._lib.RT_E_INVALID and not h.value


def _same_bits_nan_aware(a, b):
    """bit-exact, except that NaN payloads may differ between the GPU and x86"""
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("scene,split", [("door_room", 4), ("cornell", 1), ("complex_light_room", 2)])
def test_gpu_max_direction_sampling_equals_oracle(rtmi_mod, oracle_mod, gpu_ctx, scene, split):
    """sample_max_direction_from_radiance_distribution (radiance_volume.cu:246-278) after two
    frames of CDF-sampled learning: image, casts, Q, CDF, visits, irradiance and the frame
    statistics bit-exact with the restatement over two frames in max mode."""
    g, sc, rm, om = _both(rtmi_mod, oracle_mod, gpu_ctx, scene)
    try:
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=48, height=40, spp=8, spp_split=split)
        cam = rtmi_mod.camera(rtmi_mod.CAMERAS[scene])
        ocam, op = oracle_mod.camera(rtmi_mod.CAMERAS[scene]), oracle_mod.params_from(p)
        rm.render(cam, p, 2)
        om.render(ocam, op, 2)
        rm.set_sampling(rtmi_mod.sarsa.SAMPLE_MAX)
        om.set_sampling(1)
        for _ in range(2):
            img_g, casts_g = rm.render(cam, p, 1)
            img_o, casts_o = om.render(ocam, op, 1)
            assert casts_g == casts_o
            assert _same_bits_nan_aware(img_g, img_o)
            for a, b in zip(rm.read(), om.read()):
                assert np.array_equal(a, b)
            assert rm.frame_stats() == om.stats()
        # and back to CDF sampling on the greedily trained map
        rm.set_sampling(rtmi_mod.sarsa.SAMPLE_CDF)
        om.set_sampling(0)
        img_g, _ = rm.render(cam, p, 1)
        img_o, _ = om.render(ocam, op, 1)
        assert np.array_equal(img_g, img_o)
    finally:
        rm.close()
        sc.close()


@pytest.mark.gpu
def test_gpu_max_direction_sector0_pdf_is_zero(rtmi_mod, oracle_mod, gpu_ctx):
    """Frame 0 in max mode: every Q equal, so every volume's first largest sector is 0, whose
    pdf the reference computes as cdf[0] - cdf[0] = 0 (radiance_volume.cu:274): paths that
    bounce off a surface with a volume get an infinite throughput, as in the reference;
    GPU and restatement agree on which pixels are non-finite and on all the others."""
    g, sc, rm, om = _both(rtmi_mod, oracle_mod, gpu_ctx, "cornell")
    try:
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=32, height=32, spp=4)
        cam = rtmi_mod.camera(rtmi_mod.CAMERAS["cornell"])
        rm.set_sampling(rtmi_mod.sarsa.SAMPLE_MAX)
        om.set_sampling(1)
        img_g, casts_g = rm.render(cam, p, 1)
        img_o, casts_o = om.render(oracle_mod.camera(rtmi_mod.CAMERAS["cornell"]), oracle_mod.params_from(p), 1)
        assert casts_g == casts_o
        assert not np.isfinite(img_g).all()
        assert _same_bits_nan_aware(img_g, img_o)
    finally:
        rm.close()
        sc.close()


@pytest.mark.gpu
def test_gpu_q_table_load_round_trip(rtmi_mod, oracle_mod, gpu_ctx, tmp_path):
    """rt_sarsa_save_q -> rt_sarsa_load_q into a fresh map of the same scene and seed ->
    rt_sarsa_save_q: the same bytes; Q is the file's values, visits kept (zero), irradiance
    and CDF as the restatement derives them from that Q, and the next frame renders and
    learns bit-exactly like the restatement loaded with the same Q.  A map of another seed,
    a truncated file and a file with a wrong action count are refused."""
    S = rtmi_mod.sarsa
    g, sc, rm, om = _both(rtmi_mod, oracle_mod, gpu_ctx, "door_room")
    maps = [rm]
    try:
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=64, height=48, spp=8, spp_split=2)
        cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
        rm.render(cam, p, 2)
        f1, f2 = str(tmp_path / "q1.txt"), str(tmp_path / "q2.txt")
        rm.save_q(f1)
        fresh = S.RadianceMap(gpu_ctx, sc, 1984)
        maps.append(fresh)
        fresh.load_q(f1)
        fresh.save_q(f2)
        assert open(f1, "rb").read() == open(f2, "rb").read()
        q, cdf, vis, acc = fresh.read()
        _, fq = S.read_q_file(f1)
        assert np.array_equal(q, fq.astype(np.float32))
        assert not vis.any()
        om.load_q(q)
        _, ocdf, _, oacc = om.read()
        assert np.array_equal(cdf, ocdf) and np.array_equal(acc, oacc)
        img_g, casts_g = fresh.render(cam, p, 1)
        img_o, casts_o = om.render(oracle_mod.camera(rtmi_mod.CAMERAS["door_room"]), oracle_mod.params_from(p), 1)
        assert casts_g == casts_o and np.array_equal(img_g, img_o)
        for a, b in zip(fresh.read(), om.read()):
            assert np.array_equal(a, b)
        other = S.RadianceMap(gpu_ctx, sc, 7)
        maps.append(other)
        with pytest.raises(rtmi_mod.RtError):
            other.load_q(f1)
        lines = open(f1).read().splitlines()
        (tmp_path / "short.txt").write_text("\n".join(lines[:-1]) + "\n")
        with pytest.raises(rtmi_mod.RtError):
            fresh.load_q(str(tmp_path / "short.txt"))
        (tmp_path / "bad.txt").write_text("\n".join(["100"] + lines[1:]) + "\n")
        with pytest.raises(rtmi_mod.RtError):
            fresh.load_q(str(tmp_path / "bad.txt"))
    finally:
        for m in maps:
            m.close()
        sc.close()


@pytest.mark.gpu
def test_gpu_tiles_and_td_exchange_equal_single_map(rtmi_mod, gpu_ctx):
    """Two maps rendering disjoint tile sets, TD sums added on the device, then applied on
    both == one map rendering the whole frame (the multi-GPU exchange, in one process)."""
    import torch
    from rtmi import dist as rdist, tiles as rtiles
    g = geometry(rtmi_mod, "door_room")
    sc = rtmi_mod.Scene(gpu_ctx, g)
    W = H = 64
    T = 32
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=W, height=H, spp=8, spp_split=2)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
    maps = [rtmi_mod.sarsa.RadianceMap(gpu_ctx, sc, 1984) for _ in range(3)]
    dev = torch.device("cuda", 0)
    try:
        origins = rtiles.tile_origins(W, H, T)
        full = torch.zeros(len(origins), T, T, 3, device=dev)
        casts = torch.zeros(1, dtype=torch.int64, device=dev)
        maps[0].render_tiles_device(cam, p, origins, T, full.data_ptr(), casts.data_ptr(), True, 0)
        parts = []
        for r in (0, 1):
            mine = rtiles.rank_tile_indices(W, H, T, r, 2)
            assert np.array_equal(rtiles.rank_tiles(W, H, T, r, 2), origins[mine])
            out = torch.zeros(len(mine), T, T, 3, device=dev)
            maps[1 + r].render_tiles_device(cam, p, origins[mine], T, out.data_ptr(), casts.data_ptr(), False, 0)
            parts.append((torch.from_numpy(mine).to(dev), out))
        (s1, c1), (s2, c2) = [rdist.td_tensors(m, dev) for m in maps[1:]]
        tot_s, tot_c = s1 + s2, c1 + c2
        s1.copy_(tot_s), c1.copy_(tot_c), s2.copy_(tot_s), c2.copy_(tot_c)
        maps[1].apply(0)
        maps[2].apply(0)
        torch.cuda.synchronize()
        ref = maps[0].read()
        for m in maps[1:]:
            for a, b in zip(m.read(), ref):
                assert np.array_equal(a, b)
        for mine, out in parts:
            assert torch.equal(out, full[mine])
    finally:
        for m in maps:
            m.close()
        sc.close()


@pytest.mark.gpu
def test_gpu_full_size_door_room_properties(rtmi_mod, gpu_ctx):
    """BASELINE config 3 size (512^2, 256 spp per frame): finite image, reference-like
    first-frame path length, learning shortens paths, Q/CDF invariants."""
    ref = json.load(open(os.path.join(GOLDEN, "sarsa_ref_stats.json")))["door_room"]["avg_path_length"]
    g = geometry(rtmi_mod, "door_room")
    sc = rtmi_mod.Scene(gpu_ctx, g)
    rm = rtmi_mod.sarsa.RadianceMap(gpu_ctx, sc, 1984)
    try:
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=512, height=512, spp=256, spp_split=8)
        cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
        lens, logged = [], []
        for _ in range(3):
            img, casts = rm.render(cam, p, 1)
            lens.append(casts / (512 * 512 * 256))
            paths, zero = rm.frame_stats()
            logged.append(int(rm.append_stats_line(os.devnull, 512 * 512, (paths, zero)).split()[0]))
            assert paths <= casts // 256 and 0 < zero < 512 * 512 * 256
            assert np.isfinite(img).all() and (img >= 0).all()
        assert ref[0] - 0.5 <= lens[0] <= ref[0] + 2.5
        # the statistic the reference logs (floor of per-pixel floors), frame 0: 41 in its log
        assert abs(logged[0] - ref[0]) <= 1, (logged, ref[:3])
        assert lens[2] < lens[0] * 0.6, lens
        q, cdf, vis, acc = rm.read()
        assert np.all(q >= np.float32(1 / np.float32(144)) * np.float32(0.8))
        assert np.all(np.diff(cdf, axis=1) >= 0) and np.all(np.abs(cdf[:, -1] - 1) < 1e-4)
        assert np.isfinite(acc).all()
    finally:
        rm.close()
        sc.close()


@pytest.mark.gpu
def test_gpu_q_table_and_selected_volume_dumps(rtmi_mod, gpu_ctx, tmp_path):
    """rt_sarsa_save_q / rt_sarsa_save_selected write the reference's text formats
    (radiance_map_data.txt, selected_sarsa.txt) from the map's state after a frame."""
    g = geometry(rtmi_mod, "door_room")
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        rm = rtmi_mod.sarsa.RadianceMap(gpu_ctx, sc, 1984)
        try:
            p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=64, height=64, spp=16, spp_split=4)
            rm.render(rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"]), p, 1)
            vpos, vnrm, _, _ = rm.volumes()
            q, cdf, _, _ = rm.read()
            rm.save_q(str(tmp_path / "radiance_map_data.txt"))
            fpos, fq = rtmi_mod.sarsa.read_q_file(str(tmp_path / "radiance_map_data.txt"))
            assert open(tmp_path / "radiance_map_data.txt").readline().strip() == "144"
            assert fq.shape == (rm.n_volumes, 144)
            np.testing.assert_allclose(fpos, vpos, rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(fq, q, rtol=1e-5, atol=1e-9)
            sel = os.path.join(GOLDEN, "to_select.txt")
            rm.save_selected(sel, str(tmp_path / "selected_sarsa.txt"))
            spos, snrm, sdist = rtmi_mod.sarsa.read_selected_file(str(tmp_path / "selected_sarsa.txt"))
            ref = rtmi_mod.sarsa.read_selected_file(os.path.join(GOLDEN, "selected_sarsa_ref.txt"))
            assert sdist.shape == ref[2].shape
            qs = np.loadtxt(sel, ndmin=2).astype(np.float32)
            idx = rm.nearest(qs[:, :3], qs[:, 3:6])
            np.testing.assert_allclose(spos, vpos[idx], rtol=1e-5, atol=1e-6)
            assert np.array_equal(snrm, vnrm[idx])
            pdf = np.diff(cdf[idx], axis=1, prepend=0)
            np.testing.assert_allclose(sdist, pdf, rtol=1e-5, atol=1e-9)
            assert np.all(np.abs(sdist.sum(axis=1) - 1) < 1e-4)
        finally:
            rm.close()


# ------------------------------------------ in-frame TD mode (the reference's racy rule) -----
# Last in the file: its statistical gate must never stop `pytest -x` before the exact tests.

def _paired_z(a, b):
    """z score of the mean per-pixel difference of two images (channel means): the pixels'
    estimates are independent given the frame's CDFs, and under H0 both images are unbiased
    estimates of the same pixel values, so mean(d) / (std(d) / sqrt(n)) ~ N(0, 1)."""
    d = (a.mean(axis=2) - b.mean(axis=2)).ravel().astype(np.float64)
    return float(d.mean() / (d.std(ddof=1) / np.sqrt(d.size)))


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ("door_room", "cornell"))
def test_gpu_in_frame_single_lane_equals_sequential_restatement(rtmi_mod, oracle_mod, gpu_ctx, scene):
    """RT_SARSA_TD_INFRAME with one active lane (a 1 x 1 image, spp_split 1): the TD events
    then run one at a time in sample order, which is exactly the restatement's sequential
    in-frame rule (rt_oracle.c td_inframe: temporal_difference_update + expected_sarsa_irradiance,
    radiance_volume.cu:282-301, :93-112, applied in place).  Image, casts, Q, CDF, visits and
    irradiance bit-exact over three CDF frames, then two frames of max-direction sampling,
    whose argmax the in-frame mode takes from the live Q at every sample (:251-257)."""
    S = rtmi_mod.sarsa
    g, sc, rm, om = _both(rtmi_mod, oracle_mod, gpu_ctx, scene)
    try:
        rm.set_td_mode(S.TD_INFRAME)
        om.set_td_mode(1)
        assert rm.td_mode == S.TD_INFRAME
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=1, height=1, spp=512, spp_split=1)
        cam = rtmi_mod.camera(rtmi_mod.CAMERAS[scene])
        ocam, op = oracle_mod.camera(rtmi_mod.CAMERAS[scene]), oracle_mod.params_from(p)
        q0 = rm.read()[0]
        for frame in range(5):
            if frame == 3:
                rm.set_sampling(S.SAMPLE_MAX)
                om.set_sampling(1)
            img_g, casts_g = rm.render(cam, p, 1)
            img_o, casts_o = om.render(ocam, op, 1)
            assert casts_g == casts_o, (frame, casts_g, casts_o)
            assert _same_bits_nan_aware(img_g, img_o), frame
            for a, b in zip(rm.read(), om.read()):
                assert _same_bits_nan_aware(a, b), frame
        q, _, vis, _ = rm.read()
        assert vis.sum() > 100                      # the rule ran, in place
        assert not np.array_equal(q, q0)
    finally:
        rm.close()
        sc.close()


@pytest.mark.gpu
def test_gpu_in_frame_td_mode(rtmi_mod, oracle_mod, gpu_ctx):
    """RT_SARSA_TD_INFRAME on a 64^2 x 16 door_room frame, every lane racing as in the
    reference.  Exact where the rule leaves nothing to the race: frame 0 samples from the
    initial CDFs in both modes, so its image and casts equal the deterministic mode's and the
    restatement's, and so do the visit counts (integer atomics); unvisited sectors keep their
    Q; Q stays finite and >= RADIANCE_THRESHOLD.

    Statistical after that: the race decides which interleaving of the events happens, so the
    GPU's Q-table is one of many the rule allows.  Whatever the (full-support) CDFs, each
    frame is an unbiased estimate of the same pixel values, so frames 1-3 are gated against
    the sequential restatement of the rule (oracle in-frame mode) by the paired z score of
    the mean per-pixel difference (_paired_z), combined over the frames: |z| < 4 (two-sided
    p = 6e-5 under H0).  The fixed 5 % ratio this replaces failed on the driver's round-3 run
    (GPU in-frame means 0.322 / 0.308 / 0.326; the restatement's in-frame rule gives
    0.341 / 0.331 / 0.314, its frame-synchronous rule 0.341 / 0.335 / 0.334): at this size one
    frame's mean has a standard error of about 0.01 (3 %), so a 5 % bound on the ratio of two
    differently learned estimators is a 1.7-sigma gate.  Per-frame z of both rules over 4
    seeds: profiles/r4b/sarsa_inframe_probe.json (tools/sarsa_inframe_probe.py)."""
    S = rtmi_mod.sarsa
    g, sc, rm, om = _both(rtmi_mod, oracle_mod, gpu_ctx, "door_room")
    rf = S.RadianceMap(gpu_ctx, sc, 1984)
    of = oracle_mod.Sarsa(g, 1984)
    try:
        rf.set_td_mode(S.TD_INFRAME)
        of.set_td_mode(1)
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=64, height=64, spp=16, spp_split=4)
        cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
        ocam, op = oracle_mod.camera(rtmi_mod.CAMERAS["door_room"]), oracle_mod.params_from(p)
        q0 = rf.read()[0]
        img_d, casts_d = rm.render(cam, p, 1)
        img_f, casts_f = rf.render(cam, p, 1)
        img_o, casts_o = om.render(ocam, op, 1)
        img_s, casts_s = of.render(ocam, op, 1)
        assert casts_f == casts_d == casts_o == casts_s
        assert np.array_equal(img_f, img_d) and np.array_equal(img_d, img_o) and np.array_equal(img_o, img_s)
        qd, _, vd, _ = rm.read()
        qf, cf, vf, af = rf.read()
        assert np.array_equal(vf, vd) and vd.sum() > 0
        assert np.array_equal(vf, of.read()[2])
        assert np.array_equal(qf[vf == 0], q0[vf == 0])
        assert np.isfinite(qf).all() and np.isfinite(af).all() and np.isfinite(cf).all()
        assert (qf >= np.float32(0.8 / 144) * np.float32(0.999)).all()
        vis = vf > 0
        corr = np.corrcoef(of.read()[0][vis], qf[vis])[0, 1]
        assert corr > 0.9, corr
        zs = []
        for _ in range(3):
            zs.append(_paired_z(rf.render(cam, p, 1)[0], of.render(ocam, op, 1)[0]))
        z = sum(zs) / np.sqrt(len(zs))
        assert abs(z) < 4.0, (zs, z)
        assert np.isfinite(rf.read()[0]).all()
        with pytest.raises(rtmi_mod.RtError):
            rf.set_td_mode(7)
    finally:
        rf.close()
        rm.close()
        sc.close()


@pytest.mark.gpu
def test_gpu_in_frame_mode_refuses_td_exchange(rtmi_mod, gpu_ctx):
    """The in-frame rule updates the map in place: the C ABI hands out no TD sums and refuses
    a tile render that would leave them for a cross-GPU exchange (apply = 0)."""
    import torch
    S = rtmi_mod.sarsa
    g = geometry(rtmi_mod, "door_room")
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        rf = S.RadianceMap(gpu_ctx, sc, 1984)
        try:
            rf.set_td_mode(S.TD_INFRAME)
            with pytest.raises(rtmi_mod.RtError):
                rf.td_device()
            p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=32, height=32, spp=4)
            out = torch.zeros(1, 32, 32, 3, device="cuda:0")
            casts = torch.zeros(1, dtype=torch.int64, device="cuda:0")
            cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
            with pytest.raises(rtmi_mod.RtError):
                rf.render_tiles_device(cam, p, np.zeros((1, 2), np.int32), 32, out.data_ptr(), casts.data_ptr(),
                                       False, 0)
            rf.render_tiles_device(cam, p, np.zeros((1, 2), np.int32), 32, out.data_ptr(), casts.data_ptr(), True, 0)
            torch.cuda.synchronize()
            assert rf.read()[2].sum() > 0
            rf.set_td_mode(S.TD_FRAME)
            assert rf.td_device()[2] == rf.n_volumes * 144
        finally:
            rf.close()


# The reference's training runs, recovered from their own logs (tests/golden/sarsa_ref_stats.json,
# written per frame by GPU/main.cu:321-339): 720 x 720, ONE sample per pixel (the zero-contribution
# count is a count of samples: 463,054 of 518,400 in Cornell's frame 0), GPU-engine preset, the
# default AREA_PER_SAMPLE (test_volume_count_matches_reference_qtable_memory), and the reference's own
# in-frame TD rule racing at the reference GPU's concurrency.  That rule's outcome depends on how
# many paths update the table at once: the reference's GTX 1070 Ti has 19 SMs, and a
# register-bound kernel of 64-thread blocks keeps about 256 threads per SM resident -- 4,864 paths in
# flight (rt_sarsa_set_inframe_lanes).  At 2,432 - 9,728 paths every scene's whole log is matched
# (profiles/r6f/, tools/sarsa_pin.py --lanes); with the MI355X's whole occupancy (~330 k paths) the
# door room learns 17 % slower than its log, and the frame-synchronous rule slower still (up to 78 %).
REF_LANES = 4864


def _log_runs(scene):
    """the logged training runs of a scene: complex_light_room's file holds two (rows 0-41 and a
    restart at row 42, where the frame-0 values 34 / 305,873 come back), the others one"""
    ref = json.load(open(os.path.join(GOLDEN, "sarsa_ref_stats.json")))[scene]
    path = [int(x) for x in ref["avg_path_length"]]
    zero = ref["zero_contribution_paths"]
    starts = [0] + [i for i in range(1, len(path)) if path[i] == path[0] and abs(zero[i] - zero[0]) < 0.01 * zero[0]]
    ends = starts[1:] + [len(path)]
    return [(path[a:b], zero[a:b]) for a, b in zip(starts, ends)]


def _train(rtmi_mod, gpu_ctx, sc, scene, frames, mode, lanes=REF_LANES, final_spp=0):
    """(logged path length per frame, zero-contribution samples per frame, final frame's logged
    path length and image) of a 720^2 x 1 spp run from a fresh map"""
    S = rtmi_mod.sarsa
    W = H = 720
    rm = S.RadianceMap(gpu_ctx, sc, 1984)
    try:
        if mode == "inframe":
            rm.set_td_mode(S.TD_INFRAME)
            rm.set_inframe_lanes(lanes)
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=W, height=H, spp=1, spp_split=1)
        cam = rtmi_mod.camera(rtmi_mod.CAMERAS[scene])
        logged, zero = [], []
        for _ in range(frames):
            rm.render(cam, p, 1)
            paths, z = rm.frame_stats()
            logged.append(paths // (W * H))
            zero.append(z)
        final = None
        if final_spp:
            pf = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=W, height=H, spp=final_spp, spp_split=8)
            img, _ = rm.render(cam, pf, 1)
            final = (rm.frame_stats()[0] // (W * H), img)
    finally:
        rm.close()
    return logged, zero, final


def _trajectory_misses(logged, zero, rl, rz):
    """the gate: the logged path length (floor over pixels of the per-pixel floor) within 1 of the
    log's on every frame; zero-contribution samples within 1 % on frame 0 (the initial CDF), within
    6 % on every later frame and within 2 % on average over them.  Returns what missed."""
    n = min(len(logged), len(rl))
    miss = []
    dp = [abs(logged[f] - rl[f]) for f in range(n)]
    if max(dp) > 1:
        miss.append(f"path length off by {max(dp)} at frame {dp.index(max(dp))}")
    if abs(zero[0] - rz[0]) > 0.01 * rz[0]:
        miss.append(f"frame 0 zero count {zero[0]} vs {rz[0]}")
    dz = [abs(zero[f] - rz[f]) / rz[f] for f in range(1, n)]
    if dz and max(dz) > 0.06:
        miss.append(f"zero count off by {max(dz):.3f} at frame {1 + dz.index(max(dz))}")
    if dz and sum(dz) / len(dz) > 0.02:
        miss.append(f"zero count off by {sum(dz) / len(dz):.4f} on average")
    return miss


@pytest.mark.gpu
@pytest.mark.parametrize("scene", SCENES)
def test_gpu_learning_trajectory_matches_reference_logs(rtmi_mod, gpu_ctx, scene):
    """Every logged frame of the reference's Expected-SARSA training runs (100 frames; complex_light_room:
    both of its runs, 42 and 100 frames) against ours at its settings (REF_LANES): the logged path
    length and the zero-contribution samples per frame (_trajectory_misses; a path whose radiance is
    NaN in the reference -- the zero direction of a failed CDF search -- is not a zero-contribution
    one: NaN < threshold is false).  Negative controls, which the gate must refuse: the
    frame-synchronous rule, and (door_room) the in-frame rule racing at the MI355X's whole occupancy."""
    runs = _log_runs(scene)
    assert len(runs) == (2 if scene == "complex_light_room" else 1)
    frames = max(len(r[0]) for r in runs)
    with rtmi_mod.Scene(gpu_ctx, geometry(rtmi_mod, scene)) as sc:
        logged, zero, _ = _train(rtmi_mod, gpu_ctx, sc, scene, frames, "inframe")
        for rl, rz in runs:
            miss = _trajectory_misses(logged, zero, rl, rz)
            assert not miss, (miss, logged[:12], rl[:12], zero[:12], rz[:12])
        assert logged[-1] < logged[0]
        lf, zf, _ = _train(rtmi_mod, gpu_ctx, sc, scene, frames, "frame")
        assert any(_trajectory_misses(lf, zf, rl, rz) for rl, rz in runs), (scene, lf[:12], zf[:12])
        if scene == "door_room":
            lw, zw, _ = _train(rtmi_mod, gpu_ctx, sc, scene, frames, "inframe", lanes=0)
            assert _trajectory_misses(lw, zw, *runs[0]), (lw[:12], zw[:12])


# (scene, ref block-mean key, path length in the file name: sarsa_128spp_3avg_44Mb.png,
# sarsa_128spp_5avg_300Mb.png, sarsa_128_spp_avg_pl_5_max_pl_80.png)
SARSA_RENDERS = [("cornell", "cornell_sarsa_128spp", 3), ("complex_light_room", "complex_light_sarsa_128spp", 5),
                 ("door_room", "door_room_sarsa_128spp", 5)]


def _render_misses(rtmi_mod, rgb, logged_len, ref, name_len):
    rgb8 = rtmi_mod.metrics.argb_to_rgb8(rtmi_mod.pack_argb(rgb)).astype(np.float64)
    d = np.abs(rgb8.reshape(16, 45, 16, 45, 3).mean(axis=(1, 3)) - ref)
    miss = []
    if d.mean() > 1.2 or d.max() > 12.0:
        miss.append(f"block means off by {d.mean():.3f} (max {d.max():.2f})")
    if abs(logged_len - name_len) > 1:
        miss.append(f"logged path length {logged_len} vs the file name's {name_len}")
    return miss


@pytest.mark.gpu
@pytest.mark.parametrize("scene,key,name_len", SARSA_RENDERS)
def test_gpu_sarsa_render_matches_reference_sarsa_render(rtmi_mod, gpu_ctx, scene, key, name_len):
    """The reference's Expected-SARSA renders (Images/<scene>/sarsa_128spp_*.png, 720x720, 128 spp,
    block means in tests/golden/scenes_ref_stats.json) against ours after the logged training run
    (100 1-spp frames, the in-frame rule at REF_LANES): 45x45 block means within 1.2 of 255 on
    average (12 at most) and the logged path length of the 128-spp frame within 1 of the file name's.
    Negative control: the default (uniform) render of the scene fails the gate -- on its path length
    (the block means alone cannot tell an unbiased sampler's converged render from the learned one).
    The frame-synchronous rule is refused by the trajectory gate above (its zero-contribution counts);
    on the door room the render gate refuses it as well (logged path length 7).  The archway's SARSA
    render is not a target: it is 6 % darker than the reference's own default render of the scene
    (109.7 vs 116.3 of 255), which an unbiased sampler cannot be (ours: 3.5 of 255 from it in block
    mean at these settings)."""
    ref = np.array(json.load(open(os.path.join(GOLDEN, "scenes_ref_stats.json")))[key]["means"])
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS[scene])
    with rtmi_mod.Scene(gpu_ctx, geometry(rtmi_mod, scene)) as sc:
        _, _, (ln, img) = _train(rtmi_mod, gpu_ctx, sc, scene, 100, "inframe", final_spp=128)
        miss = _render_misses(rtmi_mod, img, ln, ref, name_len)
        assert not miss, miss
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=720, height=720, spp=128, spp_split=8)
        uni, casts = rtmi_mod.render(gpu_ctx, sc, cam, p)
        assert _render_misses(rtmi_mod, uni, casts // (720 * 720 * 128), ref, name_len)
        if scene == "door_room":
            _, _, (lf, imgf) = _train(rtmi_mod, gpu_ctx, sc, scene, 100, "frame", final_spp=128)
            assert _render_misses(rtmi_mod, imgf, lf, ref, name_len)
