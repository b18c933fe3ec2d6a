"""DQN Q-value path (BASELINE config 4): DyNet reader, forward pass, Q-weighted
sampling, wavefront render.

Parity levels:
  * reader, sampler: bit-exact with the oracle (same Q in -> same direction, pdf, action)
  * forward: layer 0 folded to an fp32 affine map of the ray position + bf16 MFMA
    layers 1-3, vs the oracle's forward with the same arithmetic (same fold, same
    operand and activation rounding, exact accumulation): max |dq| <= 2e-2 * max|q|,
    mean <= 2e-3 * mean|q|; vs the fp32 forward (the reference's DyNet arithmetic):
    mean <= 1e-2 * mean|q|
  * render: statistical (a Q perturbation can flip one sampled cell and change a path):
    MAPE(gpu, oracle) must not exceed the oracle's own seed-to-seed MAPE.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, MODELS

DOOR_MODEL = os.path.join(MODELS, "door_room_12_12.model")


def door(rtmi_mod):
    return rtmi_mod.obj_geometry(os.path.join(MODELS, "door_room.obj"), "door_room")


def trained(rtmi_mod):
    return rtmi_mod.dqn.split_layers(rtmi_mod.dqn.read_dynet(DOOR_MODEL))


def room_points(geom, n, seed):
    """random points on the room's surfaces (where Q is evaluated) + their triangles"""
    rng = np.random.default_rng(seed)
    tri = rng.integers(0, geom.n_surf, n)
    v = geom.tri.reshape(-1, 3, 3)[tri]
    a, b = rng.random((2, n, 1), dtype=np.float32)
    flip = (a + b) > 1
    a[flip], b[flip] = 1 - a[flip], 1 - b[flip]
    p = v[:, 0] + a * (v[:, 1] - v[:, 0]) + b * (v[:, 2] - v[:, 0])
    return p.astype(np.float32), tri.astype(np.int32)


# ---------------------------------------------------------------- CPU ----------

def test_dynet_reader_product_equals_oracle(rtmi_mod, oracle_mod):
    a = rtmi_mod.dqn.read_dynet(DOOR_MODEL)
    b = oracle_mod.read_dynet(DOOR_MODEL)
    assert [x.shape for x in a] == [(200, 342), (200,), (300, 200), (300,), (200, 300), (200,),
                                    (144, 200), (144,)]
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_oracle_forward_trained_door_room(rtmi_mod, oracle_mod):
    g = door(rtmi_mod)
    W, b = trained(rtmi_mod)
    p, _ = room_points(g, 64, 1)
    q = oracle_mod.dqn_forward(W, b, g.nn_vertices, p)
    assert q.shape == (64, 144) and np.all(q >= 0)           # ReLU output layer
    assert np.mean(q.sum(axis=1) > 0) > 0.9                  # non-degenerate distributions
    qb = oracle_mod.dqn_forward(W, b, g.nn_vertices, p, bf16=True)
    assert np.mean(np.abs(qb - q)) <= 1e-2 * np.mean(np.abs(q))


def test_oracle_sampler_properties(rtmi_mod, oracle_mod):
    g = door(rtmi_mod)
    n = 512
    p, tri = room_points(g, n, 2)
    q = np.zeros((n, 144), np.float32)
    q[:, 37] = 1.0  # all mass in one cell
    pix = np.arange(n, dtype=np.uint32)
    qc, tp, d, act = oracle_mod.dqn_sample(g.all_triangles(), q, p, tri, pix, 0, 1, 1984,
                                           np.ones((n, 3), np.float32))
    assert np.all(act == 37)
    assert np.allclose(np.linalg.norm(d, axis=1), 1.0, atol=1e-5)
    nrm = oracle_mod.normals(g.all_triangles())[tri]
    cos = np.sum(nrm * d, axis=1)
    assert np.all(cos > -1e-6)
    # pdf = (1/2pi) * 144 for a one-cell distribution: tp = cos / pdf
    assert np.allclose(tp[:, 0], cos * (2 * np.pi) / 144, rtol=1e-5, atol=1e-7)
    # all-zero Q: no cell, direction zero, throughput untouched (the reference's miss)
    _, tp0, d0, act0 = oracle_mod.dqn_sample(g.all_triangles(), np.zeros((4, 144), np.float32), p[:4],
                                             tri[:4], pix[:4], 0, 1, 1984, np.ones((4, 3), np.float32))
    assert np.all(act0 == -1) and np.all(d0 == 0) and np.all(tp0 == 1)


def test_oracle_sampler_draws_cells_by_q_cos(rtmi_mod, oracle_mod):
    """The blocked sum order is still importance_sample_direction's
    distribution: over many rays the chosen cells follow Q*cos / total (chi-square against
    the per-ray probabilities the sampler itself returns), a zero cell is never chosen, and
    every block is reached (mass spread so that each block holds some)."""
    g = door(rtmi_mod)
    n = 40000
    p, tri = room_points(g, n, 3)
    rng = np.random.default_rng(7)
    q = (rng.random((n, 144)) * (rng.random((n, 144)) < 0.5)).astype(np.float32)
    q[:, 20] = 0.0  # a cell never to be drawn
    pix = np.arange(n, dtype=np.uint32)
    qc, _, _, act = oracle_mod.dqn_sample(g.all_triangles(), q, p, tri, pix, 0, 1, 1984,
                                          np.ones((n, 3), np.float32))
    ok = qc.sum(axis=1) > 0
    assert ok.mean() > 0.99 and np.all(act[ok] >= 0)
    act = act[ok]
    prob = qc[ok] / qc[ok].sum(axis=1, keepdims=True)
    assert np.all(prob[np.arange(len(act)), act] > 0)            # never a zero-probability cell
    assert np.all(act != 20)
    obs = np.bincount(act, minlength=144)
    exp = prob.sum(axis=0)
    assert np.all(np.bincount(act // 36, minlength=4) > 0.2 * len(act) / 4)
    m = exp > 5
    chi2 = float(((obs[m] - exp[m]) ** 2 / exp[m]).sum())
    dof = int(m.sum()) - 1
    assert chi2 < dof + 5.0 * np.sqrt(2.0 * dof), (chi2, dof)    # ~5 sigma


# ---------------------------------------------------------------- GPU ----------

@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["door_room", "archway"])
def test_forward_matches_oracle(rtmi_mod, oracle_mod, gpu_ctx, kind):
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, f"{kind}.obj"), kind)
    W, b = trained(rtmi_mod) if kind == "door_room" else rtmi_mod.dqn.synthetic_weights(g.nn_vertices.size)
    pts, _ = room_points(g, 777, 3)  # not a multiple of the 64-row tile
    with rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        q = net.forward(pts)
    qe = oracle_mod.dqn_forward(W, b, g.nn_vertices, pts, bf16=True)
    qf = oracle_mod.dqn_forward(W, b, g.nn_vertices, pts, bf16=False)
    err = np.abs(q - qe)
    assert err.max() <= 2e-2 * np.abs(qe).max() + 1e-6, err.max()
    assert err.mean() <= 2e-3 * np.abs(qe).mean() + 1e-7, err.mean()
    assert np.abs(q - qf).mean() <= 1e-2 * np.abs(qf).mean()


@pytest.mark.gpu
def test_sampler_bit_exact(rtmi_mod, oracle_mod, gpu_ctx):
    g = door(rtmi_mod)
    n = 2000
    pts, tri = room_points(g, n, 4)
    rng = np.random.default_rng(5)
    q = rng.random((n, 144), dtype=np.float32) * (rng.random((n, 144)) < 0.3)
    q[:3] = 0.0  # no cell selectable
    pix = rng.integers(0, 1 << 20, n).astype(np.uint32)
    tp = rng.random((n, 3), dtype=np.float32)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        gq, gtp, gd, ga = rtmi_mod.dqn.sample(gpu_ctx, sc, 1984, q, pts, tri, pix, 3, 2, tp)
    oq, otp, od, oa = oracle_mod.dqn_sample(g.all_triangles(), q, pts, tri, pix, 3, 2, 1984, tp)
    assert np.array_equal(ga, oa)
    assert np.array_equal(gq.view(np.uint32), oq.view(np.uint32))
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
    assert np.array_equal(gtp.view(np.uint32), otp.view(np.uint32))
    assert np.all(ga[:3] == -1)


@pytest.mark.gpu
def test_dqn_render_statistical(rtmi_mod, oracle_mod, gpu_ctx):
    g = door(rtmi_mod)
    W, b = trained(rtmi_mod)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=128, height=128, spp=16)  # 80 bounces
    rect = (48, 48, 32, 32)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
    with rtmi_mod.Scene(gpu_ctx, g) as sc, rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        img, casts = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p, rect)
        img2, casts2 = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p, rect)
    assert np.array_equal(img, img2) and casts == casts2  # deterministic
    ocam = oracle_mod.camera(rtmi_mod.CAMERAS["door_room"])
    ref, rc = oracle_mod.render_dqn(g, W, b, g.nn_vertices, ocam, oracle_mod.params_from(p), rect, bf16=True)
    p2 = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=128, height=128, spp=16, seed=7)
    alt, _ = oracle_mod.render_dqn(g, W, b, g.nn_vertices, ocam, oracle_mod.params_from(p2), rect, bf16=True)
    noise = rtmi_mod.metrics.mape_f(ref, alt)
    m = rtmi_mod.metrics.mape_f(ref, img)
    assert m <= noise, (m, noise)
    assert abs(casts - rc) <= 0.05 * rc
    assert img.mean() > 0


def zscores(a, b):
    """per-channel z-score of the mean per-pixel difference a - b"""
    d = (a.astype(np.float64) - b.astype(np.float64)).reshape(-1, 3)
    se = d.std(axis=0) / np.sqrt(d.shape[0])
    return np.abs(d.mean(axis=0)) / np.maximum(se, 1e-30)


@pytest.mark.gpu
def test_config4_archway_dqn_matches_oracle(rtmi_mod, oracle_mod, gpu_ctx):
    """BASELINE config 4 at its own workload: archway (102 triangles, 918 network inputs),
    the GPU-engine preset (80 bounces), Q-weighted sampling from the fc_layer network
    (synthetic He-normal weights: the archway model is not in the reference), a 64x64
    window of the 1024x1024 frame, against the oracle's render with the kernel's bf16
    arithmetic (PretrainedPathtracer::render_frame, pre_trained_pathtracer.cu:188-491;
    importance_sample_direction, nn_rendering_helpers.cu:391-489)."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "archway.obj"), "archway")
    W, b = rtmi_mod.dqn.synthetic_weights(g.nn_vertices.size)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=1024, height=1024, spp=4)
    assert p.max_bounces == 80
    rect = (448, 448, 64, 64)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["archway"])
    with rtmi_mod.Scene(gpu_ctx, g) as sc, rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        img, casts = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p, rect)
    ocam = oracle_mod.camera(rtmi_mod.CAMERAS["archway"])
    ref, rc = oracle_mod.render_dqn(g, W, b, g.nn_vertices, ocam, oracle_mod.params_from(p), rect, bf16=True)
    p2 = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=1024, height=1024, spp=4, seed=7)
    alt, _ = oracle_mod.render_dqn(g, W, b, g.nn_vertices, ocam, oracle_mod.params_from(p2), rect, bf16=True)
    assert np.isfinite(img).all() and img.mean() > 0
    z = zscores(img, ref)
    assert np.all(z < 3.0), z
    assert abs(casts - rc) <= 0.01 * rc, (casts, rc)
    noise = rtmi_mod.metrics.mape_f(ref, alt)
    assert rtmi_mod.metrics.mape_f(ref, img) <= noise, (rtmi_mod.metrics.mape_f(ref, img), noise)


def test_oracle_bf16_q_rounding_gate(rtmi_mod, oracle_mod):
    """Statistical gate of the renderer's bf16 Q (round 4: k_dqn_mlp<.., QB> stores Q in bf16
    for the sampler; the restatement rounds the same way): the door_room frame with the
    trained network, the same paths with Q rounded and with the fp32 Q the sampler took
    before (CPU, no GPU).  Rounding can only move a CDF boundary by < 2^-9 of a cell's Q, so
    the two renders differ where a draw falls in that sliver: the per-channel z of the paired
    per-pixel differences stays below 3.5, and their MAPE stays below the seed-to-seed MAPE
    of the unrounded render."""
    g = door(rtmi_mod)
    W, b = trained(rtmi_mod)
    cam = oracle_mod.camera(rtmi_mod.CAMERAS["door_room"])
    rect = (56, 56, 16, 16)
    p = oracle_mod.params_from(rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=128, height=128, spp=8))
    p7 = oracle_mod.params_from(rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=128, height=128, spp=8, seed=7))
    rq, _ = oracle_mod.render_dqn(g, W, b, g.nn_vertices, cam, p, rect, bf16=True, q_bf16=True)
    rf, _ = oracle_mod.render_dqn(g, W, b, g.nn_vertices, cam, p, rect, bf16=True, q_bf16=False)
    alt, _ = oracle_mod.render_dqn(g, W, b, g.nn_vertices, cam, p7, rect, bf16=True, q_bf16=False)
    assert rq.mean() > 0 and not np.array_equal(rq, rf)  # the rounding does change some paths
    z = zscores(rq, rf)
    assert np.all(z < 3.5), z
    assert rtmi_mod.metrics.mape_f(rf, rq) <= rtmi_mod.metrics.mape_f(rf, alt)


def test_oracle_wavefront_render_equals_per_path(rtmi_mod, oracle_mod):
    """orc_render_dqn_wave fed by the restatement's own bf16 forward is orc_render_dqn bit for
    bit: the wavefront order and the batched Q change nothing (CPU, no GPU)."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "archway.obj"), "archway")
    W, b = rtmi_mod.dqn.synthetic_weights(g.nn_vertices.size)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=1024, height=1024, spp=2)
    rect = (480, 480, 12, 10)
    ocam = oracle_mod.camera(rtmi_mod.CAMERAS["archway"])
    op = oracle_mod.params_from(p)
    ref, rc = oracle_mod.render_dqn(g, W, b, g.nn_vertices, ocam, op, rect, bf16=True)
    got, gc, calls = oracle_mod.render_dqn_wave(
        g, ocam, op, lambda loc: oracle_mod.dqn_forward(W, b, g.nn_vertices, loc, bf16=True), rect)
    assert gc == rc and np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert len(calls) > 10 and calls[0] <= 12 * 10 * 2


@pytest.mark.gpu
def test_config4_bit_exact_downstream_of_forward(rtmi_mod, oracle_mod, gpu_ctx):
    """BASELINE config 4 (archway, 918 inputs, 80 bounces, a 64x64 window of the 1024x1024
    frame, 4 spp) bit for bit in image and ray casts: the restatement's trace, Q.cos sampler
    and sums (PretrainedPathtracer::render_frame, pre_trained_pathtracer.cu:188-491;
    importance_sample_direction, nn_rendering_helpers.cu:391-489) run on the Q values of the
    device forward itself (k_dqn_mlp via rt_dqn_forward, the same kernel the render uses).
    The only stage left out is the bf16 GEMM, gated on its own by test_forward_matches_oracle."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "archway.obj"), "archway")
    W, b = rtmi_mod.dqn.synthetic_weights(g.nn_vertices.size)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=1024, height=1024, spp=4)
    assert p.max_bounces == 80
    rect = (448, 448, 64, 64)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["archway"])
    with rtmi_mod.Scene(gpu_ctx, g) as sc, rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        img, casts = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p, rect)
        ref, rc, calls = oracle_mod.render_dqn_wave(g, oracle_mod.camera(rtmi_mod.CAMERAS["archway"]),
                                                    oracle_mod.params_from(p), net.forward, rect)
    assert len(calls) > 20
    assert casts == rc, (casts, rc)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), \
        int((img.view(np.uint32) != ref.view(np.uint32)).sum())


@pytest.mark.gpu
def test_config4_full_frame_properties(rtmi_mod, gpu_ctx):
    """The whole config-4 frame at its stated size (1024x1024, 512 spp, ~12 s per render):
    deterministic, the tile-list render equals the rectangle render, finite, and the ray casts
    per sample in the archway band."""
    torch = pytest.importorskip("torch")
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "archway.obj"), "archway")
    W, b = rtmi_mod.dqn.synthetic_weights(g.nn_vertices.size)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=1024, height=1024, spp=512)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["archway"])
    with rtmi_mod.Scene(gpu_ctx, g) as sc, rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        img, casts = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p)
        img2, casts2 = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p)
        tiles = rtmi_mod.tiles.tile_origins(1024, 1024, 32)
        out = torch.zeros((len(tiles), 32, 32, 3), dtype=torch.float32, device="cuda")
        tc = torch.zeros(1, dtype=torch.int64, device="cuda")
        rtmi_mod.dqn.render_tiles_device(gpu_ctx, sc, net, cam, p, tiles, 32, out.data_ptr(), tc.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        timg = rtmi_mod.tiles.assemble(out.cpu().numpy()[None], 1024, 1024, 32, 1)
    assert np.array_equal(img, img2) and casts == casts2
    assert np.array_equal(img, timg) and int(tc.item()) == casts
    assert np.isfinite(img).all() and img.mean() > 0
    per_sample = casts / (1024 * 1024 * 512)
    assert 30.0 < per_sample < 45.0, per_sample  # 37.5 at 512 spp (profiles/r1_configs_full.json c4)


@pytest.mark.gpu
def test_dqn_tiles_equal_rect(rtmi_mod, gpu_ctx):
    torch = pytest.importorskip("torch")
    g = door(rtmi_mod)
    W, b = trained(rtmi_mod)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=64, height=64, spp=4, max_bounces=12)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
    with rtmi_mod.Scene(gpu_ctx, g) as sc, rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        full, _ = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p)
        tiles = rtmi_mod.tiles.tile_origins(64, 64, 32)
        out = torch.zeros((len(tiles), 32, 32, 3), dtype=torch.float32, device="cuda")
        casts = torch.zeros(1, dtype=torch.int64, device="cuda")
        rtmi_mod.dqn.render_tiles_device(gpu_ctx, sc, net, cam, p, tiles, 32, out.data_ptr(),
                                         casts.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    img = rtmi_mod.tiles.assemble(out.cpu().numpy()[None], 64, 64, 32, 1)
    assert np.array_equal(img, full)


@pytest.mark.gpu
def test_dqn_samples_in_flight_bit_identical(rtmi_mod, gpu_ctx, monkeypatch):
    """Samples traced concurrently (ray = slot * pixels + pixel) give the image of one
    sample at a time: each path depends only on (pixel, sample), and the per-pixel
    totals add the slots in sample order."""
    g = door(rtmi_mod)
    W, b = trained(rtmi_mod)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=48, height=32, spp=6, max_bounces=16)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
    res = []
    with rtmi_mod.Scene(gpu_ctx, g) as sc, rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        for rays in (1, 2 * 1536, 1 << 22):   # 1, 2 (4 + 2) and all 6 samples in flight
            monkeypatch.setenv("RTMI_DQN_RAYS_IN_FLIGHT", str(rays))
            res.append(rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p))
    for img, casts in res[1:]:
        assert casts == res[0][1]
        assert np.array_equal(img.view(np.uint32), res[0][0].view(np.uint32))


@pytest.mark.gpu
def test_dqn_selected_volume_dump(rtmi_mod, oracle_mod, gpu_ctx, tmp_path):
    """rt_dqn_save_selected writes selected_deep.txt: location, normal, Q / sum(Q) of the
    network at the location (q_value_extractor.cu); the normalised Q agree with the
    oracle's fp32 (DyNet-arithmetic) forward within the bf16 tolerance."""
    g = door(rtmi_mod)
    W, b = trained(rtmi_mod)
    sel = os.path.join(GOLDEN, "to_select.txt")
    with rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        net.save_selected(sel, str(tmp_path / "selected_deep.txt"))
        pos, nrm, dist = rtmi_mod.sarsa.read_selected_file(str(tmp_path / "selected_deep.txt"))
        qs = np.loadtxt(sel, ndmin=2).astype(np.float32)
        assert np.array_equal(pos, qs[:, :3]) and np.array_equal(nrm, qs[:, 3:6])
        q = net.forward(qs[:, :3])
        np.testing.assert_allclose(dist, q / q.sum(axis=1, keepdims=True), rtol=1e-5, atol=1e-9)
    qf = oracle_mod.dqn_forward(W, b, g.nn_vertices, qs[:, :3], bf16=False)
    ref = qf / qf.sum(axis=1, keepdims=True)
    assert np.abs(dist - ref).mean() <= 1e-2 * np.abs(ref).mean()
    assert np.all(np.abs(dist.sum(axis=1) - 1) < 1e-4)


# --- Neural-Q training -------------------------------

def _tiny_net(rng, n_in=12, hidden=(7, 9, 6), n_out=144):
    dims = [n_in, *hidden, n_out]
    W = [rng.standard_normal((dims[i + 1], dims[i])) * np.sqrt(2.0 / dims[i]) for i in range(4)]
    b = [np.full(dims[i + 1], 0.1) for i in range(4)]
    return W, b


def test_train_ref_gradients_match_finite_differences(oracle_mod):
    """The fp64 learning-rule restatement's backward pass against central differences."""
    rng = np.random.default_rng(5)
    W, b = _tiny_net(rng)
    ref = oracle_mod.AdamRef(rng.standard_normal(12), W, b)
    loc = rng.uniform(-1, 1, (9, 3))
    act = rng.integers(0, 144, 9)
    act[3] = -1  # ignored row
    tgt = rng.uniform(0, 2, 9)
    loss, G = ref.loss_grads(loc, act, tgt)
    h = 1e-6
    for i in range(8):
        P = ref.P[i]
        for idx in [tuple(rng.integers(0, s) for s in P.shape) for _ in range(6)]:
            old = P[idx]
            P[idx] = old + h
            lp, _ = ref.loss_grads(loc, act, tgt)
            P[idx] = old - h
            lm, _ = ref.loss_grads(loc, act, tgt)
            P[idx] = old
            fd = (lp - lm) / (2 * h)
            assert abs(fd - G[i][idx]) <= 1e-5 * max(1.0, abs(fd)), (i, idx, fd, G[i][idx])


def test_train_ref_adam_reduces_loss_and_clips(oracle_mod):
    rng = np.random.default_rng(6)
    W, b = _tiny_net(rng)
    ref = oracle_mod.AdamRef(rng.standard_normal(12), W, b, lr=1e-2)
    loc = rng.uniform(-1, 1, (32, 3))
    act = rng.integers(0, 144, 32)
    tgt = rng.uniform(0, 3, 32)
    losses = [ref.step(loc, act, tgt)[0] for _ in range(30)]
    assert losses[-1] < 0.5 * losses[0]
    # clipping: the first Adam step moves every parameter by at most lr (|m/sqrt(v)| <= 1)
    ref2 = oracle_mod.AdamRef(rng.standard_normal(12), W, b, lr=1e-3)
    P0 = [p.copy() for p in ref2.P]
    ref2.step(loc, act, tgt * 100.0)
    assert max(float(np.max(np.abs(p - q))) for p, q in zip(ref2.P, P0)) <= 1e-3 * (1 + 1e-9)


def test_td_targets_oracle_rule(oracle_mod):
    """compute_td_targets: terminal rows take the reward; action 0 enters the max unweighted;
    cosines lie in (0, 1]."""
    rng = np.random.default_rng(7)
    n = 64
    q = rng.uniform(0, 1, (n, 144)).astype(np.float32)
    q[:8, 0] = 10.0  # action 0 dominates (no cosine)
    term = (np.arange(n) % 5 == 4).astype(np.int32)
    rw = rng.uniform(0, 1, n).astype(np.float32)
    dc = rng.uniform(0.2, 1, n).astype(np.float32)
    pix = rng.integers(0, 1 << 20, n).astype(np.uint32)
    t = oracle_mod.td_targets(1984, q, term, rw, dc, pix, 3, 2)
    assert np.array_equal(t[term == 1], rw[term == 1])
    live = (term == 0)
    ub = rw + np.maximum(q[:, 0], q[:, 1:].max(1)) * dc
    assert np.all(t[live] <= ub[live] + 1e-6)
    first = np.arange(n) < 8
    assert np.allclose(t[first & live], (rw + np.float32(10.0) * dc)[first & live])


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.gpu
def test_train_step_matches_fp64_restatement(rtmi_mod, oracle_mod, gpu_ctx):
    """Three Adam steps of the device learning rule on the trained door_room network
    (342 -> 200 -> 300 -> 200 -> 144), 777 rays (ragged), against the fp64 restatement:
    loss and gradient norm within 1e-4 relative; parameter updates within 1% of the
    learning rate on all but 0.1% of the parameters (Adam's first steps are ~sign(g) * lr,
    so a gradient that is rounding noise in one of the two may flip), never more than
    2 lr per step."""
    import torch
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "door_room.obj"), "door_room")
    W, b = trained(rtmi_mod)
    pts, _ = room_points(g, 777, 11)
    rng = np.random.default_rng(12)
    act = rng.integers(0, 144, 777).astype(np.int32)
    act[::97] = -1
    tgt = rng.uniform(0.0, 2.0, 777).astype(np.float32)
    lr = 1e-3
    ref = oracle_mod.AdamRef(g.nn_vertices, W, b, lr=lr)
    P0 = [p.copy() for p in ref.P]
    d_loc, d_act, d_tgt = _dev(pts), _dev(act), _dev(tgt)
    with rtmi_mod.dqn.DqnTrainer(gpu_ctx, g.nn_vertices, W, b, learning_rate=lr) as tr:
        for _ in range(3):
            loss, gn = tr.step_device(d_loc.data_ptr(), d_act.data_ptr(), d_tgt.data_ptr(), 777)
            rl, rg = ref.step(pts, act, tgt)
            assert abs(loss - rl) <= 1e-4 * rl, (loss, rl)
            assert abs(gn - rg) <= 1e-4 * rg, (gn, rg)
        torch.cuda.synchronize()
        Wg, bg = tr.params()
    got = Wg + bg
    n_par = sum(p.size for p in got)
    bad = 0
    for p_gpu, p_ref, p0 in zip(got, ref.P, P0):
        dg = p_gpu.astype(np.float64) - p0
        dr = p_ref - p0
        diff = np.abs(dg - dr)
        assert diff.max() <= 2 * 3 * lr * (1 + 1e-3)
        bad += int(np.count_nonzero(diff > 1e-2 * lr))
    assert bad <= 1e-3 * n_par, (bad, n_par)


@pytest.mark.gpu
def test_train_steps_reduce_loss_and_feed_inference(rtmi_mod, gpu_ctx, tmp_path):
    """Repeated steps on one batch drive its loss down; the trained parameters build an
    inference network (rt_dqn_create) whose Q moves toward the targets."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "archway.obj"), "archway")
    W, b = rtmi_mod.dqn.synthetic_weights(g.nn_vertices.size)
    pts, _ = room_points(g, 1024, 13)
    rng = np.random.default_rng(14)
    act = rng.integers(0, 144, 1024).astype(np.int32)
    tgt = rng.uniform(0.5, 1.5, 1024).astype(np.float32)
    d_loc, d_act, d_tgt = _dev(pts), _dev(act), _dev(tgt)
    with rtmi_mod.dqn.DqnTrainer(gpu_ctx, g.nn_vertices, W, b, learning_rate=1e-3) as tr:
        losses = [tr.step_device(d_loc.data_ptr(), d_act.data_ptr(), d_tgt.data_ptr(), 1024)[0]
                  for _ in range(40)]
        W2, b2 = tr.params()
    assert all(np.isfinite(losses)) and losses[-1] < 0.5 * losses[0], losses[::8]
    with rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W2, b2) as net:
        q = net.forward(pts)
    err = np.mean((q[np.arange(1024), act] - tgt) ** 2)
    assert err * 1024 < 0.6 * losses[0], (err * 1024, losses[0])
    # saved in the reference's DyNet format and loaded back: the same network, bit for bit
    path = str(tmp_path / "archway_trained.model")
    rtmi_mod.dqn.write_dynet(path, rtmi_mod.dqn.join_layers(W2, b2))
    W3, b3 = rtmi_mod.dqn.split_layers(rtmi_mod.dqn.read_dynet(path))
    with rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W3, b3) as net:
        assert np.array_equal(net.forward(pts), q)


@pytest.mark.gpu
def test_td_targets_bit_exact(rtmi_mod, oracle_mod, gpu_ctx):
    import torch
    rng = np.random.default_rng(15)
    n = 1000
    q = rng.uniform(0, 1, (n, 144)).astype(np.float32)
    term = (rng.random(n) < 0.2).astype(np.int32)
    rw = rng.uniform(0, 1, n).astype(np.float32)
    dc = rng.uniform(0.2, 1, n).astype(np.float32)
    pix = rng.integers(0, 1 << 22, n).astype(np.uint32)
    out = torch.zeros(n, dtype=torch.float32, device="cuda")
    bufs = [_dev(x) for x in (q, term, rw, dc, pix.view(np.int32))]  # kept alive over the launch
    rtmi_mod.dqn.td_targets_device(gpu_ctx, 1984, *[t.data_ptr() for t in bufs], 5, 3, n, out.data_ptr())
    torch.cuda.synchronize()
    want = oracle_mod.td_targets(1984, q, term, rw, dc, pix, 5, 3)
    assert np.array_equal(out.cpu().numpy(), want)


def test_dynet_writer_reproduces_reference_model(rtmi_mod, tmp_path):
    """rt_dynet_write of the parameters read from the reference's door_room model gives the
    reference's file back byte for byte (TextFileSaver format, neural_q_pathtracer.cu:193)."""
    params = rtmi_mod.dqn.read_dynet(DOOR_MODEL)
    out = tmp_path / "door_room_rewritten.model"
    rtmi_mod.dqn.write_dynet(str(out), params)
    assert out.read_bytes() == open(DOOR_MODEL, "rb").read()


def test_dynet_write_read_round_trip(rtmi_mod, tmp_path):
    """trained / synthetic weights -> DyNet text -> rt_dynet_read: bit-exact, shapes kept,
    extreme and denormal floats included; bad shapes are refused."""
    W, b = rtmi_mod.dqn.synthetic_weights(918, seed=7)
    W[0][0, :4] = [np.float32(1e-40), np.float32(-3.4e38), np.float32(0.0), np.float32(-0.0)]
    params = rtmi_mod.dqn.join_layers(W, b)
    out = str(tmp_path / "archway.model")
    rtmi_mod.dqn.write_dynet(out, params)
    back = rtmi_mod.dqn.read_dynet(out)
    assert [x.shape for x in back] == [x.shape for x in params]
    for x, y in zip(back, params):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
    with pytest.raises(ValueError):
        rtmi_mod.dqn.write_dynet(out, [np.zeros((2, 2, 2), np.float32)])
    # an (n, 1) matrix stays a matrix, a vector a vector
    col = np.arange(5, dtype=np.float32).reshape(5, 1)
    rtmi_mod.dqn.write_dynet(out, [col, col[:, 0]])
    text = open(out).read()
    assert "{5,1}" in text and "{5}" in text
    back = rtmi_mod.dqn.read_dynet(out)
    assert back[0].shape == (5, 1) and back[1].shape == (5,)
    # a diverged trainer's nan / inf cannot be written: DyNet's loader cannot parse them
    for bad in (np.nan, np.inf):
        x = np.ones(3, np.float32)
        x[1] = bad
        with pytest.raises(RuntimeError):
            rtmi_mod.dqn.write_dynet(out, [x])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["door_room", "archway"])
def test_gpu_weight_stationary_forward_equals_streaming(rtmi_mod, gpu_ctx, kind):
    """The weight-stationary forward (rt_dqn_ws.hip, RT_DQN_MLP_STATIONARY) and the
    weight-streaming one (the default) give the same Q bit for bit: same fragments, same K
    order of the fp32 accumulation; ragged ray counts included."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, kind + ".obj"), kind)
    W, b = trained(rtmi_mod) if kind == "door_room" else rtmi_mod.dqn.synthetic_weights(g.nn_vertices.size)
    lo, hi = g.all_triangles().reshape(-1, 3).min(0), g.all_triangles().reshape(-1, 3).max(0)
    rng = np.random.default_rng(3)
    with rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        for n in (1, 31, 33, 1000, 70_001):
            loc = (lo + (hi - lo) * rng.random((n, 3))).astype(np.float32)
            net.set_mlp(net.MLP_STATIONARY)
            qa = net.forward(loc)
            net.set_mlp(net.MLP_STREAM)
            qs = net.forward(loc)
            assert qa.shape == (n, 144) and np.isfinite(qa).all()
            assert np.array_equal(qa.view(np.uint32), qs.view(np.uint32)), n


@pytest.mark.gpu
def test_gpu_weight_stationary_render_equals_streaming(rtmi_mod, gpu_ctx):
    """Both forward kernels write the renderer's bf16 Q (k_dqn_mlp<.., QB>, k_dqn_mlp_ws): the
    archway render is the same bit for bit whichever computes it."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "archway.obj"), "archway")
    W, b = rtmi_mod.dqn.synthetic_weights(g.nn_vertices.size)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=1024, height=1024, spp=2)
    rect = (448, 448, 64, 64)
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["archway"])
    with rtmi_mod.Scene(gpu_ctx, g) as sc, rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
        img_s, casts_s = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p, rect)
        net.set_mlp(net.MLP_STATIONARY)
        img_w, casts_w = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p, rect)
        net.set_mlp(net.MLP_STREAM)
    assert casts_s == casts_w and np.array_equal(img_s.view(np.uint32), img_w.view(np.uint32))


# ------------------------------------------ reference NN renders (GPU) ----------

def _block_means8(rtmi_mod, img):
    rgb8 = rtmi_mod.metrics.argb_to_rgb8(rtmi_mod.pack_argb(img)).astype(np.float64)
    return rgb8.reshape(16, 45, 16, 45, 3).mean(axis=(1, 3))


def _transposed(W):
    """each weight matrix read in the other order: its column-major bytes taken row-major (the
    DyNet order error the gate must see)"""
    return [np.ascontiguousarray(w.ravel(order="F").reshape(w.shape)) for w in W]


@pytest.mark.gpu
@pytest.mark.parametrize("scene,model,key,casts_band", [
    # nn_128spp_32avg.png: "32avg" is the pretrained renderer's logged average path length,
    # int(sum of the last sample's ray_bounces / pixels), ray_bounces = casts - 1
    # (pre_trained_pathtracer.cu:366-375, :409, :453-464)
    ("door_room", "door_room_12_12.model", "door_room_nn_128spp", (32.0, 34.0)),
    ("cornell", "cornell_12_12.model", "cornell_nn_128spp", None),
])
def test_gpu_dqn_render_matches_reference_nn_render(rtmi_mod, gpu_ctx, scene, model, key, casts_band):
    """The pretrained renderer (PretrainedPathtracer::render_frame, pre_trained_pathtracer.cu:188-491)
    with the reference's own trained networks, against the renders the reference made with them
    (Images/door_room/nn_128spp_32avg.png, Images/cornell/nn_128spp_avg.png; 45x45 block means of
    the 8-bit images in tests/golden/scenes_ref_stats.json), at the reference's 720x720, 128 spp,
    GPU-engine preset.  A learned sampler gives zero probability to cells whose Q is 0, so its
    render is biased in a pattern of its own: the NN renders differ from the default renders of
    the same scenes by 1.26 (door room) and 1.82 (Cornell) of 255 in block mean, and ours
    reproduces the reference's NN render to 0.36 / 0.36 (profiles/r5a_nn_pin.json).  That pins the
    DyNet reader, the weight order, the layer-0 fold, the bf16 forward and the Q.cos sampler end
    to end against the reference's output.  Negative control: the same parameters read in the
    wrong matrix order render at 31 / 23 of 255 from it, with the door room's paths back at the
    uniform sampler's 51 casts."""
    import json
    from conftest import GOLDEN
    ref = np.array(json.load(open(os.path.join(GOLDEN, "scenes_ref_stats.json")))[key]["means"])
    if scene == "cornell":
        g = rtmi_mod.cornell_geometry(rtmi_mod.RT_PRESET_GPU)
    else:
        g = rtmi_mod.obj_geometry(os.path.join(MODELS, f"{scene}.obj"), scene)
    W, b = rtmi_mod.dqn.split_layers(rtmi_mod.dqn.read_dynet(os.path.join(MODELS, model)))
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS[scene])
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=720, height=720, spp=128)
    res = {}
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        for kind, WW in (("trained", W), ("transposed", _transposed(W))):
            with rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, WW, b) as net:
                img, casts = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, p)
            d = np.abs(_block_means8(rtmi_mod, img) - ref)
            res[kind] = (float(d.mean()), float(d.max()), casts / (720 * 720 * 128))
    mean_d, max_d, cps = res["trained"]
    assert mean_d <= 0.7 and max_d <= 4.0, res
    if casts_band is not None:
        assert casts_band[0] <= cps <= casts_band[1], res  # measured 33.78: 32.78 bounces
    tmean, _, tcps = res["transposed"]
    assert tmean >= 10.0, res
    if casts_band is not None:
        assert tcps > casts_band[1] + 10.0, res
