"""Neural-Q training renderer: NeuralQPathtracer::render_frame
(GPU/deep_learning/neural_q_pathtracer.cu:226-600) on the device, rt_neuralq_*.

The learning rule itself is checked against the fp64 restatement in test_dqn.py (parity
unpinned against DyNet).  Here: the renderer's estimator (with epsilon = 1 every direction
is a uniformly chosen jittered cell, pdf RHO: the GPU-preset uniform path tracer's
estimator, so the frames agree statistically), the per-sample statistics, epsilon decay,
determinism, and that rendering trains the network.
"""
import os

import numpy as np
import pytest

from conftest import MODELS

pytestmark = pytest.mark.gpu


def _cornell(rtmi_mod):
    g = rtmi_mod.cornell_geometry(rtmi_mod.RT_PRESET_GPU)
    return g, rtmi_mod.camera(rtmi_mod.CAMERAS["cornell"])


def _trainer(rtmi_mod, ctx, g, lr=1e-3):
    # the Cornell box has no OBJ vertex list: its triangles' vertices stand in
    nn = g.nn_vertices if g.nn_vertices is not None else g.all_triangles().reshape(-1).astype(np.float32)
    W, b = rtmi_mod.dqn.synthetic_weights(nn.size)
    return rtmi_mod.dqn.DqnTrainer(ctx, nn, W, b, learning_rate=lr)


def test_explore_only_frame_is_the_uniform_estimator(rtmi_mod, gpu_ctx):
    """epsilon = 1: uniform cells, throughput * cos / RHO * BRDF, light emission at the end:
    the same estimator as the GPU preset's uniform sampler.  16x16-pixel block means of a
    96x96 frame agree with a 1024-spp uniform render within 5 standard errors, and the
    frame-mean per channel within 3; the average path length of the stats rows (bounce of
    termination) is the uniform render's casts per sample minus one, within 0.1."""
    g, cam = _cornell(rtmi_mod)
    W = H = 96
    spp = 64
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=W, height=H, spp=spp)
    with rtmi_mod.Scene(gpu_ctx, g) as sc, _trainer(rtmi_mod, gpu_ctx, g) as tr, \
            rtmi_mod.dqn.NeuralQ(gpu_ctx, sc, tr, batch_size=4096, epsilon_start=1.0, epsilon_min=1.0,
                                 epsilon_decay=0.0) as nq:
        img, stats, casts = nq.render_frame(cam, p)
        pr = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=W, height=H, spp=1024, spp_split=16)
        ref, ref_casts = rtmi_mod.render(gpu_ctx, sc, cam, pr)
        pu = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=W, height=H, spp=spp)
        uni, _ = rtmi_mod.render(gpu_ctx, sc, cam, pu)
    assert np.isfinite(img).all() and stats.shape == (spp, 3)
    # per-block standard error from the uniform render at the same spp
    blk = lambda a: a.reshape(H // 16, 16, W // 16, 16, 3).mean(axis=(1, 3))
    se = np.sqrt(uni.reshape(H // 16, 16, W // 16, 16, 3).var(axis=(1, 3)) / 256.0)
    z = np.abs(blk(img) - blk(ref)) / np.maximum(se, 1e-6)
    assert np.mean(z) < 1.5 and np.max(z) < 5.0, (np.mean(z), np.max(z))
    se_all = np.sqrt(uni.reshape(-1, 3).var(axis=0) / (W * H))
    assert np.all(np.abs(img.reshape(-1, 3).mean(0) - ref.reshape(-1, 3).mean(0)) < 3 * se_all)
    avg_bounces = float(stats[:, 0].mean())
    assert abs(avg_bounces - (ref_casts / (W * H * 1024) - 1.0)) < 0.1, (avg_bounces, ref_casts / (W * H * 1024))
    assert casts > W * H * spp


def test_stats_epsilon_decay_and_learning(rtmi_mod, gpu_ctx, tmp_path):
    """Per-sample rows (path length, loss summed over the batches, zero-contribution paths),
    epsilon = max(epsilon - decay, min) after every sample, and the network's parameters
    change; the rows print as nn_training_stats.txt lines."""
    g, cam = _cornell(rtmi_mod)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=32, height=32, spp=4)
    with rtmi_mod.Scene(gpu_ctx, g) as sc, _trainer(rtmi_mod, gpu_ctx, g) as tr:
        W0, b0 = tr.params()
        with rtmi_mod.dqn.NeuralQ(gpu_ctx, sc, tr, batch_size=256, epsilon_start=0.9, epsilon_min=0.3,
                                  epsilon_decay=0.25) as nq:
            assert nq.epsilon == pytest.approx(0.9)
            img, stats, _ = nq.render_frame(cam, p)
            assert nq.epsilon == pytest.approx(0.3)
            img2, stats2, _ = nq.render_frame(cam, p)
        W1, b1 = tr.params()
    assert np.isfinite(img).all() and np.isfinite(img2).all()
    assert np.all(stats[:, 0] > 0) and np.all(stats[:, 0] <= 80)
    assert np.all(stats[:, 1] > 0) and np.isfinite(stats[:, 1]).all()
    assert np.all(stats[:, 2] >= 0) and np.all(stats[:, 2] <= 32 * 32)
    assert not all(np.array_equal(a, c) for a, c in zip(W0, W1))
    lines = rtmi_mod.dqn.NeuralQ.stats_lines(np.concatenate([stats, stats2])).splitlines()
    assert len(lines) == 8
    for ln, row in zip(lines, np.concatenate([stats, stats2])):
        a, l, z = ln.split()
        assert float(a) == pytest.approx(row[0], rel=1e-5) and int(z) == int(row[2])


def test_deterministic(rtmi_mod, gpu_ctx):
    """Same seed, same starting network: the same frame, statistics and trained parameters,
    bit for bit (fixed-order reductions, integer counters only)."""
    g, cam = _cornell(rtmi_mod)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=24, height=16, spp=2)
    out = []
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        for _ in range(2):
            with _trainer(rtmi_mod, gpu_ctx, g) as tr, rtmi_mod.dqn.NeuralQ(gpu_ctx, sc, tr, batch_size=128) as nq:
                img, stats, casts = nq.render_frame(cam, p)
                out.append((img, stats, casts, tr.params()))
    (i1, s1, c1, (W1, _)), (i2, s2, c2, (W2, _)) = out
    assert c1 == c2 and np.array_equal(i1, i2) and np.array_equal(s1, s2)
    assert all(np.array_equal(a, b) for a, b in zip(W1, W2))


def test_door_room_obj_scene_runs(rtmi_mod, gpu_ctx):
    """An OBJ scene with the reference's network shape (the door room's 342 inputs)."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "door_room.obj"), "door_room")
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=32, height=32, spp=2)
    with rtmi_mod.Scene(gpu_ctx, g) as sc, _trainer(rtmi_mod, gpu_ctx, g) as tr, \
            rtmi_mod.dqn.NeuralQ(gpu_ctx, sc, tr, batch_size=512) as nq:
        img, stats, casts = nq.render_frame(cam, p)
    assert np.isfinite(img).all() and img.mean() > 0
    assert np.isfinite(stats).all() and casts > 0


def test_trained_network_beats_the_untrained_one(rtmi_mod, gpu_ctx):
    """Two frames of Neural-Q training on the door room (from synthetic He-normal weights),
    then the pretrained-network renderer (config 4's sampler) at equal spp: the trained
    network's frame is closer to a 1024-spp uniform render than the untrained one's (MAPE),
    and its paths are shorter.  Measured at 720^2 (tools/neuralq_train.py,
    profiles/r2_neuralq_door_room_720.json): MAPE 0.63 vs 0.90, block-mean error vs the
    reference's own 128-spp render 4.2 vs 45.4 of 255, 33.6 vs 50.6 casts per sample."""
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "door_room.obj"), "door_room")
    cam = rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"])
    S = 128
    W0, b0 = rtmi_mod.dqn.synthetic_weights(g.nn_vertices.size)
    with rtmi_mod.Scene(gpu_ctx, g) as sc:
        with rtmi_mod.dqn.DqnTrainer(gpu_ctx, g.nn_vertices, W0, b0) as tr:
            with rtmi_mod.dqn.NeuralQ(gpu_ctx, sc, tr, batch_size=4096) as nq:
                p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=S, height=S, spp=2)
                for _ in range(2):
                    nq.render_frame(cam, p)
            W1, b1 = tr.params()
        pe = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=S, height=S, spp=16)
        ref, _ = rtmi_mod.render(gpu_ctx, sc, cam, rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=S, height=S,
                                                                         spp=1024, spp_split=16))
        out = {}
        for name, (W, b) in (("synthetic", (W0, b0)), ("trained", (W1, b1))):
            with rtmi_mod.dqn.Dqn(gpu_ctx, g.nn_vertices, W, b) as net:
                out[name] = rtmi_mod.dqn.render(gpu_ctx, sc, net, cam, pe)
    m = {k: float(np.mean(np.abs(v[0] - ref) / np.maximum(ref, 1e-3))) for k, v in out.items()}
    assert m["trained"] < 0.85 * m["synthetic"], m
    assert out["trained"][1] < out["synthetic"][1]


# The reference's Neural-Q training run of the door room (Radiance_Map_Data/door_room_12_12_stats.txt,
# tests/golden/nn_ref_stats.json): one row per training sample (neural_q_pathtracer.cu:545-583), the
# average path length falling linearly from 50.3 to 33.5 over 100 rows as epsilon decays from 1 by
# EPSILON_DECAY 0.01 to EPSILON_MIN 0.05 (deep_learning_settings.h:5-8), 720x720, batch 4096
# (main.cu:116-124), DyNet's Adam defaults, the network from DyNet's default Glorot initialisation.
# Measured over all 100 rows (tools/nq_pin.py, profiles/r6h/, r6j/): our rows within 0.29 of the log
# at three seeds (mean difference -0.06 ... +0.09; rows 0-19 within 0.12); a network that does not
# learn (learning rate 1e-9) drifts 3.5 above it by row 19.  The zero-contribution column is not
# gated: ours is 1.97-2.12x the log's from row 0 on (epsilon 1, uniform cells), where the equal path
# lengths already pin the sampling; the statistic counts the paths still bouncing after 80 bounces
# by their throughput, which depends on settings the row-0 path lengths do not see.
def _nq_rows(rtmi_mod, ctx, rows, lr):
    g = rtmi_mod.obj_geometry(os.path.join(MODELS, "door_room.obj"), "door_room")
    W0, b0 = rtmi_mod.dqn.glorot_weights(g.nn_vertices.size)
    out = []
    with rtmi_mod.Scene(ctx, g) as sc, rtmi_mod.dqn.DqnTrainer(ctx, g.nn_vertices, W0, b0, learning_rate=lr) as tr, \
            rtmi_mod.dqn.NeuralQ(ctx, sc, tr, batch_size=4096, epsilon_start=1.0, epsilon_min=0.05,
                                 epsilon_decay=0.01) as nq:
        p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=720, height=720, spp=1)
        for _ in range(rows):
            _, st, _ = nq.render_frame(rtmi_mod.camera(rtmi_mod.CAMERAS["door_room"]), p)
            out.append(float(st[0, 0]))
    return np.array(out)


def test_training_trajectory_matches_reference_log(rtmi_mod, gpu_ctx):
    """Rows 0-11 of the door room's logged training run (average path length within 0.3 on every
    row); negative control: the same run with a network that does not learn misses by row 11."""
    import json
    from conftest import GOLDEN
    ref = np.array(json.load(open(os.path.join(GOLDEN, "nn_ref_stats.json")))["door_room_12_12"]["avg_path_length"])
    rows = _nq_rows(rtmi_mod, gpu_ctx, 12, 1e-3)
    d = rows - ref[:12]
    assert np.abs(d).max() <= 0.3, np.round(d, 3)
    assert rows[-1] < rows[0] - 1.0
    still = _nq_rows(rtmi_mod, gpu_ctx, 12, 1e-9)
    assert np.abs(still - ref[:12]).max() > 1.0, np.round(still - ref[:12], 3)
