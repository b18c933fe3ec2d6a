"""DQN Q-value network (BASELINE config 4) on top of the C ABI.

  read_dynet(path)        the reference's DyNet text models (Radiance_Map_Data/*.model),
                          via rt_dynet_read; W row-major [out][in]
  write_dynet(path, params)   the same format out (rt_dynet_write), e.g. DqnTrainer.params()
  synthetic_weights(...)  seeded He-normal weights for scenes whose trained model the
                          reference does not ship (archway: 918 inputs)
  Dqn(ctx, nn_vertices, weights)   device network (rt_dqn_create)
  forward / sample / render / render_tiles_device
  DqnTrainer(ctx, nn_vertices, weights)   Neural-Q training (rt_dqn_trainer_*): TD targets,
                          one Adam step per batch, parameters out for a new Dqn
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._lib import check, lib
from .api import Context, Scene, _fp, _ip

HIDDEN = (200, 300, 200)  # NN_Builders/dq_network.cu:14-17
ACTIONS = 144             # GRID_RESOLUTION^2


def read_dynet(path: str) -> List[np.ndarray]:
    """Parameters of a DyNet TextFileSaver model in file order (row-major)."""
    L = lib()
    n_params, n_values = ctypes.c_int(0), ctypes.c_int64(0)
    check(L.rt_dynet_read(path.encode(), 0, None, None, None, ctypes.byref(n_params),
                          ctypes.byref(n_values)))
    rows = np.zeros(n_params.value, np.int32)
    cols = np.zeros(n_params.value, np.int32)
    vals = np.zeros(n_values.value, np.float32)
    check(L.rt_dynet_read(path.encode(), n_params.value, _ip(rows), _ip(cols), _fp(vals),
                          ctypes.byref(n_params), ctypes.byref(n_values)))
    out, off = [], 0
    for r, c in zip(rows, cols):  # cols 0: a vector ("{rows}" header)
        n = int(r) * max(int(c), 1)
        a = vals[off:off + n]
        out.append(a.copy() if c == 0 else a.reshape(int(r), int(c)).copy())
        off += n
    return out


def write_dynet(path: str, params: Sequence[np.ndarray]) -> None:
    """DyNet TextFileSaver model (neural_q_pathtracer.cu:193) of `params` in order: matrices
    row-major [rows][cols], vectors [rows]; read_dynet(path) returns them bit for bit, shapes
    included (an (n, 1) matrix stays one).  Non-finite values raise (DyNet cannot load them)."""
    arrs = [np.ascontiguousarray(p, np.float32) for p in params]
    for a in arrs:
        if a.ndim not in (1, 2) or a.size == 0:
            raise ValueError(f"DyNet parameters are non-empty vectors or matrices, got {a.shape}")
    rows = np.array([a.shape[0] for a in arrs], np.int32)
    cols = np.array([a.shape[1] if a.ndim == 2 else 0 for a in arrs], np.int32)  # 0: vector
    vals = np.concatenate([a.ravel() for a in arrs]) if arrs else np.zeros(1, np.float32)
    check(lib().rt_dynet_write(os.fsencode(path), len(arrs), _ip(rows), _ip(cols), _fp(vals)))


def join_layers(W: Sequence[np.ndarray], b: Sequence[np.ndarray]) -> list:
    """([W1..W4], [b1..b4]) -> [W1, b1, ..., W4, b4] (the reference's parameter order)"""
    return [x for pair in zip(W, b) for x in pair]


def split_layers(params: Sequence[np.ndarray]) -> Tuple[list, list]:
    """[W1, b1, ..., W4, b4] -> ([W1..W4], [b1..b4])"""
    if len(params) != 8:
        raise ValueError(f"expected 8 parameters (4 affine layers), got {len(params)}")
    return [np.ascontiguousarray(params[i], np.float32) for i in (0, 2, 4, 6)], \
           [np.ascontiguousarray(params[i], np.float32).ravel() for i in (1, 3, 5, 7)]


def synthetic_weights(n_in: int, seed: int = 1984, hidden=HIDDEN, n_out: int = ACTIONS,
                      bias: float = 0.05) -> Tuple[list, list]:
    """He-normal (std sqrt(2/fan_in)) weights from numpy's PCG64 seeded with `seed`, constant
    positive biases: a stand-in for models the reference does not ship."""
    rng = np.random.default_rng(seed)
    dims = [n_in, *hidden, n_out]
    W = [(rng.standard_normal((dims[i + 1], dims[i])) * np.sqrt(2.0 / dims[i])).astype(np.float32)
         for i in range(4)]
    b = [np.full(dims[i + 1], bias, np.float32) for i in range(4)]
    return W, b


def glorot_weights(n_in: int, seed: int = 1984, hidden=HIDDEN, n_out: int = ACTIONS) -> Tuple[list, list]:
    """DyNet's default initialiser, the one the reference's network starts from (FCLayer's
    model.add_parameters with no initializer, NN_Builders/fc_layer.cu:32-33: ParameterInitGlorot,
    gain 1): uniform in +-sqrt(6 / sum of the tensor's dims) -- sqrt(6 / (out + in)) for a weight
    matrix, sqrt(6 / out) for a bias -- here from numpy's PCG64 seeded with `seed` (DyNet's own
    random stream is not reproducible without DyNet)."""
    rng = np.random.default_rng(seed)
    dims = [n_in, *hidden, n_out]
    W, b = [], []
    for i in range(4):
        sw = np.sqrt(6.0 / (dims[i + 1] + dims[i]))
        W.append(rng.uniform(-sw, sw, (dims[i + 1], dims[i])).astype(np.float32))
        sb = np.sqrt(6.0 / dims[i + 1])
        b.append(rng.uniform(-sb, sb, dims[i + 1]).astype(np.float32))
    return W, b


class Dqn:
    def __init__(self, ctx: Context, nn_vertices: np.ndarray, W: Sequence[np.ndarray],
                 b: Sequence[np.ndarray]):
        self.ctx = ctx
        self.nn_vertices = np.ascontiguousarray(nn_vertices, np.float32).ravel()
        self.W = [np.ascontiguousarray(w, np.float32) for w in W]
        self.b = [np.ascontiguousarray(x, np.float32).ravel() for x in b]
        self.n_in = int(self.W[0].shape[1])
        if self.nn_vertices.size != self.n_in:
            raise ValueError(f"network has {self.n_in} inputs, scene has {self.nn_vertices.size}")
        hidden = np.array([w.shape[0] for w in self.W[:3]], np.int32)
        Wp = (ctypes.POINTER(ctypes.c_float) * 4)(*[_fp(w) for w in self.W])
        bp = (ctypes.POINTER(ctypes.c_float) * 4)(*[_fp(x) for x in self.b])
        self._h = ctypes.c_void_p()
        check(lib().rt_dqn_create(ctx.handle, _fp(self.nn_vertices), self.n_in, _ip(hidden),
                                  int(self.W[3].shape[0]), Wp, bp, ctypes.byref(self._h)))

    @property
    def handle(self):
        return self._h

    MLP_AUTO, MLP_STREAM, MLP_STATIONARY = 0, 1, 2  # RT_DQN_MLP_*

    def set_mlp(self, mode: int) -> None:
        """forward kernel: MLP_AUTO / MLP_STREAM (weight streaming) or MLP_STATIONARY"""
        check(lib().rt_dqn_set_mlp(self._h, mode))

    def forward(self, loc: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(loc, np.float32).reshape(-1, 3)
        q = np.zeros((x.shape[0], ACTIONS), np.float32)
        check(lib().rt_dqn_forward(self.ctx.handle, self._h, _fp(x), x.shape[0], _fp(q)))
        return q

    def forward_device(self, loc_ptr: int, n: int, q_ptr: int, stream: int = 0) -> None:
        check(lib().rt_dqn_forward_device(self.ctx.handle, self._h, ctypes.c_void_p(loc_ptr), n,
                                          ctypes.c_void_p(q_ptr), ctypes.c_void_p(stream)))

    def save_selected(self, to_select: str, out: str) -> None:
        """selected_deep.txt format for the locations of to_select.txt (rt_dqn_save_selected)."""
        check(lib().rt_dqn_save_selected(self.ctx.handle, self._h, os.fsencode(to_select), os.fsencode(out)))

    def flops_per_ray(self) -> int:
        """2 * sum(in*out) of the four layers (unpadded)"""
        return int(2 * sum(w.shape[0] * w.shape[1] for w in self.W))

    def mfma_flops_per_ray(self) -> int:
        """2 * sum(in*out) of layers 1-3, the ones executed on MFMA (unpadded); layer 0 is
        folded to a 3-input affine map on the VALU (rt_internal.hpp DqnNet)"""
        return int(2 * sum(w.shape[0] * w.shape[1] for w in self.W[1:]))

    def close(self):
        if self._h:
            lib().rt_dqn_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def sample(ctx: Context, scene: Scene, seed: int, q: np.ndarray, loc: np.ndarray, tri: np.ndarray,
           pix: np.ndarray, sample_idx: int, bounce: int, tp: np.ndarray):
    """Importance-sample directions from Q (rt_dqn_sample).  Returns (q*cos, tp, dir, action)."""
    q = np.ascontiguousarray(q, np.float32).copy()
    loc = np.ascontiguousarray(loc, np.float32)
    tri = np.ascontiguousarray(tri, np.int32)
    pix = np.ascontiguousarray(pix, np.uint32)
    tp = np.ascontiguousarray(tp, np.float32).copy()
    n = q.shape[0]
    d = np.zeros((n, 3), np.float32)
    a = np.zeros(n, np.int32)
    check(lib().rt_dqn_sample(ctx.handle, scene.handle, seed, _fp(q), _fp(loc), _ip(tri),
                              pix.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n, sample_idx,
                              bounce, _fp(tp), _fp(d), _ip(a)))
    return q, tp, d, a


def render(ctx: Context, scene: Scene, dqn: Dqn, cam, params, rect=None):
    x0, y0, w, h = rect if rect is not None else (0, 0, params.width, params.height)
    out = np.zeros((h, w, 3), np.float32)
    casts = ctypes.c_uint64(0)
    check(lib().rt_render_dqn(ctx.handle, scene.handle, dqn.handle, ctypes.byref(cam),
                              ctypes.byref(params), x0, y0, w, h, _fp(out), ctypes.byref(casts)))
    return out, int(casts.value)


def render_tiles_device(ctx: Context, scene: Scene, dqn: Dqn, cam, params, tiles: np.ndarray,
                        tile_size: int, out_ptr: int, casts_ptr: int, stream: int) -> None:
    t = np.ascontiguousarray(tiles, np.int32).reshape(-1, 2)
    check(lib().rt_render_dqn_tiles_device(ctx.handle, scene.handle, dqn.handle, ctypes.byref(cam),
                                           ctypes.byref(params), _ip(t), t.shape[0], tile_size,
                                           ctypes.c_void_p(out_ptr), ctypes.c_void_p(casts_ptr),
                                           ctypes.c_void_p(stream)))


class DqnTrainer:
    """The Neural-Q learning rule (neural_q_pathtracer.cu:420-513) on the device: fp32
    parameters + DyNet-default Adam (rt_dqn_trainer_create).  Batches are device pointers
    (e.g. torch tensors' data_ptr())."""

    def __init__(self, ctx: Context, nn_vertices: np.ndarray, W: Sequence[np.ndarray],
                 b: Sequence[np.ndarray], learning_rate: float = 1e-3):
        self.ctx = ctx
        self.nn_vertices = np.ascontiguousarray(nn_vertices, np.float32).ravel()
        W = [np.ascontiguousarray(w, np.float32) for w in W]
        b = [np.ascontiguousarray(x, np.float32).ravel() for x in b]
        self.shapes = [w.shape for w in W]
        hidden = np.array([w.shape[0] for w in W[:3]], np.int32)
        Wp = (ctypes.POINTER(ctypes.c_float) * 4)(*[_fp(w) for w in W])
        bp = (ctypes.POINTER(ctypes.c_float) * 4)(*[_fp(x) for x in b])
        self._h = ctypes.c_void_p()
        check(lib().rt_dqn_trainer_create(ctx.handle, _fp(self.nn_vertices), int(W[0].shape[1]), _ip(hidden),
                                          int(W[3].shape[0]), Wp, bp, float(learning_rate),
                                          ctypes.byref(self._h)))

    def close(self) -> None:
        if self._h:
            lib().rt_dqn_trainer_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def step_device(self, loc_ptr: int, action_ptr: int, target_ptr: int, n: int,
                    stream: int = 0, sync: bool = True) -> Optional[Tuple[float, float]]:
        """One Adam step; returns (loss, gradient L2 norm before clipping), which waits for
        the stream; sync=False leaves the step in flight and returns None."""
        loss, gn = ctypes.c_float(0.0), ctypes.c_float(0.0)
        check(lib().rt_dqn_train_step_device(self.ctx.handle, self._h, ctypes.c_void_p(loc_ptr),
                                             ctypes.c_void_p(action_ptr), ctypes.c_void_p(target_ptr), n,
                                             ctypes.byref(loss) if sync else None,
                                             ctypes.byref(gn) if sync else None, ctypes.c_void_p(stream)))
        return (float(loss.value), float(gn.value)) if sync else None

    def params(self) -> Tuple[list, list]:
        W = [np.zeros(s, np.float32) for s in self.shapes]
        b = [np.zeros(s[0], np.float32) for s in self.shapes]
        Wp = (ctypes.POINTER(ctypes.c_float) * 4)(*[_fp(w) for w in W])
        bp = (ctypes.POINTER(ctypes.c_float) * 4)(*[_fp(x) for x in b])
        check(lib().rt_dqn_trainer_params(self._h, Wp, bp))
        return W, b


class NeuralQ:
    """NeuralQPathtracer (GPU/deep_learning/neural_q_pathtracer.cu:226-600) on the device:
    epsilon-greedy sampling from the network being trained, trace_ray with rewards (light
    luminance x 200), restarts of terminated rays, the learning rule per batch of rays, one
    stats row per sample (rt_neuralq_render_frame).  The reference's run: archway, batch
    4096, epsilon 0.05 (start = min, decay 0.01), 15 frames of SAMPLES_PER_PIXEL samples."""

    def __init__(self, ctx: Context, scene: Scene, trainer: "DqnTrainer", batch_size: int = 4096,
                 epsilon_start: float = 0.05, epsilon_min: float = 0.05, epsilon_decay: float = 0.01):
        self.ctx, self.scene, self.trainer = ctx, scene, trainer
        self._h = ctypes.c_void_p()
        check(lib().rt_neuralq_create(ctx.handle, scene.handle, trainer._h, int(batch_size), float(epsilon_start),
                                      float(epsilon_min), float(epsilon_decay), ctypes.byref(self._h)))

    @property
    def epsilon(self) -> float:
        e = ctypes.c_float(0.0)
        check(lib().rt_neuralq_epsilon(self._h, ctypes.byref(e)))
        return float(e.value)

    def render_frame(self, cam, params):
        """(image H x W x 3, stats spp x 3 [average path length, loss, zero-contribution
        paths] per sample, ray casts)."""
        img = np.zeros((params.height, params.width, 3), np.float32)
        stats = np.zeros((params.spp, 3), np.float32)
        casts = ctypes.c_uint64(0)
        check(lib().rt_neuralq_render_frame(self.ctx.handle, self._h, ctypes.byref(cam), ctypes.byref(params),
                                            _fp(img), _fp(stats), ctypes.byref(casts)))
        return img, stats, int(casts.value)

    @staticmethod
    def stats_lines(stats) -> str:
        """nn_training_stats.txt lines (neural_q_pathtracer.cu:577-583): `avg_path_length
        << " " << loss << " " << total_zclp` with ostream defaults (6 significant digits)."""
        out = []
        for avg, loss, z in np.asarray(stats, np.float32):
            out.append(f"{float(avg):g} {float(loss):g} {int(z)}\n")
        return "".join(out)

    def close(self) -> None:
        if self._h:
            lib().rt_neuralq_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def td_targets_device(ctx: Context, seed: int, next_q_ptr: int, terminal_ptr: int, reward_ptr: int,
                      discount_ptr: int, pix_ptr: int, sample: int, bounce: int, n: int, target_ptr: int,
                      stream: int = 0) -> None:
    """compute_td_targets (rt_dqn_td_targets_device) on device buffers."""
    v = ctypes.c_void_p
    check(lib().rt_dqn_td_targets_device(ctx.handle, seed, v(next_q_ptr), v(terminal_ptr), v(reward_ptr),
                                         v(discount_ptr), v(pix_ptr), sample, bounce, n, v(target_ptr),
                                         v(stream)))
