"""ctypes wrapper of the CPU restatement (rt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  The product
(reinforcement-light-rays-pathtracer_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

_LIB = None
_FP = ctypes.POINTER(ctypes.c_float)
_IP = ctypes.POINTER(ctypes.c_int32)


class OrcCamera(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_float * 4), ("yaw_y", ctypes.c_float), ("yaw_x", ctypes.c_float)]


class OrcParams(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
        ("max_bounces", ctypes.c_int32), ("sampler", ctypes.c_int32), ("preset", ctypes.c_int32),
        ("hit_rule", ctypes.c_int32), ("spp_split", ctypes.c_int32), ("seed", ctypes.c_uint64),
        ("env_light", ctypes.c_float), ("t_scale", ctypes.c_float),
    ]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_philox4x32_10.argtypes = [ctypes.POINTER(ctypes.c_uint32)] * 3
        L.orc_sincos_turn.argtypes = [ctypes.c_float, _FP, _FP]
        L.orc_triangle_normals.argtypes = [_FP, ctypes.c_int, _FP]
        L.orc_cornell.argtypes = [ctypes.c_int, _FP, _FP, _FP, _IP, ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_int)]
        L.orc_intersect.argtypes = [_FP, ctypes.c_int, ctypes.c_int, _IP, _FP, _FP, ctypes.c_int,
                                    ctypes.c_float, ctypes.c_int, _FP, _IP]
        L.orc_render.argtypes = [_FP, _FP, ctypes.c_int, _FP, _IP, ctypes.c_int,
                                 ctypes.POINTER(OrcCamera), ctypes.POINTER(OrcParams),
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _FP,
                                 ctypes.POINTER(ctypes.c_uint64)]
        L.orc_render_sequential.argtypes = [_FP, _FP, ctypes.c_int, _FP, _IP, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p, _FP,
                                            ctypes.POINTER(ctypes.c_uint64)]
        L.orc_td_targets.argtypes = [ctypes.c_uint64, _FP, _IP, _FP, _FP, ctypes.POINTER(ctypes.c_uint32),
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, _FP]
        L.orc_glibc_rand.argtypes = [ctypes.c_uint, ctypes.c_int, _IP]
        L.orc_pack_argb.argtypes = [_FP, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
        L.orc_primary_hits.argtypes = [_FP, ctypes.c_int, ctypes.c_int, ctypes.POINTER(OrcCamera),
                                       ctypes.POINTER(OrcParams), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, _IP]
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_set_threads.argtypes = [ctypes.c_int]
        _LIB = L
    return _LIB


def _f(a):
    return a.ctypes.data_as(_FP)


def _i(a):
    return a.ctypes.data_as(_IP)


def philox(ctr, key) -> np.ndarray:
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    P = ctypes.POINTER(ctypes.c_uint32)
    lib().orc_philox4x32_10(c.ctypes.data_as(P), k.ctypes.data_as(P), out.ctypes.data_as(P))
    return out


def sincos_turn(r: float):
    s, c = ctypes.c_float(), ctypes.c_float()
    lib().orc_sincos_turn(ctypes.c_float(r), ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def cornell(variant: int):
    tri = np.zeros((38, 9), np.float32)
    alb = np.zeros((36, 3), np.float32)
    em = np.zeros((2, 3), np.float32)
    grp = np.zeros(2, np.int32)
    ns, nl = ctypes.c_int(), ctypes.c_int()
    lib().orc_cornell(variant, _f(tri), _f(alb), _f(em), _i(grp), ctypes.byref(ns), ctypes.byref(nl))
    return {"tri": tri[:36].copy(), "albedo": alb, "light": tri[36:].copy(), "emission": em,
            "light_group": grp}


def normals(tri_all: np.ndarray) -> np.ndarray:
    t = np.ascontiguousarray(tri_all, np.float32)
    out = np.zeros((t.shape[0], 3), np.float32)
    lib().orc_triangle_normals(_f(t), t.shape[0], _f(out))
    return out


def intersect(tri, n_surf, n_light, light_group, orig, direction, t_scale, hit_rule):
    t_all = np.ascontiguousarray(tri, np.float32)
    g = np.ascontiguousarray(light_group, np.int32)
    o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
    n = o.shape[0]
    out_t = np.zeros(n, np.float32)
    out_h = np.zeros(n, np.int32)
    lib().orc_intersect(_f(t_all), n_surf, n_light, _i(g), _f(o), _f(d), n, t_scale, hit_rule,
                        _f(out_t), _i(out_h))
    return out_t, out_h


def pass_masks(tri, orig, direction, t_scale, hit_rule):
    """[n_rays][ceil(n_tri / 64)] uint64: bit i = triangle i passes the exact test (no
    closest-hit window) -- what a candidate filter must keep (orc_pass_masks)."""
    t_all = np.ascontiguousarray(tri, np.float32).reshape(-1, 9)
    o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
    n, nt = o.shape[0], t_all.shape[0]
    out = np.zeros((n, (nt + 63) // 64), np.uint64)
    L = lib()
    L.orc_pass_masks.argtypes = [_FP, ctypes.c_int, _FP, _FP, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                 ctypes.c_void_p]
    L.orc_pass_masks(_f(t_all), nt, _f(o), _f(d), n, t_scale, hit_rule, out.ctypes.data_as(ctypes.c_void_p))
    return out


def primary_hits(tri, n_surf, n_light, cam, params, rect, s0, s1):
    """Triangle index (-1 = miss) hit by the camera ray of every pixel of rect = (x, y, w, h)
    and sample in [s0, s1): array (h, w, s1 - s0)."""
    x, y, w, h = rect
    t_all = np.ascontiguousarray(tri, np.float32)
    out = np.zeros((h, w, s1 - s0), np.int32)
    lib().orc_primary_hits(_f(t_all), n_surf, n_light, ctypes.byref(cam), ctypes.byref(params), x, y, w, h,
                           s0, s1, _i(out))
    return out


def params_from(p) -> OrcParams:
    """Copy an rtmi RtParams (or any object with the same fields) into OrcParams."""
    q = OrcParams()
    for name, _ in OrcParams._fields_:
        setattr(q, name, getattr(p, name))
    return q


def camera(pos, yaw_y=0.0, yaw_x=0.0) -> OrcCamera:
    c = OrcCamera()
    for i in range(4):
        c.pos[i] = float(pos[i])
    c.yaw_y = yaw_y
    c.yaw_x = yaw_x
    return c


def render(geom, cam: OrcCamera, params: OrcParams, rect=None):
    """geom: dict or object with tri/albedo/light/emission/light_group."""
    get = (lambda k: geom[k]) if isinstance(geom, dict) else (lambda k: getattr(geom, k))
    tri = np.ascontiguousarray(np.concatenate([get("tri"), get("light")], 0), np.float32)
    alb = np.ascontiguousarray(get("albedo"), np.float32)
    em = np.ascontiguousarray(get("emission"), np.float32)
    grp = np.ascontiguousarray(get("light_group"), np.int32)
    n_surf, n_light = get("tri").shape[0], get("light").shape[0]
    x0, y0, w, h = rect if rect is not None else (0, 0, params.width, params.height)
    out = np.zeros((h, w, 3), np.float32)
    casts = ctypes.c_uint64(0)
    lib().orc_render(_f(tri), _f(alb), n_surf, _f(em), _i(grp), n_light, ctypes.byref(cam),
                     ctypes.byref(params), x0, y0, w, h, _f(out), ctypes.byref(casts))
    return out, int(casts.value)


def render_sequential(geom, cam: OrcCamera, params: OrcParams):
    """The whole frame in the CPU engine's own order and glibc rand() stream
    (rt_oracle.c orc_render_sequential; SURVEY.md §8(c) gate 3): CPU preset only."""
    get = (lambda k: geom[k]) if isinstance(geom, dict) else (lambda k: getattr(geom, k))
    tri = np.ascontiguousarray(np.concatenate([get("tri"), get("light")], 0), np.float32)
    alb = np.ascontiguousarray(get("albedo"), np.float32)
    em = np.ascontiguousarray(get("emission"), np.float32)
    grp = np.ascontiguousarray(get("light_group"), np.int32)
    n_surf, n_light = get("tri").shape[0], get("light").shape[0]
    out = np.zeros((params.height, params.width, 3), np.float32)
    casts = ctypes.c_uint64(0)
    rc = lib().orc_render_sequential(_f(tri), _f(alb), n_surf, _f(em), _i(grp), n_light, ctypes.byref(cam),
                                     ctypes.byref(params), _f(out), ctypes.byref(casts))
    if rc != 0:
        raise ValueError("reference_sequential needs the CPU preset, uniform sampler and CPU hit rule")
    return out, int(casts.value)


def glibc_rand(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.int32)
    lib().orc_glibc_rand(seed, n, _i(out))
    return out


def pack_argb(rgb) -> np.ndarray:
    a = np.ascontiguousarray(rgb, np.float32)
    out = np.zeros(a.shape[:-1], np.uint32)
    lib().orc_pack_argb(_f(a), a.size // 3, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    return out


def num_threads() -> int:
    return int(lib().orc_num_threads())


def set_threads(n: int) -> None:
    lib().orc_set_threads(int(n))


# ---- DQN path -----------------------------------------------------------------

def read_dynet(path):
    """Independent numpy reader of a DyNet text model: [(rows, cols, row-major array)]."""
    params, shape = [], None
    with open(path) as f:
        for line in f:
            if line.startswith("#Parameter#") or line.startswith("#LookupParameter#"):
                dims = line[line.index("{") + 1:line.index("}")].split(",")
                shape = tuple(int(x) for x in dims)
            elif shape is not None:
                v = np.array(line.split(), np.float32)
                r = shape[0]
                c = shape[1] if len(shape) > 1 else 1
                a = v.reshape(c, r).T  # column-major storage
                params.append(a if c > 1 else a[:, 0])
                shape = None
    return params


def _ptrs(arrs):
    return (_FP * len(arrs))(*[a.ctypes.data_as(_FP) for a in arrs])


def dqn_forward(W, b, verts, loc, bf16=False):
    L = lib()
    L.orc_dqn_forward.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(_FP), ctypes.POINTER(_FP), _FP, _FP,
                                                        ctypes.c_int, ctypes.c_int, _FP]
    W = [np.ascontiguousarray(w, np.float32) for w in W]
    b = [np.ascontiguousarray(x, np.float32) for x in b]
    v = np.ascontiguousarray(verts, np.float32)
    x = np.ascontiguousarray(loc, np.float32).reshape(-1, 3)
    q = np.zeros((x.shape[0], W[3].shape[0]), np.float32)
    L.orc_dqn_forward(W[0].shape[1], W[0].shape[0], W[1].shape[0], W[2].shape[0], W[3].shape[0], _ptrs(W),
                      _ptrs(b), _f(v), _f(x), x.shape[0], int(bf16), _f(q))
    return q


def dqn_sample(tri_all, q, loc, tri, pix, sample, bounce, seed, tp):
    L = lib()
    U32 = ctypes.POINTER(ctypes.c_uint32)
    L.orc_dqn_sample.argtypes = [_FP, ctypes.c_int, _FP, _FP, _IP, U32, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_uint64, _FP, _FP, _IP]
    t_all = np.ascontiguousarray(tri_all, np.float32)
    q = np.ascontiguousarray(q, np.float32).copy()
    loc = np.ascontiguousarray(loc, np.float32)
    tri = np.ascontiguousarray(tri, np.int32)
    pix = np.ascontiguousarray(pix, np.uint32)
    tp = np.ascontiguousarray(tp, np.float32).copy()
    n = q.shape[0]
    d = np.zeros((n, 3), np.float32)
    a = np.zeros(n, np.int32)
    L.orc_dqn_sample(_f(t_all), t_all.shape[0], _f(q), _f(loc), _i(tri), pix.ctypes.data_as(U32), n, sample,
                     bounce, seed, _f(tp), _f(d), _i(a))
    return q, tp, d, a


def render_dqn(geom, W, b, verts, cam, params, rect=None, bf16=False, q_bf16=True):
    """orc_render_dqn; bf16: the kernel's arithmetic (bf16 forward, and with q_bf16 the
    renderer's Q rounded to bf16 before the sampler, as k_dqn_mlp<.., QB> stores it)"""
    L = lib()
    L.orc_render_dqn.argtypes = [_FP, _FP, ctypes.c_int, _FP, _IP, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.POINTER(_FP), ctypes.POINTER(_FP), _FP,
                                 ctypes.c_int, ctypes.POINTER(OrcCamera), ctypes.POINTER(OrcParams),
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _FP,
                                 ctypes.POINTER(ctypes.c_uint64)]
    get = (lambda k: geom[k]) if isinstance(geom, dict) else (lambda k: getattr(geom, k))
    tri = np.ascontiguousarray(np.concatenate([get("tri"), get("light")], 0), np.float32)
    alb = np.ascontiguousarray(get("albedo"), np.float32)
    em = np.ascontiguousarray(get("emission"), np.float32)
    grp = np.ascontiguousarray(get("light_group"), np.int32)
    W = [np.ascontiguousarray(w, np.float32) for w in W]
    b = [np.ascontiguousarray(x, np.float32) for x in b]
    v = np.ascontiguousarray(verts, np.float32)
    x0, y0, w, h = rect if rect is not None else (0, 0, params.width, params.height)
    out = np.zeros((h, w, 3), np.float32)
    casts = ctypes.c_uint64(0)
    L.orc_render_dqn(_f(tri), _f(alb), get("tri").shape[0], _f(em), _i(grp), get("light").shape[0],
                     W[0].shape[1], W[0].shape[0], W[1].shape[0], W[2].shape[0], _ptrs(W), _ptrs(b), _f(v),
                     (1 if q_bf16 else 2) if bf16 else 0, ctypes.byref(cam), ctypes.byref(params), x0, y0, w, h, _f(out),
                     ctypes.byref(casts))
    return out, int(casts.value)


ORC_Q_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                            ctypes.c_void_p)


def render_dqn_wave(geom, cam, params, q_fn, rect=None):
    """orc_render_dqn_wave: the DQN render with every bounce's Q from q_fn(loc (n, 3) float32)
    -> (n, 144) float32 (e.g. the GPU forward), in wavefront order."""
    L = lib()
    L.orc_render_dqn_wave.argtypes = [_FP, _FP, ctypes.c_int, _FP, _IP, ctypes.c_int, ctypes.POINTER(OrcCamera),
                                      ctypes.POINTER(OrcParams), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ORC_Q_FN, ctypes.c_void_p, _FP, ctypes.POINTER(ctypes.c_uint64)]
    get = (lambda k: geom[k]) if isinstance(geom, dict) else (lambda k: getattr(geom, k))
    tri = np.ascontiguousarray(np.concatenate([get("tri"), get("light")], 0), np.float32)
    alb = np.ascontiguousarray(get("albedo"), np.float32)
    em = np.ascontiguousarray(get("emission"), np.float32)
    grp = np.ascontiguousarray(get("light_group"), np.int32)
    x0, y0, w, h = rect if rect is not None else (0, 0, params.width, params.height)
    out = np.zeros((h, w, 3), np.float32)
    casts = ctypes.c_uint64(0)
    calls = []

    def cb(loc_p, n, q_p, _user):
        loc = np.ctypeslib.as_array(loc_p, shape=(n, 3)).copy()
        q = np.ascontiguousarray(q_fn(loc), np.float32)
        assert q.shape == (n, 144)
        ctypes.memmove(q_p, q.ctypes.data, q.nbytes)
        calls.append(n)

    fn = ORC_Q_FN(cb)
    L.orc_render_dqn_wave(_f(tri), _f(alb), get("tri").shape[0], _f(em), _i(grp), get("light").shape[0],
                          ctypes.byref(cam), ctypes.byref(params), x0, y0, w, h, fn, None, _f(out),
                          ctypes.byref(casts))
    return out, int(casts.value), calls


KD_DTYPE = np.dtype([("dim", "<i4"), ("leaf", "<i4"), ("left", "<i4"), ("right", "<i4"), ("data", "<f4"),
                     ("px", "<f4"), ("py", "<f4"), ("pz", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                     ("vol", "<i4")])


class Sarsa:
    """Expected-SARSA radiance map of the restatement (orc_sarsa_*)."""

    def __init__(self, geom, seed: int, area_per_sample: float = 0.001):
        L = lib()
        VP = ctypes.c_void_p
        L.orc_sarsa_create_density.restype = VP
        L.orc_sarsa_create_density.argtypes = [_FP, _FP, ctypes.c_int, _FP, _IP, ctypes.c_int, ctypes.c_uint64,
                                               ctypes.c_float]
        L.orc_sarsa_destroy.argtypes = [VP]
        L.orc_sarsa_info.argtypes = [VP, _IP, _IP]
        L.orc_sarsa_volumes.argtypes = [VP, _FP, _FP, _IP, VP]
        L.orc_sarsa_read.argtypes = [VP, _FP, _FP, ctypes.POINTER(ctypes.c_uint32), _FP]
        L.orc_sarsa_nearest.argtypes = [VP, _FP, _FP, ctypes.c_int, _IP]
        L.orc_render_sarsa.argtypes = [VP, ctypes.POINTER(OrcCamera), ctypes.POINTER(OrcParams), ctypes.c_int,
                                       _FP, ctypes.POINTER(ctypes.c_uint64)]
        L.orc_sarsa_set_sampling.argtypes = [VP, ctypes.c_int]
        L.orc_sarsa_set_td_mode.argtypes = [VP, ctypes.c_int]
        L.orc_render_sarsa_rect.argtypes = [VP, ctypes.POINTER(OrcCamera), ctypes.POINTER(OrcParams)] + \
            [ctypes.c_int] * 4 + [_FP, ctypes.POINTER(ctypes.c_uint64)]
        L.orc_sarsa_sample_stats.argtypes = [VP] + [ctypes.POINTER(ctypes.c_uint64)] * 3
        L.orc_sarsa_stats.argtypes = [VP, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.orc_sarsa_load_q.argtypes = [VP, _FP]
        L.orc_sarsa_td_rect.argtypes = [VP, ctypes.POINTER(OrcCamera), ctypes.POINTER(OrcParams), ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_uint32)]
        get = (lambda k: geom[k]) if isinstance(geom, dict) else (lambda k: getattr(geom, k))
        self._keep = [np.ascontiguousarray(np.concatenate([get("tri"), get("light")], 0), np.float32),
                      np.ascontiguousarray(get("albedo"), np.float32),
                      np.ascontiguousarray(get("emission"), np.float32),
                      np.ascontiguousarray(get("light_group"), np.int32)]
        tri, alb, em, grp = self._keep
        self._L = L
        self._h = L.orc_sarsa_create_density(_f(tri), _f(alb), get("tri").shape[0], _f(em), _i(grp),
                                             get("light").shape[0], seed, area_per_sample)
        nv, nk = ctypes.c_int32(0), ctypes.c_int32(0)
        L.orc_sarsa_info(self._h, ctypes.byref(nv), ctypes.byref(nk))
        self.n_volumes, self.n_nodes = nv.value, nk.value

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.orc_sarsa_destroy(self._h)
            self._h = None

    def volumes(self):
        n = self.n_volumes
        pos = np.zeros((n, 3), np.float32)
        nrm = np.zeros((n, 3), np.float32)
        surf = np.zeros(n, np.int32)
        kd = np.zeros(self.n_nodes, KD_DTYPE)
        self._L.orc_sarsa_volumes(self._h, _f(pos), _f(nrm), _i(surf), kd.ctypes.data_as(ctypes.c_void_p))
        return pos, nrm, surf, kd

    def read(self):
        n = self.n_volumes
        q = np.zeros((n, 144), np.float32)
        cdf = np.zeros((n, 144), np.float32)
        vis = np.zeros((n, 144), np.uint32)
        acc = np.zeros(n, np.float32)
        self._L.orc_sarsa_read(self._h, _f(q), _f(cdf), vis.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                               _f(acc))
        return q, cdf, vis, acc

    def nearest(self, pos, nrm):
        p = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
        n_ = np.ascontiguousarray(nrm, np.float32).reshape(-1, 3)
        out = np.zeros(p.shape[0], np.int32)
        self._L.orc_sarsa_nearest(self._h, _f(p), _f(n_), p.shape[0], _i(out))
        return out

    def set_sampling(self, mode: int):
        """0: CDF importance sampling, 1: sample_max_direction_from_radiance_distribution"""
        self._L.orc_sarsa_set_sampling(self._h, mode)

    def set_td_mode(self, mode: int):
        """0: frame-synchronous integer TD sums (the default), 1: the reference's in-frame rule
        applied event by event in the render's fixed order (the frame then renders on one
        thread: pixels row by row, each pixel's chunks and samples in order)"""
        self._L.orc_sarsa_set_td_mode(self._h, mode)

    def stats(self):
        """(sum over pixels of int(path length mean), zero-contribution paths) of the last frame"""
        a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._L.orc_sarsa_stats(self._h, ctypes.byref(a), ctypes.byref(b))
        return int(a.value), int(b.value)

    def sample_stats(self):
        """last frame: (CDF samples, failed ones -- the null ray --, samples of sector 0)"""
        v = [ctypes.c_uint64(0) for _ in range(3)]
        self._L.orc_sarsa_sample_stats(self._h, *[ctypes.byref(x) for x in v])
        return tuple(int(x.value) for x in v)

    def load_q(self, q):
        q = np.ascontiguousarray(q, np.float32).reshape(self.n_volumes, 144)
        self._L.orc_sarsa_load_q(self._h, _f(q))

    def td_rect(self, cam: OrcCamera, params: OrcParams, rect):
        """(int64 sums, uint32 counts), each (n_volumes * 144,): the TD accumulators that the
        rectangle (x, y, w, h) of the current frame adds (the frame is not applied)."""
        n = self.n_volumes * 144
        s = np.zeros(n, np.int64)
        c = np.zeros(n, np.uint32)
        self._L.orc_sarsa_td_rect(self._h, ctypes.byref(cam), ctypes.byref(params), *rect,
                                  s.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                  c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        return s, c

    def render_rect(self, cam: OrcCamera, params: OrcParams, rect):
        """(image (h, w, 3), casts) of the rectangle (x, y, w, h) of the current frame; the
        frame is not applied (its TD sums are dropped)"""
        x, y, w, h = rect
        out = np.zeros((h, w, 3), np.float32)
        casts = ctypes.c_uint64(0)
        self._L.orc_render_sarsa_rect(self._h, ctypes.byref(cam), ctypes.byref(params), x, y, w, h, _f(out),
                                      ctypes.byref(casts))
        return out, int(casts.value)

    def render(self, cam: OrcCamera, params: OrcParams, frames: int = 1):
        out = np.zeros((params.height, params.width, 3), np.float32)
        casts = ctypes.c_uint64(0)
        self._L.orc_render_sarsa(self._h, ctypes.byref(cam), ctypes.byref(params), frames, _f(out),
                                 ctypes.byref(casts))
        return out, int(casts.value)


# --- Neural-Q training ------------------------------------

def td_targets(seed, next_q, terminal, reward, discount, pix, sample, bounce):
    """compute_td_targets restated (rt_oracle.c orc_td_targets), float32 in and out."""
    q = np.ascontiguousarray(next_q, np.float32)
    n = q.shape[0]
    term = np.ascontiguousarray(terminal, np.int32)
    rw = np.ascontiguousarray(reward, np.float32)
    dc = np.ascontiguousarray(discount, np.float32)
    px = np.ascontiguousarray(pix, np.uint32)
    out = np.zeros(n, np.float32)
    lib().orc_td_targets(seed, _f(q), _i(term), _f(rw), _f(dc),
                         px.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), sample, bounce, n, _f(out))
    return out


class AdamRef:
    """fp64 restatement of one Neural-Q learning step (neural_q_pathtracer.cu:478-513):
    DQNetwork forward (b + W x, rectify x 4; NN_Builders/fc_layer.cu:40-72), pick, loss =
    sum (target - q_a)^2, backward, dynet::AdamTrainer update with DyNet's defaults
    (global-norm clipping at 5: scale 5/||g||; m = b1 m + (1-b1) s g; v = b2 v + (1-b2) s^2 g^2;
    x -= lr sqrt(1-b2^t)/(1-b1^t) m/(sqrt(v)+eps)).  DyNet is absent here:
    parity unpinned against DyNet itself; this is the published algorithm."""

    def __init__(self, nn_vertices, W, b, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8, clip=5.0):
        self.v = np.asarray(nn_vertices, np.float64).ravel()
        self.P = [np.asarray(w, np.float64).copy() for w in W] + [np.asarray(x, np.float64).ravel().copy() for x in b]
        self.M = [np.zeros_like(p) for p in self.P]
        self.V = [np.zeros_like(p) for p in self.P]
        self.lr, self.b1, self.b2, self.eps, self.clip = lr, b1, b2, eps, clip
        self.t = 0

    def forward(self, loc):
        loc = np.asarray(loc, np.float64).reshape(-1, 3)
        h = self.v[None, :] - np.tile(loc, (1, self.v.size // 3))
        hs = [h]
        for l in range(4):
            h = np.maximum(h @ self.P[l].T + self.P[4 + l][None, :], 0.0)
            hs.append(h)
        return hs

    def step(self, loc, action, target):
        loss, G = self.loss_grads(loc, action, target)
        gn = float(np.sqrt(sum(float(np.sum(g * g)) for g in G)))
        s = self.clip / gn if (self.clip > 0 and gn > self.clip) else 1.0
        self.t += 1
        lr_t = self.lr * np.sqrt(1.0 - self.b2 ** self.t) / (1.0 - self.b1 ** self.t)
        for i, g in enumerate(G):
            self.M[i] = self.M[i] * self.b1 + g * ((1.0 - self.b1) * s)
            self.V[i] = self.V[i] * self.b2 + (g * g) * ((1.0 - self.b2) * s * s)
            self.P[i] = self.P[i] - self.M[i] / (np.sqrt(self.V[i]) + self.eps) * lr_t
        return loss, gn

    def loss_grads(self, loc, action, target):
        """loss and its gradients [dW0..dW3, db0..db3]"""
        hs = self.forward(loc)
        q = hs[4]
        n = q.shape[0]
        act = np.asarray(action, np.int64)
        ok = (act >= 0) & (act < q.shape[1])
        rows = np.nonzero(ok)[0]
        qa = q[rows, act[ok]]
        diff = np.asarray(target, np.float64)[ok] - qa
        loss = float(np.sum(diff * diff))
        d = np.zeros_like(q)
        d[rows, act[ok]] = np.where(qa > 0.0, -2.0 * diff, 0.0)
        gW, gb = [None] * 4, [None] * 4
        for l in range(3, -1, -1):
            gW[l] = d.T @ hs[l]
            gb[l] = d.sum(0)
            if l > 0:
                d = (d @ self.P[l]) * (hs[l] > 0.0)
        return loss, gW + gb

    def params(self):
        return self.P[:4], self.P[4:]
