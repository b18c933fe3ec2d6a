"""Python mirror of the reference's scene-loader / Camera / frame-buffer /
render API for the hot path, on top of the C ABI (include/rtmi.h).

Reference names (CPU/ = Old_CPU_Rendering_Engine/Source, GPU/ =
GPU_Rendering_Engine/Source):
  get_cornell_shapes   CPU/scenes/cornell_box_scene.cpp:3   -> cornell_geometry()
  load_scene           GPU/objects/object_importer.cu:8     -> obj_geometry()
  Camera(vec4)         CPU/camera.cpp:3, GPU/camera.cu:3    -> camera()
  draw_default_path_tracing  CPU/path_tracing/default_path_tracing.cpp:5 -> render()
  Ray::closest_intersection  CPU/rays/ray.cpp:14           -> intersect()
  SDLScreen::PutPixelSDL     CPU/sdl/sdl_screen.cpp:100     -> pack_argb()
  SDLScreen::SDL_SaveImage   CPU/sdl/sdl_screen.cpp:64      -> save_bmp()
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import RtCamera, RtParams, check, lib

# Camera positions of the reference's scenes: CPU/main.cpp:77 (Cornell) and the
# presets listed in GPU/main.cu:100-104.
CAMERAS = {
    "cornell": (0.0, 0.0, -3.0, 1.0),
    "door_room": (0.0, 0.5, -0.9, 1.0),
    "archway": (-1.0, 0.2, -0.99, 1.0),
    "complex_light_room": (-1.0, -1.0, -0.4, 1.0),
}

# scene_kind of rt_obj_geometry
OBJ_KINDS = {"generic": 0, "door_room": 1, "archway": 2, "complex_light_room": 3}


def _fp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _ip(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


@dataclasses.dataclass
class Geometry:
    """Triangle soup in the reference's order: surfaces, then light triangles."""
    tri: np.ndarray          # (n_surf, 9) float32: v0, v1, v2
    albedo: np.ndarray       # (n_surf, 3) float32
    light: np.ndarray        # (n_light, 9) float32
    emission: np.ndarray     # (n_light, 3) float32
    light_group: np.ndarray  # (n_light,) int32: plane index (CPU light hit index)
    nn_vertices: Optional[np.ndarray] = None  # Scene::vertices (GPU engine) order

    @property
    def n_surf(self) -> int:
        return int(self.tri.shape[0])

    @property
    def n_light(self) -> int:
        return int(self.light.shape[0])

    @property
    def n_tri(self) -> int:
        return self.n_surf + self.n_light

    def all_triangles(self) -> np.ndarray:
        return np.concatenate([self.tri, self.light], axis=0)


def cornell_geometry(variant: int = _lib.RT_PRESET_CPU) -> Geometry:
    """get_cornell_shapes of the CPU engine (variant 0) or GPU engine (variant 1)."""
    L = lib()
    ns, nl = ctypes.c_int(), ctypes.c_int()
    check(L.rt_cornell_counts(ctypes.byref(ns), ctypes.byref(nl)))
    tri = np.zeros((ns.value, 9), np.float32)
    alb = np.zeros((ns.value, 3), np.float32)
    lv = np.zeros((nl.value, 9), np.float32)
    em = np.zeros((nl.value, 3), np.float32)
    grp = np.zeros((nl.value,), np.int32)
    check(L.rt_cornell_geometry(variant, _fp(tri), _fp(alb), _fp(lv), _fp(em), _ip(grp)))
    # the GPU engine's Scene::vertices (the network's input, 38 x 9 = 342 floats): each
    # surface's v0, v1, v2 as stored, then each light's (GPU/scenes/cornell_box_scene.cu:190-199,
    # 231-240); the CPU engine has no network
    nnv = np.concatenate([tri, lv], axis=0).ravel().copy() if variant == _lib.RT_PRESET_GPU else None
    return Geometry(tri, alb, lv, em, grp, nnv)


def obj_geometry(path: str, kind: str | int = "generic") -> Geometry:
    """load_scene with the GPU engine's semantics (object_importer.cu:8-412)."""
    L = lib()
    k = OBJ_KINDS[kind] if isinstance(kind, str) else int(kind)
    ns, nl, nn = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    null_f = ctypes.POINTER(ctypes.c_float)()
    null_i = ctypes.POINTER(ctypes.c_int32)()
    check(L.rt_obj_geometry(path.encode(), k, null_f, null_f, ctypes.byref(ns), null_f, null_f,
                            null_i, ctypes.byref(nl), null_f, ctypes.byref(nn)))
    tri = np.zeros((ns.value, 9), np.float32)
    alb = np.zeros((ns.value, 3), np.float32)
    lv = np.zeros((nl.value, 9), np.float32)
    em = np.zeros((nl.value, 3), np.float32)
    grp = np.zeros((nl.value,), np.int32)
    nnv = np.zeros((nn.value,), np.float32)
    check(L.rt_obj_geometry(path.encode(), k, _fp(tri), _fp(alb), ctypes.byref(ns), _fp(lv),
                            _fp(em), _ip(grp), ctypes.byref(nl), _fp(nnv), ctypes.byref(nn)))
    return Geometry(tri, alb, lv, em, grp, nnv)


def default_params(preset: int = _lib.RT_PRESET_CPU, **overrides) -> RtParams:
    p = RtParams()
    check(lib().rt_params_default(preset, ctypes.byref(p)))
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise AttributeError(f"rt_params has no field {k}")
        setattr(p, k, v)
    if "height" in overrides and "t_scale" not in overrides:
        p.t_scale = float(p.height)  # the reference scales by SCREEN_HEIGHT
    return p


def camera(pos=(0.0, 0.0, -3.0, 1.0), yaw_y: float = 0.0, yaw_x: float = 0.0) -> RtCamera:
    c = RtCamera()
    for i in range(4):
        c.pos[i] = float(pos[i])
    c.yaw_y = yaw_y
    c.yaw_x = yaw_x
    return c


class Context:
    """One rt_ctx per GPU (rt_ctx_create)."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        check(lib().rt_ctx_create(device, ctypes.byref(self._h)))
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().rt_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Scene:
    """A device-resident scene (rt_scene_create)."""

    def __init__(self, ctx: Context, geom: Geometry):
        self.ctx = ctx
        self.geom = geom
        self._h = ctypes.c_void_p()
        tri = np.ascontiguousarray(geom.tri, np.float32)
        alb = np.ascontiguousarray(geom.albedo, np.float32)
        lv = np.ascontiguousarray(geom.light, np.float32)
        em = np.ascontiguousarray(geom.emission, np.float32)
        grp = np.ascontiguousarray(geom.light_group, np.int32)
        check(lib().rt_scene_create(ctx.handle, _fp(tri), _fp(alb), geom.n_surf, _fp(lv), _fp(em),
                                    _ip(grp), geom.n_light, ctypes.byref(self._h)))

    @property
    def handle(self):
        return self._h

    def set_accel(self, mode: int):
        """rt_scene_set_accel: ACCEL_AUTO (BVH above 256 triangles), ACCEL_SCAN, ACCEL_BVH."""
        check(lib().rt_scene_set_accel(self._h, int(mode)))

    def accel_info(self) -> dict:
        nodes, depth, gl = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int64(0)
        check(lib().rt_scene_accel_info(self._h, ctypes.byref(nodes), ctypes.byref(depth), ctypes.byref(gl)))
        return {"nodes": nodes.value, "depth": depth.value, "plane_nodes": gl.value}

    def ctab_info(self, hit_rule: int) -> dict:
        """the bounce-ray candidate table of a hit rule: built, host build + upload seconds,
        device bytes (rt_scene_ctab_info; zeros until a render takes it)"""
        built, secs, nbytes = ctypes.c_int(0), ctypes.c_double(0.0), ctypes.c_uint64(0)
        check(lib().rt_scene_ctab_info(self._h, hit_rule, ctypes.byref(built), ctypes.byref(secs),
                                       ctypes.byref(nbytes)))
        return {"built": bool(built.value), "build_s": secs.value, "bytes": int(nbytes.value)}

    def normals(self) -> np.ndarray:
        out = np.zeros((self.geom.n_tri, 3), np.float32)
        check(lib().rt_scene_normals(self._h, _fp(out)))
        return out

    def close(self):
        if self._h:
            lib().rt_scene_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def intersect(ctx: Context, scene: Scene, orig: np.ndarray, direction: np.ndarray,
              t_scale: float, hit_rule: int) -> Tuple[np.ndarray, np.ndarray]:
    o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
    n = o.shape[0]
    t = np.zeros(n, np.float32)
    h = np.zeros(n, np.int32)
    check(lib().rt_intersect(ctx.handle, scene.handle, _fp(o), _fp(d), n, float(t_scale), hit_rule,
                             _fp(t), _ip(h)))
    return t, h


ISECT_SCAN, ISECT_FILTER, ISECT_MFMA, ISECT_BVH = 0, 1, 2, 3
ACCEL_AUTO, ACCEL_SCAN, ACCEL_BVH = 0, 1, 2


def intersect_method(ctx: Context, scene: Scene, orig: np.ndarray, direction: np.ndarray, t_scale: float,
                     hit_rule: int, method: int, count: bool = False):
    """rt_intersect_method: (t, hit) or, with count (ISECT_MFMA), (t, hit, candidates per ray)."""
    o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
    n = o.shape[0]
    t = np.zeros(n, np.float32)
    h = np.zeros(n, np.int32)
    c = np.zeros(n, np.int32) if count else None
    check(lib().rt_intersect_method(ctx.handle, scene.handle, _fp(o), _fp(d), n, float(t_scale), hit_rule,
                                    method, _fp(t), _ip(h), _ip(c) if count else None))
    return (t, h, c) if count else (t, h)


def intersect_device(ctx: Context, scene: Scene, orig_ptr: int, dir_ptr: int, n: int,
                     t_scale: float, hit_rule: int, t_ptr: int, hit_ptr: int, stream: int = 0):
    check(lib().rt_intersect_device(ctx.handle, scene.handle, ctypes.c_void_p(orig_ptr),
                                    ctypes.c_void_p(dir_ptr), n, float(t_scale), hit_rule,
                                    ctypes.c_void_p(t_ptr), ctypes.c_void_p(hit_ptr),
                                    ctypes.c_void_p(stream)))


def render(ctx: Context, scene: Scene, cam: RtCamera, params: RtParams,
           rect: Optional[Tuple[int, int, int, int]] = None) -> Tuple[np.ndarray, int]:
    """Render (x0, y0, w, h) of the image; returns (h, w, 3) float32 and the ray casts."""
    x0, y0, w, h = rect if rect is not None else (0, 0, params.width, params.height)
    out = np.zeros((h, w, 3), np.float32)
    casts = ctypes.c_uint64(0)
    check(lib().rt_render(ctx.handle, scene.handle, ctypes.byref(cam), ctypes.byref(params),
                          x0, y0, w, h, _fp(out), ctypes.byref(casts)))
    return out, int(casts.value)


def render_tiles_device(ctx: Context, scene: Scene, cam: RtCamera, params: RtParams,
                        tiles: np.ndarray, tile_size: int, out_ptr: int, casts_ptr: int,
                        stream: int) -> None:
    """Asynchronous tile-list render into device memory (rt_render_tiles_device)."""
    t = np.ascontiguousarray(tiles, np.int32).reshape(-1, 2)
    check(lib().rt_render_tiles_device(ctx.handle, scene.handle, ctypes.byref(cam),
                                       ctypes.byref(params), _ip(t), t.shape[0], tile_size,
                                       ctypes.c_void_p(out_ptr), ctypes.c_void_p(casts_ptr),
                                       ctypes.c_void_p(stream)))


def filter_records(tri_all: np.ndarray) -> np.ndarray:
    """Filter records of the two-phase hit test for a triangle soup (n, 9): (n, 20) float32."""
    t = np.ascontiguousarray(tri_all, np.float32).reshape(-1, 9)
    out = np.zeros((t.shape[0], 20), np.float32)
    check(lib().rt_filter_build(_fp(t), t.shape[0], _fp(out)))
    return out


def rect_candidates(filt: np.ndarray, cam: RtCamera, params: RtParams, px0: int, py0: int, px1: int,
                    py1: int) -> np.ndarray:
    """Boolean (n_tri,) mask: the triangles the CPU-preset primary-ray phase keeps for camera
    rays through pixels [px0, px1] x [py0, py1] (the cull of k_cull_ps, run on the host)."""
    f = np.ascontiguousarray(filt, np.float32)
    n = f.shape[0]
    words = np.zeros((n + 63) // 64, np.uint64)
    check(lib().rt_rect_candidates(_fp(f), n, ctypes.byref(cam), ctypes.byref(params), px0, py0, px1, py1,
                                   words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    return bits[:n].astype(bool)


def ctab_candidates(tri_all: np.ndarray, n_surf: int, surf: np.ndarray, orig: np.ndarray, direction: np.ndarray,
                    hit_rule: int = 0):
    """The bounce-ray candidate table of the renderers (rt_ctab_candidates, host only): the
    (n_rays, words) uint64 candidate masks of rays leaving surfaces `surf` from `orig` along unit
    `direction`, and the table's stats (patches, patches kept whole, candidate bits, grazing
    bits).  Every triangle outside a ray's mask fails the exact test (hit rule `hit_rule`; the
    CPU rule at t_scale >= 256) for it."""
    t = np.ascontiguousarray(tri_all, np.float32).reshape(-1, 9)
    s = np.ascontiguousarray(surf, np.int32).ravel()
    o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
    words = (t.shape[0] + 63) // 64
    out = np.zeros((o.shape[0], words), np.uint64)
    stats = np.zeros(4, np.int64)
    check(lib().rt_ctab_candidates(_fp(t), t.shape[0], n_surf, hit_rule, _ip(s), _fp(o), _fp(d), o.shape[0],
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                   stats.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
    return out, stats


def pack_argb(rgb: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(rgb, np.float32)
    n = a.size // 3
    out = np.zeros(a.shape[:-1], np.uint32)
    check(lib().rt_pack_argb(_fp(a), n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
    return out


def save_bmp(path: str, argb: np.ndarray) -> None:
    a = np.ascontiguousarray(argb, np.uint32)
    h, w = a.shape
    check(lib().rt_save_bmp(path.encode(), a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), w, h))


def save_png(path: str, argb: np.ndarray) -> None:
    """8-bit RGB PNG of an ARGB frame buffer (rt_save_png)."""
    a = np.ascontiguousarray(argb, np.uint32)
    h, w = a.shape
    check(lib().rt_save_png(path.encode(), a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), w, h))


def ktime_enable(on: bool = True) -> None:
    """Start (clearing the totals) or stop the library's per-kernel launch timing: HIP events
    on each launch's own stream around k_render_ps, k_render, k_sarsa_render, k_sarsa_apply,
    k_dqn_mlp, k_dqn_bounce and k_dqn_camera (rt_ktime_enable)."""
    check(lib().rt_ktime_enable(int(bool(on))))


def ktime_read() -> dict:
    """{family id: (total ms, launches)} since the last ktime_enable(True) (rt_ktime_read;
    waits for the recorded launches)."""
    out = {}
    for fam in range(_lib.RT_KT_COUNT):
        ms, n = ctypes.c_double(0.0), ctypes.c_int64(0)
        check(lib().rt_ktime_read(fam, ctypes.byref(ms), ctypes.byref(n)))
        out[fam] = (ms.value, n.value)
    return out


def ktime_name(fam: int) -> str:
    return lib().rt_ktime_name(fam).decode()
