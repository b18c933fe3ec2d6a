"""Expected-SARSA radiance volumes (BASELINE config 3) on top of the C ABI.

  RadianceMap(ctx, scene, seed)   rt_sarsa_create: volumes, Q-table, KD tree on the device
  RadianceMap(..., area_per_sample=a)   rt_sarsa_create_density: another AREA_PER_SAMPLE
  .render(cam, params, frames)    draw_reinforcement_path_tracing + update_radiance_volume_
                                  distributions per frame (rt_render_sarsa)
  .render_tiles_device(...)       one frame over a tile list; apply=False leaves the frame's TD
                                  sums for a cross-GPU sum (rtmi.dist.sarsa_frame)
  .read() / .volumes() / .nearest(pos, nrm)   Q-table, placement, KD queries (parity)
  .save_q(path) / .load_q(path)   radiance_map_data.txt out and back in (resume a trained map)
  .set_sampling(SAMPLE_MAX)       sample_max_direction_from_radiance_distribution
  .set_td_mode(TD_INFRAME)        the reference's racy in-frame TD update (one GPU)
  .frame_stats() / .append_stats_line(path)   sarsa_training_stats.txt (GPU/main.cu:321-339)
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._lib import check, lib

from .api import Context, Scene, _fp, _ip

SEARCH_KD = 0    # RT_SARSA_SEARCH_KD
SEARCH_GRID = 1  # RT_SARSA_SEARCH_GRID
SAMPLE_CDF = 0   # RT_SARSA_SAMPLE_CDF
SAMPLE_MAX = 1   # RT_SARSA_SAMPLE_MAX
TD_FRAME = 0     # RT_SARSA_TD_FRAME
TD_INFRAME = 1   # RT_SARSA_TD_INFRAME

SECTORS = 144  # GRID_RESOLUTION^2

KD_DTYPE = np.dtype([("dim", "<i4"), ("leaf", "<i4"), ("left", "<i4"), ("right", "<i4"), ("data", "<f4"),
                     ("px", "<f4"), ("py", "<f4"), ("pz", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                     ("vol", "<i4")])


class RadianceMap:
    def __init__(self, ctx: Context, scene: Scene, seed: int = 1984, area_per_sample: float | None = None):
        """area_per_sample: the volume density, floor(area / area_per_sample) volumes per
        surface (AREA_PER_SAMPLE, radiance_volumes_settings.h:12; None = the reference's 0.001)"""
        self.ctx = ctx
        self.scene = scene
        self._h = ctypes.c_void_p()
        if area_per_sample is None:
            check(lib().rt_sarsa_create(ctx.handle, scene.handle, seed, ctypes.byref(self._h)))
        else:
            check(lib().rt_sarsa_create_density(ctx.handle, scene.handle, seed, float(area_per_sample),
                                                ctypes.byref(self._h)))
        nv, nk, fr = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_uint32(0)
        check(lib().rt_sarsa_info(self._h, ctypes.byref(nv), ctypes.byref(nk), ctypes.byref(fr)))
        self.n_volumes, self.n_nodes = nv.value, nk.value

    @property
    def handle(self):
        return self._h

    @property
    def frames(self) -> int:
        fr = ctypes.c_uint32(0)
        check(lib().rt_sarsa_info(self._h, None, None, ctypes.byref(fr)))
        return int(fr.value)

    def set_search(self, mode: int) -> None:
        """RT_SARSA_SEARCH_KD (0) or RT_SARSA_SEARCH_GRID (1, default); same results."""
        check(lib().rt_sarsa_set_search(self._h, mode))

    def search_stats(self) -> dict:
        mode, ncls = ctypes.c_int32(0), ctypes.c_int32(0)
        cells, fb = ctypes.c_int64(0), ctypes.c_uint64(0)
        check(lib().rt_sarsa_search_stats(self._h, ctypes.byref(mode), ctypes.byref(ncls), ctypes.byref(cells),
                                          ctypes.byref(fb)))
        return {"mode": int(mode.value), "classes": int(ncls.value), "grid_cells": int(cells.value),
                "kd_fallbacks": int(fb.value)}

    def save_q(self, path: str) -> None:
        """radiance_map_data.txt format (RadianceMap::save_q_vals_to_file)."""
        check(lib().rt_sarsa_save_q(self._h, os.fsencode(path)))

    def load_q(self, path: str) -> None:
        """A radiance_map_data.txt of this map (same scene and seed) back into the device map:
        Q from the file, irradiance estimate and CDF recomputed, visits kept (rt_sarsa_load_q)."""
        check(lib().rt_sarsa_load_q(self._h, os.fsencode(path)))

    def set_sampling(self, mode: int) -> None:
        """SAMPLE_CDF (default) or SAMPLE_MAX (the sector of largest Q, radiance_volume.cu:246-278)."""
        check(lib().rt_sarsa_set_sampling(self._h, mode))

    def set_td_mode(self, mode: int) -> None:
        """TD_FRAME (default: frame-synchronous, deterministic) or TD_INFRAME (the reference's
        in-frame read-modify-write, radiance_volume.cu:282-301; racy, one GPU only)."""
        check(lib().rt_sarsa_set_td_mode(self._h, mode))

    def set_inframe_lanes(self, lanes: int) -> None:
        """paths in flight of the in-frame rule's render (0: the device's full occupancy;
        the reference's GTX 1070 Ti holds 38,912): rt_sarsa_set_inframe_lanes"""
        check(lib().rt_sarsa_set_inframe_lanes(self._h, lanes))

    @property
    def td_mode(self) -> int:
        """the map's TD rule, read from the library (rt_sarsa_get_td_mode)"""
        m = ctypes.c_int32(0)
        check(lib().rt_sarsa_get_td_mode(self._h, ctypes.byref(m)))
        return int(m.value)

    def frame_stats(self):
        """(sum over pixels of int(mean path length), zero-contribution paths) of the last frame."""
        a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(lib().rt_sarsa_frame_stats(self._h, ctypes.byref(a), ctypes.byref(b)))
        return int(a.value), int(b.value)

    def append_stats_line(self, path: str, pixels: int, sums=None) -> str:
        """One line of sarsa_training_stats.txt (GPU/main.cu:330-339): the average path length
        (integer division over `pixels`, printed as the float it is stored in), 0.0, the
        zero-contribution paths.  sums: (path_floor_sum, zero_paths) summed over ranks, else
        this map's frame_stats()."""
        paths, zero = self.frame_stats() if sums is None else sums
        line = stats_line(paths, zero, pixels)
        with open(path, "a") as fh:
            fh.write(line)
        return line

    def save_selected(self, to_select: str, out: str) -> None:
        """selected_sarsa.txt format for the locations of to_select.txt."""
        check(lib().rt_sarsa_save_selected(self.ctx.handle, self._h, os.fsencode(to_select), os.fsencode(out)))

    def volumes(self):
        n = self.n_volumes
        pos = np.zeros((n, 3), np.float32)
        nrm = np.zeros((n, 3), np.float32)
        surf = np.zeros(n, np.int32)
        kd = np.zeros(self.n_nodes, KD_DTYPE)
        check(lib().rt_sarsa_volumes(self._h, _fp(pos), _fp(nrm), _ip(surf), kd.ctypes.data_as(ctypes.c_void_p)))
        return pos, nrm, surf, kd

    def read(self):
        """(Q, CDF, visits) as n x 144 and the irradiance estimate accumulators (n)."""
        n = self.n_volumes
        q = np.zeros((n, SECTORS), np.float32)
        cdf = np.zeros((n, SECTORS), np.float32)
        vis = np.zeros((n, SECTORS), np.uint32)
        acc = np.zeros(n, np.float32)
        check(lib().rt_sarsa_read(self._h, _fp(q), _fp(cdf), vis.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                  _fp(acc)))
        return q, cdf, vis, acc

    def nearest(self, pos: np.ndarray, nrm: np.ndarray) -> np.ndarray:
        p = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
        n_ = np.ascontiguousarray(nrm, np.float32).reshape(-1, 3)
        out = np.zeros(p.shape[0], np.int32)
        check(lib().rt_sarsa_nearest(self.ctx.handle, self._h, _fp(p), _fp(n_), p.shape[0], _ip(out)))
        return out

    def render(self, cam, params, frames: int = 1):
        out = np.zeros((params.height, params.width, 3), np.float32)
        casts = ctypes.c_uint64(0)
        check(lib().rt_render_sarsa(self.ctx.handle, self.scene.handle, self._h, ctypes.byref(cam),
                                    ctypes.byref(params), frames, _fp(out), ctypes.byref(casts)))
        return out, int(casts.value)

    def render_tiles_device(self, cam, params, tiles: np.ndarray, tile_size: int, out_ptr: int, casts_ptr: int,
                            apply: bool, stream: int) -> None:
        t = np.ascontiguousarray(tiles, np.int32).reshape(-1, 2)
        check(lib().rt_render_sarsa_tiles_device(self.ctx.handle, self.scene.handle, self._h, ctypes.byref(cam),
                                                 ctypes.byref(params), _ip(t), t.shape[0], tile_size,
                                                 ctypes.c_void_p(out_ptr), ctypes.c_void_p(casts_ptr),
                                                 int(bool(apply)), ctypes.c_void_p(stream)))

    def td_device(self):
        """Device pointers of the frame's TD sums (int64, fixed point 2^-32) and counts (uint32)."""
        s, c, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64(0)
        check(lib().rt_sarsa_td_device(self._h, ctypes.byref(s), ctypes.byref(c), ctypes.byref(n)))
        return int(s.value or 0), int(c.value or 0), int(n.value)

    def apply(self, stream: int = 0) -> None:
        check(lib().rt_sarsa_apply(self._h, ctypes.c_void_p(stream)))

    def close(self):
        if self._h:
            lib().rt_sarsa_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def stats_line(path_floor_sum: int, zero_paths: int, pixels: int) -> str:
    """`avg << " " << 0.0 << " " << zero` with ostream defaults: avg = float(int / int)."""
    avg = np.float32(path_floor_sum // pixels)
    return f"{float(avg):g} {0.0:g} {zero_paths}\n"


def read_q_file(path: str):
    """radiance_map_data.txt -> (positions [n, 3], Q [n, 144])."""
    with open(path) as fh:
        actions = int(fh.readline())
        rows = [np.array(l.split(), np.float64) for l in fh if l.strip()]
    a = np.array(rows).reshape(len(rows), 3 + actions)
    return a[:, :3].astype(np.float32), a[:, 3:].astype(np.float32)


def read_selected_file(path: str):
    """selected_sarsa.txt / selected_deep.txt -> (positions, normals, distributions [n, 144])."""
    with open(path) as fh:
        rows = [np.array(l.split(), np.float64) for l in fh if l.strip()]
    a = np.array(rows).reshape(len(rows), -1)
    return a[:, :3].astype(np.float32), a[:, 3:6].astype(np.float32), a[:, 6:].astype(np.float32)
