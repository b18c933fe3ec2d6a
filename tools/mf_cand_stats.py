#!/usr/bin/env python3
"""Candidate statistics of the two bounce-cast filters, on the host (float64 restatement
of the filter quantities; the device roundings are far below the margins):

  fp32 filter  (closest_hit_filtered): margins at c = 2^-16, origin bound of the records
  matrix-core  (closest_hit_mf):       margins at c = 2^-12, origin bound = box + 1

For rays from surface points into the hemisphere of the surface normal (the bounce casts
of k_render_ps), prints per filter: mean candidates per ray and the mean over waves of
64 consecutive rays of the largest count in the wave (the exact phase's trip count).

    python tools/mf_cand_stats.py [--scene cornell] [--n 200000] [--c-mf -12]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402


def quantities(tri, o, d, ets):
    v0, v1, v2 = tri[:, 0:3], tri[:, 3:6], tri[:, 6:9]
    e1, e2 = v1 - v0, v2 - v0
    N = np.cross(e1, e2)
    G1, G2 = np.cross(v0, e1), np.cross(v0, e2)
    w0 = np.sum(v0 * N, axis=1)
    R = np.cross(d, o)
    A = d @ N.T
    T = w0[None, :] - o @ N.T - ets * A
    U = R @ e2.T - d @ G2.T
    V = -(R @ e1.T) + d @ G1.T
    return A, T, U, V


def margins(tri, ob, c, ets_max=1e-5 * 16384.0, dinf=2.0):
    v0, v1, v2 = tri[:, 0:3], tri[:, 3:6], tri[:, 6:9]
    a, b = v1 - v0, v2 - v0
    M = np.zeros(len(tri))
    for i in range(3):
        j, k = (i + 1) % 3, (i + 2) % 3
        M += np.abs(a[:, j] * b[:, k]) + np.abs(a[:, k] * b[:, j])
    vmax = np.abs(v0).max(axis=1)
    n1, n2 = np.abs(a).sum(axis=1), np.abs(b).sum(axis=1)
    B = ob + vmax
    eA = c * dinf * M
    EW = 2 * (c * 2 * dinf * B * n2 + c * 2 * dinf * B * n1 + eA)
    ET = c * (B + dinf * ets_max) * M + dinf * ets_max * eA
    return eA, EW, ET


def candidates(A, T, U, V, eA, EW, ET):
    sg = np.sign(A)
    sg[sg == 0] = 1
    su, sv, st = U * sg, V * sg, T * sg
    aa = np.abs(A)
    w = aa - su - sv
    m = np.minimum(np.minimum(su, sv), w)
    reject = (aa > eA) & ((m + EW < 0) | (st + ET < 0))
    return (~reject).sum(axis=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--c-mf", type=int, default=-12)
    args = ap.parse_args()
    if args.scene == "cornell":
        g = rtmi.cornell_geometry(0)
    else:
        g = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", args.scene + ".obj"), args.scene)
    tri = g.all_triangles().reshape(-1, 9).astype(np.float64)
    rng = np.random.default_rng(1)
    n = args.n
    t = tri.reshape(-1, 3, 3)
    surf = rng.integers(0, g.n_surf, n)
    u, v = rng.random(n), rng.random(n)
    f = u + v > 1
    u[f], v[f] = 1 - u[f], 1 - v[f]
    p = t[surf, 0] + u[:, None] * (t[surf, 1] - t[surf, 0]) + v[:, None] * (t[surf, 2] - t[surf, 0])
    nrm = np.cross(t[surf, 2] - t[surf, 0], t[surf, 1] - t[surf, 0])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d *= np.sign(np.sum(d * nrm, axis=1))[:, None]
    o = p + 1e-5 * d
    vmax = np.abs(tri).max()
    ob_rec = max(8.0, 2 * vmax + 1)
    ets = 1e-5 * 512
    out = {}
    for name, ob, c, dinf in (("fp32 filter", ob_rec, 2.0 ** -16, 2.0), ("matrix-core", vmax + 1, 2.0 ** args.c_mf, 2.0), ("mc tight", vmax * (1 + 2**-10) + 2**-10, 2.0 ** args.c_mf, 1.0 + 2**-10)):
        cnt = np.zeros(n, np.int64)
        for s in range(0, n, 20000):
            A, T, U, V = quantities(tri, o[s:s + 20000], d[s:s + 20000], ets)
            cnt[s:s + 20000] = candidates(A, T, U, V, *margins(tri, ob, c, dinf=dinf))
        wave = cnt[: n // 64 * 64].reshape(-1, 64).max(axis=1)
        out[name] = (cnt.mean(), wave.mean())
        print(f"{name:12s} c=2^{int(np.log2(c))} bound {ob:.1f}: mean {cnt.mean():.3f} candidates/ray, "
              f"wave max {wave.mean():.2f} (of {len(tri)} triangles)")


if __name__ == "__main__":
    main()
