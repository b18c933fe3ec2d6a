"""Per-pixel debug output of k_render_ps (RT_DEBUG_OUT build): fresh context vs after a cull call."""
import ctypes, sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import rtmi
geom = rtmi.cornell_geometry(0)
CAM = (0.0, 0.0, -3.0, 1.0)
cam = rtmi.camera(CAM)
p3 = rtmi.default_params(0, width=64, height=64, spp=8, max_bounces=1)
mode = sys.argv[1]
with rtmi.Context(0) as ctx:
    if mode == "cull1":
        p = rtmi.default_params(0, width=48, height=48, spp=64, spp_split=1)
        n = 9 * 16
        out = np.zeros(n, np.uint64); nw = ctypes.c_int64(n)
        with rtmi.Scene(ctx, geom) as sc:
            rtmi.api.check(rtmi.lib().rt_cull_masks_device(ctx.handle, sc.handle, ctypes.byref(cam), ctypes.byref(p),
                           0, 0, 40, 33, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), ctypes.byref(nw)))
    with rtmi.Scene(ctx, geom) as sc:
        img, c = rtmi.render(ctx, sc, cam, p3)
np.save(f"gpurun_out/dbg_{mode}.npy", img)
print(mode, c, flush=True)
filt = rtmi.filter_records(geom.all_triangles())
bad = []
for b in range(16):
    bx, by = (b % 4) * 16, (b // 4) * 16
    for w in range(4):
        m = rtmi.rect_candidates(filt, cam, p3, bx, by + 4 * w, bx + 15, by + 4 * w + 3)
        want = int(sum(1 << i for i in np.nonzero(m)[0]))
        got = img[by + 4 * w:by + 4 * w + 4, bx:bx + 16]
        g0 = got[..., 0].astype(np.int64); g1 = got[..., 1].astype(np.int64)
        gm = np.unique(g0 | (g1 << 24))
        if len(gm) != 1 or int(gm[0]) != want:
            bad.append((b, w, hex(want), [hex(int(x)) for x in gm[:3]]))
print(mode, "waves with wrong masks in the kernel:", len(bad), bad[:6], flush=True)
