"""Host build of the exact BVH path (rt_bvh.cpp) without a GPU: rt_bvh_check builds the
tree and grazing lists of a scene and checks their invariants (every triangle in one
leaf of each tree, nested boxes holding their triangles, planes inside their plane-space
leaves).  The bit-exactness of the
device path is in test_bvh.py (-m gpu)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import MODELS


def _check(rtmi, tri):
    tri = np.ascontiguousarray(tri, np.float32)
    stats = (ctypes.c_int64 * 4)()
    rc = rtmi.lib().rt_bvh_check(tri.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), tri.shape[0], stats)
    assert rc == 0, rtmi.lib().rt_last_error().decode()
    return list(stats)


@pytest.mark.parametrize("scene", ["bunny_cornell", "Medieval_House", "complex_light_room", "cornell"])
def test_bvh_host_invariants(rtmi_mod, scene):
    if scene == "bunny_cornell":
        from test_bvh import bunny_cornell
        g = bunny_cornell(rtmi_mod, 1)
    elif scene == "cornell":
        g = rtmi_mod.cornell_geometry(0)
    else:
        kind = scene if scene == "complex_light_room" else "generic"
        g = rtmi_mod.obj_geometry(os.path.join(MODELS, f"{scene}.obj"), kind)
    nodes, depth, pnodes, leaves = _check(rtmi_mod, g.all_triangles())
    assert 0 < depth < 24 and leaves * 4 >= g.n_tri and nodes == 2 * leaves - 1
    assert pnodes >= g.n_tri // 4


def test_bvh_host_degenerate_inputs(rtmi_mod):
    # coincident triangles (equal centroids) and a single triangle
    t = np.tile(np.array([[0, 0, 0, 1, 0, 0, 0, 1, 0]], np.float32), (40, 1))
    _check(rtmi_mod, t)
    _check(rtmi_mod, t[:1])
    rng = np.random.default_rng(0)
    _check(rtmi_mod, rng.uniform(-1, 1, (3000, 9)).astype(np.float32))
