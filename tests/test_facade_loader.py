"""The facade's OBJ loader keeps the reference's signature and HEAD semantics
(GPU/objects/object_importer.cu:8-89, GPU/scenes/scene.cu:33-39):

  load_scene(path, surfaces, lights, vertices, bool lights_in_obj)
    false -> build_surfaces + build_area_lights (archway materials and lights) == kind 2
    true  -> build_surfaces_and_lights (the OBJ's own light triangles)       == kind 3

checked through examples/scene_dump.cpp, which is the reference's own call
`scene.load_custom_scene("../Models/archway.obj", false)` (GPU/main.cu:111).
Host only (the loader touches no GPU), so these run in the CPU suite.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, MODELS, PKG

BUILD = os.path.join(PKG, "build")


def dump(path, lights_in_obj, tmp_path):
    exe = os.path.join(BUILD, "scene_dump")
    assert os.path.exists(exe), f"{exe} missing: make -C {PKG}"
    out = tmp_path / "scene.bin"
    r = subprocess.run([exe, path, str(int(lights_in_obj)), str(out)], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = out.read_bytes()
    ns, nl, nv = np.frombuffer(raw[:12], np.int32)
    body = np.frombuffer(raw[12:], np.float32)
    surf = body[:ns * 12].reshape(ns, 12)
    lig = body[ns * 12:(ns + nl) * 12].reshape(nl, 12)
    verts = body[(ns + nl) * 12:]
    assert verts.size == 3 * nv
    return surf, lig, verts


@pytest.mark.parametrize("scene,lights_in_obj,kind", [
    ("archway", False, 2),             # GPU/main.cu:111
    ("complex_light_room", True, 3),   # the config-5 scene
    ("door_room", False, 2),           # false on another OBJ: still the archway blocks at HEAD
])
def test_load_custom_scene_bool_matches_kind(rtmi_mod, scene, lights_in_obj, kind, tmp_path):
    path = os.path.join(MODELS, scene + ".obj")
    surf, lig, verts = dump(path, lights_in_obj, tmp_path)
    g = rtmi_mod.obj_geometry(path, kind)
    assert surf.shape[0] == g.n_surf and lig.shape[0] == g.n_light
    assert np.array_equal(surf[:, :9].view(np.uint32), g.tri.view(np.uint32))
    assert np.array_equal(surf[:, 9:].view(np.uint32), g.albedo.view(np.uint32))
    assert np.array_equal(lig[:, :9].view(np.uint32), g.light.view(np.uint32))
    assert np.array_equal(lig[:, 9:].view(np.uint32), g.emission.view(np.uint32))
    assert np.array_equal(verts.view(np.uint32), g.nn_vertices.view(np.uint32))
    assert g.n_light > 0  # false no longer loads an unlit scene


def test_archway_false_matches_reference_vertex_dump(rtmi_mod, tmp_path):
    """The reference's own dump of this exact call (Radiance_Map_Data/vertices.txt, written by
    Scene::save_vertices_to_file after load_custom_scene(archway, false)): the surfaces in
    (v1, v3, v2) order, then the 6 archway lights."""
    surf, lig, _ = dump(os.path.join(MODELS, "archway.obj"), False, tmp_path)
    gold = np.loadtxt(os.path.join(GOLDEN, "archway_vertices.txt"), dtype=np.float64)
    got = np.concatenate([surf[:, :9], lig[:, :9]]).astype(np.float64)
    assert got.shape == gold.shape == (102, 9)
    assert np.all(np.abs(got - gold) <= 5e-6 * np.maximum(np.abs(gold), 1.0))


def test_int_argument_does_not_compile(tmp_path):
    """An int scene kind cannot silently convert to lights_in_obj (the facade deletes the
    non-bool overloads); load_custom_scene_kind is the explicit form."""
    src = tmp_path / "bad.cpp"
    src.write_text('#include "%s"\nint main() { rtmi::Scene s; return s.load_custom_scene("x.obj", 1); }\n'
                   % os.path.join(PKG, "host", "scene.h"))
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", str(src)], capture_output=True, text=True)
    assert r.returncode != 0 and "deleted" in r.stderr
    src.write_text('#include "%s"\nint main() { rtmi::Scene s; return s.load_custom_scene("x.obj", false) + '
                   's.load_custom_scene_kind("x.obj", 1); }\n' % os.path.join(PKG, "host", "scene.h"))
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
