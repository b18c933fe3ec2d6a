"""The C ABI library loads, exports every symbol include/rtmi.h declares, and
its host-only entry points behave (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import MODELS, ROOT


def header_symbols():
    src = open(os.path.join(ROOT, "include", "rtmi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", src)))


def test_exports_every_declared_symbol(rtmi_mod):
    syms = header_symbols()
    assert len(syms) >= 16
    lib = rtmi_mod.lib()
    for s in syms:
        assert hasattr(lib, s), f"librtmi.so does not export {s}"
    assert sorted(rtmi_mod._lib.EXPORTS) == syms


def test_params_defaults(rtmi_mod):
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_CPU)
    assert (p.width, p.height, p.spp, p.max_bounces, p.hit_rule, p.seed) == (512, 512, 16, 2, 0, 1984)
    assert p.t_scale == 512.0
    g = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU)
    assert (g.width, g.height, g.spp, g.max_bounces, g.hit_rule) == (720, 720, 32, 80, 1)
    assert rtmi_mod.default_params(0, height=256).t_scale == 256.0


def test_error_codes(rtmi_mod, tmp_path):
    L = rtmi_mod.lib()
    assert L.rt_params_default(7, ctypes.byref(rtmi_mod.RtParams())) == -1
    assert b"preset" in L.rt_last_error()
    h = ctypes.c_void_p()
    assert L.rt_ctx_create(-1, ctypes.byref(h)) in (-1, -2)
    assert L.rt_pack_argb(None, -1, None) == -1
    with pytest.raises(rtmi_mod.RtError) as e:
        rtmi_mod.obj_geometry(str(tmp_path / "missing.obj"))
    assert e.value.code == -4


def test_obj_parser_formats(rtmi_mod, tmp_path):
    """'f a b c d' and 'f a/b/c ...' are fan-triangulated; other words skipped
    (GPU/objects/object_importer.cu:22-81)."""
    p = tmp_path / "quad.obj"
    p.write_text("# comment\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvt 0 0\nvn 0 0 1\n"
                 "f 1 2 3 4\nf 1/1/1 3/1/1 4/1/1\n")
    g = rtmi_mod.obj_geometry(str(p))
    assert g.n_surf == 3 and g.n_light == 0
    assert np.all(g.albedo == 0.75)
    # v*2 + (-1 - min*2), then x,y negated; Surface(v1, v3, v2)
    v1 = np.array([1.0, 1.0, -1.0]); v2 = np.array([-1.0, 1.0, -1.0]); v3 = np.array([-1.0, -1.0, -1.0])
    assert np.array_equal(g.tri[0], np.concatenate([v1, v3, v2]).astype(np.float32))
    assert np.array_equal(g.nn_vertices[:9], np.concatenate([v1, v2, v3]).astype(np.float32))


def test_save_bmp(rtmi_mod, tmp_path):
    argb = rtmi_mod.pack_argb(np.random.default_rng(1).random((5, 7, 3), dtype=np.float32))
    path = tmp_path / "x.bmp"
    rtmi_mod.save_bmp(str(path), argb)
    data = path.read_bytes()
    assert data[:2] == b"BM" and len(data) == 54 + 5 * 7 * 4
    assert np.array_equal(np.frombuffer(data[54:], np.uint32).reshape(5, 7), argb)


def test_obj_models_present():
    for k in ("door_room", "archway", "complex_light_room"):
        assert os.path.exists(os.path.join(MODELS, f"{k}.obj"))


def test_png_writer_round_trip(rtmi_mod, tmp_path):
    """rt_save_png (stored deflate) decodes to the packed RGB; BMP and PNG agree; the
    MAPE CLI (Graphing/mape.py) reads both."""
    from PIL import Image
    rng = np.random.default_rng(3)
    for h, w in [(1, 1), (7, 13), (300, 251)]:  # last: > one 64 KB deflate block
        rgb = rng.random((h, w, 3), dtype=np.float32) * 1.2
        argb = rtmi_mod.pack_argb(rgb)
        png, bmp = str(tmp_path / "f.png"), str(tmp_path / "f.bmp")
        rtmi_mod.save_png(png, argb)
        rtmi_mod.save_bmp(bmp, argb)
        want = rtmi_mod.metrics.argb_to_rgb8(argb)
        with Image.open(png) as im:
            im.load()
            assert im.mode == "RGB" and im.size == (w, h)
            assert np.array_equal(np.asarray(im), want)
        assert np.array_equal(rtmi_mod.metrics.read_rgb8(bmp), want)
        assert rtmi_mod.metrics.mape_files(png, bmp) == 0.0
    with pytest.raises(rtmi_mod.RtError):
        rtmi_mod.save_png(str(tmp_path / "missing" / "x.png"), np.zeros((2, 2), np.uint32))


def test_mape_cli_matches_formula(rtmi_mod, tmp_path, capsys):
    from PIL import Image
    rng = np.random.default_rng(4)
    a = rng.integers(0, 256, (9, 11, 3), dtype=np.uint8)
    b = np.clip(a.astype(int) + rng.integers(-3, 4, a.shape), 0, 255).astype(np.uint8)
    pa, pb = str(tmp_path / "a.png"), str(tmp_path / "b.png")
    Image.fromarray(a).save(pa)
    Image.fromarray(b).save(pb)
    gt, p = a.astype(np.intc), b.astype(np.intc)
    want = round(float(np.sum(np.abs(gt / 255 - p / 255) / ((gt + 0.01) / 255)) / gt.size), 4)
    assert rtmi_mod.metrics.main([pa, pb]) == 0
    assert float(capsys.readouterr().out.strip()) == want
    assert rtmi_mod.metrics.main([pa]) == 1
