#!/usr/bin/env python3
"""Run rt_selftest(RT_SELFTEST_RCP) for each librtmi.so variant directory given."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
from rtmi import _lib  # noqa: E402

out = {}
for v in sys.argv[1:]:
    L = ctypes.CDLL(os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd", v, "librtmi.so"))
    _lib._declare(L)
    ctx = ctypes.c_void_p()
    assert L.rt_ctx_create(0, ctypes.byref(ctx)) == 0
    res = (ctypes.c_uint64 * 2)()
    rc = L.rt_selftest(ctx, 1, res)
    out[v] = {"rc": rc, "mismatches": int(res[0]), "first_bits": hex(int(res[1]))}
print(json.dumps(out))
