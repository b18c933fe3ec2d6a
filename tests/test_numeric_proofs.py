"""Exhaustive proofs of the numeric building blocks every bit-exact claim rests on.

The kernels replace three IEEE divisions by cheaper sequences and claim the same bits:
  * rcp_rn (rt_math.hpp): 1 / x as v_rcp_f32 + one FMA Newton step (Cramer's 1/detA,
    normalize), equal to IEEE 1.0f / x for every float (out-of-range inputs divide);
  * div12: the Chiu-map grid coordinate x / 12, equal to IEEE over +0 and |x| in
    [2^-100, 2^100];
  * div_rho: the estimator's x / RHO, equal to IEEE for every float.
CPU: the host restatements of div12 / div_rho (tools/check_div12.c, check_divrho.c; IEEE fmaf
on both sides) over all 2^32 inputs.  GPU: the device functions themselves, through
rt_selftest, over all 2^32 inputs.
"""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["check_div12", "check_divrho"])
def test_host_exhaustive_division_checks(name, tmp_path):
    exe = str(tmp_path / name)
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", os.path.join(ROOT, "tools", name + ".c"),
                    "-o", exe, "-lm"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout
    words = r.stdout.split()
    tested = int(words[words.index("tested") + 1])
    assert int(words[words.index("mismatches") + 1]) == 0
    assert tested > 3_000_000_000  # (+0 and the 2^-100 .. 2^100 binades of both signs)


@pytest.mark.gpu
@pytest.mark.parametrize("which,name", [(1, "RT_SELFTEST_RCP"), (2, "RT_SELFTEST_DIV12"), (3, "RT_SELFTEST_DIVRHO")])
def test_device_exhaustive_selftest(rtmi_mod, gpu_ctx, which, name):
    res = (ctypes.c_uint64 * 2)()
    rtmi_mod.check(rtmi_mod.lib().rt_selftest(gpu_ctx.handle, which, res))
    assert int(res[0]) == 0, (name, int(res[0]), hex(int(res[1])))
    assert int(res[1]) == 0xFFFFFFFF  # no mismatching input recorded


def test_selftest_refuses_null_context(rtmi_mod):
    res = (ctypes.c_uint64 * 2)()
    assert rtmi_mod.lib().rt_selftest(None, 1, res) != 0


def test_philox_shared_prefix_equals_full(tmp_path):
    """philox_shared + philox_from (rt_math.hpp: rounds 1-3's products of the words that do not
    depend on the last counter word, computed once per ray for the DQN sampler's 47 draws and
    the TD targets' 72) give philox4x32_10's words bit for bit: 2 M random counters and keys,
    a third of them with small c3 as the sampler uses."""
    src = tmp_path / "philox_check.cpp"
    src.write_text(r'''
#include <cstdio>
#include <cstdint>
#include <random>
#include "rt_math.hpp"
int main() {
    std::mt19937 g(1);
    long bad = 0;
    for (int i = 0; i < 2000000; i++) {
        uint32_t c0 = g(), c1 = g(), c2 = g(), c3 = g(), k0 = g(), k1 = g();
        if (i % 3 == 0) c3 = i % 200;
        uint32_t a[4], b[4];
        rt::philox4x32_10(c0, c1, c2, c3, k0, k1, a);
        const rt::PhiloxShared s = rt::philox_shared(c0, c1, c2, k0, k1);
        rt::philox_from(s, c3, b);
        for (int k = 0; k < 4; k++) bad += a[k] != b[k];
    }
    printf("%ld\n", bad);
    return bad != 0;
}
''')
    exe = str(tmp_path / "philox_check")
    inc = os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", inc, str(src), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout


def _min_key(t, tri):
    """rt_trace.hpp min_key, restated"""
    import struct
    b = struct.unpack("<I", struct.pack("<f", t))[0]
    return ((b & 0x7FFFFFFF) << 32) | ((tri + 1) << 1) | (b >> 31)


def _min_unkey(k):
    import struct
    hi, lo = k >> 32, k & 0xFFFFFFFF
    return struct.unpack("<f", struct.pack("<I", (hi | ((lo & 1) << 31)) & 0xFFFFFFFF))[0], (lo >> 1) - 1


def test_rule1_min_fold_equals_index_order_window():
    """cand_exact_min (rt_trace.hpp) folds RULE 1's passes by a 64-bit minimum instead of the
    reference's index-order window (accept t < best, from best = 999999, tri -1): the same
    (t, tri) bits for every sequence -- ties (the first index wins), -0 against +0, passes at
    or above the start's 999999, and passes before or after the lane's own tests."""
    import math
    import random
    import struct
    rng = random.Random(5)
    specials = [0.0, -0.0, 999999.0, 999998.9375, 1e-30, 1.0, 2.0, 5e5, 1e6, math.inf]
    for trial in range(20000):
        n = rng.randint(0, 12)
        seq = []
        for i in range(n):
            r = rng.random()
            t = rng.choice(specials) if r < 0.5 else (rng.choice(specials[:6]) if r < 0.6 else rng.uniform(0, 2e6))
            t = struct.unpack("<f", struct.pack("<f", t))[0]
            seq.append((t, i))
        best_t, best_i = 999999.0, -1
        for t, i in seq:
            if t < best_t:
                best_t, best_i = t, i
        own = rng.randint(0, n)  # the lane's first `own` candidates tested on its lane
        h_t, h_i = 999999.0, -1
        for t, i in seq[:own]:
            if t < h_t:
                h_t, h_i = t, i
        key = _min_key(h_t, h_i)
        for t, i in seq[own:]:
            if t < 999999.0:
                key = min(key, _min_key(t, i))
        got_t, got_i = _min_unkey(key)
        assert got_i == best_i, (seq, own)
        assert struct.pack("<f", got_t) == struct.pack("<f", best_t), (seq, own)
