"""The oracle's lower-level outputs against committed golden vectors
(tests/golden/oracle_golden.json, made by tests/golden/make_golden.py) and
against an independent pure-Python restatement (tests/pyref.py)."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_binding as ob
import pyref

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))


def bits(x):
    return np.float32(x).view(np.uint32).item()


def test_wang_hash(oracle):
    for k, v in GOLD["wang_hash"].items():
        assert oracle.oracle_wang_hash(int(k)) == v == pyref.wang_hash(int(k))


def test_sample_seed(oracle):
    for a, b, c, d, e, v in GOLD["sample_seed"]:
        assert oracle.oracle_sample_seed(a, b, c, d, e) == v == pyref.sample_seed(a, b, c, d, e)


def test_rng_stream(oracle):
    for seed, ref in GOLD["rng_unilaterals_bits"].items():
        out = (C.c_float * 64)()
        oracle.oracle_rng_unilaterals(int(seed), 16, out)
        assert [bits(v) for v in out] == ref
        rs = pyref.RandomSeries(int(seed))
        py = [bits(v) for _ in range(16) for v in rs.unilaterals()]
        assert py == ref


def test_samplers(oracle):
    for strategy, x, y, idx, dim, bounce, b0, b1, b2 in GOLD["samples"]:
        out = (C.c_float * 2)()
        oracle.oracle_sample_2d(12345, strategy, x, y, idx, dim, bounce, out)
        assert [bits(out[0]), bits(out[1])] == [b0, b1]
        assert bits(oracle.oracle_sample_1d(12345, strategy, x, y, idx, dim, bounce)) == b2
        p2 = pyref.sample_2d(pyref.RandomSeries(12345), strategy, x, y, idx, dim, bounce)
        p1 = pyref.sample_1d(pyref.RandomSeries(12345), strategy, x, y, idx, dim, bounce)
        assert [bits(p2[0]), bits(p2[1]), bits(p1)] == [b0, b1, b2]


def test_stratified_covers_strata(oracle):
    """64 consecutive indices of one pixel/dimension visit each 8x8 stratum once
    (g_strata_permutation_sets rows are permutations, RT/samplers.cpp:67-72)."""
    cells = set()
    for idx in range(64):
        out = (C.c_float * 2)()
        oracle.oracle_sample_2d(99, 2, 10, 20, idx, 1, 0, out)
        cells.add((int(out[0] * 8), int(out[1] * 8)))
    assert len(cells) == 64


def test_transcendentals_golden_and_accurate(oracle):
    for xb, sb, cb in GOLD["trig_bits"]:
        x = np.uint32(xb).view(np.float32)
        assert bits(oracle.oracle_sinf(float(x))) == sb
        assert bits(oracle.oracle_cosf(float(x))) == cb
        assert abs(float(np.uint32(sb).view(np.float32)) - np.sin(float(x))) <= 4e-7 * max(1.0, abs(float(x)))
        assert abs(float(np.uint32(cb).view(np.float32)) - np.cos(float(x))) <= 4e-7 * max(1.0, abs(float(x)))
    for xb, eb in GOLD["exp_bits"]:
        x = float(np.uint32(xb).view(np.float32))
        e = float(np.uint32(eb).view(np.float32))
        assert bits(oracle.oracle_expf(x)) == eb
        ref = np.exp(x)
        assert abs(e - ref) <= 3e-7 * ref + 1e-44
    for xb, ab in GOLD["asin_bits"]:
        x = float(np.uint32(xb).view(np.float32))
        assert bits(oracle.oracle_asinf(x)) == ab
        assert abs(float(np.uint32(ab).view(np.float32)) - np.arcsin(x)) <= 4e-7
    for yb, xb, ab in GOLD["atan2_bits"]:
        y = float(np.uint32(yb).view(np.float32))
        x = float(np.uint32(xb).view(np.float32))
        assert bits(oracle.oracle_atan2f(y, x)) == ab
        assert abs(float(np.uint32(ab).view(np.float32)) - np.arctan2(y, x)) <= 5e-7


def test_mitchell_lut(rt, oracle):
    fc = rt.FilterCache()
    oracle.oracle_load_filter(b"Mitchell Netravali", C.byref(fc))
    assert [bits(v) for v in fc.cache[:256]] == GOLD["mitchell_lut_bits"]
    host = rt.load_reconstruction_kernel("Mitchell Netravali")
    assert (host.kernel_size, host.cache_size) == (2, 256)
    assert [bits(v) for v in host.cache[:256]] == GOLD["mitchell_lut_bits"]
    assert all(v == 0.0 for v in host.cache[256:])
    # B = C = 1/3: k(0) = 8/9, k(1) = 1/18, k(2) = 0
    assert abs(fc.cache[0] - 8 / 9) < 1e-6 and abs(fc.cache[255]) < 1e-6


def test_c1_hits(rt):
    scene, cam, st, fc, post = rt.load_preset("c1", 64, 64)
    rays = []
    for row in GOLD["c1_hits"]:
        f = [float(np.uint32(b).view(np.float32)) for b in row[:6]]
        rays.append(rt.abi.RayQuery(rt.V3(*f[:3]), rt.V3(*f[3:6]), 3.0e38, 0))
    hits = ob.intersect(scene.desc(), rays)
    for row, h in zip(GOLD["c1_hits"], hits):
        assert h.primitive == row[6]
        assert [bits(h.t), bits(h.n.x), bits(h.n.y), bits(h.n.z)] == row[7:11]


def test_c1_small_frame(rt):
    scene, cam, st, fc, post = rt.load_preset("c1", 64, 64)
    acc, stats = ob.render(scene.desc(), cam, st, fc, 64, 64, rng_mode=0, threads=1)
    g = GOLD["c1_64x64_frame"]
    assert hashlib.sha256(acc.tobytes()).hexdigest() == g["sha256"]
    assert (stats.closest_hit_rays, stats.shadow_rays) == (g["closest"], g["shadow"])


def test_thread_count_independence(rt):
    """The multi-threaded oracle merges tile buffers in tile order: same result for any thread count."""
    scene, cam, st, fc, post = rt.load_preset("c1", 96, 96)
    a, sa = ob.render(scene.desc(), cam, st, fc, 96, 96, rng_mode=0, threads=2)
    b, sb = ob.render(scene.desc(), cam, st, fc, 96, 96, rng_mode=0, threads=5)
    assert np.array_equal(a, b)
    c, sc_ = ob.render(scene.desc(), cam, st, fc, 96, 96, rng_mode=0, threads=1)
    assert np.abs(a - c).max() <= 1e-4 * np.abs(c).max()
    assert sa.closest_hit_rays == sb.closest_hit_rays == sc_.closest_hit_rays
