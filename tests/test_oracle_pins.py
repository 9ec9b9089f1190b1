"""The oracle is pinned against the reference itself.

1. Known-answer tests from the reference's own unit tests
   (UnitTests/main.cpp:733-786: plane and sphere t-values), run against the
   production intersection functions the oracle restates
   (RT/intersection.cpp:12-74).
2. The reference's own observed output for config C1 (BASELINE.md §2,
   SURVEY.md §8(c)): Week-6 scene, 512x512, 16 spp, depth 4, one thread,
   reference-stream RNG, C-library transcendentals.  The reference produced
   sum(rgb) = 1.975555e+07, sum(w) = 4.249201e+06 and 10,271,787 closest-hit /
   7,253,677 shadow rays; the restatement reproduces all four exactly.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_binding as ob


def _v(*a):
    return (C.c_float * 3)(*a)


@pytest.mark.parametrize("o,expected", [((0, 0, 10), 17.0710678), ((0, 2, 10), 19.0710678),
                                        ((5, -10, 10), 7.07106781)])
def test_plane_kat(oracle, o, expected):
    t = C.c_float(3.0e38)
    n = _v(0.0, 0.707106781, 0.707106781)
    assert oracle.oracle_ray_intersect_plane(_v(*o), _v(0, 0, -1), n, -5.0, C.byref(t)) == 1
    assert abs(t.value - expected) <= 0.001                  # UnitTests/main.cpp:15 EPSILON


def test_plane_kat_misses(oracle):
    t = C.c_float(3.0e38)
    assert oracle.oracle_ray_intersect_plane(_v(0, 0, 0), _v(0, 0, -1), _v(0, 1, 0), 0.0, C.byref(t)) == 0  # parallel
    assert oracle.oracle_ray_intersect_plane(_v(0, 0, -1), _v(0, 0, -1), _v(0, 0, 1), 0.0, C.byref(t)) == 0  # behind


@pytest.mark.parametrize("o,t_near", [((0, 0, 10), 6.0), ((2, 0, 10), 6.53589838), ((4, 0, 10), 10.0)])
def test_sphere_kat(oracle, o, t_near):
    t = C.c_float(3.0e38)
    assert oracle.oracle_ray_intersect_sphere(_v(*o), _v(0, 0, -1), 4.0, C.byref(t)) == 1
    assert abs(t.value - t_near) <= 0.001


def test_sphere_kat_miss_and_inside(oracle):
    t = C.c_float(3.0e38)
    assert oracle.oracle_ray_intersect_sphere(_v(6, 0, 10), _v(0, 0, -1), 4.0, C.byref(t)) == 0
    # from inside, the production function returns the far root (t_far = 4)
    assert oracle.oracle_ray_intersect_sphere(_v(0, 0, 0), _v(0, 0, -1), 4.0, C.byref(t)) == 1
    assert abs(t.value - 4.0) <= 0.001


def test_c1_reproduces_reference_output(rt, oracle):
    scene, cam, st, fc, post = rt.load_preset("c1", 512, 512)
    assert (st.samples_per_pixel, st.max_bounce_count) == (16, 4)
    oracle.oracle_set_math_mode(1)
    try:
        acc, stats = ob.render(scene.desc(), cam, st, fc, 512, 512, rng_mode=1, threads=1)
    finally:
        oracle.oracle_set_math_mode(0)
    assert f"{acc[..., :3].astype(np.float64).sum():.6e}" == "1.975555e+07"
    assert f"{acc[..., 3].astype(np.float64).sum():.6e}" == "4.249201e+06"
    assert stats.closest_hit_rays == 10271787
    assert stats.shadow_rays == 7253677
