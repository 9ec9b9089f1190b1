"""Closed-form fixtures and hand-computed intersection KATs.

The reference pins only plane and sphere t-values (UnitTests/main.cpp:733-786).  These
tests pin the rest of the path against answers derived by hand from the rendering
equation and from the intersection formulas of RT/intersection.cpp, not from either
implementation:

* analytic scenes (tests/analytic_scenes.py): white furnace, emitter only, one diffuse
  bounce off a plane / a mesh / a box -- checked on the CPU oracle here and on the GPU
  (`-m gpu`) through the C ABI;
* Moller-Trumbore triangle KATs (RT/intersection.cpp:135-182) including the inclusive
  edge v + w = 1, the back side (no culling), a parallel ray and a transformed instance;
* box KATs (RT/intersection.cpp:76-105, normal :544-561) including the reference's NaN
  slab quirk: an axis-parallel ray that misses the box geometrically is reported as a
  hit, because the ternary max/min (MathLib/my_math.h) drop the NaN slabs.
"""
import math

import numpy as np
import pytest

import analytic_scenes as asc
import oracle_binding as ob


W, H = 96, 64


@pytest.mark.parametrize("name", sorted(asc.SCENES))
def test_analytic_scene_oracle(rt, name):
    s, cam, st, fc, expected = asc.SCENES[name](rt, W, H)
    frame, stats = ob.render(s.desc(), cam, st, fc, W, H, rng_mode=0, threads=8)
    r = asc.check(frame, expected, st.samples_per_pixel)
    if name == "emitter":
        assert abs(r - asc.disc_fraction(W, H)) < 0.02


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(asc.SCENES))
def test_analytic_scene_gpu(rt, name):
    s, cam, st, fc, expected = asc.SCENES[name](rt, W, H)
    dev = rt.DeviceScene(s, 0)
    try:
        frame, stats = dev.render(cam, st, fc, W, H)
    finally:
        dev.close()
    r = asc.check(frame, expected, st.samples_per_pixel)
    if name == "emitter":
        assert abs(r - asc.disc_fraction(W, H)) < 0.02
    cpu, cstats = ob.render(s.desc(), cam, st, fc, W, H, rng_mode=0, threads=8)
    assert (stats.closest_hit_rays, stats.shadow_rays) == (cstats.closest_hit_rays, cstats.shadow_rays)


def _tri_scene(rt, transform=None, flat=False):
    """The triangle (0,0,0), (2,0,0), (0,2,0); unless `flat`, a second triangle off to the side at
    z = -1 gives the mesh's boxes depth (a zero-thickness box never passes the reference's slab
    test, RT/intersection.cpp:107-133: tn < tf fails when a slab has no width)."""
    s = rt.Scene()
    m = s.add_diffuse_material((0.5, 0.5, 0.5), 1.0)
    tris = [[[0, 0, 0], [2, 0, 0], [0, 2, 0]]]
    if not flat:
        tris.append([[10, 10, -1], [11, 10, -1], [10, 11, -1]])
    tris = np.array(tris, np.float32)
    mesh = s.create_mesh(tris)
    s.add_mesh(m, mesh, transform if transform is not None else rt.translate((0.0, 0.0, 0.0)))
    s.create_scene_bvh()
    return s


def _box_scene(rt):
    s = rt.Scene()
    m = s.add_diffuse_material((0.5, 0.5, 0.5), 1.0)
    s.add_box(m, (1.0, 2.0, 3.0), rt.translate((0.0, 0.0, 0.0)))
    s.create_scene_bvh()
    return s


def _norm(v):
    v = np.asarray(v, np.float64)
    return tuple(v / np.linalg.norm(v))


# (origin, direction, expected t or None for a miss, expected normal or None)
TRI_KATS = [
    ((0.5, 0.5, 5.0), (0.0, 0.0, -1.0), 5.0, (0.0, 0.0, 1.0)),      # front face
    ((0.5, 0.5, -3.0), (0.0, 0.0, 1.0), 3.0, (0.0, 0.0, 1.0)),      # back face: no culling
    ((1.0, 1.0, 5.0), (0.0, 0.0, -1.0), 5.0, (0.0, 0.0, 1.0)),      # on the edge: v = w = 0.5, v + w = 1 kept
    ((0.0, 0.0, 5.0), (0.0, 0.0, -1.0), 5.0, (0.0, 0.0, 1.0)),      # on a vertex: v = w = 0
    ((1.5, 1.5, 5.0), (0.0, 0.0, -1.0), None, None),                # outside: v + w = 1.5
    ((-0.5, 0.5, 5.0), (0.0, 0.0, -1.0), None, None),               # outside: v < 0
    ((0.5, 0.5, 0.0), (1.0, 0.0, 0.0), None, None),                 # parallel: |det| < 1e-9
    ((0.5, 0.5, 5.0), (0.0, 0.0, 1.0), None, None),                 # pointing away: t < 1e-9
]
# instance under translate(10, 0, 0) * scale(2): the world triangle is (10,0,0), (14,0,0), (10,4,0)
TRI_KATS_XF = [
    ((11.0, 1.0, 5.0), (0.0, 0.0, -1.0), 5.0),
    ((12.0, 2.0, -7.0), (0.0, 0.0, 1.0), 7.0),                      # on the hypotenuse, back side
    ((13.0, 3.0, 5.0), (0.0, 0.0, -1.0), None),
]
# Axis-parallel rays hit the reference's NaN-slab quirk: with d = 0 on an axis, inv_d = inf and
# that slab's t1/t2 are NaN when o is 0 there (inf * 0); the ternary max/min (mx(a, b) = a > b ? a
# : b) drop a NaN in the first two slots and keep one in the last, so the outcome depends on
# which axes are zero (worked by hand in each comment, RT/intersection.cpp:76-105).
BOX_KATS = [
    ((0.0, 0.0, 10.0), (0.0, 0.0, -1.0), 7.0, (0.0, 0.0, 1.0)),     # NaN in x, y: dropped -> tn 7, tf 13
    ((0.5, 0.5, -10.0), (0.0, 0.0, 1.0), 7.0, (0.0, 0.0, -1.0)),    # x, y slabs -inf / NaN: tn 7, tf 13
    ((2.0, 0.0, 10.0), (0.0, 0.0, -1.0), 7.0, (1.0, 0.0, 0.0)),     # a geometric miss (x = 2 > 1) reported at z = 3;
                                                                    # normal: major axis of (2, 0, 3) / r = x
    ((0.0, 10.0, 0.0), (0.0, -1.0, 0.0), None, None),               # NaN in z (last): tn = NaN -> miss
    ((0.0, 0.0, 0.0), (1.0, 0.0, 0.0), None, None),                 # from inside along x: NaN last -> miss
    ((-5.0, 0.25, 0.5), (1.0, 0.0, 0.0), None, None),               # tf = NaN -> miss
    ((2.0, 0.0, 10.0), _norm((0.001, 0.001, -1.0)), None, None),    # the quirk ray tilted: a true miss
    ((0.0, 0.0, 10.0), (0.0, 0.0, 1.0), None, None),                # box behind the ray: tf < 0
]


def _tilted_box_kats():
    """Oblique rays with t from float64 slab geometry (entry distance into the box)."""
    rng = np.random.default_rng(5)
    r = np.array([1.0, 2.0, 3.0])
    out = []
    for _ in range(64):
        target = rng.uniform(-0.8, 0.8, 3) * r
        o = target + rng.normal(size=3) * 8.0
        d = target - o
        d /= np.linalg.norm(d)
        d32 = d.astype(np.float32).astype(np.float64)
        o32 = o.astype(np.float32).astype(np.float64)
        t1 = (-r - o32) / d32
        t2 = (r - o32) / d32
        tn = np.max(np.minimum(t1, t2))
        tf = np.min(np.maximum(t1, t2))
        if tn < tf and tn > 0:
            rel = np.abs((o32 + tn*d32) / r)
            axis = int(np.argmax(rel))
            if np.sort(rel)[-2] > rel[axis] - 1e-3:
                continue                                  # near an edge: the major axis is ambiguous
            n = [0.0, 0.0, 0.0]
            n[axis] = float(np.sign((o32 + tn*d32)[axis]))
            out.append((tuple(o32), tuple(d32), float(tn), tuple(n)))
    return out


def _queries(rt, kats):
    from buas_pathtracer_amd.abi import RayQuery, V3
    return [RayQuery(V3(*k[0]), V3(*k[1]), 3.0e38, 0) for k in kats]


def _check_kats(hits, kats, with_normals=True):
    for h, k in zip(hits, kats):
        t_exp = k[2]
        if t_exp is None:
            assert h.primitive == 0xFFFFFFFF, (k, h.t)
            continue
        assert h.primitive != 0xFFFFFFFF, k
        assert abs(h.t - t_exp) <= 1e-6 * max(1.0, t_exp), (k, h.t)
        if with_normals and len(k) > 3 and k[3] is not None:
            assert np.allclose([h.n.x, h.n.y, h.n.z], k[3], atol=1e-6), (k, (h.n.x, h.n.y, h.n.z))


def test_triangle_kats_oracle(rt):
    s = _tri_scene(rt)
    _check_kats(ob.intersect(s.desc(), _queries(rt, TRI_KATS)), TRI_KATS)
    s2 = _tri_scene(rt, rt.mul(rt.translate((10.0, 0.0, 0.0)), rt.scale((2.0, 2.0, 2.0))))
    _check_kats(ob.intersect(s2.desc(), _queries(rt, TRI_KATS_XF)), TRI_KATS_XF, with_normals=False)


def test_flat_mesh_is_invisible_oracle(rt):
    """Reference quirk: a mesh whose bounding box has zero thickness is never hit."""
    s = _tri_scene(rt, flat=True)
    hits = ob.intersect(s.desc(), _queries(rt, TRI_KATS[:4]))
    assert all(h.primitive == 0xFFFFFFFF for h in hits)


def test_box_kats_oracle(rt):
    s = _box_scene(rt)
    _check_kats(ob.intersect(s.desc(), _queries(rt, BOX_KATS)), BOX_KATS)
    tilted = _tilted_box_kats()
    assert len(tilted) > 40
    hits = ob.intersect(s.desc(), _queries(rt, tilted))
    for h, k in zip(hits, tilted):
        assert h.primitive != 0xFFFFFFFF and abs(h.t - k[2]) <= 1e-5 * k[2], (k, h.t)
        assert (h.n.x, h.n.y, h.n.z) == k[3]


@pytest.mark.gpu
def test_triangle_and_box_kats_gpu(rt):
    """The same KATs through the GPU's intersection kernels (rt_debug_intersect), which must
    also agree with the oracle bit for bit."""
    xf = rt.mul(rt.translate((10.0, 0.0, 0.0)), rt.scale((2.0, 2.0, 2.0)))
    flat_kats = [k[:2] + (None, None) for k in TRI_KATS[:4]]
    cases = [(_tri_scene(rt), TRI_KATS, True), (_tri_scene(rt, xf), TRI_KATS_XF, False),
             (_tri_scene(rt, flat=True), flat_kats, False), (_box_scene(rt), BOX_KATS, True)]
    for s, kats, normals in cases:
        dev = rt.DeviceScene(s, 0)
        try:
            hits = dev.intersect(_queries(rt, kats), False)
        finally:
            dev.close()
        _check_kats(hits, kats, with_normals=normals)
        ref = ob.intersect(s.desc(), _queries(rt, kats))
        for a, b in zip(hits, ref):
            assert a.primitive == b.primitive and (a.primitive == 0xFFFFFFFF or a.t == b.t)
    s = _box_scene(rt)
    tilted = _tilted_box_kats()
    dev = rt.DeviceScene(s, 0)
    try:
        hits = dev.intersect(_queries(rt, tilted), False)
    finally:
        dev.close()
    for h, k in zip(hits, tilted):
        assert h.primitive != 0xFFFFFFFF and abs(h.t - k[2]) <= 1e-5 * k[2], (k, h.t)
        assert (h.n.x, h.n.y, h.n.z) == k[3]
