"""Edge cases of the render path through the GPU against the oracle: degenerate scenes (sky only,
planes only, no meshes, a one-triangle mesh), ragged and tiny frames, and the settings' limits
(one sample per pixel, the deepest path the ABI accepts, and the first one it rejects).

Each case is checked as tests/test_gpu_scenes.py checks a scene (`_compare`): per-sample radiance
bit-exact on a random sample list (>= 99.9 %), the exact-splat frame against the oracle's
single-thread frame (the reference's splat order, RT/raytracer.cpp:187-259) bit for bit on
>= 99.9 % of pixels and rel L2 <= 1e-6, the streaming splat within rel L2 <= 1e-5, equal ray counts.
"""
import numpy as np
import pytest

import oracle_binding as ob
from test_gpu_scenes import _compare


KINDS = ["sky", "planes", "sphere_light", "one_triangle", "flat_triangle"]


def _camera(rt, w, h, p=(0.0, 1.0, -5.0), at=(0.0, 1.0, 0.0)):
    cam = rt.abi.Camera()
    cam.vfov = rt.DEG_TO_RAD * 50.0
    cam.aspect_ratio = w / h
    cam.lens_radius = 0.0
    cam.focus_distance = 10.0
    cam.p = rt.v3(*p)
    rt.aim_camera_at(cam, at)
    rt.recompute_camera(cam)
    return cam


def degenerate_scene(rt, kind):
    """A scene that exercises one empty or minimal part of the scene model (RT/scene.h): no
    primitive at all (only the reference's null primitive 0), planes without a BVH, analytic
    primitives without a mesh, a mesh of one triangle (a one-leaf mesh BVH), and the same triangle
    lying in z = 0, whose zero-thickness box no ray enters: the reference's slab test needs
    tn < tf strictly (RT/intersection.cpp:128), so the triangle is invisible there and here."""
    s = rt.Scene()
    m = s.add_diffuse_material((0.6, 0.5, 0.4), 1.5)
    light = s.add_emissive_material((8.0, 7.0, 6.0))
    if kind in ("planes", "sphere_light"):
        s.add_plane(m, (0.0, 1.0, 0.0), -1.0)
    if kind == "sphere_light":
        s.add_sphere(m, 1.0, rt.translate((0.0, 1.0, 0.0)))
    if kind in ("sphere_light", "one_triangle", "flat_triangle"):
        s.add_sphere(light, 0.5, rt.translate((0.0, 3.0, -3.0)))   # above the camera's view
    if kind in ("one_triangle", "flat_triangle"):
        dz = 0.5 if kind == "one_triangle" else 0.0
        tris = np.array([[[-1.0, 0.0, dz], [0.0, 2.0, 0.0], [1.0, 0.0, -dz]]], np.float32)   # normal towards -z
        s.add_mesh(m, s.create_mesh(tris), rt.identity())
    s.set_sky((0.6, 0.7, 0.9), (0.1, 0.1, 0.1))
    s.create_scene_bvh()
    return s


def test_degenerate_scenes_render_on_the_oracle(rt):
    """CPU: the oracle renders every degenerate scene deterministically, and the scenes differ
    where they should: a frame with no diffuse surface in view sends no shadow ray (sky only, the
    flat triangle), the tilted triangle is seen."""
    w, h = 16, 12
    cam = _camera(rt, w, h)
    st, _ = rt.default_settings()
    st.samples_per_pixel = 2
    fc = rt.load_reconstruction_kernel("Mitchell Netravali")
    frames = {}
    for kind in KINDS:
        scene = degenerate_scene(rt, kind)          # desc() points into the live host scene
        d = scene.desc()
        a, sa = ob.render(d, cam, st, fc, w, h, rng_mode=0, threads=2)
        b, sb = ob.render(d, cam, st, fc, w, h, rng_mode=0, threads=2)
        assert np.array_equal(a, b) and sa.closest_hit_rays == sb.closest_hit_rays
        frames[kind] = (a, sa)
    assert frames["sky"][1].shadow_rays == 0 and frames["flat_triangle"][1].shadow_rays == 0
    assert frames["one_triangle"][1].shadow_rays > 0 and frames["sphere_light"][1].shadow_rays > 0
    assert not np.array_equal(frames["flat_triangle"][0], frames["one_triangle"][0])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_degenerate_scene_gpu_matches_oracle(rt, kind):
    w, h = 48, 36
    cam = _camera(rt, w, h)
    st, _ = rt.default_settings()
    st.samples_per_pixel = 8
    fc = rt.load_reconstruction_kernel("Mitchell Netravali")
    _compare(rt, f"degenerate_{kind}", degenerate_scene(rt, kind), cam, st, fc, w, h)


def plane_room(rt, n):
    """A room of n planes (floor, ceiling, walls, then planes tilted outside it, each also tested by
    every ray) with a sphere light and a glass sphere: the ray prologue loads the planes four per
    scalar load (DevScene::plane_nd), so n = 4 fills one batch exactly and n = 9 ends in a partial one;
    a shadow ray stops at the first plane that occludes it (RT/intersection.cpp:424-433)."""
    s = rt.Scene()
    m = [s.add_diffuse_material(c, 1.5) for c in ((0.6, 0.5, 0.4), (0.8, 0.2, 0.2), (0.2, 0.7, 0.3))]
    glass = s.add_translucent_material((0.1, 0.1, 0.1), 1.5, 0.0)
    light = s.add_emissive_material((9.0, 8.0, 7.0))
    planes = [((0.0, 1.0, 0.0), -1.0), ((0.0, -1.0, 0.0), -6.0), ((1.0, 0.0, 0.0), -4.0), ((-1.0, 0.0, 0.0), -4.0),
              ((0.0, 0.0, -1.0), -6.0), ((0.6, 0.8, 0.0), -9.0), ((-0.6, 0.0, 0.8), -9.0), ((0.0, -0.6, -0.8), -9.0),
              ((0.48, 0.6, 0.64), -12.0)]
    for i, (nrm, d) in enumerate(planes[:n]):
        s.add_plane(m[i % 3], nrm, d)
    s.add_sphere(light, 0.5, rt.translate((0.0, 4.5, 1.0)))
    s.add_sphere(glass, 0.8, rt.translate((1.0, 0.0, 2.0)))
    s.set_sky((0.6, 0.7, 0.9), (0.1, 0.1, 0.1))
    s.create_scene_bvh()
    return s


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 9])
def test_plane_batches_gpu_match_oracle(rt, n):
    w, h = 48, 36
    cam = _camera(rt, w, h, p=(0.0, 1.5, -3.0), at=(0.0, 1.0, 2.0))
    st, _ = rt.default_settings()
    st.samples_per_pixel = 8
    fc = rt.load_reconstruction_kernel("Mitchell Netravali")
    _compare(rt, f"plane_room_{n}", plane_room(rt, n), cam, st, fc, w, h)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(1, 1), (5, 3), (65, 33), (130, 7)])
def test_ragged_frames_gpu_match_oracle(rt, w, h):
    """Frames smaller than one 64x64 tile, one pixel past a tile in each direction, and a
    strip: the tile grid, the pixel map and the resolve's edges (RT/raytracer.cpp:366-372)."""
    scene, cam, st, fc, post = rt.load_preset("c1", w, h)
    st.samples_per_pixel = 4
    _compare(rt, f"ragged_{w}x{h}", scene, cam, st, fc, w, h)


@pytest.mark.gpu
@pytest.mark.parametrize("spp,bounces", [(1, 4), (4, 63)])
def test_settings_limits_gpu_match_oracle(rt, spp, bounces):
    """One sample per pixel, and the deepest path the material stack allows (max_bounce_count
    63): in the closed Cornell box without Russian roulette a sample traces ~54 closest-hit rays,
    most paths run all 63 bounces."""
    w, h = 64, 48
    scene, cam, st, fc, post = rt.load_preset("cornell_box", w, h)
    st.samples_per_pixel = spp
    st.max_bounce_count = bounces
    st.russian_roulette = 0
    _compare(rt, f"limits_spp{spp}_depth{bounces}", scene, cam, st, fc, w, h)


@pytest.mark.gpu
def test_max_bounce_count_over_limit_rejected(rt):
    """max_bounce_count 64 is past the 64-entry material stack's levels: RT_ERROR_INVALID, no
    frame (DESIGN.md §2 Errors)."""
    w, h = 16, 16
    scene, cam, st, fc, post = rt.load_preset("c1", w, h)
    st.max_bounce_count = 64
    dev = rt.DeviceScene(scene, 0)
    try:
        with pytest.raises(rt.RenderError) as e:
            dev.render(cam, st, fc, w, h)
        assert e.value.code == rt.abi.RT_ERROR_INVALID
        st.max_bounce_count = 63
        frame, stats = dev.render(cam, st, fc, w, h)
        assert stats.samples == w * h * st.samples_per_pixel
    finally:
        dev.close()


def test_desc_keeps_its_scene_alive(rt):
    """CPU: rt_scene_desc's arrays point into the host scene; the struct the Python host returns
    holds the Scene, so a desc taken from a temporary stays valid (it once read freed memory)."""
    import gc
    d = degenerate_scene(rt, "planes").desc()
    gc.collect()
    assert d.plane_count == 1 and d.planes[0].transform_index < d.transform_count
    cam = _camera(rt, 8, 6)
    st, _ = rt.default_settings()
    st.samples_per_pixel = 1
    fc = rt.load_reconstruction_kernel("Box")
    frame, stats = ob.render(d, cam, st, fc, 8, 6, rng_mode=0, threads=1)
    assert stats.samples == 48 and np.isfinite(frame).all()


class _DescOverride:
    """A scene whose rt_scene_desc differs from its host scene's: mesh `m` without its BVH
    (node_count 0), which rt_scene_upload accepts and the reference renders as a mesh whose
    triangles are never tested (intersect_mesh counts the call, RT/intersection.cpp:254, then
    skips everything under `if (bvh)`, :259)."""

    def __init__(self, rt, scene, m):
        self.scene = scene
        d = scene.desc()
        n = d.mesh_count
        self._meshes = (rt.abi.Mesh * n)(*[d.meshes[i] for i in range(n)])
        self._meshes[m].node_count = 0
        self._meshes[m].nodes = None
        self._desc = rt.abi.SceneDesc.from_buffer_copy(d)
        self._desc.meshes = self._meshes

    def desc(self):
        return self._desc


@pytest.mark.gpu
def test_mesh_without_bvh(rt):
    """a mesh uploaded without a BVH.  Frames and samples against the oracle as every
    scene here (the mesh is invisible on both sides), the reference's TraversalStats units
    (rt_scene_config::traversal_ref) against its own walk: the call is counted, no root pop."""
    from parity_report import REPORT
    from test_gpu_fullscale import check_traversal_ref
    w, h = 96, 54
    scene, cam, st, fc, post = rt.load_preset("c4", w, h)
    st.samples_per_pixel = 8
    sc = _DescOverride(rt, scene, 0)
    _compare(rt, "mesh_without_bvh", sc, cam, st, fc, w, h)
    dev = rt.DeviceScene(sc, 0)
    try:
        with dev.configured(traversal_ref=1):
            _, gs = dev.render(cam, st, fc, w, h)
    finally:
        dev.close()
    _, cs = ob.render(sc.desc(), cam, st, fc, w, h, rng_mode=0, threads=8)
    REPORT["mesh_without_bvh_traversal_ref"] = check_traversal_ref(gs, cs)
    for k in range(2):
        assert gs.traversal_ref[k].mesh_intersection_count == cs.traversal[k].mesh_intersection_count
