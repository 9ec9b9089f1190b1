"""Host scene model (include/rt_host.h): BVH builders, presets, asset formats,
output — the inputs and outputs on either side of the hot path."""
import ctypes as C
import math
import os
import re
import struct

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _nodes(desc_nodes, n):
    return [desc_nodes[i] for i in range(n)]


def _check_bvh(nodes, prim_boxes, count_total):
    """every primitive in exactly one leaf; every child box inside its parent (+ulp slack)."""
    seen = []
    stack = [0]
    while stack:
        i = stack.pop()
        nd = nodes[i]
        lo = np.array([nd.bv_p.x - nd.bv_r.x, nd.bv_p.y - nd.bv_r.y, nd.bv_p.z - nd.bv_r.z])
        hi = np.array([nd.bv_p.x + nd.bv_r.x, nd.bv_p.y + nd.bv_r.y, nd.bv_p.z + nd.bv_r.z])
        slack = 1e-5 * (1 + np.abs(lo) + np.abs(hi))
        if nd.count:
            for k in range(nd.left_first, nd.left_first + nd.count):
                seen.append(k)
                plo, phi = prim_boxes(k)
                assert np.all(plo >= lo - slack) and np.all(phi <= hi + slack)
        else:
            assert i != 1, "node 1 is the cache-line padding node"
            stack += [nd.left_first, nd.left_first + 1]
    assert sorted(seen) == list(range(count_total))


@pytest.mark.parametrize("method", [0, 1, 2])
def test_mesh_bvh_invariants(rt, method):
    n = rt.lib().rth_generate_mesh(800 if method == 2 else 5000, 7, None, None)
    tris = np.zeros((n, 3, 3), np.float32)
    nrm = np.zeros((n, 3, 3), np.float32)
    rt.lib().rth_generate_mesh(800 if method == 2 else 5000, 7, tris.ctypes.data_as(C.POINTER(rt.V3)),
                               nrm.ctypes.data_as(C.POINTER(rt.V3)))
    s = rt.Scene()
    mid = s.create_mesh(tris, nrm, method=method)
    s.create_scene_bvh()
    m = s.desc().meshes[mid]
    assert m.triangle_count == n and m.has_normals
    idx = np.array([m.indices[i] for i in range(n)])
    assert sorted(idx.tolist()) == list(range(n))
    bt = np.array([[m.triangles[3 * i + k].x, m.triangles[3 * i + k].y, m.triangles[3 * i + k].z]
                   for i in range(n) for k in range(3)], np.float32).reshape(n, 3, 3)
    assert np.array_equal(bt, tris[idx])           # MeshBVH::triangles = triangles[indices[i]]
    nodes = _nodes(m.nodes, m.node_count)
    _check_bvh(nodes, lambda k: (bt[k].min(0), bt[k].max(0)), n)
    info = s.bvh_info(mid)
    # a leaf holds <= 4 entries unless no split improves the SAH (RT/bvh.cpp:236, :254-255)
    assert info["max_leaf_size"] <= 16
    assert info["max_depth"] < 62


def test_scene_bvh_and_lights(rt):
    scene, cam, st, fc, post = rt.load_preset("week_6", 64, 64)
    d = scene.desc()
    assert d.plane_count == 6
    assert d.primitive_count == 5              # null + box + 2 spheres + light
    assert d.light_count == 1 and d.lights[0] == 4
    assert d.materials[0].flags == 0           # null material
    idx = sorted(d.bvh_indices[i] for i in range(d.bvh_index_count))
    assert idx == [1, 2, 3, 4]                 # create_scene_bvh over primitives 1..n
    # camera: aim_camera(v3(0,0,-1)) -> z = (0,0,-1), film distance 1/tan(vfov)
    assert (cam.z.x, cam.z.y, cam.z.z) == (0.0, 0.0, -1.0)
    assert abs(cam.film_distance - 1.0 / math.tan(math.radians(45.0))) < 1e-5
    assert (cam.focus_distance, cam.lens_radius) == (pytest.approx(19.77), 10.0)


@pytest.mark.parametrize("name", ["week_1", "week_2", "week_3", "week_4", "week_5", "week_6", "week_7",
                                  "week_7_nicer", "cornell_box", "dragon", "platforms", "nested_dielectrics",
                                  "c1", "c2", "c3", "c4"])
def test_presets_load(rt, name):
    scene, cam, st, fc, post = rt.load_preset(name, 160, 90)
    d = scene.desc()
    assert d.bvh_node_count >= 1
    assert st.integrator == 0 and st.max_bounce_count <= 63
    if name in ("c2", "c3", "cornell_box"):
        assert d.mesh_count == 1 and d.meshes[0].triangle_count >= 69000
    if name == "c4":
        tris = sum(d.meshes[d.primitives[i].mesh_index].triangle_count for i in range(d.primitive_count)
                   if d.primitives[i].type == 4)
        assert tris >= 250000                  # ~250k-tri multi-mesh scene
        assert d.mesh_count == 4               # four distinct meshes, not one instanced
    if name in ("c3", "c4", "dragon", "platforms"):
        assert d.skydome_w == 2048 and d.skydome_h == 1024


def test_obj_round_trip(rt, tmp_path):
    path = str(tmp_path / "m.obj")
    assert rt.lib().rth_write_synthetic_obj(path.encode(), 3000, 4)
    s = rt.Scene()
    mid = s.load_obj_mesh(path)
    m = s.desc().meshes[mid]
    n = rt.lib().rth_generate_mesh(3000, 4, None, None)
    tris = np.zeros((n, 3, 3), np.float32)
    rt.lib().rth_generate_mesh(3000, 4, tris.ctypes.data_as(C.POINTER(rt.V3)), None)
    got = np.array([[m.triangles[3 * i + k].x, m.triangles[3 * i + k].y, m.triangles[3 * i + k].z]
                    for i in range(n) for k in range(3)], np.float32).reshape(n, 3, 3)
    idx = np.array([m.indices[i] for i in range(n)])
    assert np.array_equal(got, tris[idx])      # %.9g text round-trips float32 exactly
    assert m.has_normals


def test_obj_fan_triangulation_and_negative_indices(rt, tmp_path):
    path = tmp_path / "quad.obj"
    path.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nf 1 2 3 4\nf -4 -3 -2\n")
    s = rt.Scene()
    mid = s.load_obj_mesh(str(path))
    assert s.desc().meshes[mid].triangle_count == 3      # quad -> 2-triangle fan, + 1 triangle


def test_hdr_round_trip(rt, tmp_path):
    path = str(tmp_path / "sky.hdr")
    assert rt.lib().rth_write_synthetic_hdr(path.encode(), 256, 128, 9)
    s = rt.Scene()
    s.load_environment_map(path)
    d = s.desc()
    assert (d.skydome_w, d.skydome_h) == (256, 128)
    px = np.ctypeslib.as_array(C.cast(d.skydome, C.POINTER(C.c_float)), shape=(128, 256, 3))
    assert np.all(px >= 0) and px.max() > 1000          # the sun disk
    assert px[100:, :, 2].mean() > px[:20, :, 2].mean()  # row h-1 is "up": blue sky vs ground


def test_bitmap_and_resolve(rt, tmp_path):
    acc = np.zeros((2, 3, 4), np.float32)
    acc[0, 0] = (1, 1, 1, 1)
    acc[0, 1] = (np.nan, 0, 0, 1)
    acc[0, 2] = (0, 0, 0, -1)
    _, post = rt.default_settings()
    px = rt.resolve_bgra8(acc, post)
    assert px[0, 1] == 0xFF00FFFF                        # NaN -> (0,255,255)
    assert px[0, 2] == 0xFFFF00FF                        # negative weight -> magenta
    assert px[1, 0] == 0xFF000000                        # untouched -> black
    path = str(tmp_path / "out.bmp")
    rt.write_bitmap(path, px)
    raw = open(path, "rb").read()
    assert raw[:2] == b"BM" and struct.unpack("<i", raw[22:26])[0] == -2   # top-down
    assert len(raw) == 54 + 4 * 6


def test_filters(rt):
    for name, r in [("Box", 0), ("Gaussian 3", 3), ("Gaussian 12", 12), ("Mitchell Netravali", 2),
                    ("Lanczos 3", 3), ("Lanczos 4", 4), ("Lanczos 6", 6), ("Lanczos 12", 12), ("nope", 0)]:
        fc = rt.load_reconstruction_kernel(name)
        assert fc.kernel_size == r and fc.cache_size == (256 if r else 0)


def test_transforms(rt):
    t = rt.translate((1, 2, 3)) * rt.rotate_y(0.3) * rt.scale(2.0)
    f = np.array(t.forward.e)
    i = np.array(t.inverse.e)
    assert np.allclose(f @ i, np.eye(4), atol=1e-6)
