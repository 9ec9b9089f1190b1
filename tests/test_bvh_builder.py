"""The device BVH builder (rt_build_bvh) against the host builder, which
restates the reference's (RT/bvh.cpp:26-326, rt_host.cpp; its layout checks are in
tests/test_layouts.py and tests/test_host_model.py).

CPU: the parallel form of partition_objects the device uses (stop lists A and B, swaps
(A[k], B[k]) for k < K, split index min(A[K], B[K-1], n - 1); rt_bvh_build.hip) is checked
against the sequential two-pointer loop of RT/bvh.cpp:26-51 on many arrays with ties.
GPU: node arrays and entry orders bit-identical to the host's, for meshes, random entry soups
(duplicates, signed zeros, flat axes, every size from 5 to 40), the top level of C4, and both
methods; a scene built with the device builder renders the same frame.
"""
import ctypes as C

import numpy as np
import pytest


def sequential_partition(v, split):
    """partition_objects (RT/bvh.cpp:26-51) on a list of keys: returns (permutation, split index)."""
    e = list(range(len(v)))
    n = len(v)
    i, j = -1, n
    while True:
        i += 1
        while i < n - 1 and v[e[i]] < split:
            i += 1
        j -= 1
        while j > 0 and v[e[j]] > split:
            j -= 1
        if i >= j:
            break
        e[i], e[j] = e[j], e[i]
    return e, i


def parallel_partition(v, split):
    """The device's form (rt_bvh_build.hip, k_bvh_level)."""
    n = len(v)
    A = [i for i in range(n) if not (v[i] < split)]
    B = [i for i in range(n - 1, -1, -1) if not (v[i] > split)]
    K = 0
    while K < min(len(A), len(B)) and A[K] < B[K]:
        K += 1
    e = list(range(n))
    for k in range(K):
        e[A[k]], e[B[k]] = e[B[k]], e[A[k]]
    si = n - 1
    if K < len(A):
        si = min(si, A[K])
    if K > 0:
        si = min(si, B[K - 1])
    return e, si


def test_parallel_partition_matches_sequential():
    rng = np.random.default_rng(1)
    cases = 0
    for n in range(1, 40):
        for _ in range(60):
            v = list(rng.integers(0, 5, n).astype(float))       # many ties with the split value
            for split in (-1.0, 0.0, 1.5, 2.0, 4.0, 9.0):
                assert parallel_partition(v, split) == sequential_partition(v, split), (v, split)
                cases += 1
    assert cases > 10000


def _entries(rng, n, kind):
    if kind == "soup":
        c = rng.normal(size=(n, 3)).astype(np.float32)
        r = np.abs(rng.normal(size=(n, 3)) * 0.1).astype(np.float32)
    elif kind == "dupes":
        c = rng.integers(-2, 3, size=(n, 3)).astype(np.float32)
        r = np.full((n, 3), 0.5, np.float32)
    elif kind == "zeros":
        c = rng.choice(np.array([-0.0, 0.0, 1.0, -1.0], np.float32), size=(n, 3))
        r = rng.choice(np.array([0.0, -0.0, 0.25], np.float32), size=(n, 3))
    else:                                                       # flat: every centre on one plane
        c = rng.normal(size=(n, 3)).astype(np.float32)
        c[:, 1] = 0.0
        r = np.abs(rng.normal(size=(n, 3)) * 0.1).astype(np.float32)
        r[:, 1] = 0.0
    return np.ascontiguousarray(c), np.ascontiguousarray(r)


def _build(rt, c, r, method, device):
    from buas_pathtracer_amd.abi import BvhNode, V3
    n = c.shape[0]
    nodes = (BvhNode * (2 * n + 2))()
    order = np.zeros(n, np.uint32)
    cnt = C.c_uint32()
    P = C.POINTER(V3)
    if device is None:
        rt.lib().rth_set_bvh_device(-1)
        err = rt.lib().rth_build_bvh_entries(n, c.ctypes.data_as(P), r.ctypes.data_as(P), method, nodes, C.byref(cnt),
                                             order.ctypes.data_as(C.POINTER(C.c_uint32)))
    else:
        err = rt.lib().rt_build_bvh(device, n, c.ctypes.data_as(P), r.ctypes.data_as(P), method, nodes, C.byref(cnt),
                                    order.ctypes.data_as(C.POINTER(C.c_uint32)))
    assert err == 0, rt.lib().rt_build_bvh_last_error()
    raw = np.frombuffer(bytes(nodes), np.uint8).reshape(2 * n + 2, 32)[:cnt.value]
    return raw, order


def _mesh_entries(rt, tris):
    t = tris.reshape(-1, 3, 3)
    mn, mx = t.min(axis=1), t.max(axis=1)
    return (np.float32(0.5) * (mn + mx)).astype(np.float32), (np.float32(0.5) * (mx - mn)).astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("method", [0, 1])
@pytest.mark.parametrize("kind", ["soup", "dupes", "zeros", "flat"])
def test_device_builder_bit_identical_small(rt, method, kind):
    rng = np.random.default_rng(7)
    for n in list(range(1, 41)) + [97, 256, 1000, 5000]:
        c, r = _entries(rng, n, kind)
        hn, ho = _build(rt, c, r, method, None)
        dn, do = _build(rt, c, r, method, 0)
        assert np.array_equal(ho, do), (n, kind)
        assert np.array_equal(hn, dn), (n, kind)


@pytest.mark.gpu
@pytest.mark.parametrize("method", [0, 1])
def test_device_builder_bit_identical_meshes(rt, method):
    """The synthetic 70k-triangle mesh of C2/C3, the 62.5k one of C4/C5 and a 400k one."""
    import time
    from parity_report import REPORT
    for tris_n, seed in [(70000, 1), (62500, 3), (400000, 5)]:
        n = rt.lib().rth_generate_mesh(tris_n, seed, None, None)
        tris = np.zeros((n, 3, 3), np.float32)
        rt.lib().rth_generate_mesh(tris_n, seed, tris.ctypes.data_as(C.POINTER(rt.abi.V3)), None)
        c, r = _mesh_entries(rt, tris)
        t0 = time.perf_counter()
        hn, ho = _build(rt, c, r, method, None)
        t1 = time.perf_counter()
        dn, do = _build(rt, c, r, method, 0)
        t2 = time.perf_counter()
        REPORT[f"bvh_build_{tris_n}_m{method}"] = {"nodes": int(len(hn)), "identical": bool(np.array_equal(hn, dn)),
                                                   "host_ms": (t1 - t0) * 1e3, "device_ms": (t2 - t1) * 1e3}
        assert np.array_equal(ho, do)
        assert np.array_equal(hn, dn)


@pytest.mark.gpu
def test_scene_built_on_device_renders_the_same(rt):
    """C4 (4 mesh instances + top level) with every BVH built on the device: same BVHs, same frame."""
    rt.lib().rth_set_bvh_device(-1)
    host = rt.load_preset("c4", 128, 72)
    rt.lib().rth_set_bvh_device(0)
    try:
        dev_built = rt.load_preset("c4", 128, 72)
    finally:
        rt.lib().rth_set_bvh_device(-1)
    hd, dd = host[0].desc(), dev_built[0].desc()
    assert hd.bvh_node_count == dd.bvh_node_count
    assert bytes((rt.abi.BvhNode * hd.bvh_node_count).from_address(C.addressof(hd.bvh_nodes.contents))) == \
        bytes((rt.abi.BvhNode * dd.bvh_node_count).from_address(C.addressof(dd.bvh_nodes.contents)))
    for m in range(hd.mesh_count):
        a, b = hd.meshes[m], dd.meshes[m]
        assert a.node_count == b.node_count
        assert bytes((rt.abi.BvhNode * a.node_count).from_address(C.addressof(a.nodes.contents))) == \
            bytes((rt.abi.BvhNode * b.node_count).from_address(C.addressof(b.nodes.contents)))
    scene, cam, st, fc, post = dev_built
    st.samples_per_pixel = 16
    dev = rt.DeviceScene(scene, 0)
    try:
        got, _ = dev.render(cam, st, fc, 128, 72)
    finally:
        dev.close()
    hs, hcam, hst, hfc, _ = host
    hst.samples_per_pixel = 16
    dev = rt.DeviceScene(hs, 0)
    try:
        ref, _ = dev.render(hcam, hst, hfc, 128, 72)
    finally:
        dev.close()
    assert np.array_equal(got, ref)
