"""Parity at the bench's own scale.

The default production path -- rt_render at the BASELINE configs' full sizes, with everything the
bench's frames run: four partitions, 8.4M-path pools, the streaming splat's record ring and resolve
chunks, the fused drain -- against the oracle's frame of the same samples (RT_RNG_PER_SAMPLE, the
reference-order splat, RT/raytracer.cpp:366-495, :692-757):

* C2 (1920x1080, 64 spp, r05), C3 (1920x1080, 256 spp) and C4 (1920x1080, 256 spp, ~250k
  triangles): the whole frame, rel L2
  <= 1e-5 (the streaming splat sums a pixel pass by pass, the reference tile by tile) and the same
  closest-hit and shadow ray counts, call for call;
* the frame's TraversalStats (rt_stats::traversal, RT/intersection.h:33-40): the GPU counts its own
  walk (include/rt_abi.h), so its mesh_intersection_count must equal, query kind by query kind, the
  oracle's restatement of that walk (oracle_gpu_walk_stats), and its leaves entered must agree with
  the restatement's (which leaves out the GPU's pruning for rays with an exactly-zero direction
  component); the reference's own counts from the same render (BVH2 pops, front-to-back order) are
  reported beside them;
* C5 (3840x2160, 1024 spp, blue noise): the GPU renders the tiles t % 85 == 42 of the frame
  (RT_SHARD_TILES, shard 42 of 85: 24 tiles spread over the frame) and the oracle the same tiles:
  every pixel, filter halos included, rel L2 <= 1e-5, and identical ray counts.

The oracle runs on the box's cores (bench.host_cores, 16 on a one-GPU box): ~30 s for C3.
"""
import ctypes as C
import importlib.util
import os

import numpy as np
import pytest

import oracle_binding as ob
from parity_report import REPORT

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _threads():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.host_cores()["cores"]


def rel_l2(a, b):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("preset,spp", [("c2", 64), ("c3", 256), ("c4", 256)])
def test_full_frame_default_path(rt, preset, spp):
    w, h = 1920, 1080
    scene, cam, st, fc, post = rt.load_preset(preset, w, h)
    assert st.samples_per_pixel == spp
    dev = rt.DeviceScene(scene, 0)
    try:
        gpu, gs = dev.render(cam, st, fc, w, h)
        # the auto shadow launch (rt_scene_config::shadow_launch): a scene's first whole frame traces its
        # shadow rays in a launch of their own; later frames merge them into the trace launch when the
        # last frame traced >= 0.15 shadow rays per extension ray (C2 / C3: ~0.26; C4: ~0.11) -- the
        # bench's timed frames.  Both schedules trace the same rays; the frame is held to the same bar.
        gpu2, gs2 = dev.render(cam, st, fc, w, h)
        rs = None
        if preset == "c3":         # the reference's own TraversalStats units (rt_scene_config::traversal_ref)
            with dev.configured(traversal_ref=1):
                rgpu, rs = dev.render(cam, st, fc, w, h)
    finally:
        dev.close()
    assert gs.splat_mode == rt.abi.RT_SPLAT_STREAM
    share = gs.traced_rays[1] / gs.traced_rays[0]
    assert gs.shadow_launch == rt.abi.RT_SHADOW_LAUNCH_SEPARATE
    assert gs2.shadow_launch == (rt.abi.RT_SHADOW_LAUNCH_MERGED if share >= 0.15 else rt.abi.RT_SHADOW_LAUNCH_SEPARATE)
    assert gs2.shadow_launch == (rt.abi.RT_SHADOW_LAUNCH_SEPARATE if preset == "c4" else rt.abi.RT_SHADOW_LAUNCH_MERGED)
    assert (gs.closest_hit_rays, gs.shadow_rays, tuple(gs.traced_rays)) == \
        (gs2.closest_hit_rays, gs2.shadow_rays, tuple(gs2.traced_rays))
    threads = _threads()
    with ob.gpu_walk() as walk:
        cpu, cs = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=threads)
    err = rel_l2(gpu, cpu)
    trav = traversal_report(gs, cs, walk.result)
    REPORT[f"fullscale_{preset}_1080p_{spp}spp"] = {
        "rel_l2": err, "max_abs_weight_diff": float(np.abs(gpu[..., 3] - cpu[..., 3]).max()),
        "gpu_rays": [int(gs.closest_hit_rays), int(gs.shadow_rays)], "oracle_rays": [int(cs.closest_hit_rays), int(cs.shadow_rays)],
        "samples": int(gs.samples), "iterations": int(gs.iterations), "oracle_threads": threads,
        "shadow_rays_per_extension_ray": share, "second_frame_shadow_launch": int(gs2.shadow_launch),
        "second_frame_bitwise_equal": bool(np.array_equal(gpu, gpu2)), "second_frame_rel_l2": rel_l2(gpu2, cpu),
        "gpu_seconds": gs.seconds, "traversal": trav}
    assert gs.samples == cs.samples == w * h * spp
    assert (gs.closest_hit_rays, gs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays)
    assert np.isfinite(gpu).all() and np.isfinite(cpu).all()
    assert err <= 1e-5 and rel_l2(gpu2, cpu) <= 1e-5
    check_traversal(gs, walk.result)
    if rs is not None:
        ref_report = check_traversal_ref(rs, cs)
        REPORT[f"fullscale_{preset}_1080p_{spp}spp"]["traversal_ref_units"] = ref_report
        assert (rs.closest_hit_rays, rs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays)
        assert rel_l2(rgpu, cpu) <= 1e-5


def check_traversal_ref(rs, cs, tol=1e-3):
    """rt_stats::traversal_ref (the GPU walk counting the reference's units, RT/intersection.cpp:254,
    :274-380) against the reference's own counts of the same frame (the oracle's reference walk):
    within `tol` per field and query kind.  Returns the report."""
    out = {}
    for k, kind in enumerate(("closest", "shadow")):
        g, r = rs.traversal_ref[k].as_dict(), cs.traversal[k].as_dict()
        out[kind] = {"gpu_ref_units": g, "reference_walk": r,
                     "rel_diff": {f: (g[f] - r[f]) / max(r[f], 1) for f in g}}
    for kind in ("closest", "shadow"):
        for f, d in out[kind]["rel_diff"].items():
            assert abs(d) <= tol, (kind, f, out[kind])
    return out


def traversal_report(gs, cs, walk):
    """The frame's TraversalStats: the GPU's (its walk, BVH4 units), the oracle's restatement of that
    walk, and the reference's own counts (BVH2 pops in its front-to-back walk)."""
    out = {}
    for k, kind in enumerate(("closest", "shadow")):
        g = gs.traversal[k].as_dict()
        g["trace_steps"] = int(gs.trace_steps[k])
        out[kind] = {"gpu": g,
                     "gpu_walk_restated": {"mesh_intersection_count": walk["calls"][k],
                                           "instances_entered": walk["entries"][k],
                                           "mesh_bvh_traversals": walk["bvh"][k],
                                           "mesh_node_traversals": walk["nodes"][k],
                                           "mesh_leaf_traversals": walk["leaves"][k]},
                     "reference_walk": cs.traversal[k].as_dict()}
    return out


def check_traversal(gs, walk):
    for k in range(2):
        t = gs.traversal[k]
        # the instances the walk reaches: exact, query kind by query kind
        assert t.mesh_intersection_count == walk["calls"][k], (k, t.mesh_intersection_count, walk["calls"][k])
        # leaves entered, BVH4 nodes expanded, BVH4 steps: the restatement walks each mesh BVH2 front to
        # back with the GPU's degenerate-axis pruning, counting the even-depth interior nodes (the BVH4's)
        # and the triangle steps (two triangles each).  The BVH4 skips a level's box test, and where float
        # rounding lets a child pass a test its parent fails (or a tie at tn == t) the GPU takes a few more
        # (measured: leaves +1 to +188 per frame, at most 3.0e-7, on C3, C4 and the C5 shard)
        for f, key in (("mesh_leaf_traversals", "leaves"), ("mesh_node_traversals", "nodes"),
                       ("mesh_bvh_traversals", "bvh")):
            g, r = getattr(t, f), walk[key][k]
            assert abs(g - r) <= 1e-6 * r, (k, f, g, r)
        # the extend / connect launches' steps: the fused drain's are in the counts but not in
        # trace_steps (r05; every BASELINE scene is walked from the prologue's mesh lists: no top steps)
        assert 0 < gs.trace_steps[k] <= t.mesh_bvh_traversals


def test_c5_tile_shard_exact(rt):
    """C5 at 4K, 1024 spp: shard 42 of 85 by tiles (the tiles t % 85 == 42: 24 tiles evenly spread
    over the 60 x 34 tile frame) on the GPU against the same tiles in the oracle."""
    w, h = 3840, 2160
    scene, cam, st, fc, post = rt.load_preset("c5", w, h)
    assert st.samples_per_pixel == 1024
    tcx, tcy = (w + 63) // 64, (h + 63) // 64
    count, index = 85, 42
    tiles = [t for t in range(tcx * tcy - 1, -1, -1) if t % count == index]    # the reference's queue order
    assert len(tiles) == 24
    dev = rt.DeviceScene(scene, 0)
    try:
        with dev.configured(shard_mode=rt.abi.RT_SHARD_TILES):
            gpu, gs = dev.render(cam, st, fc, w, h, shard_index=index, shard_count=count)
    finally:
        dev.close()
    lib = ob.load()
    cpu = np.zeros((h, w, 4), np.float32)
    buf = rt.abi.AccumulationBuffer(w, h, 0, cpu.ctypes.data_as(C.POINTER(C.c_float)))
    arr = (C.c_uint32 * len(tiles))(*tiles)
    cs = rt.abi.Stats()
    with ob.gpu_walk() as walk:
        assert lib.oracle_render_tiles(C.byref(scene.desc()), C.byref(cam), C.byref(st), C.byref(fc), 64, 64, 0, 0,
                                       _threads(), len(tiles), arr, C.byref(buf), C.byref(cs)) == 0
    err = rel_l2(gpu, cpu)
    touched = int((cpu[..., 3] != 0).sum())
    REPORT["fullscale_c5_4k_1024spp_shard42of85"] = {
        "rel_l2_every_pixel": err, "tiles": tiles, "pixels_with_weight": touched,
        "gpu_rays": [int(gs.closest_hit_rays), int(gs.shadow_rays)], "oracle_rays": [int(cs.closest_hit_rays), int(cs.shadow_rays)],
        "samples": int(gs.samples), "gpu_seconds": gs.seconds, "iterations": int(gs.iterations),
        "traversal": traversal_report(gs, cs, walk.result)}
    area = sum((min(64, w - (t % tcx)*64)) * (min(64, h - (t // tcx)*64)) for t in tiles)   # bottom-row tiles: 48 rows
    assert gs.samples == cs.samples == area * 1024
    assert (gs.closest_hit_rays, gs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays)
    assert np.isfinite(gpu).all() and np.isfinite(cpu).all()
    assert touched > 24 * 64 * 64
    assert err <= 1e-5
    check_traversal(gs, walk.result)
