"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Tolerances:
* intersection queries: bit-exact (t, primitive, hit point, normal);
* per-sample radiance (RT_RNG_PER_SAMPLE, spec transcendentals on both
  sides, -ffp-contract=off, IEEE div/sqrt): >= 99.9 % of samples bit-exact,
  the rest within 1e-3 relative (rare branch flips on exact ties only);
* accumulated frames: relative L2 <= 1e-3 (north star); with the gather
  splat (k_resolve) the GPU frame is additionally compared bit for bit with
  the oracle's single-threaded frame, which splats in the reference's order.
"""
import numpy as np
import pytest

import oracle_binding as ob

pytestmark = pytest.mark.gpu

from parity_report import REPORT      # noqa: E402  (written to gpurun_out/parity_report.json at session end)


def rel_l2(a, b):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def c1(rt):
    scene, cam, st, fc, post = rt.load_preset("c1", 256, 256)
    dev = rt.DeviceScene(scene, 0)
    yield rt, scene, cam, st, fc, dev
    dev.close()


@pytest.fixture(scope="module")
def c3small(rt):
    scene, cam, st, fc, post = rt.load_preset("c3", 192, 108)
    dev = rt.DeviceScene(scene, 0)
    yield rt, scene, cam, st, fc, dev
    dev.close()


@pytest.fixture(scope="module")
def c4small(rt):
    """C4 topology (4 mesh instances, boxes, 3 sphere lights, nested dielectric shell)."""
    scene, cam, st, fc, post = rt.load_preset("c4", 192, 108)
    dev = rt.DeviceScene(scene, 0)
    yield rt, scene, cam, st, fc, dev
    dev.close()


@pytest.fixture(scope="module")
def c5small(rt):
    """C5 sampler: OptimizedBlueNoise; 320 spp so indices past 256 take the stratified fallback
    (RT/samplers.cpp:27-28)."""
    scene, cam, st, fc, post = rt.load_preset("c5", 96, 54)
    st.samples_per_pixel = 320
    dev = rt.DeviceScene(scene, 0)
    yield rt, scene, cam, st, fc, dev
    dev.close()


@pytest.fixture(scope="module")
def c1uniform(rt):
    """C1 with SamplingStrategy_Uniform (the third sampler)."""
    scene, cam, st, fc, post = rt.load_preset("c1", 128, 128)
    st.sampling_strategy = rt.abi.RT_SAMPLING_UNIFORM
    dev = rt.DeviceScene(scene, 0)
    yield rt, scene, cam, st, fc, dev
    dev.close()


def random_rays(rng, n, center, spread):
    rays = []
    o = center + spread * (rng.random((n, 3)) - 0.5)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    from buas_pathtracer_amd.abi import RayQuery, V3
    for i in range(n):
        rays.append(RayQuery(V3(*o[i]), V3(*d[i]), 3.0e38, 0))
    return rays


@pytest.mark.parametrize("which", ["c1", "c3small", "c4small"])
@pytest.mark.parametrize("occlusion", [False, True])
def test_intersect_bit_exact(which, occlusion, request):
    rt, scene, cam, st, fc, dev = request.getfixturevalue(which)
    rng = np.random.default_rng(7)
    rays = random_rays(rng, 4096, np.array([0.0, 6.0, -4.0]), np.array([14.0, 10.0, 10.0]))
    g = dev.intersect(rays, occlusion)
    o = ob.intersect(scene.desc(), rays, occlusion)
    mism = 0
    for a, b in zip(g, o):
        if occlusion:
            # intersect_shadow_ray returns a b32 (RT/intersection.cpp:600-604): compare hit / miss only
            mism += (a.primitive == 0xFFFFFFFF) != (b.primitive == 0xFFFFFFFF)
        elif a.primitive != b.primitive or (a.primitive != 0xFFFFFFFF and (
                a.t != b.t or tuple(a.n) != tuple(b.n) or tuple(a.hit_p) != tuple(b.hit_p))):
            mism += 1
    REPORT[f"intersect_{which}_{'occ' if occlusion else 'closest'}"] = {"rays": len(rays), "mismatches": int(mism)}
    assert mism == 0, f"{mism} of {len(rays)} hit records differ"


@pytest.mark.parametrize("occlusion", [False, True])
def test_axis_parallel_rays_bit_exact(occlusion, c3small):
    """Rays with exactly-zero direction components (inv_d = inf, the NaN slab
    case) through and around the mesh: the GPU prunes nodes the reference
    visits uselessly, and must still return the reference's hits."""
    rt, scene, cam, st, fc, dev = c3small
    from buas_pathtracer_amd.abi import RayQuery, V3
    rng = np.random.default_rng(3)
    rays = []
    for i in range(6000):
        o = np.array([5.0, 2.0, -3.0]) + rng.uniform(-6, 6, 3)
        a = rng.uniform(0, 2 * np.pi)
        kind = i % 3
        if kind == 0:
            d = (np.cos(a), 0.0, np.sin(a))          # horizontal (d.y == 0)
        elif kind == 1:
            d = (0.0, np.cos(a), np.sin(a))          # d.x == 0
        else:
            d = (0.0, 1.0 if a < np.pi else -1.0, 0.0)   # two zero components
        d = np.array(d, np.float32)
        rays.append(RayQuery(V3(*o.astype(np.float32)), V3(*d), 3.0e38 if not occlusion else 20.0, 0))
    g = dev.intersect(rays, occlusion)
    o = ob.intersect(scene.desc(), rays, occlusion)
    mism = 0
    for a, b in zip(g, o):
        if occlusion:
            mism += (a.primitive == 0xFFFFFFFF) != (b.primitive == 0xFFFFFFFF)
        elif a.primitive != b.primitive or (a.primitive != 0xFFFFFFFF and (
                a.t != b.t or tuple(a.n) != tuple(b.n) or tuple(a.hit_p) != tuple(b.hit_p))):
            mism += 1
    hits = sum(b.primitive != 0xFFFFFFFF for b in o)
    REPORT[f"axis_parallel_{'occ' if occlusion else 'closest'}"] = {"rays": len(rays), "hits": int(hits),
                                                                     "mismatches": int(mism)}
    assert hits > 1000
    assert mism == 0, f"{mism} of {len(rays)} hit records differ"


def _sample_list(rng, w, h, n, spp):
    xy = np.stack([rng.integers(0, w, n), rng.integers(0, h, n)], axis=1).astype(np.uint32)
    s = rng.integers(0, spp, n).astype(np.uint32)
    return xy, s


@pytest.mark.parametrize("which,w,h", [("c1", 256, 256), ("c3small", 192, 108), ("c4small", 192, 108),
                                       ("c5small", 96, 54), ("c1uniform", 128, 128)])
def test_trace_samples_bitwise(which, w, h, request):
    rt, scene, cam, st, fc, dev = request.getfixturevalue(which)
    rng = np.random.default_rng(11)
    xy, s = _sample_list(rng, w, h, 20000, st.samples_per_pixel)
    gpu, gstats = dev.trace_samples(cam, st, w, h, xy, s)
    cpu, cstats = ob.trace_samples(scene.desc(), cam, st, w, h, xy, s)
    exact = np.all(gpu == cpu, axis=1) | np.all(np.isnan(gpu) == np.isnan(cpu), axis=1) & np.all(
        (gpu == cpu) | np.isnan(cpu), axis=1)
    frac = exact.mean()
    REPORT[f"trace_samples_{which}"] = {"samples": int(len(exact)), "bit_exact_fraction": float(frac),
                                        "gpu_closest": int(gstats.closest_hit_rays),
                                        "cpu_closest": int(cstats.closest_hit_rays)}
    assert frac >= 0.999, f"only {frac:.5f} of samples bit-exact"
    assert gstats.closest_hit_rays == cstats.closest_hit_rays or frac < 1.0
    diff = np.abs(gpu[:, :3] - cpu[:, :3]).sum() / max(np.abs(cpu[:, :3]).sum(), 1e-30)
    assert diff <= 1e-3


@pytest.mark.parametrize("which,w,h", [("c1", 256, 256), ("c3small", 192, 108), ("c4small", 192, 108),
                                       ("c5small", 96, 54), ("c1uniform", 128, 128)])
def test_frame_rel_l2(which, w, h, request):
    rt, scene, cam, st, fc, dev = request.getfixturevalue(which)
    gpu, gstats = dev.render(cam, st, fc, w, h)
    cpu, cstats = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=8)
    REPORT[f"frame_vs_mt_oracle_{which}"] = {"rel_l2": rel_l2(gpu, cpu), "gpu_rays": [int(gstats.closest_hit_rays),
                                             int(gstats.shadow_rays)], "cpu_rays": [int(cstats.closest_hit_rays),
                                             int(cstats.shadow_rays)]}
    assert rel_l2(gpu, cpu) <= 1e-3
    assert gstats.samples == cstats.samples == w * h * st.samples_per_pixel
    # ray counts: identical unless a tie flipped a branch somewhere
    assert abs(int(gstats.closest_hit_rays) - int(cstats.closest_hit_rays)) <= 1e-4 * cstats.closest_hit_rays
    assert abs(int(gstats.shadow_rays) - int(cstats.shadow_rays)) <= 1e-4 * cstats.shadow_rays


@pytest.mark.parametrize("strip", ["4row", "8row"])
@pytest.mark.parametrize("which,w,h", [("c1", 256, 256), ("c3small", 192, 108), ("c4small", 192, 108),
                                       ("c5small", 96, 54), ("c1uniform", 128, 128)])
def test_frame_bitwise_vs_reference_order(which, w, h, strip, request, monkeypatch):
    """The exact splat (RT_SPLAT_EXACT, k_resolve) sums each pixel's contributions in the
    single-threaded reference order, so the GPU frame equals the oracle's threads=1 frame
    bit for bit wherever every contributing sample is bit-exact (>= 99.9 % of pixels).
    Both strip heights of k_resolve run: 4 rows, and the 8 rows whole-frame shards of
    >= 1.6M pixels use (forced here by RT_RES_TALL_PIXELS=1)."""
    rt, scene, cam, st, fc, dev = request.getfixturevalue(which)
    with dev.configured(resolve_tall_pixels=1 if strip == "8row" else 0xFFFFFFFF, splat_mode=rt.abi.RT_SPLAT_EXACT):
        gpu, gs = dev.render(cam, st, fc, w, h)
    assert gs.splat_mode == rt.abi.RT_SPLAT_EXACT
    cpu, _ = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=1)
    same = np.all(gpu == cpu, axis=2).mean()
    REPORT[f"frame_bitwise_{which}_{strip}"] = {"pixels_bit_identical": float(same), "rel_l2": rel_l2(gpu, cpu),
                                                "frame_equal": bool(np.array_equal(gpu, cpu))}
    assert same >= 0.999
    assert rel_l2(gpu, cpu) <= 1e-6


@pytest.mark.parametrize("which,w,h", [("c1", 256, 256), ("c3small", 192, 108), ("c4small", 192, 108),
                                       ("c5small", 96, 54)])
def test_stream_splat_vs_reference_order(which, w, h, request):
    """The streaming splat (the default, k_resolve_tiles) sums pass by pass: the frame
    equals the reference-order frame up to float summation order (rel L2 <= 1e-5), with
    the same sample and ray counts."""
    rt, scene, cam, st, fc, dev = request.getfixturevalue(which)
    gpu, gs = dev.render(cam, st, fc, w, h)
    assert gs.splat_mode == rt.abi.RT_SPLAT_STREAM
    cpu, cs = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=1)
    err = rel_l2(gpu, cpu)
    wdiff = float(np.abs(gpu[..., 3] - cpu[..., 3]).max())
    REPORT[f"frame_stream_{which}"] = {"rel_l2": err, "max_abs_weight_diff": wdiff}
    assert (gs.closest_hit_rays, gs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays)
    assert err <= 1e-5
    assert np.isfinite(gpu).all()
    assert np.isfinite(cpu).all()


@pytest.mark.parametrize("env", [{"splat_chunk": 1, "splat_ring": 1}, {"splat_chunk": 3, "splat_ring": 5},
                                 {"splat_chunk": 1000}])
def test_stream_splat_deterministic_in_chunking(c3small, env):
    """k_resolve_tiles' result does not depend on how the passes are split between its
    launches or on the record ring's size (a one-pass ring throttles the sample claims):
    the frames are bit-identical to the default streaming frame, and to a second run."""
    rt, scene, cam, st, fc, dev = c3small
    st = type(st).from_buffer_copy(st)
    st.samples_per_pixel = 24
    ref, rs = dev.render(cam, st, fc, 192, 108)
    again, _ = dev.render(cam, st, fc, 192, 108)
    assert np.array_equal(ref, again)
    with dev.configured(**env):
        got, gs = dev.render(cam, st, fc, 192, 108)
    REPORT["stream_chunking_" + "_".join(f"{k}={v}" for k, v in env.items())] = {
        "frame_equal": bool(np.array_equal(ref, got)), "iterations": [int(rs.iterations), int(gs.iterations)]}
    assert (gs.closest_hit_rays, gs.shadow_rays) == (rs.closest_hit_rays, rs.shadow_rays)
    assert np.array_equal(ref, got)


def test_stream_splat_box_filter_bit_exact(c1):
    """With one partition the streaming splat of the box filter adds each pixel's samples in
    sample order, the reference's order: bit-identical to the oracle's frame."""
    rt, scene, cam, st, fc, dev = c1
    box = rt.load_reconstruction_kernel("Box")
    with dev.configured(partitions=1):
        gpu, _ = dev.render(cam, st, box, 256, 256)
    cpu, _ = ob.render(scene.desc(), cam, st, box, 256, 256, rng_mode=0, threads=1)
    assert np.array_equal(gpu, cpu)


def test_sharded_frames_sum_to_full(c1):
    """Tiles t % G == r per GPU, summed (the RCCL reduce) == the single-GPU frame."""
    rt, scene, cam, st, fc, dev = c1
    full, _ = dev.render(cam, st, fc, 256, 256)
    parts = [dev.render(cam, st, fc, 256, 256, shard_index=r, shard_count=3)[0] for r in range(3)]
    assert rel_l2(sum(parts), full) <= 1e-5


def test_box_filter_and_progressive_frames(c1):
    rt, scene, cam, st, fc, dev = c1
    box = rt.load_reconstruction_kernel("Box")
    acc, stats = dev.render(cam, st, box, 256, 256)
    # box filter: every sample adds weight exactly 1 to its own pixel
    assert np.all(acc[..., 3] == st.samples_per_pixel)
    acc2, _ = dev.render(cam, st, box, 256, 256, accum=acc.copy(), frame_count=st.samples_per_pixel,
                         total_frame_index=1)
    assert np.all(acc2[..., 3] == 2 * st.samples_per_pixel)
    cpu = np.zeros_like(acc)
    ob.render(scene.desc(), cam, st, box, 256, 256, rng_mode=0, threads=8, accum=cpu)
    ob.render(scene.desc(), cam, st, box, 256, 256, rng_mode=0, threads=8, accum=cpu,
              frame_count=st.samples_per_pixel, total_frame_index=1)
    assert rel_l2(acc2, cpu) <= 1e-5


def test_golden_frame_hash(rt):
    """The GPU frame of C1 at 64x64 equals the committed oracle golden frame byte for byte."""
    import hashlib
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))["c1_64x64_frame"]
    scene, cam, st, fc, post = rt.load_preset("c1", 64, 64)
    dev = rt.DeviceScene(scene, 0)
    with rt.splat_mode(rt.abi.RT_SPLAT_EXACT):
        acc, stats = dev.render(cam, st, fc, 64, 64)
    dev.close()
    REPORT["golden_c1_64"] = {"sha256_equal": hashlib.sha256(acc.tobytes()).hexdigest() == gold["sha256"],
                              "rays": [int(stats.closest_hit_rays), int(stats.shadow_rays)],
                              "golden_rays": [gold["closest"], gold["shadow"]]}
    assert (stats.closest_hit_rays, stats.shadow_rays) == (gold["closest"], gold["shadow"])
    assert hashlib.sha256(acc.tobytes()).hexdigest() == gold["sha256"]


@pytest.mark.parametrize("frame", [0, 5])
def test_postprocess_bit_exact(c1, frame):
    """The output pass (k_post via rt_postprocess) equals oracle_postprocess byte for byte
    (spec transcendentals on both sides) on a rendered frame plus special pixels, for
    several post settings."""
    rt, scene, cam, st, fc, dev = c1
    acc, _ = dev.render(cam, st, fc, 256, 256)
    acc = acc.copy()
    acc[0, 0] = [np.nan, 1, 1, 1]
    acc[0, 1] = [1, 1, 1, 0]
    acc[0, 2] = [0, 0, 0, -0.75]
    acc[0, 3] = [1e30, 1, 0, 1]
    settings = [rt.abi.PostSettings(0.0, 1, 1, 0.5, 0.0), rt.abi.PostSettings(0.75, 1, 1, 0.45, 0.35),
                rt.abi.PostSettings(-1.0, 0, 0, 0.5, 0.0), rt.abi.PostSettings(0.0, 1, 0, 0.6, 1.0)]
    same = []
    for post in settings:
        gpu = rt.postprocess(acc, post, total_frame_index=frame)
        cpu = ob.postprocess(acc, post, total_frame_index=frame)
        same.append(float((gpu == cpu).mean()))
        assert np.array_equal(gpu, cpu), f"{(gpu != cpu).sum()} pixels differ"
    REPORT[f"postprocess_frame{frame}"] = {"pixels_bit_identical": same}


@pytest.mark.parametrize("env", [{}, {"RT_TOP_PROLOGUE": "0"}, {"RT_MLIST_MAX": "1"}, {"RT_MLIST_MAX": "0"}])
def test_top_level_paths(rt, env, monkeypatch):
    """The three ways a queued ray meets the top level (ray prologue):
    the trace kernel walks all of it (RT_TOP_PROLOGUE=0), the prologue tests the
    analytic primitives and the kernel re-walks everything because the mesh list
    overflowed (RT_MLIST_MAX=1 on C4's four instances, and 0), or the default mesh
    list.  Per-sample results stay bit-exact against the oracle, and the TraversalStats
    (rt_stats::traversal) are those of the oracle's restatement of each walk."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    scene, cam, st, fc, post = rt.load_preset("c4", 192, 108)
    dev = rt.DeviceScene(scene, 0)
    try:
        rng = np.random.default_rng(5)
        xy, s = _sample_list(rng, 192, 108, 20000, st.samples_per_pixel)
        gpu, gstats = dev.trace_samples(cam, st, 192, 108, xy, s)
    finally:
        dev.close()
    with ob.gpu_walk(mlist_max=int(env.get("RT_MLIST_MAX", 4)), top_prologue=env.get("RT_TOP_PROLOGUE") != "0") as walk:
        cpu, cstats = ob.trace_samples(scene.desc(), cam, st, 192, 108, xy, s)
    same = np.all((gpu == cpu) | (np.isnan(gpu) & np.isnan(cpu)), axis=1).mean()
    calls = [int(gstats.traversal[k].mesh_intersection_count) for k in range(2)]
    leaves = [int(gstats.traversal[k].mesh_leaf_traversals) for k in range(2)]
    REPORT["top_level_" + ("_".join(f"{k}={v}" for k, v in env.items()) or "default")] = {
        "bit_exact_fraction": float(same), "gpu_calls": calls, "restated_calls": walk.result["calls"],
        "gpu_leaves": leaves, "restated_leaves": walk.result["leaves"],
        "reference_walk_calls": [int(cstats.traversal[k].mesh_intersection_count) for k in range(2)]}
    assert same >= 0.999
    assert gstats.closest_hit_rays == cstats.closest_hit_rays or same < 1.0
    assert calls == walk.result["calls"]
    for k in range(2):
        # leaves entered: the restated walk applies the GPU's degenerate-axis pruning; the BVH4's skipped
        # level can let a few more through (test_gpu_fullscale.py: at most 3e-7 of them)
        assert abs(leaves[k] - walk.result["leaves"][k]) <= max(2, 1e-5 * walk.result["leaves"][k]), \
            (k, leaves[k], walk.result["leaves"][k])
        for f, key in (("mesh_node_traversals", "nodes"), ("mesh_bvh_traversals", "bvh")):
            g, r = int(getattr(gstats.traversal[k], f)), walk.result[key][k]
            assert abs(g - r) <= max(4, 1e-5 * r), (k, f, g, r)


@pytest.mark.parametrize("how", ["budget", "mode"])
def test_atomic_splat_fallback(rt, monkeypatch, how):
    """Frames whose sample records exceed the HBM budget (even a one-pass ring), or
    RT_SPLAT_ATOMIC, splat with float atomics: the same image up to float summation order."""
    scene, cam, st, fc, post = rt.load_preset("c1", 128, 128)
    dev = rt.DeviceScene(scene, 0)
    try:
        if how == "budget":
            dev.configure(sample_budget_gb=0.0)
            gpu, stats = dev.render(cam, st, fc, 128, 128)
        else:
            with rt.splat_mode(rt.abi.RT_SPLAT_ATOMIC):
                gpu, stats = dev.render(cam, st, fc, 128, 128)
        assert stats.splat_mode == rt.abi.RT_SPLAT_ATOMIC
    finally:
        dev.close()
    cpu, cstats = ob.render(scene.desc(), cam, st, fc, 128, 128, rng_mode=0, threads=8)
    REPORT[f"atomic_splat_c1_128_{how}"] = {"rel_l2": rel_l2(gpu, cpu)}
    assert (stats.closest_hit_rays, stats.shadow_rays) == (cstats.closest_hit_rays, cstats.shadow_rays)
    assert rel_l2(gpu, cpu) <= 1e-5


def test_rcp_cr_exhaustive(rt):
    """The kernels' 3-instruction reciprocal (rt_dmath.h rcp_cr: v_rcp_f32 + one FMA
    Newton step, full division outside [2^-125, 2^125]) equals the correctly rounded
    IEEE 1.0f / x for all 2^32 inputs, so using it in the ray setup, the triangle test
    and normalize leaves every result bit-identical."""
    import ctypes as C
    bad, first = C.c_uint64(), C.c_uint32()
    assert rt.lib().rt_debug_verify_rcp(0, C.byref(bad), C.byref(first)) == 0
    REPORT["rcp_cr_exhaustive"] = {"inputs": 1 << 32, "mismatches": bad.value}
    assert bad.value == 0, f"first mismatch at bits 0x{first.value:08x}"


@pytest.mark.parametrize("which,w,h,spp", [("c3small", 192, 108, 24), ("c4small", 192, 108, 16), ("c1", 256, 256, 16)])
def test_fused_drain_matches_separate_kernels(which, w, h, spp, request):
    """The frame's drain fused into k_drain (each lane runs a path's remaining bounces) computes
    the same per-sample bits as the separate extend / shade / connect launches: frames (exact and
    streaming splat), per-sample radiance of the explicit-sample path and every ray count are
    identical whether the drain is never fused (RT_FUSE_PATHS=0), fused at the default count
    or fused with every path still alive (a count above the pool)."""
    rt, scene, cam, st, fc, dev = request.getfixturevalue(which)
    st = type(st).from_buffer_copy(st)
    st.samples_per_pixel = spp
    rng = np.random.default_rng(11)
    xy = rng.integers(0, [w, h], size=(20000, 2)).astype(np.uint32)
    s = rng.integers(0, spp, size=20000).astype(np.uint32)
    out = {}
    for name, val in (("off", 0), ("default", -1), ("all", 1000000000)):
        with dev.configured(fuse_paths=val):
            with dev.configured(splat_mode=rt.abi.RT_SPLAT_EXACT):
                ex, es = dev.render(cam, st, fc, w, h)
            sm, ss = dev.render(cam, st, fc, w, h)
            samp, ts = dev.trace_samples(cam, st, w, h, xy, s)
        out[name] = (ex, sm, samp, [(int(x.closest_hit_rays), int(x.shadow_rays), int(x.traced_rays[0]),
                                     int(x.traced_rays[1])) for x in (es, ss, ts)], int(ss.iterations))
    ref = out["off"]
    REPORT[f"fused_drain_{which}"] = {k: {"frames_equal": bool(np.array_equal(v[0], ref[0]) and np.array_equal(v[1], ref[1])),
                                          "samples_equal": bool(np.array_equal(v[2], ref[2])), "rays": v[3],
                                          "iterations": v[4]} for k, v in out.items()}
    for name in ("default", "all"):
        ex, sm, samp, rays, _ = out[name]
        assert rays == ref[3], name
        assert np.array_equal(ex, ref[0]), name
        assert np.array_equal(sm, ref[1]), name
        assert np.array_equal(samp, ref[2]), name
    assert out["all"][4] < out["off"][4]          # the fused drain ended the frame in fewer iterations


@pytest.mark.parametrize("mode", ["separate", "merged"])
@pytest.mark.parametrize("which", ["c3small", "c4small"])
def test_fused_drain_any_cadence(which, mode, request):
    """Counters::fused is safe whatever iterations carry the drain kernels (rt_scene_config::
    drain_every, r06).  With the drain kernels on only every 2nd ... 7th iteration, k_bookkeep sets
    `fused` in iterations that run the separate extend / shade / connect launches, and iterations
    without the drain kernels follow the drain.  r05's every-4th carry lost the radiance of one claim
    batch on C4-small (82.6 % of pixels identical: stale pool slots re-shaded after the drain, see
    k_drain_list).  Every cadence must give the default's exact-splat frame bit for bit (and so the
    oracle's, test_frame_bitwise_vs_reference_order), the same ray counts, and the same per-sample
    radiance through rt_trace_samples; also with the drain fused at once (every path alive)."""
    rt, scene, cam, st, fc, dev = request.getfixturevalue(which)
    w, h = 192, 108
    rng = np.random.default_rng(13)
    xy, s = _sample_list(rng, w, h, 20000, st.samples_per_pixel)
    launch = rt.abi.RT_SHADOW_LAUNCH_SEPARATE if mode == "separate" else rt.abi.RT_SHADOW_LAUNCH_MERGED

    def run(**cfg):
        with dev.configured(splat_mode=rt.abi.RT_SPLAT_EXACT, shadow_launch=launch, **cfg):
            fr, fs = dev.render(cam, st, fc, w, h)
            samp, ss = dev.trace_samples(cam, st, w, h, xy, s)
        rays = [(int(x.closest_hit_rays), int(x.shadow_rays), int(x.traced_rays[0]), int(x.traced_rays[1]))
                for x in (fs, ss)]
        return fr, samp, rays, int(fs.iterations)

    ref = run()
    report = {}
    for every in (2, 3, 4, 7):
        for fuse in (-1, 1000000000):
            fr, samp, rays, iters = run(drain_every=every, fuse_paths=fuse)
            same = float(np.all(fr == ref[0], axis=2).mean())
            report[f"every{every}_fuse{'all' if fuse > 0 else 'auto'}"] = {
                "pixels_identical": same, "samples_identical": bool(np.array_equal(samp, ref[1])),
                "rays_equal": rays == ref[2], "iterations": [iters, ref[3]]}
            assert rays == ref[2], (every, fuse)
            assert np.array_equal(fr, ref[0]), (every, fuse, same)
            assert np.array_equal(samp, ref[1]), (every, fuse)
    REPORT[f"fused_drain_cadence_{which}_{mode}"] = report


@pytest.mark.parametrize("which", ["c1", "c3small", "c4small"])
def test_shadow_launch_modes_identical(which, request):
    """rt_scene_config::shadow_launch (r06): the NEE shadow rays traced in a launch of their own after
    k_shade (SEPARATE, the full frame's default) or in the next iteration's trace launch (MERGED, the
    default of small pools) give the same bits: exact-splat frames (equal to the oracle's single-thread
    frame on >= 99.9 % of pixels), streaming frames, per-sample radiance, ray counts, TraversalStats."""
    rt, scene, cam, st, fc, dev = request.getfixturevalue(which)
    w, h = (256, 256) if which == "c1" else (192, 108)
    rng = np.random.default_rng(31)
    xy, s = _sample_list(rng, w, h, 20000, st.samples_per_pixel)
    out = {}
    for name, launch in (("separate", rt.abi.RT_SHADOW_LAUNCH_SEPARATE), ("merged", rt.abi.RT_SHADOW_LAUNCH_MERGED)):
        with dev.configured(shadow_launch=launch):
            with dev.configured(splat_mode=rt.abi.RT_SPLAT_EXACT):
                ex, es = dev.render(cam, st, fc, w, h)
            sm, ss = dev.render(cam, st, fc, w, h)
            samp, ts = dev.trace_samples(cam, st, w, h, xy, s)
        stats = [(int(x.closest_hit_rays), int(x.shadow_rays), int(x.traced_rays[0]), int(x.traced_rays[1]),
                  [x.traversal[k].as_dict() for k in range(2)]) for x in (es, ss, ts)]
        assert es.shadow_launch == ss.shadow_launch == ts.shadow_launch == launch   # rt_stats reports the mode used
        out[name] = (ex, sm, samp, stats, int(ss.iterations))
    cpu, _ = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=1)
    a, b = out["separate"], out["merged"]
    REPORT[f"shadow_launch_{which}"] = {"frames_equal": bool(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])),
                                        "samples_equal": bool(np.array_equal(a[2], b[2])), "stats_equal": a[3] == b[3],
                                        "iterations": [a[4], b[4]],
                                        "separate_pixels_vs_oracle": float(np.all(a[0] == cpu, axis=2).mean())}
    assert a[3] == b[3]
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert np.all(a[0] == cpu, axis=2).mean() >= 0.999


@pytest.mark.parametrize("depth", [0, 1, 2])
def test_fused_drain_shallow_paths(c1, depth):
    """max_bounce_count 0 (nothing traced: every path finished at generation), 1 and 2: the fused
    drain gives the separate kernels' frame and ray counts, and the oracle's frame."""
    rt, scene, cam, st, fc, dev = c1
    st = type(st).from_buffer_copy(st)
    st.max_bounce_count = depth
    st.samples_per_pixel = 8
    out = []
    for val in (0, 1000000000):
        with dev.configured(fuse_paths=val, splat_mode=rt.abi.RT_SPLAT_EXACT):
            out.append(dev.render(cam, st, fc, 256, 256))
    cpu, cs = ob.render(scene.desc(), cam, st, fc, 256, 256, rng_mode=0, threads=1)
    (a, as_), (b, bs) = out
    REPORT[f"fused_drain_depth{depth}"] = {"frames_equal": bool(np.array_equal(a, b)),
                                          "oracle_pixels_bit_identical": float(np.all(b == cpu, axis=2).mean())}
    assert np.array_equal(a, b)
    assert (as_.closest_hit_rays, as_.shadow_rays) == (bs.closest_hit_rays, bs.shadow_rays) == \
        (cs.closest_hit_rays, cs.shadow_rays)
    assert np.all(b == cpu, axis=2).mean() >= 0.999
