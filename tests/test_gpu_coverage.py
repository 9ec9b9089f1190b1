"""GPU parity for the configurations and options tests/test_gpu_parity.py does not reach:

* C2 (Cornell box + the 70k-triangle mesh, no environment map, 64 spp): samples and frames;
* every reconstruction filter of g_filters (RT/reconstruction_filters.cpp:97-106) in both
  deterministic splats: Box, Gaussian 3 / 12, Mitchell-Netravali, Lanczos 3 / 4 / 6 / 12
  (radius 12 exercises k_resolve_tiles' widest staging);
* the bokeh polygon (f_factor != 0, RT/raytracer.cpp:86-94) with DOF;
* the render-to-bitmap entry point (rth_take_picture -> rt_render_picture -> write_bitmap,
  RT/raytracer.cpp:2031-2185) against the oracle's output pass;
* rt_cancel in the middle of a frame (discard_current_render, RT/raytracer.cpp:686-690) and a
  bit-exact frame right after it;
* frames sharded over 2, 4 and 8 ranks (tiles t % N) summing to the single-rank frame, in the
  streaming splat (each rank resolves only the blocks its tiles reach) and the exact one.
"""
import os
import threading

import numpy as np
import pytest

import oracle_binding as ob
from parity_report import REPORT
from test_gpu_parity import rel_l2, _sample_list

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2small(rt):
    scene, cam, st, fc, post = rt.load_preset("c2", 192, 108)
    dev = rt.DeviceScene(scene, 0)
    yield rt, scene, cam, st, fc, post, dev
    dev.close()


def test_c2_trace_samples_bitwise(c2small):
    rt, scene, cam, st, fc, post, dev = c2small
    rng = np.random.default_rng(21)
    xy, s = _sample_list(rng, 192, 108, 20000, st.samples_per_pixel)
    gpu, gs = dev.trace_samples(cam, st, 192, 108, xy, s)
    cpu, cs = ob.trace_samples(scene.desc(), cam, st, 192, 108, xy, s)
    same = np.all((gpu == cpu) | (np.isnan(gpu) & np.isnan(cpu)), axis=1).mean()
    REPORT["trace_samples_c2small"] = {"samples": int(len(xy)), "bit_exact_fraction": float(same)}
    assert same >= 0.999
    assert gs.closest_hit_rays == cs.closest_hit_rays or same < 1.0


@pytest.mark.parametrize("mode", ["exact", "stream"])
def test_c2_frame(c2small, mode):
    rt, scene, cam, st, fc, post, dev = c2small
    m = rt.abi.RT_SPLAT_EXACT if mode == "exact" else rt.abi.RT_SPLAT_STREAM
    with rt.splat_mode(m):
        gpu, gs = dev.render(cam, st, fc, 192, 108)
    cpu, cs = ob.render(scene.desc(), cam, st, fc, 192, 108, rng_mode=0, threads=1)
    REPORT[f"frame_c2small_{mode}"] = {"rel_l2": rel_l2(gpu, cpu), "bit_identical": bool(np.array_equal(gpu, cpu))}
    assert (gs.closest_hit_rays, gs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays)
    if mode == "exact":
        assert np.all(gpu == cpu, axis=2).mean() >= 0.999
        assert rel_l2(gpu, cpu) <= 1e-6
    else:
        assert rel_l2(gpu, cpu) <= 1e-5


FILTERS = ["Box", "Gaussian 3", "Gaussian 12", "Mitchell Netravali", "Lanczos 3", "Lanczos 4", "Lanczos 6",
           "Lanczos 12"]


@pytest.mark.parametrize("name", FILTERS)
def test_every_reconstruction_filter(rt, name):
    """Each g_filters entry through both deterministic splats against the oracle's
    single-threaded splat_filter (C1 at 128x96, 8 spp; Lanczos lobes give negative weights)."""
    scene, cam, st, fc, post = rt.load_preset("c1", 128, 96)
    st.samples_per_pixel = 8
    filt = rt.load_reconstruction_kernel(name)
    ref = ob.load()
    ofc = type(filt)()
    assert ref.oracle_load_filter(name.encode(), ofc) == 0
    assert (ofc.kernel_size, ofc.cache_size) == (filt.kernel_size, filt.cache_size)
    assert np.array_equal(np.ctypeslib.as_array(ofc.cache), np.ctypeslib.as_array(filt.cache))
    dev = rt.DeviceScene(scene, 0)
    try:
        with rt.splat_mode(rt.abi.RT_SPLAT_EXACT):
            exact, es = dev.render(cam, st, filt, 128, 96)
        stream, ss = dev.render(cam, st, filt, 128, 96)
    finally:
        dev.close()
    cpu, _ = ob.render(scene.desc(), cam, st, filt, 128, 96, rng_mode=0, threads=1)
    REPORT[f"filter_{name}"] = {"exact_pixels_bit_identical": float(np.all(exact == cpu, axis=2).mean()),
                                "stream_rel_l2": rel_l2(stream, cpu), "stream_mode": int(ss.splat_mode)}
    assert es.splat_mode == rt.abi.RT_SPLAT_EXACT and ss.splat_mode == rt.abi.RT_SPLAT_STREAM
    assert np.all(exact == cpu, axis=2).mean() >= 0.999
    assert rel_l2(exact, cpu) <= 1e-6
    assert rel_l2(stream, cpu) <= 1e-5


@pytest.mark.parametrize("f_factor,edges", [(0.5, 6.0), (1.0, 5.0), (0.25, 3.0)])
def test_bokeh_polygon(rt, f_factor, edges):
    """transform_bokeh_sample with f_factor != 0 (RT/raytracer.cpp:86-94): the polygonal
    aperture of diaphragm_edges blades, rotated by f * phi_shutter_max, on C3's DOF camera."""
    scene, cam, st, fc, post = rt.load_preset("c3", 192, 108)
    assert cam.lens_radius > 0
    st.f_factor = f_factor
    st.diaphragm_edges = edges
    st.samples_per_pixel = 32
    dev = rt.DeviceScene(scene, 0)
    try:
        rng = np.random.default_rng(9)
        xy, s = _sample_list(rng, 192, 108, 20000, st.samples_per_pixel)
        gpu, _ = dev.trace_samples(cam, st, 192, 108, xy, s)
        with rt.splat_mode(rt.abi.RT_SPLAT_EXACT):
            frame, _ = dev.render(cam, st, fc, 192, 108)
    finally:
        dev.close()
    cpu, _ = ob.trace_samples(scene.desc(), cam, st, 192, 108, xy, s)
    same = np.all((gpu == cpu) | (np.isnan(gpu) & np.isnan(cpu)), axis=1).mean()
    cframe, _ = ob.render(scene.desc(), cam, st, fc, 192, 108, rng_mode=0, threads=1)
    REPORT[f"bokeh_f{f_factor}_n{edges}"] = {"bit_exact_fraction": float(same), "frame_rel_l2": rel_l2(frame, cframe)}
    assert same >= 0.999
    assert rel_l2(frame, cframe) <= 1e-6


@pytest.mark.parametrize("mode", ["exact", "stream"])
def test_take_picture_bitmap(rt, tmp_path, mode):
    """rth_take_picture renders frame T on the device, runs the output pass with the dither of
    frame T + 1 and writes the BMP: its pixels equal oracle_postprocess of the same frame."""
    w, h, T = 192, 108, 5
    scene, cam, st, fc, post = rt.load_preset("c3", w, h)
    path = tmp_path / "picture.bmp"
    m = rt.abi.RT_SPLAT_EXACT if mode == "exact" else rt.abi.RT_SPLAT_STREAM
    with rt.splat_mode(m):
        stats = rt.take_picture(scene, cam, st, fc, post, w, h, 16, path, total_frame_index=T)
        st.samples_per_pixel = 16
        dev = rt.DeviceScene(scene, 0)
        try:
            frame, _ = dev.render(cam, st, fc, w, h, total_frame_index=T)
        finally:
            dev.close()
    pic = rt.read_bitmap(path, w, h)
    assert stats.samples == w * h * 16
    assert np.array_equal(pic, ob.postprocess(frame, post, total_frame_index=T + 1))
    if mode == "exact":
        cpu, _ = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=1, total_frame_index=T)
        ref = ob.postprocess(cpu, post, total_frame_index=T + 1)
        REPORT["take_picture_exact"] = {"pixels_equal": float((pic == ref).mean())}
        assert (pic == ref).mean() >= 0.999


def test_cancel_mid_frame(rt):
    """rt_cancel from another thread while a long frame renders returns RT_ERROR_CANCELLED
    (after the partitions' in-flight work has drained), and the next frame is bit-exact."""
    scene, cam, st, fc, post = rt.load_preset("c3", 1920, 1080)
    st.samples_per_pixel = 1024                      # ~1.2 s: the cancel lands mid-frame
    dev = rt.DeviceScene(scene, 0)
    try:
        timer = threading.Timer(0.15, dev.cancel)
        timer.start()
        with pytest.raises(rt.RenderError) as ei:
            dev.render(cam, st, fc, 1920, 1080)
        timer.join()
        assert ei.value.code == rt.abi.RT_ERROR_CANCELLED
        small = type(st).from_buffer_copy(st)
        small.samples_per_pixel = 16
        with rt.splat_mode(rt.abi.RT_SPLAT_EXACT):
            gpu, gs = dev.render(cam, small, fc, 192, 108)
    finally:
        dev.close()
    cpu, cs = ob.render(scene.desc(), cam, small, fc, 192, 108, rng_mode=0, threads=1)
    REPORT["cancel_then_render"] = {"bit_identical": bool(np.array_equal(gpu, cpu))}
    assert (gs.closest_hit_rays, gs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays)
    assert np.all(gpu == cpu, axis=2).mean() >= 0.999


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("mode", ["stream", "exact"])
def test_sharded_frames_sum(rt, n, mode):
    """Ranks' shares (tiles t % N, each rendered as a whole frame of its own) sum to the
    single-rank frame: the per-rank sample keys make the shares disjoint, and every filter
    footprint crossing a tile border lands in the right buffer."""
    scene, cam, st, fc, post = rt.load_preset("c3", 320, 200)
    st.samples_per_pixel = 16
    m = rt.abi.RT_SPLAT_EXACT if mode == "exact" else rt.abi.RT_SPLAT_STREAM
    dev = rt.DeviceScene(scene, 0)
    try:
        with rt.splat_mode(m):
            full, fs = dev.render(cam, st, fc, 320, 200)
            parts = [dev.render(cam, st, fc, 320, 200, shard_index=r, shard_count=n) for r in range(n)]
    finally:
        dev.close()
    total = sum(p[0].astype(np.float64) for p in parts)
    REPORT[f"sharded_{mode}_{n}"] = {"rel_l2": rel_l2(total, full)}
    assert sum(p[1].samples for p in parts) == fs.samples
    assert sum(p[1].closest_hit_rays for p in parts) == fs.closest_hit_rays
    assert rel_l2(total, full) <= 1e-5


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("mode", ["stream", "atomic"])
def test_pass_sharded_frames_sum(rt, n, mode):
    """RT_SHARD_PASSES: shard i of n renders every tile over sample passes [spp*i/n, spp*(i+1)/n).
    The shares sum to the single-rank frame (same sample keys, so the same samples and rays, only
    the float sums regrouped), including a pass count that does not divide evenly (n = 3), and an
    exact-splat request renders as the streaming splat."""
    scene, cam, st, fc, post = rt.load_preset("c3", 320, 200)
    st.samples_per_pixel = 16
    m = rt.abi.RT_SPLAT_ATOMIC if mode == "atomic" else rt.abi.RT_SPLAT_STREAM
    dev = rt.DeviceScene(scene, 0)
    try:
        with rt.splat_mode(m):
            full, fs = dev.render(cam, st, fc, 320, 200)
            rt.set_shard_mode(rt.abi.RT_SHARD_PASSES)
            try:
                parts = [dev.render(cam, st, fc, 320, 200, shard_index=r, shard_count=n) for r in range(n)]
            finally:
                rt.set_shard_mode(rt.abi.RT_SHARD_TILES)
        with rt.splat_mode(rt.abi.RT_SPLAT_EXACT):
            rt.set_shard_mode(rt.abi.RT_SHARD_PASSES)
            try:
                ex, es = dev.render(cam, st, fc, 320, 200, shard_index=0, shard_count=n)
            finally:
                rt.set_shard_mode(rt.abi.RT_SHARD_TILES)
        # the last shard too: its passes start past 0, so a misplaced record would show here
        with rt.splat_mode(rt.abi.RT_SPLAT_EXACT):
            rt.set_shard_mode(rt.abi.RT_SHARD_PASSES)
            try:
                exl, esl = dev.render(cam, st, fc, 320, 200, shard_index=n - 1, shard_count=n)
            finally:
                rt.set_shard_mode(rt.abi.RT_SHARD_TILES)
    finally:
        dev.close()
    total = sum(p[0].astype(np.float64) for p in parts)
    REPORT[f"pass_sharded_{mode}_{n}"] = {"rel_l2": rel_l2(total, full), "samples": [int(p[1].samples) for p in parts]}
    assert [p[1].samples for p in parts] == [320 * 200 * (16 * (r + 1) // n - 16 * r // n) for r in range(n)]
    assert sum(p[1].closest_hit_rays for p in parts) == fs.closest_hit_rays
    assert sum(p[1].shadow_rays for p in parts) == fs.shadow_rays
    assert rel_l2(total, full) <= (1e-5 if mode == "stream" else 1e-4)
    assert es.splat_mode == esl.splat_mode == rt.abi.RT_SPLAT_STREAM
    assert (np.array_equal(ex, parts[0][0]) and np.array_equal(exl, parts[-1][0])) or mode == "atomic"


@pytest.mark.parametrize("want", ["stream", "exact"])
def test_pass_shards_wide_filter(rt, want):
    """A filter radius past what k_resolve_tiles stages (kernel_size 16 > 12): a whole frame takes
    the exact gather, a pass shard the atomic splat (its records would otherwise be placed at its
    first pass in an array sized for its own passes).  Every shard of 3, the last one
    included, sums with the others to the single-rank frame."""
    scene, cam, st, fc, post = rt.load_preset("c1", 160, 128)
    st.samples_per_pixel = 9
    wide = rt.abi.FilterCache.from_buffer_copy(fc)
    wide.kernel_size = 16                     # the Mitchell LUT stretched over a 16-pixel radius
    dev = rt.DeviceScene(scene, 0)
    try:
        m = rt.abi.RT_SPLAT_EXACT if want == "exact" else rt.abi.RT_SPLAT_STREAM
        dev.configure(splat_mode=m)
        full, fs = dev.render(cam, st, wide, 160, 128)
        dev.configure(shard_mode=rt.abi.RT_SHARD_PASSES)
        parts = [dev.render(cam, st, wide, 160, 128, shard_index=r, shard_count=3) for r in range(3)]
    finally:
        dev.close()
    total = sum(p[0].astype(np.float64) for p in parts)
    cpu, cs = ob.render(scene.desc(), cam, st, wide, 160, 128, rng_mode=0, threads=8)
    REPORT[f"pass_shards_wide_filter_{want}"] = {"rel_l2_sum_vs_full": rel_l2(total, full), "rel_l2_full_vs_oracle": rel_l2(full, cpu),
                                                 "modes": [int(fs.splat_mode)] + [int(p[1].splat_mode) for p in parts]}
    assert fs.splat_mode == rt.abi.RT_SPLAT_EXACT
    assert all(p[1].splat_mode == rt.abi.RT_SPLAT_ATOMIC for p in parts)
    assert (fs.closest_hit_rays, fs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays)
    assert sum(p[1].closest_hit_rays for p in parts) == fs.closest_hit_rays
    assert rel_l2(full, cpu) <= 1e-6
    assert rel_l2(total, full) <= 1e-4


def test_scene_config_is_per_scene(rt, monkeypatch):
    """rt_scene_config: two scenes in one process render with their own splat modes; the
    environment is read once at upload (a variable set afterwards changes nothing); a bad
    value is rejected with RT_ERROR_INVALID and leaves the configuration as it was."""
    scene, cam, st, fc, post = rt.load_preset("c1", 128, 128)
    st.samples_per_pixel = 4
    a, b = rt.DeviceScene(scene, 0), None
    try:
        monkeypatch.setenv("RT_PARTITIONS", "1")
        b = rt.DeviceScene(scene, 0)                     # uploaded with the override
        monkeypatch.setenv("RT_SPLAT", "2")              # after both uploads: ignored
        assert a.config().partitions == 0 and b.config().partitions == 1
        a.configure(splat_mode=rt.abi.RT_SPLAT_EXACT)
        fa, sa = a.render(cam, st, fc, 128, 128)
        fb, sb = b.render(cam, st, fc, 128, 128)
        assert sa.splat_mode == rt.abi.RT_SPLAT_EXACT and sb.splat_mode == rt.abi.RT_SPLAT_STREAM
        assert (sa.closest_hit_rays, sa.shadow_rays) == (sb.closest_hit_rays, sb.shadow_rays)
        assert rel_l2(fa, fb) <= 1e-5
        before = a.config()
        with pytest.raises(rt.RenderError):
            a.configure(partitions=9)
        with pytest.raises(rt.RenderError):
            a.configure(splat_mode=7)
        assert bytes(a.config()) == bytes(before)
    finally:
        a.close()
        if b is not None:
            b.close()


@pytest.mark.parametrize("var,value", [("RT_SPLAT", "exact"), ("RT_SPLAT", "3"), ("RT_PARTITIONS", "9"),
                                       ("RT_FUSE_PATHS", "-1"), ("RT_SAMPLE_BUDGET_GB", "lots"),
                                       ("RT_TOP_PROLOGUE", "off"), ("RT_MLIST_MAX", "9"), ("RT_LDS_SCENE", "no"),
                                       ("RT_TRACE_GRID_PCT", "0"), ("RT_DRAIN_GRID_PCT", "75%"),
                                       ("RT_DRAIN_GRID_PCT", "200")])
def test_bad_override_rejected(rt, monkeypatch, var, value):
    """A malformed test-override variable fails rt_scene_upload with RT_ERROR_INVALID naming it,
    instead of silently becoming 0 (RT_SPLAT=exact read as RT_SPLAT_STREAM)."""
    scene, cam, st, fc, post = rt.load_preset("c1", 32, 32)
    monkeypatch.setenv(var, value)
    with pytest.raises(rt.RenderError) as e:
        rt.DeviceScene(scene, 0)
    assert e.value.code == rt.abi.RT_ERROR_INVALID and var in str(e.value)


@pytest.mark.parametrize("preset", ["c3", "c4"])
def test_traversal_ref_units(rt, preset):
    """rt_scene_config::traversal_ref: the trace kernels walk the top level in the reference's order and
    count TraversalStats in its BVH2 units (rt_stats::traversal_ref); against the reference's own counts
    of the same frame (the oracle's reference walk) within 1e-3, the frame and ray counts unchanged."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("fullscale", os.path.join(os.path.dirname(__file__), "test_gpu_fullscale.py"))
    fs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(fs)
    w, h = 320, 180
    scene, cam, st, fc, post = rt.load_preset(preset, w, h)
    st.samples_per_pixel = 16
    dev = rt.DeviceScene(scene, 0)
    try:
        with dev.configured(traversal_ref=1):
            gpu, gs = dev.render(cam, st, fc, w, h)
        plain, ps = dev.render(cam, st, fc, w, h)
    finally:
        dev.close()
    cpu, cs = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=8)
    REPORT[f"traversal_ref_{preset}_{w}x{h}_16spp"] = fs.check_traversal_ref(gs, cs)
    assert all(v == 0 for k in range(2) for v in ps.traversal_ref[k].as_dict().values())   # off: not counted
    assert (gs.closest_hit_rays, gs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays) == (ps.closest_hit_rays, ps.shadow_rays)
    assert rel_l2(gpu, cpu) <= 1e-5 and rel_l2(plain, cpu) <= 1e-5
