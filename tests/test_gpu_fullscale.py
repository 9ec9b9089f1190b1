"""Parity at the bench's own scale.

The default production path -- rt_render at the BASELINE configs' full sizes, with everything the
bench's frames run: four partitions, 8.4M-path pools, the streaming splat's record ring and resolve
chunks, the fused drain -- against the oracle's frame of the same samples (RT_RNG_PER_SAMPLE, the
reference-order splat, RT/raytracer.cpp:366-495, :692-757):

* C3 (1920x1080, 256 spp) and C4 (1920x1080, 256 spp, ~250k triangles): the whole frame, rel L2
  <= 1e-5 (the streaming splat sums a pixel pass by pass, the reference tile by tile) and the same
  closest-hit and shadow ray counts, call for call;
* C5 (3840x2160, 1024 spp, blue noise): the GPU renders the whole frame; the oracle renders an
  evenly spaced subset of its 64x64 tiles (oracle_render_tiles), compared on the pixels whose
  whole filter window lies in a rendered tile (at least kernel_size px inside it).

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


@pytest.mark.parametrize("preset", ["c3", "c4"])
def test_full_frame_default_path(rt, preset):
    w, h = 1920, 1080
    scene, cam, st, fc, post = rt.load_preset(preset, w, h)
    assert st.samples_per_pixel == 256
    dev = rt.DeviceScene(scene, 0)
    try:
        gpu, gs = dev.render(cam, st, fc, w, h)
    finally:
        dev.close()
    assert gs.splat_mode == rt.abi.RT_SPLAT_STREAM
    threads = _threads()
    cpu, cs = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=threads)
    err = rel_l2(gpu, cpu)
    REPORT[f"fullscale_{preset}_1080p_256spp"] = {
        "rel_l2": err, "max_abs_weight_diff": float(np.abs(gpu[..., 3] - cpu[..., 3]).max()),
        "gpu_rays": [int(gs.closest_hit_rays), int(gs.shadow_rays)], "oracle_rays": [int(cs.closest_hit_rays), int(cs.shadow_rays)],
        "samples": int(gs.samples), "iterations": int(gs.iterations), "oracle_threads": threads,
        "gpu_seconds": gs.seconds}
    assert gs.samples == cs.samples == w * h * 256
    assert (gs.closest_hit_rays, gs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays)
    assert np.isfinite(gpu).all() == np.isfinite(cpu).all()
    assert err <= 1e-5


def test_c5_tile_subset(rt):
    w, h = 3840, 2160
    scene, cam, st, fc, post = rt.load_preset("c5", w, h)
    assert st.samples_per_pixel == 1024
    dev = rt.DeviceScene(scene, 0)
    try:
        gpu, gs = dev.render(cam, st, fc, w, h)
    finally:
        dev.close()
    tcx, tcy = (w + 63) // 64, (h + 63) // 64
    n_tiles = 24
    step = tcx * tcy // n_tiles
    tiles = [k * step + step // 2 for k in range(n_tiles)]
    lib = ob.load()
    cpu = np.zeros((h, w, 4), np.float32)
    buf = rt.abi.AccumulationBuffer(w, h, 0, cpu.ctypes.data_as(C.POINTER(C.c_float)))
    arr = (C.c_uint32 * len(tiles))(*tiles)
    cs = rt.abi.Stats()
    assert lib.oracle_render_tiles(C.byref(scene.desc()), C.byref(cam), C.byref(st), C.byref(fc), 64, 64, 0, 0,
                                   _threads(), len(tiles), arr, C.byref(buf), C.byref(cs)) == 0
    ks = int(fc.kernel_size)
    mask = np.zeros((h, w), bool)
    for t in tiles:
        x0, y0 = (t % tcx) * 64, (t // tcx) * 64
        x1, y1 = min(x0 + 64, w), min(y0 + 64, h)
        mask[y0 + ks:y1 - ks, x0 + ks:x1 - ks] = True
    err = rel_l2(gpu[mask], cpu[mask])
    REPORT["fullscale_c5_4k_1024spp_tiles"] = {"rel_l2": err, "tiles": tiles, "pixels_compared": int(mask.sum()),
                                               "kernel_size": ks, "gpu_rays": [int(gs.closest_hit_rays), int(gs.shadow_rays)],
                                               "oracle_rays_subset": [int(cs.closest_hit_rays), int(cs.shadow_rays)],
                                               "gpu_seconds": gs.seconds, "iterations": int(gs.iterations)}
    assert gs.samples == w * h * 1024
    assert mask.sum() >= n_tiles * (64 - 2 * ks) ** 2 // 2
    assert np.isfinite(gpu).all()
    assert err <= 1e-5
