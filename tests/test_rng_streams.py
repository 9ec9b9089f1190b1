"""Noise-aware comparison of the GPU's per-sample RNG with the reference's tile stream.

The reference draws every random number of a 64x64 tile from one xorshift RandomSeries seeded
from (total_frame_index, frame_count, tile) and consumed serially pixel by pixel, sample by
sample (RT/raytracer.cpp:588-593) -- a stream no parallel renderer can reproduce.  The GPU
seeds a RandomSeries per sample from the same tile seed plus the pixel and the sample index
(RT_RNG_PER_SAMPLE) and keeps the reference's draw order inside a sample.  Both
are unbiased estimators of the same pixel integrals, so their frames agree in distribution:

* the frame sums sum(rgb) and sum(w) over SEEDS frames (total_frame_index 0..SEEDS-1) have means
  within K sigma of each other, sigma estimated from the frames of each side;
* the same holds per 64x64 tile (the unit of the reference's stream), and for the closest-hit
  and shadow rays per sample.

The CPU test runs the oracle in both modes (RT_RNG_PER_SAMPLE is bit-exact with the GPU,
tests/test_gpu_parity.py); the GPU tests compare the GPU's own frames with the oracle's
tile-stream frames (the oracle's tile-stream mode reproduces the reference's C1 output exactly,
tests/test_oracle_pins.py).

Power.  The CPU test runs SEEDS = 48 frames per side: the smallest relative bias of a statistic it
detects is K * se / mean, se = sqrt(var_a / 48 + var_b / 48), recorded per statistic in the parity
report ("min_detectable_rel_bias"; DESIGN.md section 3 quotes it).  The GPU spot check keeps 8.
"""
import numpy as np
import pytest

import oracle_binding as ob

K = 4.5          # sigma bound; with ~100 tile comparisons a false alarm at 4.5 sigma is < 1e-3
SEEDS = 48       # frames per side on the CPU
GPU_SEEDS = 8    # frames per side of the GPU spot check


def _frames(render, seeds=SEEDS):
    out = []
    for t in range(seeds):
        frame, stats = render(t)
        out.append((frame.astype(np.float64), stats.closest_hit_rays / stats.samples, stats.shadow_rays / stats.samples))
    return out


def _tile_sums(frame, tile=64):
    h, w, _ = frame.shape
    ty, tx = (h + tile - 1) // tile, (w + tile - 1) // tile
    pad = np.zeros((ty * tile, tx * tile, 4))
    pad[:h, :w] = frame
    return pad.reshape(ty, tile, tx, tile, 4).sum(axis=(1, 3))       # (ty, tx, 4)


def _z(a, b):
    a, b = np.asarray(a), np.asarray(b)
    se = np.sqrt(a.var(axis=0, ddof=1) / len(a) + b.var(axis=0, ddof=1) / len(b))
    diff = a.mean(axis=0) - b.mean(axis=0)
    with np.errstate(divide="ignore", invalid="ignore"):
        z = np.where(se > 0, diff / np.where(se > 0, se, 1), np.where(diff == 0, 0.0, np.inf))
    return z


def _min_bias(a, b):
    """The smallest relative difference of the means that reaches K sigma."""
    a, b = np.asarray(a), np.asarray(b)
    se = np.sqrt(a.var(axis=0, ddof=1) / len(a) + b.var(axis=0, ddof=1) / len(b))
    return K * se / np.abs(0.5 * (a.mean(axis=0) + b.mean(axis=0)))


def compare(per_sample, tile_stream, report=None):
    fa = [f for f, _, _ in per_sample]
    fb = [f for f, _, _ in tile_stream]
    tot_a = [[f[..., :3].sum(), f[..., 3].sum()] for f in fa]
    tot_b = [[f[..., :3].sum(), f[..., 3].sum()] for f in fb]
    z_tot = _z(tot_a, tot_b)
    tiles_a = [_tile_sums(f)[..., :3].sum(axis=-1) for f in fa]
    tiles_b = [_tile_sums(f)[..., :3].sum(axis=-1) for f in fb]
    z_tile = _z(tiles_a, tiles_b)
    rays_a, rays_b = [[c, s] for _, c, s in per_sample], [[c, s] for _, c, s in tile_stream]
    z_rays = _z(rays_a, rays_b)
    if report is not None:
        mb_tot, mb_rays = _min_bias(tot_a, tot_b), _min_bias(rays_a, rays_b)
        report.update({"frames_per_side": len(fa),
                       "z_sum_rgb": float(z_tot[0]), "z_sum_w": float(z_tot[1]),
                       "max_abs_z_tile_rgb": float(np.abs(z_tile).max()), "tiles": int(z_tile.size),
                       "z_tile_rgb": [round(float(x), 3) for x in np.ravel(z_tile)],
                       "z_closest_per_sample": float(z_rays[0]), "z_shadow_per_sample": float(z_rays[1]),
                       "min_detectable_rel_bias": {"sum_rgb": float(mb_tot[0]), "sum_w": float(mb_tot[1]),
                                                   "closest_per_sample": float(mb_rays[0]),
                                                   "shadow_per_sample": float(mb_rays[1]),
                                                   "median_tile_rgb": float(np.median(_min_bias(tiles_a, tiles_b)))},
                       "mean_sum_rgb": [float(np.mean([t[0] for t in tot_a])), float(np.mean([t[0] for t in tot_b]))]})
    assert np.all(np.abs(z_tot) <= K), z_tot
    assert np.all(np.abs(z_tile) <= K), np.abs(z_tile).max()
    assert np.all(np.abs(z_rays) <= K), z_rays


@pytest.mark.parametrize("preset,w,h,spp", [("c1", 192, 192, 16), ("c3", 128, 72, 32), ("c4", 128, 72, 32)])
def test_per_sample_vs_tile_stream_oracle(rt, preset, w, h, spp):
    """CPU, 48 frames per side: the oracle's per-sample RNG (the GPU's scheme, bit-exact with it)
    against its tile-stream RNG (the reference's): C1 (depth 4) and C3-, C4-small (depth 12)."""
    from parity_report import REPORT
    scene, cam, st, fc, post = rt.load_preset(preset, w, h)
    st.samples_per_pixel = spp
    desc = scene.desc()
    a = _frames(lambda t: ob.render(desc, cam, st, fc, w, h, rng_mode=0, threads=8, total_frame_index=t))
    b = _frames(lambda t: ob.render(desc, cam, st, fc, w, h, rng_mode=1, threads=8, total_frame_index=t))
    rep = {}
    try:
        compare(a, b, rep)
    finally:
        REPORT[f"rng_stream_cpu_{preset}_{w}x{h}_{spp}spp"] = rep
    # what 48 frames per side resolve: a bias of the rays per sample well under 0.1 %
    assert rep["min_detectable_rel_bias"]["closest_per_sample"] <= 1e-3
    assert rep["min_detectable_rel_bias"]["shadow_per_sample"] <= 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("preset,w,h,spp", [("c1", 512, 512, 16), ("c3", 192, 108, 256), ("c4", 192, 108, 256)])
def test_gpu_vs_reference_tile_stream(rt, preset, w, h, spp):
    """GPU frames (per-sample RNG) against the oracle's reference-stream frames."""
    from parity_report import REPORT
    scene, cam, st, fc, post = rt.load_preset(preset, w, h)
    st.samples_per_pixel = spp
    dev = rt.DeviceScene(scene, 0)
    try:
        a = _frames(lambda t: dev.render(cam, st, fc, w, h, total_frame_index=t), GPU_SEEDS)
    finally:
        dev.close()
    b = _frames(lambda t: ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=1, threads=16, total_frame_index=t),
                GPU_SEEDS)
    rep = {}
    try:
        compare(a, b, rep)
    finally:
        REPORT[f"rng_stream_{preset}_{w}x{h}_{spp}spp"] = rep
