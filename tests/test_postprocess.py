"""The output pass (RT/raytracer.cpp:2103-2171) on the CPU: the dither data and the
oracle's restatement.  The GPU kernel is compared with it in test_gpu_parity.py."""
import hashlib
import os

import numpy as np

import oracle_binding as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tex():
    d = np.fromfile(os.path.join(ROOT, "data", "dither_rgb1_256.u8"), np.uint8)
    return d.reshape(8, 256, 256, 3)


def test_dither_textures_pinned():
    """data/dither_rgb1_256.u8 = the reference's LDR_RGB1_{0..7}.png as R8G8B8 (tools/extract_noise.py).
    Each channel of each texture is a blue-noise permutation: every value occurs exactly 256 times."""
    raw = open(os.path.join(ROOT, "data", "dither_rgb1_256.u8"), "rb").read()
    assert hashlib.sha256(raw).hexdigest() == "aba3ac02000300ef9323e37a8b1024251ad1484f25fa9793bb65f093a03c4f57"
    t = _tex()
    for k in range(8):
        for c in range(3):
            assert np.all(np.bincount(t[k, :, :, c].ravel(), minlength=256) == 256)


def _post(rt, exposure=0.0, tonemapping=1, srgb=1, midpoint=0.5, contrast=0.0):
    return rt.abi.PostSettings(exposure, tonemapping, srgb, midpoint, contrast)


def test_special_pixels(rt, oracle):
    acc = np.zeros((2, 4, 4), np.float32)
    acc[0, 0] = [np.nan, 0, 0, 1]           # NaN -> (0, 255, 255)
    acc[0, 1] = [1, 1, 1, 0]                # weight 0 -> black
    acc[0, 2] = [0, 0, 0, -0.5]             # negative weight -> magenta 127
    acc[0, 3] = [1e30, 1e30, 1e30, 1]       # tonemapped to white
    acc[1, :] = [0.25, 0.5, 1.0, 1.0]
    out = ob.postprocess(acc, _post(rt), total_frame_index=3)
    assert out[0, 0] == 0xFF00FFFF
    assert out[0, 1] == 0xFF000000
    assert out[0, 2] == 0xFF7F007F
    assert out[0, 3] == 0xFFFFFFFF
    assert np.all((out >> 24) == 255)


def test_matches_host_resolve_up_to_dither(rt, oracle):
    """With libm transcendentals the oracle equals the host library's undithered resolve
    (rth_resolve_bgra8, which adds 0.5) within the TPDF dither's +-1 per channel."""
    rng = np.random.default_rng(7)
    acc = np.abs(rng.standard_normal((64, 96, 4))).astype(np.float32) * 3
    acc[..., 3] = rng.uniform(0.5, 4, (64, 96)).astype(np.float32)
    for post in (_post(rt), _post(rt, exposure=0.5, contrast=0.4, midpoint=0.45), _post(rt, tonemapping=0, srgb=0)):
        oracle.oracle_set_math_mode(1)
        try:
            got = ob.postprocess(acc, post, total_frame_index=5)
        finally:
            oracle.oracle_set_math_mode(0)
        host = rt.resolve_bgra8(acc, post)
        for sh in (0, 8, 16):
            d = ((got >> sh) & 255).astype(int) - ((host >> sh) & 255).astype(int)
            assert np.abs(d).max() <= 1
            assert np.abs(d).mean() > 0.05        # the dither is actually applied


def test_dither_texture_follows_frame_index(rt, oracle):
    acc = np.full((256, 256, 4), 0.3, np.float32)
    outs = [ob.postprocess(acc, _post(rt), total_frame_index=i) for i in (0, 1, 8)]
    assert np.array_equal(outs[0], outs[2])          # texture total_frame_index % 8
    assert not np.array_equal(outs[0], outs[1])
