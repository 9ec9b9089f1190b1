#!/usr/bin/env python3
"""Regenerate tests/golden/*.json from the CPU oracle (oracle/liboracle.so).

Run from the repo root after `make -C oracle`:  python tests/golden/make_golden.py
The oracle itself is pinned against the reference's own observations
(tests/test_oracle_pins.py); these vectors freeze its lower-level outputs
(RNG, samplers, transcendentals, hit records, a small frame) so that any
change to the restatement or to the HIP kernels is caught exactly.
"""
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import conftest  # noqa: E402

rt = conftest._import_package()
import oracle_binding as ob  # noqa: E402


def f2h(x):
    return np.float32(x).view(np.uint32).item()


def main():
    lib = ob.load()
    g = {}
    g["wang_hash"] = {str(k): lib.oracle_wang_hash(k) for k in [0, 1, 2, 3, 12345, 0xDEADBEEF, 0xFFFFFFFF]}
    g["sample_seed"] = [[a, b, c, d, e, lib.oracle_sample_seed(a, b, c, d, e)]
                        for (a, b, c, d, e) in [(0, 0, 0, 0, 0), (0, 0, 509, 1920 * 1079 + 7, 255), (3, 16, 5, 77, 19)]]
    rng = {}
    for seed in [0, 1, 2, 0x9E3779B9]:
        out = (C.c_float * 64)()
        lib.oracle_rng_unilaterals(seed, 16, out)
        rng[str(seed)] = [f2h(v) for v in out]
    g["rng_unilaterals_bits"] = rng
    samp = []
    for strategy in (0, 1, 2):
        for (x, y, idx, dim, bounce) in [(0, 0, 0, 0, 0), (17, 3, 5, 1, 0), (200, 100, 63, 2, 0), (5, 9, 255, 3, 0),
                                         (5, 9, 256, 3, 0), (5, 9, 300, 3, 0), (5, 9, 10, 5, 0), (5, 9, 10, 6, 0),
                                         (5, 9, 10, 1, 1)]:
            out = (C.c_float * 2)()
            lib.oracle_sample_2d(12345, strategy, x, y, idx, dim, bounce, out)
            s1 = lib.oracle_sample_1d(12345, strategy, x, y, idx, dim, bounce)
            samp.append([strategy, x, y, idx, dim, bounce, f2h(out[0]), f2h(out[1]), f2h(s1)])
    g["samples"] = samp
    xs = np.linspace(-20.0, 20.0, 97, dtype=np.float32)
    g["trig_bits"] = [[f2h(x), f2h(lib.oracle_sinf(float(x))), f2h(lib.oracle_cosf(float(x)))] for x in xs]
    es = np.linspace(-90.0, 80.0, 61, dtype=np.float32)
    g["exp_bits"] = [[f2h(x), f2h(lib.oracle_expf(float(x)))] for x in es]
    asx = np.linspace(-1.0, 1.0, 41, dtype=np.float32)
    g["asin_bits"] = [[f2h(x), f2h(lib.oracle_asinf(float(x)))] for x in asx]
    at = [(0.3, -0.7), (-0.2, -0.9), (1.0, 0.0), (0.0, -1.0), (-0.5, 0.5), (2.0, 3.0)]
    g["atan2_bits"] = [[f2h(y), f2h(x), f2h(lib.oracle_atan2f(y, x))] for (y, x) in at]
    fc = rt.FilterCache()
    lib.oracle_load_filter(b"Mitchell Netravali", C.byref(fc))
    g["mitchell_lut_bits"] = [f2h(v) for v in fc.cache[:256]]
    # hit records on the C1 scene for fixed rays
    scene, cam, st, fcache, post = rt.load_preset("c1", 64, 64)
    r = np.random.default_rng(5)
    rays = []
    for i in range(64):
        o = np.array([0.0, 7.0, -10.0]) + r.uniform(-6, 6, 3)
        d = r.normal(size=3)
        d /= np.linalg.norm(d)
        rays.append(rt.abi.RayQuery(rt.V3(*o.astype(np.float32)), rt.V3(*d.astype(np.float32)), 3.0e38, 0))
    hits = ob.intersect(scene.desc(), rays)
    g["c1_hits"] = [[f2h(q.o.x), f2h(q.o.y), f2h(q.o.z), f2h(q.d.x), f2h(q.d.y), f2h(q.d.z), h.primitive, f2h(h.t),
                     f2h(h.n.x), f2h(h.n.y), f2h(h.n.z)] for q, h in zip(rays, hits)]
    # a small frame: C1 at 64x64, 16 spp, per-sample RNG, single thread
    acc, stats = ob.render(scene.desc(), cam, st, fcache, 64, 64, rng_mode=0, threads=1)
    g["c1_64x64_frame"] = {"sha256": hashlib.sha256(acc.tobytes()).hexdigest(),
                           "sum_rgb": float(acc[..., :3].astype(np.float64).sum()),
                           "sum_w": float(acc[..., 3].astype(np.float64).sum()),
                           "closest": int(stats.closest_hit_rays), "shadow": int(stats.shadow_rays)}
    with open(os.path.join(HERE, "oracle_golden.json"), "w") as f:
        json.dump(g, f, indent=0)
    print("wrote", os.path.join(HERE, "oracle_golden.json"))


if __name__ == "__main__":
    main()
