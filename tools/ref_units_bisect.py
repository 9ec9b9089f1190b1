"""Find samples whose reference-unit TraversalStats (rt_stats::traversal_ref) differ from the oracle's
reference walk (diagnostic): python tools/ref_units_bisect.py c3 640 360 [spp]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402
import oracle_binding as ob  # noqa: E402

rt = conftest._import_package()
preset, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
scene, cam, st, fc, post = rt.load_preset(preset, w, h)
dev = rt.DeviceScene(scene, 0)
dev.configure(traversal_ref=1)
desc = scene.desc()


def diff(xy, s):
    _, g = dev.trace_samples(cam, st, w, h, xy, s)
    _, c = ob.trace_samples(desc, cam, st, w, h, xy, s)
    out = []
    for k in range(2):
        gd, cd = g.traversal_ref[k].as_dict(), c.traversal[k].as_dict()
        out.append({f: gd[f] - cd[f] for f in gd})
    return out, g, c


spp = int(sys.argv[4]) if len(sys.argv) > 4 else 1
ys, xs = np.mgrid[0:h, 0:w]
xy1 = np.stack([xs.ravel(), ys.ravel()], axis=1).astype(np.uint32)
xy = np.concatenate([xy1] * spp)
s = np.repeat(np.arange(spp, dtype=np.uint32), len(xy1))
d, _, _ = diff(xy, s)
print(f"all pixels, samples 0..{spp - 1}:", json.dumps(d), flush=True)
found = []


def bisect(lo, hi, depth=0):
    if len(found) >= 6:
        return
    d, g, c = diff(xy[lo:hi], s[lo:hi])
    bad = any(v != 0 for k in range(2) for v in d[k].values())
    if not bad:
        return
    if hi - lo == 1:
        found.append((int(xy[lo][0]), int(xy[lo][1])))
        print("sample", xy[lo].tolist(), int(s[lo]), json.dumps(d), "gpu", json.dumps([g.traversal_ref[k].as_dict() for k in range(2)]),
              "ref", json.dumps([c.traversal[k].as_dict() for k in range(2)]), flush=True)
        return
    mid = (lo + hi) // 2
    bisect(lo, mid, depth + 1)
    bisect(mid, hi, depth + 1)


bisect(0, len(xy))
dev.close()
