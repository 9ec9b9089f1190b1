"""Reference-unit TraversalStats by render path (diagnostic): the same samples (every pixel, passes
0..spp-1) as a frame (rt_render) and as an explicit sample list (rt_trace_samples), GPU and oracle.
  python tools/ref_units_paths.py c3 640 360 16"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402
import oracle_binding as ob  # noqa: E402

rt = conftest._import_package()
preset, w, h, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
scene, cam, st, fc, post = rt.load_preset(preset, w, h)
st.samples_per_pixel = spp
dev = rt.DeviceScene(scene, 0)
dev.configure(traversal_ref=1)
desc = scene.desc()
ys, xs = np.mgrid[0:h, 0:w]
xy1 = np.stack([xs.ravel(), ys.ravel()], axis=1).astype(np.uint32)
xy = np.concatenate([xy1] * spp)
s = np.repeat(np.arange(spp, dtype=np.uint32), len(xy1))
_, gl = dev.trace_samples(cam, st, w, h, xy, s)
_, cl = ob.trace_samples(desc, cam, st, w, h, xy, s)
_, gr = dev.render(cam, st, fc, w, h)
_, cr = ob.render(desc, cam, st, fc, w, h, rng_mode=0, threads=16)
dev.close()
for name, st_ in (("gpu_list", gl), ("oracle_list", cl), ("gpu_render", gr), ("oracle_render", cr)):
    t = st_.traversal_ref if name.startswith("gpu") else st_.traversal
    print(name, st_.closest_hit_rays, st_.shadow_rays, json.dumps([t[k].as_dict() for k in range(2)]), flush=True)
