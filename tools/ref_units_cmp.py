"""rt_stats::traversal_ref against the oracle's reference walk for one preset frame (diagnostic):
  python tools/ref_units_cmp.py c3 320 180 256"""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402
import oracle_binding as ob  # noqa: E402

rt = conftest._import_package()
preset, w, h, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
scene, cam, st, fc, post = rt.load_preset(preset, w, h)
st.samples_per_pixel = spp
dev = rt.DeviceScene(scene, 0)
with dev.configured(traversal_ref=1):
    _, gs = dev.render(cam, st, fc, w, h)
dev.close()
_, cs = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=16)
for k, kind in enumerate(("closest", "shadow")):
    g, r = gs.traversal_ref[k].as_dict(), cs.traversal[k].as_dict()
    print(json.dumps({"frame": [preset, w, h, spp], "kind": kind, "diff": {f: g[f] - r[f] for f in g}, "ref": r}), flush=True)
