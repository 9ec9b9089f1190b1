"""rt_stats::traversal_ref of one preset frame under a few schedule settings (diagnostic).
  python tools/ref_units_diag.py c3 1920 1080"""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("buas_pathtracer_amd", os.path.join(ROOT, "buas-pathtracer_amd", "__init__.py"),
                                              submodule_search_locations=[os.path.join(ROOT, "buas-pathtracer_amd")])
rt = importlib.util.module_from_spec(spec)
sys.modules["buas_pathtracer_amd"] = rt
spec.loader.exec_module(rt)
preset, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
scene, cam, st, fc, post = rt.load_preset(preset, w, h)
dev = rt.DeviceScene(scene, 0)
for cfg in ({}, {"fuse_paths": 0}, {"partitions": 1}, {"partitions": 1, "fuse_paths": 0}):
    with dev.configured(traversal_ref=1, **cfg):
        _, s = dev.render(cam, st, fc, w, h)
    print(json.dumps({"cfg": cfg, "rays": [s.closest_hit_rays, s.shadow_rays],
                      "closest": s.traversal_ref[0].as_dict(), "shadow": s.traversal_ref[1].as_dict()}), flush=True)
dev.close()
