"""Diagnostic (GPU box): TraversalStats leaves of the device against the oracle's restatement of its
walk, for the library in RT_MI355X_LIB, on C3 / C4 at a reduced size.  Prints GPU - restated per kind.
  RT_MI355X_LIB=... python tools/leaf_diag.py c3 480 270"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import conftest                     # noqa: E402
import oracle_binding as ob         # noqa: E402

rt = conftest._import_package()
preset, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
scene, cam, st, fc, post = rt.load_preset(preset, w, h)
dev = rt.DeviceScene(scene, 0)
try:
    gpu, gs = dev.render(cam, st, fc, w, h)
finally:
    dev.close()
with ob.gpu_walk() as walk:
    cpu, cs = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=16)
res = walk.result
print(preset, w, h, "rays", gs.closest_hit_rays, gs.shadow_rays, "oracle", cs.closest_hit_rays, cs.shadow_rays)
for k, kind in enumerate(("closest", "shadow")):
    g = gs.traversal[k]
    print(f"  {kind}: calls {g.mesh_intersection_count} / {res['calls'][k]}  leaves {g.mesh_leaf_traversals} / "
          f"{res['leaves'][k]}  diff {g.mesh_leaf_traversals - res['leaves'][k]} "
          f"({(g.mesh_leaf_traversals - res['leaves'][k]) / max(1, res['leaves'][k]):.2e})")
