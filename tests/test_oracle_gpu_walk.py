"""The oracle's restatement of the GPU library's traversal walk (oracle_gpu_walk_stats, the reference
for rt_stats::traversal), on the CPU: its counts do not depend on how the frame
is split over threads, a scene without meshes counts nothing, and the BVH4 figures relate to the
reference's own BVH2 counts as the layout says (a BVH4 interior node stands for one or two BVH2 ones)."""
import oracle_binding as ob


def _walk(rt, preset, w, h, spp, threads):
    scene, cam, st, fc, post = rt.load_preset(preset, w, h)
    st.samples_per_pixel = spp
    with ob.gpu_walk() as g:
        _, cs = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=threads)
    return g.result, cs


def test_walk_counts_independent_of_threads(rt):
    a, _ = _walk(rt, "c3", 64, 36, 4, 1)
    b, _ = _walk(rt, "c3", 64, 36, 4, 4)
    assert a == b
    assert all(a["calls"]) and all(a["leaves"])


def test_walk_counts_zero_without_meshes(rt):
    r, cs = _walk(rt, "c1", 32, 32, 2, 2)
    assert cs.closest_hit_rays > 0
    assert all(v == [0, 0] for v in r.values())


def test_walk_bvh4_against_bvh2(rt):
    r, cs = _walk(rt, "c3", 64, 36, 4, 4)
    for k in range(2):
        # every BVH4 step is an entry, a node or a triangle step; a node stands for at most two BVH2 nodes
        assert r["bvh"][k] >= r["entries"][k] + r["nodes"][k] + r["leaves"][k]
        assert r["nodes"][k] > 0 and r["entries"][k] <= r["calls"][k]
    # closest-hit queries: the reference walks more BVH2 interior nodes than the BVH4 has nodes
    assert r["nodes"][0] < cs.traversal[0].mesh_node_traversals
