"""Host-side device layouts (no GPU): the mesh BVH4 and the ray prologue's top-level
sequences must visit nodes in exactly the reference's order.

* BVH4 (rt_debug_mesh_bvh4): each interior node of the caller's BVH2 merged with its
  interior children.  The reference's mesh traversal (RT/intersection.cpp:269-376)
  pops a node, box-tests it and pushes (left, left+1) or (left+1, left) by
  d_is_negative[split_axis].  For random rays, the leaves the BVH4 walk reaches must
  come in the same order as the BVH2 walk's.
* Top-level sequences (rt_debug_top_sequences): per direction octant, the walk that
  jumps past a failing node's subtree must visit the same nodes, in the same order,
  as the reference's stack walk of the top level (:444-520) for any pass/fail pattern.
"""
import ctypes as C
import numpy as np
import pytest

EMPTY4 = 0xFFFFFFFF


def _box_hit(o, inv_d, p, r):
    """The slab test of ray_intersect_bounding_volume (RT/intersection.cpp:107-133) in
    float64, NaN slabs dropped like the reference's ternary max/min; no far clip."""
    with np.errstate(invalid="ignore", over="ignore"):
        n = inv_d * (o - p)
        k = np.abs(inv_d) * r
        t1, t2 = -n - k, -n + k
    tn, tf = t1[0], t2[0]
    for a in (1, 2):
        tn = tn if tn > t1[a] else t1[a]
        tf = tf if tf < t2[a] else t2[a]
    return bool(tn < tf and tf > 0.0)


def _node_box(n):
    return (np.array([n.bv_p.x, n.bv_p.y, n.bv_p.z]), np.array([n.bv_r.x, n.bv_r.y, n.bv_r.z]))


def _bvh2_leaves(nodes, o, d, inv_d):
    """Leaves (first, count) of the reference's mesh traversal without far-clip culling."""
    neg = d < 0
    out, stack = [], [0]
    while stack:
        i = stack.pop()
        n = nodes[i]
        if not _box_hit(o, inv_d, *_node_box(n)):
            continue
        if n.count:
            out.append((n.left_first, n.count))
        elif neg[n.split_axis]:
            stack += [n.left_first, n.left_first + 1]
        else:
            stack += [n.left_first + 1, n.left_first]
    return out


def _bvh4_leaves(q, qb, root, nodes, o, d, inv_d):
    """The same rays through the BVH4 as k_trace's push_children4 walks it (the root's box
    is tested first, as the TM_LEAF step does for the mesh root)."""
    neg = [bool(x) for x in (d < 0)]
    out = []
    if not _box_hit(o, inv_d, *_node_box(nodes[0])):
        return out

    def leaf(rec):
        if rec & 0x80000000:                       # index form: the BVH2 node
            n = nodes[rec & 0x7FFFFFFF]
            return (n.left_first, n.count)
        return (rec & 0x1FFFFFF, (rec >> 25) & 31)

    stack = [root]
    while stack:
        rec = stack.pop()
        if rec & 0x80000000 or (rec >> 30) & 1:
            out.append(leaf(rec))
            continue
        f = q[rec]
        recs = [int(x) for x in qb[rec][24:28]]
        meta = int(qb[rec][28])
        hit = []
        for c in range(4):
            p = np.array([f[0 + c], f[4 + c], f[8 + c]])
            r = np.array([f[12 + c], f[16 + c], f[20 + c]])
            hit.append(recs[c] != EMPTY4 and _box_hit(o, inv_d, p, r))
        g = int(neg[meta & 3])
        fa, fb = int(neg[(meta >> 2) & 3]), int(neg[(meta >> 4) & 3])
        f1, f2 = (fb, fa) if g else (fa, fb)
        v = [2 * g + f1, 2 * g + 1 - f1, 2 * (1 - g) + f2, 2 * (1 - g) + 1 - f2]
        for k in (3, 2, 1, 0):
            if hit[v[k]]:
                stack.append(recs[v[k]])
    return out


def _mesh(rt, preset):
    scene, cam, st, fc, post = rt.load_preset(preset, 32, 32)
    d = scene.desc()
    return scene, d


def test_mesh_bvh4_keeps_bvh2_leaf_order(rt):
    lib = rt.lib()
    scene, d = _mesh(rt, "c3")
    m = d.meshes[0]
    nodes = m.nodes
    cnt, root = C.c_uint32(), C.c_uint32()
    assert lib.rt_debug_mesh_bvh4(nodes, m.node_count, None, 0, C.byref(cnt), C.byref(root)) == 0
    # a BVH4 node absorbs an interior BVH2 node and its interior children: about half of
    # the BVH2's interior nodes (which are half of all its nodes)
    assert m.node_count // 8 < cnt.value < m.node_count // 2
    buf = (C.c_float * (32 * cnt.value))()
    assert lib.rt_debug_mesh_bvh4(nodes, m.node_count, buf, cnt.value, C.byref(cnt), C.byref(root)) == 0
    q = np.frombuffer(buf, dtype=np.float32).reshape(cnt.value, 32).astype(np.float64)
    qb = np.frombuffer(buf, dtype=np.uint32).reshape(cnt.value, 32)     # records and axes as bits
    box_p, box_r = _node_box(nodes[0])
    rng = np.random.default_rng(17)
    total = same = 0
    for i in range(150):
        o = box_p + box_r * rng.uniform(-1.6, 1.6, 3)
        d = rng.normal(size=3)
        axis_parallel = i % 10 == 0
        if axis_parallel:
            d[i // 10 % 3] = 0.0
        d /= np.linalg.norm(d)
        with np.errstate(divide="ignore"):
            inv_d = 1.0 / d
        a = _bvh2_leaves(nodes, o, d, inv_d)
        b = _bvh4_leaves(q, qb, root.value, nodes, o, d, inv_d)
        # the reference's leaves, in the reference's order
        assert [x for x in b if x in a] == a
        if axis_parallel:
            # d == 0 on an axis makes that slab NaN, and the ternary max/min then drop a
            # NEIGHBOURING slab's bound too, depending on the NaN's position: a child can
            # pass where its parent fails.  Skipping the merged level's test then visits
            # extra nodes -- never fewer, so no hit the reference finds is lost, and the
            # extra ones lie outside the ray's geometric path (test_gpu_parity.py
            # test_axis_parallel_rays_bit_exact checks the hits on the GPU).
            continue
        total += 1
        same += a == b
    assert same >= 0.99 * total


def _walk_sequence(seq, bits, length, passes):
    """The prologue's walk: entries failing `passes` jump past their subtree."""
    out, i = [], 0
    while i < length:
        e = seq[8 * i: 8 * i + 8]
        key = tuple(np.round(e[:6], 6))
        info, skip = int(bits[8 * i + 6]), int(bits[8 * i + 7])
        if not passes(key):
            i = skip
            continue
        out.append(key)
        i = skip if info >> 31 else i + 1
    return out


def _walk_reference(nodes, octant, passes):
    out, stack = [], [0]
    while stack:
        n = nodes[stack.pop()]
        key = tuple(np.round(np.array([n.bv_p.x, n.bv_p.y, n.bv_p.z, n.bv_r.x, n.bv_r.y, n.bv_r.z],
                                      dtype=np.float32).astype(np.float64), 6))
        if not passes(key):
            continue
        out.append(key)
        if n.count:
            continue
        if (octant >> n.split_axis) & 1:
            stack += [n.left_first, n.left_first + 1]
        else:
            stack += [n.left_first + 1, n.left_first]
    return out


@pytest.mark.parametrize("preset", ["c3", "c4", "platforms"])
def test_top_sequences_match_reference_walk(rt, preset):
    lib = rt.lib()
    scene, d = _mesh(rt, preset)
    n = C.c_uint32()
    assert lib.rt_debug_top_sequences(d.bvh_nodes, d.bvh_node_count, d.bvh_index_count, None, 0, C.byref(n)) == 0
    assert n.value >= 1
    buf = (C.c_float * (8 * 8 * n.value))()
    assert lib.rt_debug_top_sequences(d.bvh_nodes, d.bvh_node_count, d.bvh_index_count, buf, 8 * n.value,
                                      C.byref(n)) == 0
    seqs = np.frombuffer(buf, dtype=np.float32).astype(np.float64).reshape(8, 8 * n.value)
    bits = np.frombuffer(buf, dtype=np.uint32).reshape(8, 8 * n.value)
    rng = np.random.default_rng(3)
    for trial in range(40):
        salt = int(rng.integers(1 << 30))
        keep = 0.5 if trial else 1.0
        passes = (lambda key, salt=salt, keep=keep:
                  keep >= 1.0 or (hash((key, salt)) % 1000) / 1000.0 < keep)
        for octant in range(8):
            assert _walk_sequence(seqs[octant], bits[octant], n.value, passes) == \
                _walk_reference(d.bvh_nodes, octant, passes)
