"""ctypes binding of oracle/liboracle.so (the CPU restatement — TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes as C
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    import importlib
    import sys
    abi = sys.modules["buas_pathtracer_amd"].abi if "buas_pathtracer_amd" in sys.modules else importlib.import_module("buas_pathtracer_amd").abi
    if not os.path.exists(LIB):
        raise RuntimeError(f"{LIB} missing: run make -C oracle (or __graft_entry__.build())")
    lib = C.CDLL(LIB)
    P = C.POINTER
    fns = {
        "oracle_render": (C.c_int, [P(abi.SceneDesc), P(abi.Camera), P(abi.Settings), P(abi.FilterCache),
                                    P(abi.TileSet), C.c_uint32, C.c_int, C.c_int, P(abi.AccumulationBuffer),
                                    P(abi.Stats)]),
        "oracle_render_tiles": (C.c_int, [P(abi.SceneDesc), P(abi.Camera), P(abi.Settings), P(abi.FilterCache),
                                          C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_uint32,
                                          P(C.c_uint32), P(abi.AccumulationBuffer), P(abi.Stats)]),
        "oracle_trace_samples": (C.c_int, [P(abi.SceneDesc), P(abi.Camera), P(abi.Settings), C.c_uint32,
                                           C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                           C.c_uint32, P(C.c_uint32), P(C.c_uint32), P(C.c_float),
                                           P(abi.Stats)]),
        "oracle_debug_intersect": (C.c_int, [P(abi.SceneDesc), C.c_uint32, P(abi.RayQuery), C.c_int,
                                             P(abi.HitRecord)]),
        "oracle_wang_hash": (C.c_uint32, [C.c_uint32]),
        "oracle_sample_seed": (C.c_uint32, [C.c_uint32] * 5),
        "oracle_rng_unilaterals": (None, [C.c_uint32, C.c_uint32, P(C.c_float)]),
        "oracle_sample_2d": (None, [C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                    C.c_uint32, P(C.c_float)]),
        "oracle_sample_1d": (C.c_float, [C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                         C.c_uint32]),
        "oracle_ray_intersect_plane": (C.c_int, [P(C.c_float), P(C.c_float), P(C.c_float), C.c_float,
                                                 P(C.c_float)]),
        "oracle_ray_intersect_sphere": (C.c_int, [P(C.c_float), P(C.c_float), C.c_float, P(C.c_float)]),
        "oracle_sinf": (C.c_float, [C.c_float]),
        "oracle_cosf": (C.c_float, [C.c_float]),
        "oracle_expf": (C.c_float, [C.c_float]),
        "oracle_logf": (C.c_float, [C.c_float]),
        "oracle_atan2f": (C.c_float, [C.c_float, C.c_float]),
        "oracle_asinf": (C.c_float, [C.c_float]),
        "oracle_set_math_mode": (None, [C.c_int]),
        "oracle_set_env_sampling": (None, [C.c_int]),
        "oracle_load_filter": (C.c_int, [C.c_char_p, P(abi.FilterCache)]),
        "oracle_postprocess": (None, [P(abi.AccumulationBuffer), P(abi.PostSettings), C.c_uint32, P(C.c_uint32)]),
        "oracle_gpu_walk_stats": (None, [C.c_int, C.c_uint32, C.c_int]),
        "oracle_gpu_walk_result": (None, [P(C.c_uint64)]),
    }
    for name, (res, args) in fns.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def render(desc, cam, st, fc, w, h, rng_mode=0, threads=1, tile=64, shard_index=0, shard_count=1,
           frame_count=0, total_frame_index=0, accum=None):
    import numpy as np
    import sys
    abi = sys.modules["buas_pathtracer_amd"].abi
    lib = load()
    if accum is None:
        accum = np.zeros((h, w, 4), np.float32)
    buf = abi.AccumulationBuffer(w, h, frame_count, accum.ctypes.data_as(C.POINTER(C.c_float)))
    tiles = abi.TileSet(tile, tile, shard_index, shard_count)
    stats = abi.Stats()
    err = lib.oracle_render(C.byref(desc), C.byref(cam), C.byref(st), C.byref(fc), C.byref(tiles),
                            total_frame_index, rng_mode, threads, C.byref(buf), C.byref(stats))
    assert err == 0, err
    return accum, stats


def trace_samples(desc, cam, st, w, h, xy, s, frame_count=0, total_frame_index=0, tile=64):
    import numpy as np
    import sys
    abi = sys.modules["buas_pathtracer_amd"].abi
    lib = load()
    xy = np.ascontiguousarray(xy, np.uint32).reshape(-1, 2)
    s = np.ascontiguousarray(s, np.uint32).reshape(-1)
    out = np.zeros((xy.shape[0], 5), np.float32)
    stats = abi.Stats()
    err = lib.oracle_trace_samples(C.byref(desc), C.byref(cam), C.byref(st), w, h, tile, tile, frame_count,
                                   total_frame_index, xy.shape[0], xy.ctypes.data_as(C.POINTER(C.c_uint32)),
                                   s.ctypes.data_as(C.POINTER(C.c_uint32)), out.ctypes.data_as(C.POINTER(C.c_float)),
                                   C.byref(stats))
    assert err == 0, err
    return out, stats


def intersect(desc, rays, occlusion=False):
    import sys
    abi = sys.modules["buas_pathtracer_amd"].abi
    n = len(rays)
    q = (abi.RayQuery * n)(*rays)
    out = (abi.HitRecord * n)()
    assert load().oracle_debug_intersect(C.byref(desc), n, q, int(bool(occlusion)), out) == 0
    return list(out)


def postprocess(accum, post, total_frame_index=0):
    """oracle_postprocess: the reference's output pass (RT/raytracer.cpp:2103-2171) -> BGRA8 (h, w) u32."""
    import numpy as np
    import sys
    abi = sys.modules["buas_pathtracer_amd"].abi
    accum = np.ascontiguousarray(accum, np.float32)
    h, w, _ = accum.shape
    out = np.zeros((h, w), np.uint32)
    buf = abi.AccumulationBuffer(w, h, 0, accum.ctypes.data_as(C.POINTER(C.c_float)))
    load().oracle_postprocess(C.byref(buf), C.byref(post), total_frame_index, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out


class env_sampling:
    """with env_sampling(1): oracle renders with environment-map NEE (oracle_set_env_sampling)."""

    def __init__(self, mode=1):
        self.mode = mode

    def __enter__(self):
        load().oracle_set_env_sampling(self.mode)
        return self

    def __exit__(self, *exc):
        load().oracle_set_env_sampling(0)
        return False


class gpu_walk:
    """with gpu_walk() as g: the oracle's renders also restate the GPU library's own traversal walk
    (oracle_gpu_walk_stats); afterwards g.result = {"calls": [closest, shadow], "entries": [...],
    "leaves": [...], "nodes": [...], "bvh": [...]}: the GPU's rt_stats::traversal
    mesh_intersection_count, the mesh instances its trace kernels enter, its mesh_leaf_traversals,
    mesh_node_traversals (BVH4 nodes) and mesh_bvh_traversals (entries + nodes + triangle steps)."""

    def __init__(self, mlist_max=4, top_prologue=True):
        self.mlist_max, self.top = mlist_max, top_prologue
        self.result = None

    def __enter__(self):
        load().oracle_gpu_walk_stats(1, self.mlist_max, int(self.top))
        return self

    def __exit__(self, *exc):
        out = (C.c_uint64 * 10)()
        load().oracle_gpu_walk_result(out)
        load().oracle_gpu_walk_stats(0, 4, 1)
        g = lambda i: [int(out[i]), int(out[5 + i])]
        self.result = {"calls": g(0), "entries": g(1), "leaves": g(2), "nodes": g(3),
                       "bvh": [g(1)[k] + g(3)[k] + g(4)[k] for k in range(2)]}
        return False
