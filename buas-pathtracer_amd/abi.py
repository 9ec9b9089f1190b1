"""ctypes mirror of include/rt_abi.h and include/rt_host.h.

The structs below are field-for-field copies of the C ABI (which in turn
mirrors the reference's Material / Primitive / Camera / SceneSettings /
FilterCache / AccumulationBuffer, RT/scene.h:15-120, RT/Raytracer.h:34-48).
No torch types cross the boundary: pointers and sizes only.
"""
import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "librt_mi355x.so")

RT_OK = 0
RT_ERROR_INVALID = 1
RT_ERROR_DEVICE = 2
RT_ERROR_OUT_OF_MEMORY = 3
RT_ERROR_CANCELLED = 4
RT_ERROR_NO_DEVICE = 5

RT_MATERIAL_MIRROR = 0x1
RT_MATERIAL_CHECKERS = 0x2
RT_MATERIAL_EMISSIVE = 0x4

RT_PRIMITIVE_NONE, RT_PRIMITIVE_PLANE, RT_PRIMITIVE_SPHERE, RT_PRIMITIVE_BOX, RT_PRIMITIVE_MESH = range(5)
RT_SAMPLING_UNIFORM, RT_SAMPLING_OPTIMIZED_BLUE_NOISE, RT_SAMPLING_STRATIFIED = range(3)
RT_SPLAT_STREAM, RT_SPLAT_EXACT, RT_SPLAT_ATOMIC = range(3)          # rt_splat_mode
RT_SHARD_TILES, RT_SHARD_PASSES = range(2)                           # rt_shard_mode
RT_SHADOW_LAUNCH_AUTO, RT_SHADOW_LAUNCH_SEPARATE, RT_SHADOW_LAUNCH_MERGED = range(3)   # rt_shadow_launch (ABI 8)
RT_RNG_PER_SAMPLE, RT_RNG_TILE_STREAM = 0, 1
RT_HIT_MISS = 0xFFFFFFFF
RT_HIT_PLANE_BIT = 0x80000000
RTH_BVH_MIDPOINT_SPLIT, RTH_BVH_SAH_BINNED, RTH_BVH_SAH_FULL = range(3)

RT_KERNEL_NAMES = ("generate", "extend", "shade", "connect", "splat", "resolve")
RT_KERNEL_COUNT = 6


class V3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]

    def __iter__(self):
        return iter((self.x, self.y, self.z))

    def __repr__(self):
        return f"V3({self.x}, {self.y}, {self.z})"


def v3(x, y=None, z=None):
    if y is None:
        return V3(x, x, x)
    return V3(x, y, z)


class M4x4(C.Structure):
    _fields_ = [("e", (C.c_float * 4) * 4)]


class M4x4Inv(C.Structure):
    _fields_ = [("forward", M4x4), ("inverse", M4x4)]


class Material(C.Structure):          # RT/scene.h:15-29
    _fields_ = [("flags", C.c_uint32), ("albedo", V3), ("checker_color", V3), ("emission_color", V3),
                ("ior", C.c_float), ("metallic", C.c_float), ("roughness", C.c_float),
                ("is_participating_medium", C.c_int32), ("absorb", V3)]


class Primitive(C.Structure):         # RT/primitives.h:92-106
    _fields_ = [("transform_index", C.c_uint32), ("material_id", C.c_uint32), ("type", C.c_uint32),
                ("mesh_index", C.c_uint32), ("p", C.c_float * 4)]


class BvhNode(C.Structure):           # RT/bvh.h:31-37
    _fields_ = [("bv_p", V3), ("bv_r", V3), ("left_first", C.c_uint32), ("count", C.c_uint16),
                ("split_axis", C.c_uint16)]


class Mesh(C.Structure):
    _fields_ = [("triangle_count", C.c_uint32), ("has_normals", C.c_uint32),
                ("triangles", C.POINTER(V3)), ("indices", C.POINTER(C.c_uint32)),
                ("normals", C.POINTER(V3)), ("node_count", C.c_uint32), ("nodes", C.POINTER(BvhNode))]


class SceneDesc(C.Structure):         # RT/scene.h:92-120
    _fields_ = [("material_count", C.c_uint32), ("materials", C.POINTER(Material)),
                ("primitive_count", C.c_uint32), ("primitives", C.POINTER(Primitive)),
                ("plane_count", C.c_uint32), ("planes", C.POINTER(Primitive)),
                ("transform_count", C.c_uint32), ("transforms", C.POINTER(M4x4Inv)),
                ("light_count", C.c_uint32), ("lights", C.POINTER(C.c_uint32)),
                ("mesh_count", C.c_uint32), ("meshes", C.POINTER(Mesh)),
                ("bvh_node_count", C.c_uint32), ("bvh_nodes", C.POINTER(BvhNode)),
                ("bvh_index_count", C.c_uint32), ("bvh_indices", C.POINTER(C.c_uint32)),
                ("top_sky_color", V3), ("bot_sky_color", V3),
                ("skydome_w", C.c_uint32), ("skydome_h", C.c_uint32), ("skydome", C.POINTER(V3))]


class Camera(C.Structure):            # RT/scene.h:31-46
    _fields_ = [("p", V3), ("x", V3), ("y", V3), ("z", V3), ("vfov", C.c_float), ("aspect_ratio", C.c_float),
                ("lens_radius", C.c_float), ("focus_distance", C.c_float), ("film_distance", C.c_float),
                ("half_film_w", C.c_float), ("half_film_h", C.c_float)]


class Settings(C.Structure):          # RT/scene.h:64-82
    _fields_ = [("next_event_estimation", C.c_int32), ("importance_sample_lights", C.c_int32),
                ("importance_sample_diffuse", C.c_int32), ("use_mis", C.c_int32),
                ("russian_roulette", C.c_int32), ("caustics", C.c_int32),
                ("sampling_strategy", C.c_int32), ("use_path_guide", C.c_int32),
                ("vignette_strength", C.c_float), ("lens_distortion", C.c_float), ("f_factor", C.c_float),
                ("diaphragm_edges", C.c_float), ("phi_shutter_max", C.c_float),
                ("samples_per_pixel", C.c_uint32), ("max_bounce_count", C.c_uint32), ("integrator", C.c_int32)]


class FilterCache(C.Structure):       # RT/Raytracer.h:34-40
    _fields_ = [("kernel_size", C.c_uint32), ("cache_size", C.c_uint32), ("cache", C.c_float * 512)]


class AccumulationBuffer(C.Structure):  # RT/Raytracer.h:44-48
    _fields_ = [("w", C.c_uint32), ("h", C.c_uint32), ("frame_count", C.c_uint32), ("pixels", C.POINTER(C.c_float))]


class TileSet(C.Structure):
    _fields_ = [("tile_w", C.c_uint32), ("tile_h", C.c_uint32), ("shard_index", C.c_uint32), ("shard_count", C.c_uint32)]


TRAVERSAL_FIELDS = ("mesh_intersection_count", "mesh_bvh_traversals", "mesh_node_traversals", "mesh_leaf_traversals")


class TraversalStats(C.Structure):    # TraversalStats RT/intersection.h:33-40 (rt_traversal_stats)
    _fields_ = [(f, C.c_uint64) for f in TRAVERSAL_FIELDS]

    def as_dict(self):
        return {f: getattr(self, f) for f in TRAVERSAL_FIELDS}


class Stats(C.Structure):
    _fields_ = [("closest_hit_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("samples", C.c_uint64),
                ("iterations", C.c_uint64), ("seconds", C.c_double),
                ("kernel_ms", C.c_double * RT_KERNEL_COUNT), ("kernel_launches", C.c_uint64 * RT_KERNEL_COUNT),
                ("traced_rays", C.c_uint64 * 2), ("splat_mode", C.c_int32), ("shadow_launch", C.c_int32),
                ("traversal", TraversalStats * 2), ("trace_steps", C.c_uint64 * 2),
                ("traversal_ref", TraversalStats * 2)]       # ABI 7: rt_scene_config::traversal_ref

    def traversal_total(self):
        """The reference's TraversalStats: both query kinds summed."""
        return {f: getattr(self.traversal[0], f) + getattr(self.traversal[1], f) for f in TRAVERSAL_FIELDS}

    def as_dict(self):
        return {"closest_hit_rays": self.closest_hit_rays, "shadow_rays": self.shadow_rays,
                "samples": self.samples, "iterations": self.iterations, "seconds": self.seconds,
                "kernel_ms": {RT_KERNEL_NAMES[i]: self.kernel_ms[i] for i in range(6)},
                "kernel_launches": {RT_KERNEL_NAMES[i]: self.kernel_launches[i] for i in range(6)},
                "traced_rays": [self.traced_rays[0], self.traced_rays[1]], "splat_mode": self.splat_mode,
                "traversal": [self.traversal[0].as_dict(), self.traversal[1].as_dict()],
                "trace_steps": [self.trace_steps[0], self.trace_steps[1]],
                "traversal_ref": [self.traversal_ref[0].as_dict(), self.traversal_ref[1].as_dict()]}


class RayQuery(C.Structure):
    _fields_ = [("o", V3), ("d", V3), ("max_t", C.c_float), ("ignored_primitive", C.c_uint32)]


class HitRecord(C.Structure):
    _fields_ = [("t", C.c_float), ("primitive", C.c_uint32), ("hit_p", V3), ("n", V3)]


class PostSettings(C.Structure):      # RT/scene.h:84-90
    _fields_ = [("exposure", C.c_float), ("tonemapping", C.c_int32), ("srgb_transform", C.c_int32),
                ("midpoint", C.c_float), ("contrast", C.c_float)]


RT_CONFIG_INHERIT = -1


class SceneConfig(C.Structure):       # rt_scene_config (per-scene schedule and splat settings)
    _fields_ = [("splat_mode", C.c_int32), ("shard_mode", C.c_int32), ("env_sampling", C.c_int32),
                ("partitions", C.c_int32), ("path_pool", C.c_int64), ("fuse_paths", C.c_int64),
                ("splat_chunk", C.c_int32), ("splat_ring", C.c_int32), ("sample_budget_gb", C.c_double),
                ("resolve_tall_pixels", C.c_int64), ("debug_traversal", C.c_int32), ("traversal_ref", C.c_int32),
                ("drain_every", C.c_int32), ("shadow_launch", C.c_int32),  # ABI 8
                ("reserved", C.c_int32 * 4)]


class BvhInfo(C.Structure):
    _fields_ = [("node_count", C.c_uint32), ("leaf_count", C.c_uint32), ("max_depth", C.c_uint32),
                ("max_leaf_size", C.c_uint32)]


P = C.POINTER

# name -> (restype, argtypes)
ABI_FUNCTIONS = {
    "rt_abi_version": (C.c_int, []),
    "rt_last_error": (C.c_char_p, []),
    "rt_device_count": (C.c_int, [P(C.c_int)]),
    "rt_scene_upload": (C.c_int, [P(SceneDesc), C.c_int, P(C.c_void_p)]),
    "rt_scene_free": (C.c_int, [C.c_void_p]),
    "rt_render": (C.c_int, [C.c_void_p, P(Camera), P(Settings), P(FilterCache), P(TileSet), C.c_uint32,
                            P(AccumulationBuffer), P(Stats)]),
    "rt_render_device": (C.c_int, [C.c_void_p, P(Camera), P(Settings), P(FilterCache), P(TileSet), C.c_uint32,
                                   C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, P(Stats)]),
    "rt_trace_samples": (C.c_int, [C.c_void_p, P(Camera), P(Settings), C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P(C.c_uint32), P(C.c_uint32),
                                   P(C.c_float), P(Stats)]),
    "rt_debug_intersect": (C.c_int, [C.c_void_p, C.c_uint32, P(RayQuery), C.c_int, P(HitRecord)]),
    "rt_debug_mesh_bvh4": (C.c_int, [P(BvhNode), C.c_uint32, P(C.c_float), C.c_uint32, P(C.c_uint32),
                                     P(C.c_uint32)]),
    "rt_debug_top_sequences": (C.c_int, [P(BvhNode), C.c_uint32, C.c_uint32, P(C.c_float), C.c_uint32,
                                         P(C.c_uint32)]),
    "rt_debug_verify_rcp": (C.c_int, [C.c_int, P(C.c_uint64), P(C.c_uint32)]),
    "rt_set_profiling": (C.c_int, [C.c_int]),
    "rt_set_profiling_stages": (C.c_int, [C.c_uint32]),
    "rt_set_path_pool": (C.c_int, [C.c_uint32]),
    "rt_set_splat_mode": (C.c_int, [C.c_int]),
    "rt_set_shard_mode": (C.c_int, [C.c_int]),
    "rt_set_env_sampling": (C.c_int, [C.c_int]),
    "rt_build_bvh": (C.c_int, [C.c_int, C.c_uint32, P(V3), P(V3), C.c_int, P(BvhNode), P(C.c_uint32), P(C.c_uint32)]),
    "rt_build_bvh_last_error": (C.c_char_p, []),
    "rt_render_picture": (C.c_int, [C.c_void_p, P(Camera), P(Settings), P(FilterCache), P(TileSet), C.c_uint32,
                                    C.c_uint32, C.c_uint32, P(PostSettings), P(C.c_uint32), P(Stats)]),
    "rt_cancel": (C.c_int, [C.c_void_p]),
    "rt_scene_default_config": (C.c_int, [P(SceneConfig)]),
    "rt_scene_get_config": (C.c_int, [C.c_void_p, P(SceneConfig)]),
    "rt_scene_set_config": (C.c_int, [C.c_void_p, P(SceneConfig)]),
    "rt_postprocess_device": (C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_uint32, P(PostSettings), C.c_uint32,
                                        C.c_void_p, C.c_void_p]),
    "rt_postprocess": (C.c_int, [C.c_int, P(AccumulationBuffer), P(PostSettings), C.c_uint32, P(C.c_uint32)]),
}

HOST_FUNCTIONS = {
    "rth_last_error": (C.c_char_p, []),
    "rth_scene_create": (C.c_void_p, []),
    "rth_scene_destroy": (None, [C.c_void_p]),
    "rth_add_material": (C.c_uint32, [C.c_void_p, P(Material)]),
    "rth_add_diffuse_material": (C.c_uint32, [C.c_void_p, V3, C.c_float, C.c_float, C.c_int32, V3]),
    "rth_add_translucent_material": (C.c_uint32, [C.c_void_p, V3, C.c_float, C.c_float]),
    "rth_add_emissive_material": (C.c_uint32, [C.c_void_p, V3]),
    "rth_add_plane": (C.c_uint32, [C.c_void_p, C.c_uint32, V3, C.c_float]),
    "rth_add_sphere": (C.c_uint32, [C.c_void_p, C.c_uint32, C.c_float, P(M4x4Inv)]),
    "rth_add_box": (C.c_uint32, [C.c_void_p, C.c_uint32, V3, P(M4x4Inv)]),
    "rth_add_mesh": (C.c_uint32, [C.c_void_p, C.c_uint32, C.c_uint32, P(M4x4Inv)]),
    "rth_create_mesh": (C.c_uint32, [C.c_void_p, C.c_uint32, P(V3), P(V3), C.c_int32]),
    "rth_load_obj_mesh": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32, P(C.c_uint32)]),
    "rth_mesh_bvh_info": (C.c_int, [C.c_void_p, C.c_uint32, P(BvhInfo)]),
    "rth_scene_bvh_info": (C.c_int, [C.c_void_p, P(BvhInfo)]),
    "rth_set_sky": (None, [C.c_void_p, V3, V3]),
    "rth_load_environment_map": (C.c_int, [C.c_void_p, C.c_char_p]),
    "rth_set_environment_map": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(V3)]),
    "rth_create_scene_bvh": (C.c_int, [C.c_void_p]),
    "rth_set_bvh_device": (None, [C.c_int]),
    "rth_build_bvh_entries": (C.c_int, [C.c_uint32, P(V3), P(V3), C.c_int32, P(BvhNode), P(C.c_uint32), P(C.c_uint32)]),
    "rth_scene_desc": (P(SceneDesc), [C.c_void_p]),
    "rth_transform_identity": (M4x4Inv, []),
    "rth_transform_translate": (M4x4Inv, [V3]),
    "rth_transform_scale": (M4x4Inv, [V3]),
    "rth_transform_rotate_x_axis": (M4x4Inv, [C.c_float]),
    "rth_transform_rotate_y_axis": (M4x4Inv, [C.c_float]),
    "rth_transform_rotate_z_axis": (M4x4Inv, [C.c_float]),
    "rth_transform_mul": (M4x4Inv, [M4x4Inv, M4x4Inv]),
    "rth_aim_camera": (None, [P(Camera), V3]),
    "rth_aim_camera_at": (None, [P(Camera), V3]),
    "rth_recompute_camera": (None, [P(Camera)]),
    "rth_default_settings": (None, [P(Settings), P(PostSettings)]),
    "rth_load_reconstruction_kernel": (None, [C.c_char_p, P(FilterCache)]),
    "rth_load_preset": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, C.c_char_p, P(C.c_void_p), P(Camera),
                                  P(Settings), P(FilterCache), P(PostSettings)]),
    "rth_generate_mesh": (C.c_uint32, [C.c_uint32, C.c_uint32, P(V3), P(V3)]),
    "rth_write_synthetic_obj": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32]),
    "rth_write_synthetic_hdr": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32]),
    "rth_resolve_bgra8": (None, [P(AccumulationBuffer), P(PostSettings), P(C.c_uint32)]),
    "rth_write_bitmap": (C.c_int, [C.c_char_p, P(C.c_uint32), C.c_uint32, C.c_uint32]),
    "rth_take_picture": (C.c_int, [C.c_void_p, P(Camera), P(Settings), P(FilterCache), P(PostSettings),
                                   C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_char_p, P(Stats)]),
    "rth_read_bitmap": (C.c_int, [C.c_char_p, P(C.c_uint32), C.c_uint32, C.c_uint32]),
}


def bind(lib, table):
    for name, (res, args) in table.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None


def load_library(path=None):
    """Load librt_mi355x.so.  There is no fallback: a missing library is an error.

    RT_MI355X_LIB names another build of the same library (tuning variants)."""
    global _LIB
    if path is None:
        path = os.environ.get("RT_MI355X_LIB") or LIB_PATH
    if _LIB is None:
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: run __graft_entry__.build() (make -C buas-pathtracer_amd/csrc)")
        lib = C.CDLL(path)
        bind(lib, ABI_FUNCTIONS)
        bind(lib, HOST_FUNCTIONS)
        _LIB = lib
    return _LIB
