"""MI355X wavefront path tracer — Python host mirror of the reference's interface.

The hot path (render_tile -> advanced_integrator -> intersect_scene /
intersect_shadow_ray -> samplers -> splat_filter, RT/raytracer.cpp:366-495)
runs as gfx950 HIP kernels in lib/librt_mi355x.so behind the C ABI of
include/rt_abi.h.  This module is a thin ctypes host over that ABI and over
the scene model of include/rt_host.h, keeping the reference's names:

    scene = Scene()                         # clear_scene + init_scene
    m = scene.add_diffuse_material(...)     # RT/scene.cpp:23-37
    scene.add_sphere(m, 2.0, translate(...))
    scene.create_scene_bvh()                # RT/scene.cpp:173-242
    dev = DeviceScene(scene, device=0)      # rt_scene_upload
    acc = dev.render(camera, settings, filter_cache, w, h)   # render_all_tiles

There is no CPU fallback: without a visible MI355X, DeviceScene raises.
"""
import ctypes as C
import math

import numpy as np

from . import abi
from .abi import (V3, v3, M4x4Inv, Material, Camera, Settings, FilterCache, PostSettings, TileSet, Stats,
                  AccumulationBuffer, RayQuery, HitRecord, BvhInfo)

__all__ = ["Scene", "DeviceScene", "RenderError", "load_preset", "default_settings", "load_reconstruction_kernel",
           "translate", "scale", "rotate_x", "rotate_y", "rotate_z", "identity", "aim_camera", "aim_camera_at",
           "recompute_camera", "resolve_bgra8", "postprocess", "write_bitmap", "lib", "abi", "v3", "PI_32", "DEG_TO_RAD",
           "set_splat_mode", "splat_mode", "take_picture", "read_bitmap"]

PI_32 = 3.14159265359
DEG_TO_RAD = 6.28318530717 / 360.0


class RenderError(RuntimeError):
    def __init__(self, code, message):
        super().__init__(f"rt error {code}: {message}")
        self.code = code


def lib():
    return abi.load_library()


def _check(code):
    if code != abi.RT_OK:
        raise RenderError(code, (lib().rt_last_error() or b"").decode())


def _v(x):
    if isinstance(x, V3):
        return x
    x = tuple(x) if not isinstance(x, (int, float)) else (x, x, x)
    return V3(*[float(c) for c in x])


# ---- transforms (MathLib/my_math.h:1009-1069)
def identity():
    return lib().rth_transform_identity()


def translate(t):
    return lib().rth_transform_translate(_v(t))


def scale(s):
    return lib().rth_transform_scale(_v(s))


def rotate_x(a):
    return lib().rth_transform_rotate_x_axis(float(a))


def rotate_y(a):
    return lib().rth_transform_rotate_y_axis(float(a))


def rotate_z(a):
    return lib().rth_transform_rotate_z_axis(float(a))


def mul(a, b):
    return lib().rth_transform_mul(a, b)


M4x4Inv.__mul__ = lambda a, b: lib().rth_transform_mul(a, b)


# ---- camera (RT/raytracer.cpp:26-59)
def aim_camera(cam, d):
    lib().rth_aim_camera(C.byref(cam), _v(d))


def aim_camera_at(cam, at):
    lib().rth_aim_camera_at(C.byref(cam), _v(at))


def recompute_camera(cam):
    lib().rth_recompute_camera(C.byref(cam))


def default_settings():
    """init_scene defaults (RT/raytracer.cpp:1430-1452) -> (Settings, PostSettings)."""
    st, post = Settings(), PostSettings()
    lib().rth_default_settings(C.byref(st), C.byref(post))
    return st, post


def load_reconstruction_kernel(name="Mitchell Netravali"):
    """load_reconstruction_kernel(find_filter(name)) (RT/raytracer.cpp:164-185)."""
    fc = FilterCache()
    lib().rth_load_reconstruction_kernel(name.encode(), C.byref(fc))
    return fc


class Scene:
    """Host scene (RT/scene.h:92-120): materials, primitives, planes, lights, BVHs."""

    def __init__(self, handle=None):
        self._h = handle if handle is not None else lib().rth_scene_create()
        if not self._h:
            raise MemoryError("rth_scene_create failed")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            try:
                lib().rth_scene_destroy(h)
            except Exception:
                pass

    @property
    def handle(self):
        return self._h

    # materials (RT/scene.cpp:9-61)
    def add_material(self, flags=0, albedo=0.0, checker_color=0.0, emission_color=0.0, ior=0.0, metallic=0.0,
                     roughness=0.0, is_participating_medium=False, absorb=0.0):
        m = Material(flags, _v(albedo), _v(checker_color), _v(emission_color), ior, metallic, roughness,
                     int(bool(is_participating_medium)), _v(absorb))
        return lib().rth_add_material(self._h, C.byref(m))

    def add_diffuse_material(self, diffuse_color, ior, roughness=0.0, checkers=False, checker_color=0.1):
        return lib().rth_add_diffuse_material(self._h, _v(diffuse_color), float(ior), float(roughness),
                                              int(bool(checkers)), _v(checker_color))

    def add_translucent_material(self, absorb, ior, roughness=0.0):
        return lib().rth_add_translucent_material(self._h, _v(absorb), float(ior), float(roughness))

    def add_emissive_material(self, emission_color):
        return lib().rth_add_emissive_material(self._h, _v(emission_color))

    # primitives (RT/scene.cpp:70-159)
    def add_plane(self, material_id, n, d):
        return lib().rth_add_plane(self._h, material_id, _v(n), float(d))

    def add_sphere(self, material_id, r, transform=None):
        return lib().rth_add_sphere(self._h, material_id, float(r), C.byref(transform) if transform else None)

    def add_box(self, material_id, r, transform=None):
        return lib().rth_add_box(self._h, material_id, _v(r), C.byref(transform) if transform else None)

    def add_mesh(self, material_id, mesh_id, transform=None):
        return lib().rth_add_mesh(self._h, material_id, mesh_id, C.byref(transform) if transform else None)

    def create_mesh(self, triangles, normals=None, method=abi.RTH_BVH_SAH_BINNED):
        """triangles: float32 array [n,3,3]; normals: optional [n,3,3] (per-vertex)."""
        t = np.ascontiguousarray(triangles, dtype=np.float32).reshape(-1, 3, 3)
        n = None if normals is None else np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3, 3)
        mid = lib().rth_create_mesh(self._h, t.shape[0], t.ctypes.data_as(C.POINTER(V3)),
                                    None if n is None else n.ctypes.data_as(C.POINTER(V3)), method)
        if mid == 0xFFFFFFFF:
            raise RuntimeError(f"rth_create_mesh failed: {(lib().rth_last_error() or b'').decode()}")
        return mid

    def load_obj_mesh(self, path, method=abi.RTH_BVH_SAH_BINNED):
        out = C.c_uint32()
        if not lib().rth_load_obj_mesh(self._h, str(path).encode(), method, C.byref(out)):
            raise ValueError(lib().rth_last_error().decode())
        return out.value

    def set_sky(self, top, bot):
        lib().rth_set_sky(self._h, _v(top), _v(bot))

    def load_environment_map(self, path):
        if not lib().rth_load_environment_map(self._h, str(path).encode()):
            raise ValueError(lib().rth_last_error().decode())

    def set_environment_map(self, pixels):
        """An environment map from an (h, w, 3) float32 array (row 0 = v = 0, the bottom)."""
        a = np.ascontiguousarray(pixels, dtype=np.float32)
        h, w = a.shape[:2]
        if not lib().rth_set_environment_map(self._h, w, h, a.ctypes.data_as(C.POINTER(abi.V3))):
            raise ValueError(lib().rth_last_error().decode())

    def create_scene_bvh(self):
        if not lib().rth_create_scene_bvh(self._h):
            raise RuntimeError(f"rth_create_scene_bvh failed: {(lib().rth_last_error() or b'').decode()}")

    def bvh_info(self, mesh_id=None):
        info = BvhInfo()
        if mesh_id is None:
            lib().rth_scene_bvh_info(self._h, C.byref(info))
        else:
            lib().rth_mesh_bvh_info(self._h, mesh_id, C.byref(info))
        return {k: getattr(info, k) for k, _ in BvhInfo._fields_}

    def desc(self):
        """The flattened scene (rt_scene_desc).  Its arrays point into this host scene, so the
        returned struct keeps the Scene alive (`Scene(...).desc()` on a temporary is safe)."""
        d = lib().rth_scene_desc(self._h).contents
        d._scene = self
        return d


def load_preset(name, w, h, asset_dir=None):
    """load_scene(g_scenes[...]) or a BASELINE config ('c1'..'c5').
    Returns (Scene, Camera, Settings, FilterCache, PostSettings)."""
    handle = C.c_void_p()
    cam, st, fc, post = Camera(), Settings(), FilterCache(), PostSettings()
    ok = lib().rth_load_preset(name.encode(), w, h, asset_dir.encode() if asset_dir else None, C.byref(handle),
                               C.byref(cam), C.byref(st), C.byref(fc), C.byref(post))
    if not ok:
        why = lib().rth_last_error()
        why = why.decode() if isinstance(why, bytes) else why
        raise ValueError(f"preset {name!r}: " + (why or "unknown preset"))
    return Scene(handle.value), cam, st, fc, post


class DeviceScene:
    """A scene resident on one MI355X (rt_scene_upload)."""

    def __init__(self, scene, device=0):
        self.scene = scene          # keep the host arrays alive
        self.device = device
        h = C.c_void_p()
        _check(lib().rt_scene_upload(C.byref(scene.desc()), device, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().rt_scene_free(self._h)
            self._h = C.c_void_p()

    __del__ = close

    def render(self, camera, settings, filter_cache, w, h, accum=None, frame_count=0, total_frame_index=0,
               tile=64, shard_index=0, shard_count=1):
        """rt_render: adds one frame into `accum` (float32 [h,w,4], host) and returns (accum, stats)."""
        if accum is None:
            accum = np.zeros((h, w, 4), np.float32)
        assert accum.dtype == np.float32 and accum.flags.c_contiguous and accum.shape == (h, w, 4)
        buf = AccumulationBuffer(w, h, frame_count, accum.ctypes.data_as(C.POINTER(C.c_float)))
        tiles = TileSet(tile, tile, shard_index, shard_count)
        stats = Stats()
        _check(lib().rt_render(self._h, C.byref(camera), C.byref(settings), C.byref(filter_cache), C.byref(tiles),
                               total_frame_index, C.byref(buf), C.byref(stats)))
        return accum, stats

    def render_device(self, camera, settings, filter_cache, w, h, d_pixels, stream=None, frame_count=0,
                      total_frame_index=0, tile=64, shard_index=0, shard_count=1):
        """rt_render_device into a device pointer (e.g. torch tensor .data_ptr())."""
        tiles = TileSet(tile, tile, shard_index, shard_count)
        stats = Stats()
        _check(lib().rt_render_device(self._h, C.byref(camera), C.byref(settings), C.byref(filter_cache),
                                      C.byref(tiles), total_frame_index, w, h, frame_count, C.c_void_p(d_pixels),
                                      C.c_void_p(stream) if stream else None, C.byref(stats)))
        return stats

    def trace_samples(self, camera, settings, w, h, pixel_xy, sample_offset, frame_count=0, total_frame_index=0,
                      tile=64):
        xy = np.ascontiguousarray(pixel_xy, np.uint32).reshape(-1, 2)
        s = np.ascontiguousarray(sample_offset, np.uint32).reshape(-1)
        out = np.zeros((xy.shape[0], 5), np.float32)
        stats = Stats()
        _check(lib().rt_trace_samples(self._h, C.byref(camera), C.byref(settings), w, h, tile, tile, frame_count,
                                      total_frame_index, xy.shape[0], xy.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      s.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(stats)))
        return out, stats

    def intersect(self, rays, occlusion=False):
        n = len(rays)
        q = (RayQuery * n)(*rays)
        out = (HitRecord * n)()
        _check(lib().rt_debug_intersect(self._h, n, q, int(bool(occlusion)), out))
        return list(out)

    def cancel(self):
        lib().rt_cancel(self._h)

    def config(self):
        """rt_scene_get_config: this scene's schedule and splat settings (abi.SceneConfig)."""
        c = abi.SceneConfig()
        _check(lib().rt_scene_get_config(self._h, C.byref(c)))
        return c

    def configure(self, **fields):
        """rt_scene_set_config with the named fields changed, e.g. configure(partitions=1,
        splat_mode=abi.RT_SPLAT_EXACT).  Returns the previous configuration (pass it to
        set_config to restore it)."""
        old = self.config()
        c = abi.SceneConfig.from_buffer_copy(old)
        for k, v in fields.items():
            if k not in dict(abi.SceneConfig._fields_):
                raise AttributeError(f"rt_scene_config has no field {k!r}")
            setattr(c, k, v)
        self.set_config(c)
        return old

    def set_config(self, c):
        _check(lib().rt_scene_set_config(self._h, C.byref(c)))

    def configured(self, **fields):
        """with dev.configured(partitions=1): ... -- the scene's configuration restored after."""
        dev = self

        class _Ctx:
            def __enter__(self):
                self.old = dev.configure(**fields)
                return dev

            def __exit__(self, *exc):
                dev.set_config(self.old)
                return False
        return _Ctx()


def resolve_bgra8(accum, post):
    h, w, _ = accum.shape
    out = np.zeros((h, w), np.uint32)
    buf = AccumulationBuffer(w, h, 0, accum.ctypes.data_as(C.POINTER(C.c_float)))
    lib().rth_resolve_bgra8(C.byref(buf), C.byref(post), out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out


def postprocess(accum, post, total_frame_index=0, device=0):
    """The output pass on the GPU (rt_postprocess; RT/raytracer.cpp:2103-2171): host float4 (h, w, 4) in,
    BGRA8 (h, w) u32 out, with the reference's TPDF blue-noise dither."""
    accum = np.ascontiguousarray(accum, np.float32)
    h, w, _ = accum.shape
    out = np.zeros((h, w), np.uint32)
    buf = AccumulationBuffer(w, h, 0, accum.ctypes.data_as(C.POINTER(C.c_float)))
    _check(lib().rt_postprocess(device, C.byref(buf), C.byref(post), total_frame_index,
                                out.ctypes.data_as(C.POINTER(C.c_uint32))))
    return out


def write_bitmap(path, bgra):
    h, w = bgra.shape
    b = np.ascontiguousarray(bgra, np.uint32)
    if not lib().rth_write_bitmap(str(path).encode(), b.ctypes.data_as(C.POINTER(C.c_uint32)), w, h):
        raise OSError(lib().rth_last_error().decode())


def set_splat_mode(mode):
    """rt_set_splat_mode: abi.RT_SPLAT_STREAM (default), RT_SPLAT_EXACT (the reference's splat
    order, bit-identical frames) or RT_SPLAT_ATOMIC."""
    _check(lib().rt_set_splat_mode(int(mode)))


def set_shard_mode(mode):
    """rt_set_shard_mode: abi.RT_SHARD_TILES (default: tile t to shard t % n) or RT_SHARD_PASSES
    (every tile, a contiguous range of the sample passes per shard)."""
    _check(lib().rt_set_shard_mode(int(mode)))


class splat_mode:
    """with splat_mode(abi.RT_SPLAT_EXACT): ... restores the default (streaming) splat after."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        set_splat_mode(self.mode)
        return self

    def __exit__(self, *exc):
        set_splat_mode(abi.RT_SPLAT_STREAM)
        return False


def set_env_sampling(mode):
    """rt_set_env_sampling: 1 = environment-map importance sampling in the NEE (beyond the
    reference, whose environment CDF is never read), 0 = the reference's estimator (default)."""
    _check(lib().rt_set_env_sampling(int(mode)))


class env_sampling:
    """with env_sampling(1): ... turns environment-map sampling off again after."""

    def __init__(self, mode=1):
        self.mode = mode

    def __enter__(self):
        set_env_sampling(self.mode)
        return self

    def __exit__(self, *exc):
        set_env_sampling(0)
        return False


def read_bitmap(path, w, h):
    """The BGRA8 pixels (h, w) u32 of a bitmap write_bitmap wrote."""
    out = np.zeros((h, w), np.uint32)
    if not lib().rth_read_bitmap(str(path).encode(), out.ctypes.data_as(C.POINTER(C.c_uint32)), w, h):
        raise OSError(lib().rth_last_error().decode())
    return out


def take_picture(scene, camera, settings, filter_cache, post, w, h, spp, path, total_frame_index=0, device=0):
    """rth_take_picture: the reference's "Take picture" (RT/raytracer.cpp:2031-2185) -> BMP at `path`."""
    stats = Stats()
    _check(lib().rth_take_picture(scene.handle, C.byref(camera), C.byref(settings), C.byref(filter_cache),
                                  C.byref(post), w, h, spp, total_frame_index, device, str(path).encode(),
                                  C.byref(stats)))
    return stats


def device_count():
    n = C.c_int()
    lib().rt_device_count(C.byref(n))
    return n.value
