"""Scenes with closed-form answers ("white furnace; emitter-only; one
diffuse bounce against a closed form"), built through the host scene model exactly as a
reference preset would be (RT/scene.cpp add_* functions, RT/raytracer.cpp:26-59 camera).

Every scene returns (Scene, Camera, Settings, FilterCache, expected) where `expected`
describes the closed form the rendered radiance (accum.rgb / accum.w, box filter) must meet.
The expectations come from the rendering equation, not from either implementation:

* furnace: a diffuse sphere of albedo 1 under a uniform sky of radiance c.  The sphere is
  convex, so a path leaves it after one scattering event: a Fresnel reflection (weight
  lerp(1, albedo, metallic) = 1, RT/integrators.cpp:684-696) or a cosine-sampled diffuse
  bounce (weight pi * albedo / pi = 1, :777-789).  Without Russian roulette every sample
  returns c (to float rounding): the sphere disappears.
* emitter: an emissive sphere on a black sky seen directly.  A camera ray's first hit on
  an emitter is counted (is_specular_bounce starts true, :651-660), so every sample is Le
  or 0, and a pixel all of whose samples hit the sphere resolves to exactly Le.
* bounce: an infinite diffuse plane of albedo a (ior 1: no Fresnel reflection) under a
  uniform sky c.  The outgoing radiance of a Lambertian surface under uniform incident
  radiance c is a * c, and a bounced ray never meets the plane again: every pixel is a * c.
* bounce_mesh / bounce_box: the same closed form with the diffuse surface being a large
  two-triangle mesh quad (mesh BVH + Moller-Trumbore, RT/intersection.cpp:135-401) or the
  top face of a box (RT/intersection.cpp:76-105).
"""
import math


def camera(rt, w, h, p, at, vfov_deg=40.0):
    cam = rt.abi.Camera()
    cam.vfov = rt.DEG_TO_RAD * vfov_deg
    cam.aspect_ratio = w / h
    cam.lens_radius = 0.0
    cam.focus_distance = 1.0
    cam.p = rt.v3(*p)
    rt.aim_camera_at(cam, at)
    rt.recompute_camera(cam)
    return cam


def settings(rt, spp=16, bounces=8):
    st, post = rt.default_settings()
    st.samples_per_pixel = spp
    st.max_bounce_count = bounces
    st.russian_roulette = 0
    st.vignette_strength = 0.0
    st.lens_distortion = 0.0
    return st


def furnace(rt, w, h, spp=16, sky=(0.5, 0.25, 0.75)):
    s = rt.Scene()
    m = s.add_diffuse_material((1.0, 1.0, 1.0), 1.5)          # Fresnel reflections happen (ior 1.5)
    s.add_sphere(m, 2.0, rt.translate((0.0, 0.0, 0.0)))
    s.set_sky(sky, sky)
    s.create_scene_bvh()
    cam = camera(rt, w, h, (0.0, 0.0, -7.0), (0.0, 0.0, 0.0), 40.0)
    return s, cam, settings(rt, spp), rt.load_reconstruction_kernel("Box"), {"kind": "uniform", "value": sky}


def emitter(rt, w, h, spp=16, le=(2.0, 3.0, 4.0)):
    s = rt.Scene()
    m = s.add_emissive_material(le)
    s.add_sphere(m, 3.0, rt.translate((0.0, 0.0, 0.0)))
    s.set_sky((0.0, 0.0, 0.0), (0.0, 0.0, 0.0))
    s.create_scene_bvh()
    cam = camera(rt, w, h, (0.0, 0.0, -10.0), (0.0, 0.0, 0.0), 30.0)
    return s, cam, settings(rt, spp), rt.load_reconstruction_kernel("Box"), {"kind": "emitter", "value": le}


def _bounce_common(rt, s, w, h, spp, sky, albedo):
    s.set_sky(sky, sky)
    s.create_scene_bvh()
    cam = camera(rt, w, h, (0.0, 10.0, -2.0), (0.0, 0.0, 0.5), 30.0)
    return s, cam, settings(rt, spp, bounces=4), rt.load_reconstruction_kernel("Box"), {
        "kind": "uniform", "value": tuple(a * c for a, c in zip(albedo, sky))}


def bounce(rt, w, h, spp=16, sky=(0.8, 0.6, 0.4), albedo=(0.25, 0.5, 0.75)):
    s = rt.Scene()
    m = s.add_diffuse_material(albedo, 1.0)
    s.add_plane(m, (0.0, 1.0, 0.0), 0.0)
    return _bounce_common(rt, s, w, h, spp, sky, albedo)


def bounce_mesh(rt, w, h, spp=16, sky=(0.8, 0.6, 0.4), albedo=(0.25, 0.5, 0.75)):
    import numpy as np
    s = rt.Scene()
    m = s.add_diffuse_material(albedo, 1.0)
    big = 1000.0
    # face normals cross(b - a, c - a) point up.  A third small triangle below the quad gives the
    # mesh's boxes some height: the reference's slab test (tn < tf, RT/intersection.cpp:107-133)
    # never passes a box of zero thickness, so a perfectly flat mesh is invisible.
    tris = np.array([[[-big, 0, -big], [-big, 0, big], [big, 0, big]],
                     [[-big, 0, -big], [big, 0, big], [big, 0, -big]],
                     [[0, -1, 0], [1, -1, 0], [0, -1, 1]]], np.float32)
    mesh = s.create_mesh(tris)
    s.add_mesh(m, mesh, rt.translate((0.0, 0.0, 0.0)))
    return _bounce_common(rt, s, w, h, spp, sky, albedo)


def bounce_box(rt, w, h, spp=16, sky=(0.8, 0.6, 0.4), albedo=(0.25, 0.5, 0.75)):
    s = rt.Scene()
    m = s.add_diffuse_material(albedo, 1.0)
    s.add_box(m, (1000.0, 1.0, 1000.0), rt.translate((0.0, -1.0, 0.0)))   # top face at y = 0
    return _bounce_common(rt, s, w, h, spp, sky, albedo)


SCENES = {"furnace": furnace, "emitter": emitter, "bounce": bounce, "bounce_mesh": bounce_mesh,
          "bounce_box": bounce_box}


def check(frame, expected, spp):
    """Assert the rendered frame (h, w, 4) meets the closed form; returns the max relative error."""
    import numpy as np
    w = frame[..., 3]
    assert np.all(w == spp), "box filter: every pixel weighs exactly spp"
    rad = frame[..., :3] / w[..., None]
    val = np.array(expected["value"], np.float64)
    if expected["kind"] == "uniform":
        err = float(np.max(np.abs(rad - val) / val))
        assert err <= 1e-5, f"max relative deviation {err}"
        return err
    # emitter: every pixel is a mix of Le and 0 with the same proportion in every channel,
    # the fully covered centre is exactly Le, the corners exactly 0
    h, wd = w.shape
    frac = rad / val
    assert np.all(frac >= -1e-7) and np.all(frac <= 1 + 1e-6)
    assert np.max(np.abs(frac - frac[..., :1])) <= 1e-6
    assert np.array_equal(rad[h // 2, wd // 2], val.astype(np.float32))
    assert np.all(rad[0, 0] == 0) and np.all(rad[-1, -1] == 0)
    # the covered fraction of the image approaches the sphere's projected disc
    return float(frac[..., 0].mean())


def disc_fraction(w, h, r=3.0, dist=10.0, vfov_deg=30.0):
    """Fraction of the film the sphere covers (pinhole, the reference's film: half height 0.5 at
    film distance 1/tan(vfov), RT/raytracer.cpp:37, :397; the x flip does not matter)."""
    film_d = 1.0 / math.tan(math.radians(vfov_deg))
    half_h, half_w = 0.5, 0.5 * w / h
    ang = math.asin(r / dist)                     # angular radius of the sphere
    rad_film = film_d * math.tan(ang)
    return math.pi * rad_film ** 2 / (4 * half_w * half_h)


# ---- environment-map sampling (rt_set_env_sampling; beyond the reference, see include/rt_abi.h)

def env_plane(rt, w, h, spp=16, c=(0.8, 0.6, 0.4), albedo=(0.25, 0.5, 0.75)):
    """`bounce` under a constant environment MAP of radiance c (64 x 32 texels) instead of the
    sky colours.  With environment NEE the estimate per sample is random, but its expectation is
    still a * c: the NEE term and the MIS-weighted escape split the one bounce."""
    import numpy as np
    s = rt.Scene()
    m = s.add_diffuse_material(albedo, 1.0)
    s.add_plane(m, (0.0, 1.0, 0.0), 0.0)
    s.set_environment_map(np.broadcast_to(np.array(c, np.float32), (32, 64, 3)))
    s.create_scene_bvh()
    cam = camera(rt, w, h, (0.0, 10.0, -2.0), (0.0, 0.0, 0.5), 30.0)
    return s, cam, settings(rt, spp, bounces=4), rt.load_reconstruction_kernel("Box"), {
        "kind": "mean", "value": tuple(a * x for a, x in zip(albedo, c))}


def env_sun(rt, w, h, spp=16, lights=False):
    """A diffuse floor and sphere under a dim sky with a small, very bright sun (128 x 64 map,
    the sun 4 x 2 texels at 400): the case environment sampling exists for.  `lights` adds a
    sphere light (the NEE then picks the environment with probability 1/2)."""
    import numpy as np
    env = np.full((64, 128, 3), 0.1, np.float32)
    env[40:42, 70:74] = (400.0, 380.0, 300.0)
    s = rt.Scene()
    floor = s.add_diffuse_material((0.6, 0.6, 0.6), 1.0)
    ball = s.add_diffuse_material((0.2, 0.4, 0.8), 1.0)
    s.add_plane(floor, (0.0, 1.0, 0.0), 0.0)
    s.add_sphere(ball, 1.5, rt.translate((0.0, 1.5, 0.0)))
    if lights:
        lm = s.add_emissive_material((20.0, 20.0, 18.0))
        s.add_sphere(lm, 0.5, rt.translate((-3.0, 5.0, 2.0)))
    s.set_environment_map(env)
    s.create_scene_bvh()
    cam = camera(rt, w, h, (0.0, 4.0, -9.0), (0.0, 1.0, 0.0), 40.0)
    st = settings(rt, spp, bounces=6)
    return s, cam, st, rt.load_reconstruction_kernel("Box"), None
