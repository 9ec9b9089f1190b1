"""Seeded random scenes for GPU-vs-oracle fuzzing (tests/test_gpu_scenes.py).

Each scene mixes everything the scene model offers, in proportions no preset has:
rotated / scaled spheres and boxes, several distinct meshes (with and without vertex
normals) instanced more often than the ray prologue's 63-entry mesh list holds, planes,
sphere lights, dielectrics with absorption nested inside each other, rough metals,
checkers, and either an environment map or the two sky colours.  The camera sits inside
the scene at a random place.  Nothing here is compared with a closed form: the oracle is
the answer, bit for bit.
"""
import math

import numpy as np


def _mesh(rt, s, rng, n_tris, seed, normals):
    n = rt.lib().rth_generate_mesh(n_tris, seed, None, None)
    tris = np.zeros((n, 3, 3), np.float32)
    nn = np.zeros((n, 3, 3), np.float32)
    import ctypes as C
    rt.lib().rth_generate_mesh(n_tris, seed, tris.ctypes.data_as(C.POINTER(rt.abi.V3)),
                               nn.ctypes.data_as(C.POINTER(rt.abi.V3)))
    return s.create_mesh(tris, nn if normals else None)


def _xf(rt, rng, pos, max_scale=1.0):
    t = rt.translate(tuple(float(x) for x in pos))
    t = t * rt.rotate_y(float(rng.uniform(0, 2 * math.pi)))
    t = t * rt.rotate_x(float(rng.uniform(-0.6, 0.6)))
    if max_scale != 1.0:
        t = t * rt.scale(tuple(float(x) for x in rng.uniform(0.5, max_scale, 3)))
    return t


def random_scene(rt, seed, w, h, spp=8, mesh_instances=70):
    rng = np.random.default_rng(seed)
    s = rt.Scene()
    mats = []
    for _ in range(4):
        mats.append(s.add_diffuse_material(tuple(rng.uniform(0.1, 0.9, 3)), float(rng.uniform(1.0, 1.6)),
                                           checkers=bool(rng.random() < 0.3)))
    for _ in range(2):
        mats.append(s.add_material(0, tuple(rng.uniform(0.5, 1.0, 3)), 0.0, 0.0, 1.5, 1.0,
                                   float(rng.choice([0.0, 0.1, 0.4]))))
    glass = [s.add_translucent_material(tuple(rng.uniform(0.0, 0.5, 3)), float(rng.uniform(1.3, 1.8)))
             for _ in range(2)]
    air = s.add_translucent_material((0.0, 0.0, 0.0), 1.0)
    lights = [s.add_emissive_material(tuple(rng.uniform(2.0, 15.0, 3))) for _ in range(2)]
    # planes: a floor and a back wall
    s.add_plane(mats[0], (0.0, 1.0, 0.0), -2.0)
    s.add_plane(mats[1], (0.0, 0.0, -1.0), -40.0)
    # distinct meshes, one without normals
    meshes = [_mesh(rt, s, rng, int(rng.integers(200, 3000)), int(rng.integers(1, 1000)), normals=k != 1)
              for k in range(3)]
    for i in range(mesh_instances):
        pos = rng.uniform((-20, -2, -5), (20, 8, 35))
        s.add_mesh(int(rng.choice(mats + glass)), meshes[i % len(meshes)], _xf(rt, rng, pos, 3.0))
    for _ in range(int(rng.integers(10, 30))):
        pos = rng.uniform((-15, -1, 0), (15, 6, 30))
        r = float(rng.uniform(0.3, 2.0))
        if rng.random() < 0.5:
            s.add_sphere(int(rng.choice(mats + glass)), r, rt.translate(tuple(float(x) for x in pos)))
        else:
            s.add_box(int(rng.choice(mats + glass)), tuple(float(x) for x in rng.uniform(0.2, 2.0, 3)),
                      _xf(rt, rng, pos))
    # a glass shell with an air bubble and a glass core (three nested media)
    c = tuple(float(x) for x in rng.uniform((-5, 1, 5), (5, 4, 15)))
    s.add_sphere(glass[0], 2.5, rt.translate(c))
    s.add_sphere(air, 2.0, rt.translate(c))
    s.add_sphere(glass[1], 1.0, rt.translate(c))
    for k, lm in enumerate(lights):
        s.add_sphere(lm, float(rng.uniform(0.5, 1.5)), rt.translate(tuple(float(x) for x in
                                                                           rng.uniform((-10, 8, 0), (10, 15, 25)))))
    if seed % 2:
        env = rng.uniform(0.0, 0.6, (32, 64, 3)).astype(np.float32)
        env[20:22, 10:14] = 50.0
        s.set_environment_map(env)
    else:
        s.set_sky(tuple(rng.uniform(0.2, 0.8, 3)), tuple(rng.uniform(0.0, 0.3, 3)))
    s.create_scene_bvh()
    cam = rt.abi.Camera()
    cam.vfov = rt.DEG_TO_RAD * float(rng.uniform(30, 70))
    cam.aspect_ratio = w / h
    cam.lens_radius = float(rng.choice([0.0, 0.0, 2.0]))
    cam.focus_distance = float(rng.uniform(5, 20))
    cam.p = rt.v3(float(rng.uniform(-5, 5)), float(rng.uniform(1, 6)), float(rng.uniform(-12, -4)))
    rt.aim_camera_at(cam, tuple(float(x) for x in rng.uniform((-3, 0, 5), (3, 3, 20))))
    rt.recompute_camera(cam)
    st, post = rt.default_settings()
    st.samples_per_pixel = spp
    st.max_bounce_count = int(rng.integers(3, 13))
    st.russian_roulette = int(rng.random() < 0.7)
    st.caustics = int(rng.random() < 0.5)
    st.sampling_strategy = int(rng.choice([0, 1, 2]))
    fc = rt.load_reconstruction_kernel(str(rng.choice(["Mitchell Netravali", "Box", "Gaussian 3", "Lanczos 3"])))
    # the reference's integrator switches (RT/raytracer.cpp:1974-1977): one of their 16 combinations
    # (drawn last, so the scenes themselves do not change with it)
    combo = int(rng.integers(0, 16))
    for i, k in enumerate(("next_event_estimation", "importance_sample_lights", "use_mis", "importance_sample_diffuse")):
        setattr(st, k, (combo >> i) & 1)
    return s, cam, st, fc
