// rt_presets.cpp — scene presets (g_scenes, RT/raytracer.cpp:795-1422) and the
// benchmark configurations c1..c5 of BASELINE.json, plus the render-to-bitmap
// entry point.  Preset parameters are the reference's, value for value; the
// missing assets (.MISSING_LARGE_BLOBS) come from seeded synthetic generators.
#include "../../../include/rt_host.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <sys/stat.h>
#include <unistd.h>
#include <atomic>

std::vector<uint8_t> rth_synthetic_hdr_bytes(uint32_t w, uint32_t h, uint32_t seed);
int rth_load_environment_map_bytes(rth_scene* s, std::vector<char>& file);

namespace {

const float PI_32 = 3.14159265359f;
const float DEG_TO_RAD = 6.28318530717f / 360.0f;

rt_v3 v3(float x, float y, float z) { return {x, y, z}; }
rt_v3 v3(float s) { return {s, s, s}; }
rt_v3 sc(float s, rt_v3 a) { return {s*a.x, s*a.y, s*a.z}; }

rt_m4x4inv translate(rt_v3 t) { return rth_transform_translate(t); }
rt_m4x4inv scale(rt_v3 s) { return rth_transform_scale(s); }
rt_m4x4inv roty(float a) { return rth_transform_rotate_y_axis(a); }
rt_m4x4inv rotx(float a) { return rth_transform_rotate_x_axis(a); }
rt_m4x4inv operator*(rt_m4x4inv a, rt_m4x4inv b) { return rth_transform_mul(a, b); }

// RandomSeries for preset generation (RT/samplers.h:29-108): scalar restatement
struct Series { uint32_t e[4]; };
uint32_t wang(uint32_t k) { k += ~(k << 15); k ^= (k >> 10); k += (k << 3); k ^= (k >> 6); k += ~(k << 11); k ^= (k >> 16); return k; }
void next_set(Series* s, uint32_t o[4]) {
    for (int i = 0; i < 4; ++i) { uint32_t r = s->e[i]; r ^= r << 13; r ^= r >> 17; r ^= r << 5; s->e[i] = r; o[i] = r; }
}
Series seed_series(uint32_t seed) {
    Series r; if (seed == 0) seed = 0xFFFFFFFFu;
    uint32_t h = wang(seed); r.e[0] = r.e[1] = r.e[2] = r.e[3] = h;
    uint32_t a[4], b[4], c[4], d[4];
    next_set(&r, a); next_set(&r, b); next_set(&r, c); next_set(&r, d);
    r.e[0] = wang(a[0]); r.e[1] = wang(b[1]); r.e[2] = wang(c[2]);
    return r;
}
void unilaterals(Series* s, float o[4]) {
    uint32_t b[4]; next_set(s, b);
    for (int i = 0; i < 4; ++i) { uint32_t u = (127u << 23) | (b[i] >> 9); float f; memcpy(&f, &u, 4); o[i] = f - 1.0f; }
}
void bilaterals(Series* s, float o[4]) { unilaterals(s, o); for (int i = 0; i < 4; ++i) o[i] = o[i]*2.0f - 1.0f; }
uint32_t random_range(Series* s, uint32_t mn, uint32_t mx) {       // RT/samplers.h:47-66
    uint32_t r = s->e[0]; r ^= r << 13; r ^= r >> 17; r ^= r << 5; s->e[0] = r;
    return mx > mn ? mn + (r % (mx - mn)) : mn;
}

struct Ctx {
    rth_scene* s;
    rt_camera* cam;
    rt_settings* st;
    rt_filter_cache* filter;
    rth_post_settings* post;
    uint32_t w, h;
    std::string asset_dir;
    bool failed = false;             // a mesh or BVH build failed (rth_last_error says why)
};

bool exists(const std::string& p) { struct stat st; return stat(p.c_str(), &st) == 0; }

// A synthetic asset is written under a name private to this process and call, then renamed into
// place: rename() within a directory is atomic, so a process that finds the file (ranks started
// together sharing an asset directory) never parses a half-written one.
template <class W>
void write_asset(const std::string& path, W write) {
    static std::atomic<uint32_t> seq{0};
    const std::string tmp = path + ".tmp." + std::to_string((long)getpid()) + "." + std::to_string(seq++);
    if (write(tmp.c_str()) && rename(tmp.c_str(), path.c_str()) == 0) return;
    remove(tmp.c_str());                  // the caller then finds no file and builds the asset in memory
}

// load_mesh (RT/raytracer.cpp:148-158) with the synthetic stand-in for dragon_mcguire.obj.
// The presets build the mesh BVH with binned SAH (the north star's SAH BVH);
// the reference's load_mesh used BVH_MidpointSplit (:154).
uint32_t load_mesh(Ctx& c, uint32_t triangles, uint32_t seed) {
    if (!c.asset_dir.empty()) {
        std::string path = c.asset_dir + "/synthetic_mesh_" + std::to_string(triangles) + "_s" + std::to_string(seed) + ".obj";
        if (!exists(path)) write_asset(path, [&](const char* f) { return rth_write_synthetic_obj(f, triangles, seed) != 0; });
        uint32_t id;
        if (rth_load_obj_mesh(c.s, path.c_str(), RTH_BVH_SAH_BINNED, &id)) return id;
    }
    uint32_t n = rth_generate_mesh(triangles, seed, nullptr, nullptr);
    std::vector<rt_v3> t(3*(size_t)n), nn(3*(size_t)n);
    rth_generate_mesh(triangles, seed, t.data(), nn.data());
    const uint32_t id = rth_create_mesh(c.s, n, t.data(), nn.data(), RTH_BVH_SAH_BINNED);
    if (id == 0xFFFFFFFFu) c.failed = true;      // e.g. out of memory in the BVH build
    return id;
}

// load_environment_map with the synthetic stand-in for the missing 2k .hdr files.
void load_env(Ctx& c, uint32_t seed) {
    const uint32_t W = 2048, H = 1024;
    if (!c.asset_dir.empty()) {
        std::string path = c.asset_dir + "/synthetic_sky_s" + std::to_string(seed) + ".hdr";
        if (!exists(path)) write_asset(path, [&](const char* f) { return rth_write_synthetic_hdr(f, W, H, seed) != 0; });
        if (rth_load_environment_map(c.s, path.c_str())) return;
    }
    std::vector<uint8_t> b = rth_synthetic_hdr_bytes(W, H, seed);
    std::vector<char> f(b.begin(), b.end());
    f.push_back(0);
    rth_load_environment_map_bytes(c.s, f);
}

void set_filter(Ctx& c, const char* name) { rth_load_reconstruction_kernel(name, c.filter); }

uint32_t add_diffuse(Ctx& c, rt_v3 col, float ior, float rough = 0.0f, bool checkers = false, rt_v3 cc = {0.1f, 0.1f, 0.1f}) {
    return rth_add_diffuse_material(c.s, col, ior, rough, checkers, cc);
}
uint32_t add_mat(Ctx& c, uint32_t flags, rt_v3 albedo, rt_v3 checker, float ior, float metallic, float rough) {
    rt_material m = {};
    m.flags = flags; m.albedo = albedo; m.checker_color = checker; m.ior = ior; m.metallic = metallic; m.roughness = rough;
    return rth_add_material(c.s, &m);
}
void sphere(Ctx& c, uint32_t m, float r, rt_m4x4inv t) { rth_add_sphere(c.s, m, r, &t); }
void box(Ctx& c, uint32_t m, rt_v3 r, rt_m4x4inv t) { rth_add_box(c.s, m, r, &t); }
void plane(Ctx& c, uint32_t m, rt_v3 n, float d) { rth_add_plane(c.s, m, n, d); }

void camera_basic(Ctx& c, float vfov_deg, float lens_radius, float focus) {
    c.cam->vfov = DEG_TO_RAD*vfov_deg;
    c.cam->aspect_ratio = (float)c.w / (float)c.h;
    c.cam->lens_radius = lens_radius;
    c.cam->focus_distance = focus;
}

// ---- g_scenes (RT/raytracer.cpp:798-1407)
void week_1(Ctx& c) {
    camera_basic(c, 60.0f, 0.0f, 1.0f);
    c.cam->p = v3(0, 4, -10); rth_aim_camera(c.cam, v3(0, 0, -1));
    c.st->lens_distortion = 0.0f; set_filter(c, "Box"); c.post->tonemapping = 0;
    uint32_t g = add_diffuse(c, v3(1), 1.0f, 0.0f, true, v3(0.0f));
    plane(c, g, v3(0, 1, 0), 0.0f);
}
void week_2(Ctx& c) {
    week_1(c);
    uint32_t sm = add_diffuse(c, v3(1.0f, 0.0f, 0.0f), 1.0f);
    sphere(c, sm, 4.0f, translate(v3(0, 4, 0)));
}
void week_3(Ctx& c) {
    week_2(c);
    uint32_t lm = rth_add_emissive_material(c.s, v3(12500));
    sphere(c, lm, 0.1f, translate(v3(8, 16, -8)));
}
void week_4(Ctx& c) {
    camera_basic(c, 60.0f, 0.0f, 1.0f);
    c.cam->p = v3(0, 4, -10); rth_aim_camera(c.cam, v3(0, 0, -1));
    c.st->lens_distortion = 0.0f; set_filter(c, "Box"); c.post->tonemapping = 0;
    uint32_t g = add_diffuse(c, v3(1), 1.0f, 0.0f, true, v3(0.0f));
    uint32_t sm = add_mat(c, 0, v3(0.5f), v3(0), 1.5f, 0.5f, 0.05f);
    uint32_t lm = rth_add_emissive_material(c.s, v3(12500));
    plane(c, g, v3(0, 1, 0), 0.0f);
    sphere(c, sm, 4.0f, translate(v3(0, 4, 0)));
    sphere(c, lm, 0.1f, translate(v3(8, 16, -8)));
}
void week_5(Ctx& c) {                                                      // :891-924
    camera_basic(c, 50.0f, 0.0f, 1.0f);
    c.cam->p = v3(-5, 8, -15); rth_aim_camera(c.cam, v3(0, 0, -1));
    c.st->lens_distortion = 0.0f; c.st->max_bounce_count = 12; c.st->caustics = 0;
    set_filter(c, "Gaussian 3"); c.post->tonemapping = 1;
    rth_set_sky(c.s, v3(0.1f, 0.7f, 2.0f), v3(0.1f, 0.7f, 2.0f));
    uint32_t g = add_diffuse(c, v3(1.0f, 0.0f, 0.0f), 1.0f, 0.0f, true, v3(1.0f, 1.0f, 0.0f));
    uint32_t glass = rth_add_translucent_material(c.s, v3(0), 1.8f, 0.0f);
    uint32_t metal = add_mat(c, 0, v3(0.95f), v3(0), 1.5f, 0.8f, 0.0f);
    uint32_t air = rth_add_translucent_material(c.s, v3(0.0f), 1.0f, 0.0f);
    uint32_t light = rth_add_emissive_material(c.s, v3(325000000));
    box(c, g, v3(16, 1, 20), translate(v3(0, -1.0f, 16)));
    sphere(c, glass, 4.0f, translate(v3(-5, 8, 0)));
    sphere(c, air, 3.8f, translate(v3(-5, 8, 0)));
    sphere(c, metal, 4.0f, translate(v3(0, 5, 8)));
    sphere(c, light, 10.0f, translate(sc(10000.0f, v3(-1, 10, -8))));
}
void week_6(Ctx& c) {                                                      // :926-978
    camera_basic(c, 45.0f, 10.0f, 1.0f);
    c.cam->p = v3(0, 7.5f, -25); rth_aim_camera(c.cam, v3(0, 0, -1));
    c.cam->focus_distance = 19.77f;
    c.st->lens_distortion = 0.0f;
    uint32_t ground = add_diffuse(c, v3(0.55f, 0.55f, 0.55f), 1.0f);
    (void)add_diffuse(c, v3(0.75f, 0.75f, 0.75f), 1.1f, 0.25f);
    uint32_t red = add_diffuse(c, v3(0.95f, 0.1f, 0.1f), 1.0f);
    uint32_t green = add_diffuse(c, v3(0.1f, 0.95f, 0.1f), 1.0f);
    uint32_t blue = add_diffuse(c, v3(0.1f, 0.1f, 0.95f), 1.0f);
    uint32_t glass = rth_add_translucent_material(c.s, v3(0.15f), 1.5f, 0.0f);
    (void)rth_add_translucent_material(c.s, v3(0.0f, 0.1f, 0.1f), 1.6f, 0.0f);
    (void)rth_add_translucent_material(c.s, v3(0.0f), 1.0f, 0.0f);
    uint32_t metal = add_mat(c, 0, v3(0.85f, 0.85f, 0.85f), v3(0), 0.2f, 1.0f, 0.0f);
    uint32_t mixed = add_mat(c, 0, v3(0.05f, 0.05f, 0.95f), v3(0), 1.5f, 0.15f, 0.0f);
    uint32_t white_light = rth_add_emissive_material(c.s, sc(6.0f, v3(10.0f, 10.0f, 10.0f)));
    (void)rth_add_emissive_material(c.s, sc(10.0f, v3(10.0f, 2.0f, 0.0f)));
    (void)rth_add_emissive_material(c.s, sc(3.0f, v3(2.0f, 6.0f, 10.0f)));
    (void)rth_add_emissive_material(c.s, sc(3.0f, v3(1.0f, 10.0f, 2.0f)));
    box(c, metal, v3(2.0f, 6.0f, 2.0f), translate(v3(-3, 3, 1))*roty(-0.125f*PI_32));
    sphere(c, glass, 2.0f, translate(v3(-3, 2.3f, -5)));
    sphere(c, mixed, 2.0f, translate(v3(3, 2.0f, -4)));
    plane(c, ground, v3(0, 1, 0), 0.0f);
    plane(c, ground, v3(0, -1, 0), -15.0f);
    plane(c, ground, v3(0, 0, -1), -8.0f);
    plane(c, blue, v3(0, 0, 1), -8.0f);
    plane(c, red, v3(1, 0, 0), -7.5f);
    plane(c, green, v3(-1, 0, 0), -7.5f);
    sphere(c, white_light, 1.5f, translate(v3(0, 13.4f, -2)));
}
void week_7_common(Ctx& c, bool nicer) {                                   // :980-1104
    camera_basic(c, 39.0f, nicer ? 6.0f : 0.0f, 1.0f);
    c.cam->p = v3(0, nicer ? 8.0f : 7.0f, -15); rth_aim_camera_at(c.cam, v3(0, 0, 0));
    c.cam->focus_distance = 10.8f;
    c.st->lens_distortion = nicer ? -0.5f : 0.0f;
    c.st->vignette_strength = nicer ? 1.0f : 0.0f;
    c.st->caustics = 0;
    rth_set_sky(c.s, v3(0.2f, 0.7f, 0.95f), v3(0.2f, 0.7f, 0.95f));
    if (nicer) c.post->contrast = 0.1f;
    set_filter(c, "Gaussian 3");
    uint32_t ground = add_diffuse(c, v3(0.55f, 0.55f, 0.55f), 1.0f);
    uint32_t sm = add_mat(c, 0, v3(0.85f, 0.85f, 0.85f), v3(0), 1.5f, 1.0f, 0.0f);
    plane(c, ground, v3(0, 1, 0), 0.0f);
    sphere(c, sm, 1.0f, translate(v3(0, 1.0f, 0)));
    if (nicer) {
        uint32_t wl = rth_add_emissive_material(c.s, sc(25.0f, v3(10.0f, 7.0f, 4.0f)));
        sphere(c, wl, 1000.0f, translate(sc(100.0f, v3(-50, 100.0f, -50))));
    } else {
        uint32_t wl = rth_add_emissive_material(c.s, sc(3.0f, v3(10.0f, 10.0f, 10.0f)));
        sphere(c, wl, 30.0f, translate(v3(-50, 100.0f, -50)));
    }
    Series e = seed_series(nicer ? 1 : 2);
    for (int x = -100; x <= 100; ++x)
        for (int y = -100; y <= 100; ++y) {
            if ((x < -2 || x > 2) || (y < -2 || y > 2)) {
                float rnd[4], rnd2[4], rnd3[4];
                unilaterals(&e, rnd); unilaterals(&e, rnd2); unilaterals(&e, rnd3);
                rt_v3 col = v3(0.25f + 0.75f*rnd3[0], 0.25f + 0.75f*rnd3[1], 0.25f + 0.75f*rnd3[2]);
                uint32_t bm;
                if (!nicer) bm = add_diffuse(c, col, 1.5f, 0.75f);
                else if (rnd3[3] > 0.67f && rnd3[3] < 0.90f)
                    bm = rth_add_translucent_material(c.s, v3(1.0f - col.x, 1.0f - col.y, 1.0f - col.z), 1.5f, 0.0f);
                else if (rnd3[3] > 0.90f) bm = add_mat(c, 0, col, v3(0), 1.5f, 1.0f, 0.0f);
                else bm = add_diffuse(c, col, 1.5f, 0.25f);
                rt_m4x4inv m = translate(v3(2.0f*(-.5f + rnd[0] + (float)x), 1.0f, 2.0f*(-0.5f + rnd[1] + (float)y)));
                m = m*roty(PI_32*rnd[2]);
                m = m*rotx(-0.25f + 0.5f*PI_32*rnd[3]);
                box(c, bm, v3(0.25f + rnd2[0], 0.5f + rnd2[1], 0.25f + rnd2[2]), m);
            }
        }
}
void week_7(Ctx& c) { week_7_common(c, false); }
void week_7_nicer(Ctx& c) { week_7_common(c, true); }

void cornell_box(Ctx& c, uint32_t mesh_tris) {                              // :1106-1165
    camera_basic(c, 45.0f, 10.0f, 1.0f);
    c.cam->p = v3(0, 7.5f, -25); rth_aim_camera(c.cam, v3(0, 0, -1));
    c.cam->focus_distance = 19.77f;
    c.st->lens_distortion = 1.0f;
    uint32_t ground = add_diffuse(c, v3(0.55f, 0.55f, 0.55f), 1.0f);
    (void)add_diffuse(c, v3(0.75f, 0.75f, 0.75f), 1.1f, 0.25f);
    uint32_t red = add_diffuse(c, v3(0.95f, 0.1f, 0.1f), 1.0f);
    uint32_t green = add_diffuse(c, v3(0.1f, 0.95f, 0.1f), 1.0f);
    (void)add_diffuse(c, v3(0.1f, 0.1f, 0.95f), 1.0f);
    uint32_t glass = rth_add_translucent_material(c.s, v3(0.15f), 1.5f, 0.0f);
    (void)rth_add_translucent_material(c.s, v3(0.0f, 0.1f, 0.1f), 1.6f, 0.0f);
    (void)rth_add_translucent_material(c.s, v3(0.0f), 1.0f, 0.0f);
    uint32_t metal = add_mat(c, 0, v3(0.85f, 0.75f, 0.45f), v3(0), 0.2f, 1.0f, 0.0f);
    uint32_t mixed = add_mat(c, 0, v3(0.05f, 0.05f, 0.95f), v3(0), 1.5f, 0.15f, 0.0f);
    uint32_t white_light = rth_add_emissive_material(c.s, sc(6.0f, v3(10.0f, 10.0f, 10.0f)));
    (void)rth_add_emissive_material(c.s, sc(10.0f, v3(10.0f, 2.0f, 0.0f)));
    (void)rth_add_emissive_material(c.s, sc(3.0f, v3(2.0f, 6.0f, 10.0f)));
    (void)rth_add_emissive_material(c.s, sc(3.0f, v3(1.0f, 10.0f, 2.0f)));
    box(c, metal, v3(2.5f, 8.0f, 2.5f), translate(v3(-3, 4, 1))*roty(-0.125f*PI_32));
    box(c, metal, v3(0.5f, 2.0f, 0.5f), translate(v3(-5, 2, -5)));
    sphere(c, glass, 2.0f, translate(v3(-5, 6.0f, -5)));
    if (mesh_tris) {
        uint32_t dragon = load_mesh(c, mesh_tris, 1);
        rt_m4x4inv t = translate(v3(5, 2.0f, -3))*scale(v3(10.0f))*roty(0.25f*PI_32);
        rth_add_mesh(c.s, mixed, dragon, &t);
    }
    plane(c, ground, v3(0, 1, 0), 0.0f);
    plane(c, ground, v3(0, -1, 0), -15.0f);
    plane(c, ground, v3(0, 0, -1), -8.0f);
    plane(c, red, v3(1, 0, 0), -10.5f);
    plane(c, green, v3(-1, 0, 0), -10.5f);
    sphere(c, white_light, 1.5f, translate(v3(0, 13.4f, -2)));
}

// unique: the BASELINE C4/C5 "~250k-tri multi-mesh scene" as four distinct meshes (seeds 1..4),
// so 250k triangles are resident; the reference scene instances one dragon four times.
void dragon(Ctx& c, uint32_t mesh_tris, bool nested, uint32_t env_seed, bool unique = false) {  // :1167-1225
    camera_basic(c, 40.0f, 6.0f, 1.0f);
    c.cam->p = v3(-25, 6, 0); rth_aim_camera_at(c.cam, v3(1, 5, 0));
    uint32_t ground = add_diffuse(c, v3(0.55f, 0.55f, 0.55f), 1.0f, 0.0f, true);
    (void)add_diffuse(c, v3(0.55f, 0.85f, 0.55f), 1.0f, 0.0f, true, v3(0.65f, 0.15f, 0.65f));
    (void)add_diffuse(c, v3(0.25f, 0.35f, 0.55f), 1.3f);
    uint32_t blue_glass = rth_add_translucent_material(c.s, v3(0.98f, 0.35f, 0.15f), 1.5f, 0.0f);
    uint32_t red_glass = rth_add_translucent_material(c.s, v3(0.15f, 0.35f, 0.95f), 1.5f, 0.0f);
    (void)rth_add_translucent_material(c.s, v3(0.98f, 0.35f, 0.15f), 1.5f, 0.0f);
    uint32_t marble = rth_add_translucent_material(c.s, v3(0.0f, 0.0f, 0.0f), 1.5f, 0.0f);
    uint32_t air = rth_add_translucent_material(c.s, v3(0.0f, 0.0f, 0.0f), 1.0f, 0.0f);
    (void)rth_add_translucent_material(c.s, v3(0.0f, 0.1f, 0.2f), 1.5f, 0.0f);
    uint32_t rough = add_mat(c, 0, v3(0.15f, 0.5f, 0.8f), v3(0), 1.3f, 0.0f, 0.75f);
    uint32_t metal = add_mat(c, 0, v3(0.85f, 0.85f, 0.85f), v3(0), 0.0f, 1.0f, 0.0f);
    uint32_t white_light = rth_add_emissive_material(c.s, sc(8.0f, v3(10.0f, 10.0f, 9.0f)));
    uint32_t red_light = rth_add_emissive_material(c.s, sc(10.0f, v3(10.0f, 2.0f, 0.0f)));
    uint32_t blue_light = rth_add_emissive_material(c.s, sc(3.0f, v3(2.0f, 6.0f, 10.0f)));
    (void)rth_add_emissive_material(c.s, sc(3.0f, v3(1.0f, 10.0f, 2.0f)));
    load_env(c, env_seed);
    uint32_t d = load_mesh(c, mesh_tris, 1);
    uint32_t d1 = unique ? load_mesh(c, mesh_tris, 2) : d;
    uint32_t d2 = unique ? load_mesh(c, mesh_tris, 3) : d;
    uint32_t d3 = unique ? load_mesh(c, mesh_tris, 4) : d;
    rt_m4x4inv t0 = translate(v3(0, 6.0f, 0))*scale(v3(14.0f));
    rt_m4x4inv t1 = translate(v3(-5, 3.7f, 0))*scale(v3(6.0f));
    rt_m4x4inv t2 = translate(v3(-5, 3.7f, -7))*scale(v3(6.0f));
    rt_m4x4inv t3 = translate(v3(-5, 3.7f, 7))*scale(v3(6.0f));
    rth_add_mesh(c.s, blue_glass, d, &t0);
    rth_add_mesh(c.s, red_glass, d1, &t1);
    rth_add_mesh(c.s, rough, d2, &t2);
    rth_add_mesh(c.s, metal, d3, &t3);
    box(c, ground, v3(10, 1, 10), translate(v3(0, 1.0f, 0)));
    box(c, ground, v3(40, 1, 40), translate(v3(8.0f, -1.0f, 0)));
    if (nested) {
        // nested dielectrics: a glass shell around an air bubble, as week_5_scene (:920-921)
        sphere(c, marble, 2.5f, translate(v3(-7.0f, 4.5f, -3.5f)));
        sphere(c, air, 2.3f, translate(v3(-7.0f, 4.5f, -3.5f)));
    }
    sphere(c, blue_light, 2, translate(v3(-5.0f, 25.0f, 5)));
    sphere(c, red_light, 2, translate(v3(5.0f, 35.0f, 8)));
    sphere(c, white_light, 2, translate(v3(0.0f, 15.0f, 12)));
}

void platforms(Ctx& c) {                                                    // :1227-1347
    camera_basic(c, 40.0f, 10.0f, 15.0f);
    c.cam->p = v3(0, 3, -18); rth_aim_camera_at(c.cam, v3(0, 0, 0));
    c.st->lens_distortion = 2.0f; c.st->caustics = 0;
    load_env(c, 4);
    (void)add_diffuse(c, v3(0.8f, 0.1f, 0.1f), 1.0f, 0.0f, true, v3(0.8f, 0.8f, 0.1f));
    uint32_t marble = rth_add_translucent_material(c.s, v3(0.5f, 0.25f, 0.0f), 1.5f, 0.0f);
    (void)add_diffuse(c, v3(0.85f, 0.85f, 0.35f), 1.5f);
    (void)rth_add_translucent_material(c.s, v3(0.0f), 1.0f, 0.0f);
    uint32_t pedestal = add_diffuse(c, v3(0.5f, 0.5f, 0.5f), 1.0f);
    uint32_t checker = add_mat(c, RT_MATERIAL_CHECKERS, v3(0.5f), v3(0.25f), 1.1f, 0.0f, 0.0f);
    (void)add_mat(c, 0, v3(0.95f), v3(0), 1.5f, 1.0f, 0.0f);
    (void)add_mat(c, 0, v3(0.95f), v3(0), 1.5f, 1.0f, 0.10f);
    (void)add_mat(c, 0, v3(0.95f), v3(0), 1.5f, 1.0f, 0.20f);
    (void)add_mat(c, 0, v3(0.95f), v3(0), 1.5f, 1.0f, 0.4f);
    for (float x : {-9.0f, -3.0f, 3.0f, 9.0f}) sphere(c, marble, 2.5f, translate(v3(x, 0.0f, 0.0f)));
    box(c, checker, v3(50.0f, 1.0f, 50.0f), translate(v3(0.0f, -10.0f, 0.0f)));
    box(c, pedestal, v3(10.0f, 1.0f, 10.0f), translate(v3(-35.0f, -6.5f, 0.0f)));
    box(c, pedestal, v3(10.0f, 1.0f, 10.0f), translate(v3(35.0f, 3.5f, 0.0f)));
    box(c, pedestal, v3(10.0f, 1.0f, 10.0f), translate(v3(0.0f, 9.5f, -35.0f)));
    box(c, pedestal, v3(10.0f, 1.0f, 10.0f), translate(v3(0.0f, 0.5f, 35.0f)));
    uint32_t pink = rth_add_emissive_material(c.s, sc(50.0f, v3(10.0f, 1.0f, 10.0f)));
    uint32_t redl = rth_add_emissive_material(c.s, sc(50.0f, v3(10.0f, 1.0f, 1.0f)));
    uint32_t greenl = rth_add_emissive_material(c.s, sc(50.0f, v3(1.0f, 10.0f, 1.0f)));
    uint32_t bluel = rth_add_emissive_material(c.s, sc(50.0f, v3(1.0f, 1.0f, 10.0f)));
    sphere(c, bluel, 2, translate(v3(-35.0f, -6.5f + 10.0f, 0.0f)));
    sphere(c, redl, 2, translate(v3(35.0f, 3.5f + 10.0f, 0.0f)));
    sphere(c, pink, 2, translate(v3(0.0f, 9.5f + 10.0f, -35.0f)));
    sphere(c, greenl, 2, translate(v3(0.0f, 0.5f + 10.0f, 35.0f)));
    sphere(c, greenl, 0.25f, translate(v3(0.0f, 20.0f, 0.0f)));
}

void nested_dielectrics(Ctx& c, uint32_t seed) {                            // :1349-1407
    camera_basic(c, 40.0f, 6.0f, 1.0f);
    c.cam->p = v3(-25, 6, 0); rth_aim_camera_at(c.cam, v3(1, 5, 0));
    (void)rth_add_translucent_material(c.s, v3(0.0f), 1.5f, 0.0f);
    (void)rth_add_translucent_material(c.s, v3(0.6f, 0.3f, 0.0f), 1.5f, 0.0f);
    (void)rth_add_translucent_material(c.s, v3(0.0f), 1.0f, 0.0f);
    uint32_t ground = add_diffuse(c, v3(0.55f, 0.55f, 0.55f), 1.0f, 0.0f, true);
    uint32_t wl = rth_add_emissive_material(c.s, sc(8.0f, v3(10.0f, 10.0f, 9.0f)));
    load_env(c, 5);
    box(c, ground, v3(10, 1, 10), translate(v3(0, 1.0f, 0)));
    box(c, ground, v3(40, 1, 40), translate(v3(8.0f, -1.0f, 0)));
    const float floor_h = 2.0f;
    // the reference seeds with SDL_GetTicks() (nondeterministic); a fixed seed here
    Series e = seed_series(seed);
    uint32_t count = random_range(&e, 20, 40);
    for (uint32_t m = 0; m < count; ++m) {
        float u[4]; unilaterals(&e, u);
        uint32_t mm = rth_add_translucent_material(c.s, v3(0.25f + 0.75f*u[0], 0.25f + 0.75f*u[1], 0.25f + 0.75f*u[2]), 1.5f, 0.0f);
        float b[4]; bilaterals(&e, b);
        float mx = 8.0f*b[0], my = 8.0f*b[1];
        unilaterals(&e, u);
        float r = 0.6f + u[0];
        rt_v3 p = v3(mx, floor_h + r, my);
        sphere(c, mm, r, translate(p));
        uint32_t bubbles = random_range(&e, 5, 12);
        for (uint32_t i = 0; i < bubbles; ++i) {
            float r1[4]; bilaterals(&e, r1);
            float br = 0.05f + ((r1[3] - -1.0f) / (1.0f - -1.0f))*0.15f;
            float maxoff = r - br - 0.05f;
            unilaterals(&e, u);
            float off = maxoff*u[0];
            rt_v3 bp = v3(p.x + off*r1[0], p.y + off*r1[1], p.z + off*r1[2]);
            sphere(c, ground, br, translate(bp));
        }
    }
    sphere(c, wl, 2, translate(v3(0.0f, 15.0f, 12)));
}

}  // namespace

extern "C" int rth_load_preset(const char* name_c, uint32_t w, uint32_t h, const char* asset_dir,
                               rth_scene** out_scene, rt_camera* cam, rt_settings* st,
                               rt_filter_cache* filter, rth_post_settings* post) {
    std::string name(name_c ? name_c : "");
    rth_post_settings post_local;
    if (!post) post = &post_local;
    rth_scene* s = rth_scene_create();
    memset(cam, 0, sizeof(*cam));
    rth_default_settings(st, post);                                      // init_scene :1424-1453
    rth_load_reconstruction_kernel("Mitchell Netravali", filter);
    Ctx c{s, cam, st, filter, post, w, h, asset_dir ? asset_dir : ""};
    bool ok = true;
    if (name == "week_1") week_1(c);
    else if (name == "week_2") week_2(c);
    else if (name == "week_3") week_3(c);
    else if (name == "week_4") week_4(c);
    else if (name == "week_5") week_5(c);
    else if (name == "week_6") week_6(c);
    else if (name == "week_7") week_7(c);
    else if (name == "week_7_nicer") week_7_nicer(c);
    else if (name == "cornell_box") cornell_box(c, 70000);
    else if (name == "dragon") dragon(c, 62500, false, 3);
    else if (name == "platforms") platforms(c);
    else if (name == "nested_dielectrics") nested_dielectrics(c, 1234);
    // ---- BASELINE.json configs
    else if (name == "c1") { week_6(c); st->samples_per_pixel = 16; st->max_bounce_count = 4; }
    else if (name == "c2") { cornell_box(c, 70000); st->samples_per_pixel = 64; }
    else if (name == "c3") { cornell_box(c, 70000); load_env(c, 2); st->samples_per_pixel = 256; }
    else if (name == "c4") { dragon(c, 62500, true, 3, true); st->samples_per_pixel = 256; }
    else if (name == "c4i") { dragon(c, 62500, true, 3); st->samples_per_pixel = 256; }   // one mesh, 4 instances
    else if (name == "c5") { dragon(c, 62500, true, 3, true); st->samples_per_pixel = 1024;
                             st->sampling_strategy = RT_SAMPLING_OPTIMIZED_BLUE_NOISE; }
    else ok = false;
    // a failed mesh or scene BVH build fails the preset (rth_last_error says why) instead of leaving an
    // out-of-range mesh id or no top level in the scene
    if (!ok || c.failed) { rth_scene_destroy(s); return 0; }
    st->integrator = RT_INTEGRATOR_ADVANCED;   // the hot path is the Advanced Pathtracer
    rth_recompute_camera(cam);                 // render_all_tiles -> recompute_camera (:717)
    if (!rth_create_scene_bvh(s)) { rth_scene_destroy(s); return 0; }   // load_scene (:1465)
    *out_scene = s;
    return 1;
}

extern "C" int rth_take_picture(rth_scene* s, const rt_camera* camera, const rt_settings* settings,
                                const rt_filter_cache* filter, const rth_post_settings* post,
                                uint32_t w, uint32_t h, uint32_t spp, uint32_t total_frame_index, int device,
                                const char* bmp_path, rt_stats* stats_out) {
    // "Take picture" (RT/raytracer.cpp:2037-2041): discard the render, samples_per_pixel = picture_spp;
    // render_all_tiles renders the frame, the output pass dithers it into BGRA8 (:2103-2173) and
    // write_bitmap stores it (:2175-2179, RT/assets.cpp:693-724).  The frame and its output pass run
    // on the device (rt_render_picture); only the BGRA8 picture comes back.
    rt_scene* dev = nullptr;
    int err = rt_scene_upload(rth_scene_desc(s), device, &dev);
    if (err) return err;
    rt_settings st = *settings;
    st.samples_per_pixel = spp;
    rt_tile_set tiles = {64, 64, 0, 1};
    rt_post_settings pp = {post->exposure, post->tonemapping, post->srgb_transform, post->midpoint, post->contrast};
    rt_stats stats = {};
    std::vector<uint32_t> bgra((size_t)w*h);
    err = rt_render_picture(dev, camera, &st, filter, &tiles, total_frame_index, w, h, &pp, bgra.data(), &stats);
    rt_scene_free(dev);
    if (err) return err;
    if (!rth_write_bitmap(bmp_path, bgra.data(), w, h)) return RT_ERROR_INVALID;
    printf("Took %ux%u %uspp image in %f seconds.\n", w, h, spp, stats.seconds);   // :2177-2179
    if (stats_out) *stats_out = stats;
    return RT_OK;
}
