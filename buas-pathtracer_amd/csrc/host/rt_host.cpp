// rt_host.cpp — host-side scene model (see include/rt_host.h).
//
// Restates the reference's host code that produces the hot path's inputs:
// scene building (RT/scene.cpp), BVH construction (RT/bvh.cpp), camera setup
// (RT/raytracer.cpp:26-59), presets (RT/raytracer.cpp:795-1470), asset
// formats (RT/assets.cpp) and output (RT/raytracer.cpp:2103-2185).  The
// result is flattened into rt_scene_desc for the device path.
#include "../../../include/rt_host.h"

#include <cmath>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>
#include <array>
#include <chrono>
#include <sys/stat.h>

namespace {

thread_local std::string g_err;
void set_err(const std::string& s) { g_err = s; }

const float PI_32 = 3.14159265359f;     // MathLib/my_math.h:15
const float DEG_TO_RAD = 6.28318530717f / 360.0f;
const float EPSILON = 0.001f;           // RT/common.h:35

// ---------------------------------------------------------------- MathLib
struct V3 { float x, y, z; };
inline V3 v3(float x, float y, float z) { return {x, y, z}; }
inline V3 v3(float s) { return {s, s, s}; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator/(V3 a, V3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
inline V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline V3 operator/(float s, V3 a) { return {s / a.x, s / a.y, s / a.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline float dot(V3 a, V3 b) { return a.x*b.x + a.y*b.y + a.z*b.z; }
inline V3 cross(V3 a, V3 b) { return {a.y*b.z - a.z*b.y, a.z*b.x - a.x*b.z, a.x*b.y - a.y*b.x}; }
inline float length_sq(V3 a) { return dot(a, a); }
inline float length(V3 a) { return sqrtf(dot(a, a)); }
inline V3 normalize(V3 a) { float r = 1.0f / length(a); return a*r; }
inline V3 noz(V3 a) {                                        // MathLib/my_math.h:492-500
    V3 r = {0, 0, 0};
    float lsq = length_sq(a);
    if ((lsq > 0.0001f) && (lsq < INFINITY)) r = a / sqrtf(lsq);
    return r;
}
inline float fmin_(float a, float b) { return a < b ? a : b; }
inline float fmax_(float a, float b) { return a > b ? a : b; }
inline V3 vmin(V3 a, V3 b) { return {fmin_(a.x, b.x), fmin_(a.y, b.y), fmin_(a.z, b.z)}; }
inline V3 vmax(V3 a, V3 b) { return {fmax_(a.x, b.x), fmax_(a.y, b.y), fmax_(a.z, b.z)}; }
inline float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
inline rt_v3 rv(V3 a) { return {a.x, a.y, a.z}; }
inline V3 vr(rt_v3 a) { return {a.x, a.y, a.z}; }

struct AABB { V3 min, max; };
inline AABB inverted_infinity_aabb() { return {v3(FLT_MAX), v3(-FLT_MAX)}; }
inline AABB union_of(AABB a, AABB b) { return {vmin(a.min, b.min), vmax(a.max, b.max)}; }
inline AABB grow(AABB a, V3 p) { return {vmin(a.min, p), vmax(a.max, p)}; }
inline AABB aabb_cr(V3 p, V3 r) { return {p - r, p + r}; }
inline uint32_t largest_axis(AABB a) {                      // MathLib/my_math.h:1113-1129
    V3 d = a.max - a.min;
    uint32_t ax = 0; float m = d.x;
    if (m < d.y) { m = d.y; ax = 1; }
    if (m < d.z) { m = d.z; ax = 2; }
    return ax;
}
inline float surface_area(AABB a) {                         // :1131-1138
    V3 d = a.max - a.min;
    return 2.0f*(d.x*d.y + d.x*d.z + d.y*d.z);
}

rt_m4x4 m_identity() { rt_m4x4 m = {}; for (int i = 0; i < 4; ++i) m.e[i][i] = 1; return m; }
rt_m4x4 m_mul(const rt_m4x4& a, const rt_m4x4& b) {       // :910-921
    rt_m4x4 r = {};
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) for (int k = 0; k < 4; ++k)
        r.e[i][j] += a.e[i][k]*b.e[k][j];
    return r;
}
V3 m_xform(const rt_m4x4& a, V3 p) {                        // transform(a, p, 1) :947-954
    return {p.x*a.e[0][0] + p.y*a.e[0][1] + p.z*a.e[0][2] + 1.0f*a.e[0][3],
            p.x*a.e[1][0] + p.y*a.e[1][1] + p.z*a.e[1][2] + 1.0f*a.e[1][3],
            p.x*a.e[2][0] + p.y*a.e[2][1] + p.z*a.e[2][2] + 1.0f*a.e[2][3]};
}
rt_m4x4 m_translate(V3 t) { rt_m4x4 m = m_identity(); m.e[0][3] = t.x; m.e[1][3] = t.y; m.e[2][3] = t.z; return m; }
rt_m4x4 m_scale(V3 s) { rt_m4x4 m = m_identity(); m.e[0][0] = s.x; m.e[1][1] = s.y; m.e[2][2] = s.z; return m; }
rt_m4x4 m_rot_x(float a) { float c = cosf(a), s = sinf(a); rt_m4x4 m = m_identity();
    m.e[1][1] = c; m.e[1][2] = -s; m.e[2][1] = s; m.e[2][2] = c; return m; }
rt_m4x4 m_rot_y(float a) { float c = cosf(a), s = sinf(a); rt_m4x4 m = m_identity();
    m.e[0][0] = c; m.e[0][2] = s; m.e[2][0] = -s; m.e[2][2] = c; return m; }
rt_m4x4 m_rot_z(float a) { float c = cosf(a), s = sinf(a); rt_m4x4 m = m_identity();
    m.e[0][0] = c; m.e[0][1] = -s; m.e[1][0] = s; m.e[1][1] = c; return m; }

inline rt_m4x4inv T_identity() { return {m_identity(), m_identity()}; }
inline rt_m4x4inv T_translate(V3 t) { return {m_translate(t), m_translate(-t)}; }
inline rt_m4x4inv T_scale(V3 s) { return {m_scale(s), m_scale(1.0f / s)}; }
inline rt_m4x4inv T_rot_x(float a) { return {m_rot_x(a), m_rot_x(-a)}; }
inline rt_m4x4inv T_rot_y(float a) { return {m_rot_y(a), m_rot_y(-a)}; }
inline rt_m4x4inv T_rot_z(float a) { return {m_rot_z(a), m_rot_z(-a)}; }
inline rt_m4x4inv operator*(const rt_m4x4inv& a, const rt_m4x4inv& b) {   // :1009-1015
    return {m_mul(a.forward, b.forward), m_mul(b.inverse, a.inverse)};
}

// ------------------------------------------------------------------ BVH
struct SortEntry { uint32_t index; V3 p, r; };               // BVHSortEntry RT/bvh.h:25-29

struct Partition { uint32_t split_axis = 0, split_index = 0; };

void compute_bv(uint32_t n, const SortEntry* e, AABB* bv, AABB* cr) {      // RT/bvh.cpp:6-17
    AABB b = inverted_infinity_aabb(), c = inverted_infinity_aabb();
    for (uint32_t i = 0; i < n; ++i) { b = union_of(b, aabb_cr(e[i].p, e[i].r)); c = grow(c, e[i].p); }
    *bv = b; *cr = c;
}

Partition partition_objects(uint32_t n, SortEntry* e, float split_p, uint32_t axis) {   // :26-51
    int64_t i = -1, j = (int64_t)n;
    for (;;) {
        do { ++i; } while (i < (int64_t)n - 1 && comp(e[i].p, axis) < split_p);
        do { --j; } while (j > 0 && comp(e[j].p, axis) > split_p);
        if (i >= j) break;
        std::swap(e[i], e[j]);
    }
    Partition r; r.split_axis = axis; r.split_index = (uint32_t)i;
    return r;
}

Partition partition_midpoint(SortEntry* e, AABB bv, uint32_t n) {         // :53-61
    uint32_t axis = largest_axis(bv);
    V3 mid = 0.5f*(bv.min + bv.max);
    return partition_objects(n, e, comp(mid, axis), axis);
}

float evaluate_sah(uint32_t n, const SortEntry* e, float split_p, uint32_t axis) {   // :63-100
    uint32_t lc = 0, rc = 0;
    V3 lmin = v3(FLT_MAX), lmax = v3(-FLT_MAX), rmin = v3(FLT_MAX), rmax = v3(-FLT_MAX);
    for (uint32_t i = 0; i < n; ++i) {
        if (comp(e[i].p, axis) <= split_p) { ++lc; lmin = vmin(lmin, e[i].p - e[i].r); lmax = vmax(lmax, e[i].p + e[i].r); }
        else { ++rc; rmin = vmin(rmin, e[i].p - e[i].r); rmax = vmax(rmax, e[i].p + e[i].r); }
    }
    V3 ld = lmax - lmin, rd = rmax - rmin;
    float la = 2.0f*(ld.x*ld.y + ld.x*ld.z + ld.y*ld.z);
    float ra = 2.0f*(rd.x*rd.y + rd.x*rd.z + rd.y*rd.z);
    return la*(float)lc + ra*(float)rc;
}

Partition partition_sah_full(SortEntry* e, AABB bv, AABB cr, uint32_t n) {      // :102-131
    float parent = (float)n*surface_area(bv);
    float best = parent, best_p = 0.0f;
    uint32_t axis = largest_axis(cr), best_axis = 0;
    for (uint32_t i = 0; i < n; ++i) {
        float sp = comp(e[i].p, axis);
        float s = evaluate_sah(n, e, sp, axis);
        if (best > s) { best = s; best_p = sp; best_axis = axis; }
    }
    Partition r;
    if (best < parent) r = partition_objects(n, e, best_p, best_axis);
    return r;
}

Partition partition_sah_binned(SortEntry* e, AABB bv, AABB cr, uint32_t n) {    // :138-213 (Wald 2007)
    float parent = (float)n*surface_area(bv);
    float best = parent, split_p = 0.0f;
    uint32_t axis = largest_axis(cr);
    const int B = 16;
    struct Bin { uint32_t count; AABB b; };
    Bin bins[B], ls[B], rs[B];
    for (int i = 0; i < B; ++i) { bins[i] = {0, inverted_infinity_aabb()}; ls[i] = rs[i] = bins[i]; }
    float k0 = comp(cr.min, axis);
    float k1 = ((float)B*(1.0f - EPSILON)) / (comp(cr.max, axis) - comp(cr.min, axis));
    for (uint32_t i = 0; i < n; ++i) {
        float f = k1*(comp(e[i].p, axis) - k0);
        uint32_t bi = (f == f && f > 0.0f) ? (uint32_t)f : 0u;   // (u32)NaN -> 0 as on x64
        if (bi >= (uint32_t)B) bi = B - 1;
        bins[bi].count += 1;
        bins[bi].b.min = vmin(bins[bi].b.min, e[i].p - e[i].r);
        bins[bi].b.max = vmax(bins[bi].b.max, e[i].p + e[i].r);
    }
    Bin empty = {0, inverted_infinity_aabb()};
    for (int i = 0; i < B - 1; ++i) {
        const Bin& prev = i > 0 ? ls[i - 1] : empty;
        ls[i].count = prev.count + bins[i].count;
        ls[i].b = union_of(prev.b, bins[i].b);
    }
    for (int i = B - 1; i >= 1; --i) {
        const Bin& prev = i < B - 1 ? rs[i + 1] : empty;
        rs[i].count = prev.count + bins[i].count;
        rs[i].b = union_of(prev.b, bins[i].b);
        float l = (float)ls[i].count*surface_area(ls[i].b);
        float r = (float)rs[i].count*surface_area(rs[i].b);
        float s = l + r;
        if ((s > 0.0f) && (s < best)) { best = s; split_p = k0 + ((float)i / k1); }
    }
    Partition r;
    if (best < parent) r = partition_objects(n, e, split_p, axis);
    return r;
}

struct BvhBuild {
    std::vector<rt_bvh_node> nodes;
    uint32_t node_count = 0;
    SortEntry* data = nullptr;
    int method = RTH_BVH_SAH_BINNED;
};

void construct(BvhBuild& st, uint32_t node_index, uint32_t count, uint32_t first) {   // :222-287
    AABB bv, cr;
    compute_bv(count, st.data + first, &bv, &cr);
    {
        rt_bvh_node& p = st.nodes[node_index];
        p.bv_p = rv(0.5f*(bv.min + bv.max));
        p.bv_r = rv(0.5f*(bv.max - bv.min));
    }
    bool make_leaf = count <= 4;                                 // MIN_PRIMITIVES_PER_BVH_LEAF RT/bvh.h:23
    if (!make_leaf) {
        Partition part;
        switch (st.method) {
            case RTH_BVH_MIDPOINT_SPLIT: part = partition_midpoint(st.data + first, bv, count); break;
            case RTH_BVH_SAH_FULL: part = partition_sah_full(st.data + first, bv, cr, count); break;
            default: part = partition_sah_binned(st.data + first, bv, cr, count); break;
        }
        if ((part.split_index == 0) || (part.split_index > (count - 1))) {
            make_leaf = true;
        } else {
            uint32_t l = st.node_count++;
            uint32_t r = st.node_count++;
            st.nodes[node_index].split_axis = (uint16_t)part.split_axis;
            st.nodes[node_index].left_first = l;
            construct(st, l, part.split_index, first);
            construct(st, r, count - part.split_index, first + part.split_index);
        }
    }
    if (make_leaf) {
        st.nodes[node_index].left_first = first;
        st.nodes[node_index].count = (uint16_t)count;
    }
}

// construct_bvh_internal (:289-326): root at 0, node 1 is padding so sibling pairs share a cache line.
std::vector<rt_bvh_node> build_bvh(std::vector<SortEntry>& entries, int method) {
    BvhBuild st;
    st.nodes.assign(2*(size_t)entries.size() + 2, rt_bvh_node{});
    st.node_count = 2;
    st.data = entries.data();
    st.method = method;
    construct(st, 0, (uint32_t)entries.size(), 0);
    st.nodes.resize(st.node_count);
    return st.nodes;
}

void bvh_info(const std::vector<rt_bvh_node>& nodes, rth_bvh_info* out) {
    memset(out, 0, sizeof(*out));
    out->node_count = (uint32_t)nodes.size();
    if (nodes.empty()) return;
    std::vector<std::pair<uint32_t, uint32_t>> st;
    st.push_back({0, 1});
    while (!st.empty()) {
        auto [n, d] = st.back(); st.pop_back();
        if (d > out->max_depth) out->max_depth = d;
        const rt_bvh_node& nd = nodes[n];
        if (nd.count) { out->leaf_count++; if (nd.count > out->max_leaf_size) out->max_leaf_size = nd.count; }
        else if (n == 0 && nd.left_first == 0) { /* empty tree */ }
        else { st.push_back({nd.left_first, d + 1}); st.push_back({nd.left_first + 1, d + 1}); }
    }
}

// ------------------------------------------------------------ scene data
struct Mesh {
    std::vector<rt_v3> tris;      // BVH order
    std::vector<uint32_t> indices;
    std::vector<rt_v3> normals;   // original order
    std::vector<rt_bvh_node> nodes;
    bool has_normals = false;
};

}  // namespace

struct rth_scene {
    std::vector<rt_material> materials;
    std::vector<rt_primitive> primitives;
    std::vector<rt_primitive> planes;
    std::vector<rt_m4x4inv> transforms;
    std::vector<uint32_t> lights;
    std::vector<Mesh> meshes;
    std::vector<rt_bvh_node> bvh_nodes;
    std::vector<uint32_t> bvh_indices;
    rt_v3 top_sky = {0, 0, 0}, bot_sky = {0, 0, 0};
    uint32_t sky_w = 0, sky_h = 0;
    std::vector<rt_v3> sky;
    std::vector<float> sky_cdf;
    std::vector<rt_mesh> mesh_descs;
    rt_scene_desc desc = {};
};

namespace {

uint32_t add_primitive(rth_scene* s, uint32_t type, uint32_t material_id, const rt_m4x4inv* transform) {  // RT/scene.cpp:70-103
    auto& buf = (type == RT_PRIMITIVE_PLANE) ? s->planes : s->primitives;
    uint32_t id = (uint32_t)buf.size();
    rt_primitive p = {};
    p.type = type;
    p.material_id = material_id;
    if (transform) {                                   // push_transform :63-68
        p.transform_index = (uint32_t)s->transforms.size();
        s->transforms.push_back(*transform);
    } else {
        p.transform_index = 0;                         // static identity_transform :76
    }
    buf.push_back(p);
    if (material_id < s->materials.size() && (s->materials[material_id].flags & RT_MATERIAL_EMISSIVE))
        s->lights.push_back(id);
    return id;
}

// ------------------------------------------------------------ assets
bool read_file(const char* path, std::vector<char>& out) {
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    out.resize((size_t)n + 1);
    size_t got = fread(out.data(), 1, (size_t)n, f);
    fclose(f);
    out[got] = 0;
    out.resize(got + 1);
    return got == (size_t)n;
}

bool file_exists(const std::string& p) { struct stat st; return stat(p.c_str(), &st) == 0; }

// parse_obj (RT/assets.cpp:187-400), CounterClockwise winding: fan-triangulates faces.
bool parse_obj(char* input, std::vector<rt_v3>& tris, std::vector<rt_v3>& normals) {
    std::vector<rt_v3> verts(1, rt_v3{0, 0, 0}), tex(1, rt_v3{0, 0, 0}), nrm(1, rt_v3{0, 0, 0});
    std::vector<rt_v3> t_tris, t_tex, t_nrm;
    char* at = input;
    while (*at) {
        while (*at && (*at == ' ' || *at == '\t' || *at == '\r' || *at == '\n')) ++at;
        char* line_end = at;
        while (*line_end && *line_end != '\r' && *line_end != '\n') ++line_end;
        char* next = line_end;
        if (*next == '\r') ++next;
        if (*next == '\n') ++next;
        if (!*at) break;
        char c = *at++;
        if (c == 'v') {
            std::vector<rt_v3>* target = &verts;
            if (*at == 'n') { ++at; target = &nrm; }
            else if (*at == 't') { ++at; target = &tex; }
            float v[3] = {0, 0, 0};
            for (int i = 0; i < 3; ++i) { char* end; float e = strtof(at, &end); if (end != at) v[i] = e; at = end; }
            target->push_back(rt_v3{v[0], v[1], v[2]});
        } else if (c == 'f') {
            struct Face { uint32_t count = 0; uint32_t idx[32]; } faces[3];
            uint32_t src_counts[3] = {(uint32_t)verts.size(), (uint32_t)tex.size(), (uint32_t)nrm.size()};
            for (;;) {
                for (int fi = 0; fi < 3; ++fi) {
                    Face& f = faces[fi];
                    if (f.count >= 32) { set_err("OBJ PARSE ERROR: Too many vertices for face"); return false; }
                    char* end;
                    long long index = strtoll(at, &end, 0);
                    if (index < 0) index = (long long)src_counts[fi] + index;
                    if (end != at) f.idx[f.count++] = (uint32_t)index;
                    at = end;
                    if (*at == '/') { ++at; }
                    else { while (*at == ' ') ++at; break; }
                }
                if (at >= line_end) break;
            }
            std::vector<rt_v3>* srcs[3] = {&verts, &tex, &nrm};
            std::vector<rt_v3>* dsts[3] = {&t_tris, &t_tex, &t_nrm};
            for (int fi = 0; fi < 3; ++fi) {
                Face& f = faces[fi];
                if (!f.count) continue;
                if (f.count < 3) { set_err("OBJ PARSE ERROR: Not enough vertices to make a face."); return false; }
                for (uint32_t i = 1; i < f.count - 1; ++i) {
                    for (uint32_t k : {f.idx[0], f.idx[i], f.idx[i + 1]}) {
                        if (k >= srcs[fi]->size()) { set_err("OBJ PARSE ERROR: index out of range"); return false; }
                        dsts[fi]->push_back((*srcs[fi])[k]);
                    }
                }
            }
        }
        at = next;
    }
    if (!t_tex.empty() && t_tex.size() != t_tris.size()) { set_err("OBJ PARSE ERROR: Texture coordinates don't match triangles"); return false; }
    if (!t_nrm.empty() && t_nrm.size() != t_tris.size()) { set_err("OBJ PARSE ERROR: Normals don't match triangles"); return false; }
    tris.swap(t_tris);
    if (nrm.size() > 1) normals.swap(t_nrm); else normals.clear();
    return true;
}

// parse_hdr (RT/assets.cpp:423-618) + decode_radiance_color (:411-421)
// match_word_ (:115-129): leading spaces (only ' ') skipped, then a prefix match
bool match_word(char** s, const char* w) {
    char* at = *s;
    while (*at == ' ') ++at;
    size_t n = strlen(w);
    if (strncmp(at, w, n) == 0) { *s = at + n; return true; }
    return false;
}
// parse_u32 (:147-160): strtoul with base 0 (its own whitespace skip; "010" is octal)
bool parse_u32(char** s, uint32_t* out) {
    char* end;
    unsigned long v = strtoul(*s, &end, 0);
    if (end == *s) return false;
    *out = (uint32_t)v; *s = end; return true;
}
bool parse_f32(char** s, float* out) {                 // :132-145
    char* end;
    float v = strtof(*s, &end);
    if (end == *s) return false;
    *out = v; *s = end; return true;
}

bool parse_hdr(const std::vector<char>& file, uint32_t* w_out, uint32_t* h_out, std::vector<rt_v3>& pixels) {
    char* at = const_cast<char*>(file.data());
    const char* file_end = file.data() + file.size() - 1;
    int x_adv = 1, y_adv = -1;
    // the header (:446-492): up to the first empty line; FORMAT and PRIMARIES are read, a
    // missing '=' after either is a malformed header, every other line is skipped.  The XYZ
    // format and unknown formats are read as RGB (the reference warns and goes on).
    while (at < file_end && *at) {
        if (*at == '\n') { ++at; break; }
        if (match_word(&at, "FORMAT")) {
            if (!match_word(&at, "=")) { set_err("HDR PARSE ERROR: Malformed header."); return false; }
            if (!match_word(&at, "32-bit_rle_rgbe")) (void)match_word(&at, "32-bit_rle_xyz");
        } else if (match_word(&at, "PRIMARIES")) {
            if (!match_word(&at, "=")) { set_err("HDR PARSE ERROR: Malformed header."); return false; }
            float prim[8];                                 // parsed and unused, as in the reference
            for (int i = 0; i < 8 && parse_f32(&at, &prim[i]); ++i) {}
        }
        while (at < file_end && *at && *at != '\n') ++at;
        if (at < file_end && *at == '\n') ++at;
    }
    if (at >= file_end || !*at) { set_err("HDR PARSE ERROR: Unexpected end of file while parsing header."); return false; }
    uint32_t w = 0, h = 0;
    if (match_word(&at, "+Y")) y_adv = 1; else if (match_word(&at, "-Y")) y_adv = -1;
    else { set_err("HDR PARSE ERROR: Failed to parse resolution string (+/-Y)."); return false; }
    if (!parse_u32(&at, &h)) { set_err("HDR PARSE ERROR: vertical resolution"); return false; }
    if (match_word(&at, "+X")) x_adv = 1; else if (match_word(&at, "-X")) x_adv = -1;
    else { set_err("HDR PARSE ERROR: Failed to parse resolution string (+/-X)."); return false; }
    if (!parse_u32(&at, &w)) { set_err("HDR PARSE ERROR: horizontal resolution"); return false; }
    if (*at++ != '\n') { set_err("HDR PARSE ERROR: Expected newline after resolution string."); return false; }
    if (!w || !h) { set_err("HDR PARSE ERROR: Malformed resolution."); return false; }
    std::vector<uint8_t> rgbe((size_t)w*h*4, 0);
    const uint8_t* p = (const uint8_t*)at;
    const uint8_t* pend = (const uint8_t*)file_end;
    int64_t row = 0;
    if (x_adv < 0) row += (int64_t)w - 1;
    if (y_adv < 0) row += (int64_t)w*(h - 1);
    for (uint32_t y = 0; y < h; ++y) {
        if (p + 4 > pend) { set_err("HDR PARSE ERROR: truncated"); return false; }
        uint16_t sig = (uint16_t)((p[0] << 8) | p[1]); p += 2;
        if (sig != 0x0202) { set_err("HDR PARSE ERROR: .hdr format unsupported."); return false; }
        uint16_t len = (uint16_t)((p[0] << 8) | p[1]); p += 2;
        if (len != w) { set_err("HDR PARSE ERROR: Scanline length did not match image width."); return false; }
        for (int ch = 0; ch < 4; ++ch) {
            int64_t dst = row;
            for (uint32_t x = 0; x < w;) {
                if (p >= pend) { set_err("HDR PARSE ERROR: truncated"); return false; }
                uint8_t code = *p++;
                if (code > 128) {
                    uint8_t n = code & 127, v = *p++;
                    while (n-- && x < w) { rgbe[4*(size_t)dst + ch] = v; dst += x_adv; ++x; }
                } else {
                    uint8_t n = code;
                    while (n-- && x < w) { rgbe[4*(size_t)dst + ch] = *p++; dst += x_adv; ++x; }
                }
            }
        }
        row += (int64_t)y_adv*(int64_t)w;
    }
    pixels.resize((size_t)w*h);
    for (size_t i = 0; i < (size_t)w*h; ++i) {
        const uint8_t* c = &rgbe[4*i];
        rt_v3 r = {0, 0, 0};
        if (c[3] > 9) {
            uint32_t bits = (uint32_t)(c[3] - 9) << 23;
            float mul; memcpy(&mul, &bits, 4);
            r = rt_v3{mul*((float)c[0] + 0.5f), mul*((float)c[1] + 0.5f), mul*((float)c[2] + 0.5f)};
        }
        pixels[i] = r;
    }
    *w_out = w; *h_out = h;
    return true;
}

// RGBE encode (inverse of decode_radiance_color: value = 2^(e-136) * (m + 0.5))
void encode_rgbe(rt_v3 c, uint8_t out[4]) {
    float v = fmax_(c.x, fmax_(c.y, c.z));
    if (!(v > 1e-32f)) { out[0] = out[1] = out[2] = out[3] = 0; return; }
    int e;
    frexpf(v, &e);                 // v = f * 2^e, f in [0.5,1)
    float scale = ldexpf(1.0f, 8 - e);
    auto q = [&](float x) { float m = x*scale - 0.5f; if (m < 0) m = 0; if (m > 255) m = 255; return (uint8_t)lrintf(m); };
    out[0] = q(c.x); out[1] = q(c.y); out[2] = q(c.z);
    out[3] = (uint8_t)(e + 128);   // decode: 2^((e+128)-9-127) = 2^(e-8)
}

void write_rle_channel(std::vector<uint8_t>& out, const uint8_t* data, uint32_t n) {
    uint32_t i = 0;
    while (i < n) {
        uint32_t run = 1;
        while (i + run < n && run < 127 && data[i + run] == data[i]) ++run;
        if (run >= 3) { out.push_back((uint8_t)(128 + run)); out.push_back(data[i]); i += run; continue; }
        uint32_t lit = 0;
        while (i + lit < n && lit < 128) {
            uint32_t r2 = 1;
            while (i + lit + r2 < n && r2 < 3 && data[i + lit + r2] == data[i + lit]) ++r2;
            if (r2 >= 3) break;
            ++lit;
        }
        out.push_back((uint8_t)lit);
        for (uint32_t k = 0; k < lit; ++k) out.push_back(data[i + k]);
        i += lit;
    }
}

uint32_t hash32(uint32_t x) { x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x; }
float hash_unit(uint32_t seed, uint32_t i) { return (float)(hash32(seed*0x9E3779B9u ^ hash32(i)) >> 8) * (1.0f / 16777216.0f); }

// Synthetic equirect sky: gradient + ground + sun disk (~1e4) + seeded cloud noise.
std::vector<rt_v3> synth_sky(uint32_t w, uint32_t h, uint32_t seed) {
    std::vector<rt_v3> px((size_t)w*h);
    float sun_phi = (float)(2.0*M_PI) * hash_unit(seed, 1) - (float)M_PI;
    float sun_th = 0.35f + 0.5f*hash_unit(seed, 2);
    V3 sun = v3(cosf(sun_th)*cosf(sun_phi), sinf(sun_th), cosf(sun_th)*sinf(sun_phi));
    for (uint32_t y = 0; y < h; ++y) {
        // row y of the image maps to v = (y+0.5)/h; theta = (v-0.5)*pi (sample_sky RT/integrators.cpp:272-295)
        float theta = (((float)y + 0.5f) / (float)h - 0.5f) * (float)M_PI;
        for (uint32_t x = 0; x < w; ++x) {
            float phi = (((float)x + 0.5f) / (float)w - 0.5f) * (float)(2.0*M_PI);
            V3 d = v3(cosf(theta)*cosf(phi), sinf(theta), cosf(theta)*sinf(phi));
            V3 c;
            if (d.y >= 0) {
                float t = powf(d.y, 0.4f);
                c = (1.0f - t)*v3(1.2f, 1.25f, 1.35f) + t*v3(0.25f, 0.45f, 1.1f);
                float n = 0.5f + 0.5f*sinf(7.0f*phi + 3.0f*hash_unit(seed, 3))*sinf(11.0f*theta + 5.0f*hash_unit(seed, 4));
                c = c*(0.85f + 0.3f*n);
            } else {
                c = v3(0.18f, 0.16f, 0.14f)*(0.7f + 0.3f*hash_unit(seed, 1000 + (x/8) + 4096*(y/8)));
            }
            float cs = dot(d, sun);
            if (cs > 0.99985f) c = c + v3(1.0e4f, 0.95e4f, 0.85e4f);
            px[(size_t)y*w + x] = rv(c);
        }
    }
    return px;
}

// Synthetic closed mesh with vertex normals (stands in for dragon_mcguire.obj):
// a seeded, displaced latitude/longitude sphere of radius ~0.35.
void synth_mesh(uint32_t target, uint32_t seed, std::vector<rt_v3>& tris, std::vector<rt_v3>& nrms) {
    uint32_t nv = (uint32_t)std::max(3.0, std::round(0.5 + std::sqrt((double)target / 4.0)));
    uint32_t nu = 2*nv;
    float amp[6], fu[6], fv[6], ph[6];
    for (int k = 0; k < 6; ++k) {
        amp[k] = 0.05f + 0.09f*hash_unit(seed, 10 + k);
        fu[k] = (float)(1 + (hash32(seed*31 + k) % 6));
        fv[k] = (float)(1 + (hash32(seed*57 + k) % 5));
        ph[k] = 6.2831853f*hash_unit(seed, 40 + k);
    }
    auto radius = [&](float th, float phi) {
        float r = 1.0f;
        for (int k = 0; k < 6; ++k) r += amp[k]*sinf(fv[k]*th + ph[k])*cosf(fu[k]*phi + 0.7f*ph[k]);
        return 0.35f*r / 1.4f;
    };
    // vertex grid: row 0 = north pole, row nv = south pole
    std::vector<V3> P((size_t)(nv + 1)*nu);
    for (uint32_t j = 0; j <= nv; ++j) {
        float th = (float)M_PI*(float)j / (float)nv;
        for (uint32_t i = 0; i < nu; ++i) {
            float phi = 6.2831853f*(float)i / (float)nu;
            float r = radius(th, (j == 0 || j == nv) ? 0.0f : phi);
            P[(size_t)j*nu + i] = v3(r*sinf(th)*cosf(phi), r*cosf(th), r*sinf(th)*sinf(phi));
        }
    }
    auto vid = [&](uint32_t j, uint32_t i) { return (size_t)j*nu + (i % nu); };
    std::vector<std::array<size_t, 3>> faces;
    faces.reserve((size_t)4*nv*nv);
    for (uint32_t j = 0; j < nv; ++j)
        for (uint32_t i = 0; i < nu; ++i) {
            size_t a = vid(j, i), b = vid(j, i + 1), c = vid(j + 1, i), d = vid(j + 1, i + 1);
            // outward-facing counter-clockwise winding
            if (j != 0) faces.push_back({a, b, c});
            if (j != nv - 1) faces.push_back({b, d, c});
        }
    std::vector<V3> vn(P.size(), v3(0.0f));
    for (auto& f : faces) {
        V3 n = cross(P[f[1]] - P[f[0]], P[f[2]] - P[f[0]]);
        for (size_t k : f) vn[k] = vn[k] + n;
    }
    // poles: all pole copies share one normal
    for (uint32_t pole : {0u, nv}) {
        V3 s = v3(0.0f);
        for (uint32_t i = 0; i < nu; ++i) s = s + vn[vid(pole, i)];
        for (uint32_t i = 0; i < nu; ++i) vn[vid(pole, i)] = s;
    }
    for (auto& n : vn) n = noz(n);
    tris.clear(); nrms.clear();
    tris.reserve(faces.size()*3); nrms.reserve(faces.size()*3);
    for (auto& f : faces)
        for (size_t k : f) { tris.push_back(rv(P[k])); nrms.push_back(rv(vn[k])); }
}

}  // namespace

// ======================================================================
// C ABI
// ======================================================================
extern "C" {

const char* rth_last_error(void) { return g_err.c_str(); }

rth_scene* rth_scene_create(void) {
    rth_scene* s = new rth_scene();
    s->materials.push_back(rt_material{});      // null material (RT/raytracer.cpp:1426)
    s->primitives.push_back(rt_primitive{});    // null primitive (:1427)
    s->transforms.push_back(T_identity());      // identity_transform (RT/scene.cpp:76)
    return s;
}

void rth_scene_destroy(rth_scene* s) { delete s; }

uint32_t rth_add_material(rth_scene* s, const rt_material* m) {           // RT/scene.cpp:9-21
    uint32_t id = (uint32_t)s->materials.size();
    rt_material mm = *m;
    if (mm.emission_color.x + mm.emission_color.y + mm.emission_color.z > 0.0f) mm.flags |= RT_MATERIAL_EMISSIVE;
    s->materials.push_back(mm);
    return id;
}
uint32_t rth_add_diffuse_material(rth_scene* s, rt_v3 c, float ior, float rough, int32_t checkers, rt_v3 cc) { // :23-37
    rt_material m = {};
    if (checkers) m.flags |= RT_MATERIAL_CHECKERS;
    m.checker_color = cc; m.albedo = c; m.ior = ior; m.roughness = rough;
    s->materials.push_back(m);
    return (uint32_t)s->materials.size() - 1;
}
uint32_t rth_add_translucent_material(rth_scene* s, rt_v3 absorb, float ior, float rough) {  // :39-50
    rt_material m = {};
    m.is_participating_medium = 1; m.absorb = absorb; m.ior = ior; m.roughness = rough;
    s->materials.push_back(m);
    return (uint32_t)s->materials.size() - 1;
}
uint32_t rth_add_emissive_material(rth_scene* s, rt_v3 e) {                // :52-61
    rt_material m = {};
    m.flags |= RT_MATERIAL_EMISSIVE; m.emission_color = e;
    s->materials.push_back(m);
    return (uint32_t)s->materials.size() - 1;
}

uint32_t rth_add_plane(rth_scene* s, uint32_t mat, rt_v3 n, float d) {      // :105-114
    uint32_t id = add_primitive(s, RT_PRIMITIVE_PLANE, mat, nullptr);
    V3 nn = noz(vr(n));
    rt_primitive& p = s->planes[id];
    p.p[0] = nn.x; p.p[1] = nn.y; p.p[2] = nn.z; p.p[3] = d;
    return id;
}
uint32_t rth_add_sphere(rth_scene* s, uint32_t mat, float r, const rt_m4x4inv* t) {   // :116-129
    uint32_t id = add_primitive(s, RT_PRIMITIVE_SPHERE, mat, t);
    s->primitives[id].p[0] = r;
    return id;
}
uint32_t rth_add_box(rth_scene* s, uint32_t mat, rt_v3 r, const rt_m4x4inv* t) {      // :131-144
    uint32_t id = add_primitive(s, RT_PRIMITIVE_BOX, mat, t);
    s->primitives[id].p[0] = r.x; s->primitives[id].p[1] = r.y; s->primitives[id].p[2] = r.z;
    return id;
}
uint32_t rth_add_mesh(rth_scene* s, uint32_t mat, uint32_t mesh_id, const rt_m4x4inv* t) {  // :146-159
    if (mesh_id >= s->meshes.size()) { set_err("rth_add_mesh: bad mesh id"); return 0; }
    uint32_t id = add_primitive(s, RT_PRIMITIVE_MESH, mat, t);
    s->primitives[id].mesh_index = mesh_id;
    return id;
}

// The BVH builder the scene model uses: the host restatement, or (rth_set_bvh_device) the
// device builder rt_build_bvh for the methods it has (midpoint, binned SAH), bit-identical.
static int g_bvh_device = -1;
void rth_set_bvh_device(int device) { g_bvh_device = device; }

static int build_entries(std::vector<SortEntry>& in, int method, std::vector<rt_bvh_node>& nodes) {
    if (g_bvh_device >= 0 && in.size() > 0 && (method == RTH_BVH_MIDPOINT_SPLIT || method == RTH_BVH_SAH_BINNED)) {
        const size_t n = in.size();
        std::vector<rt_v3> p(n), r(n);
        for (size_t i = 0; i < n; ++i) { p[i] = rv(in[i].p); r[i] = rv(in[i].r); }
        nodes.assign(2*n + 2, rt_bvh_node{});
        std::vector<uint32_t> order(n);
        uint32_t count = 0;
        const int err = rt_build_bvh(g_bvh_device, (uint32_t)n, p.data(), r.data(),
                                     method == RTH_BVH_MIDPOINT_SPLIT ? RT_BVH_BUILD_MIDPOINT : RT_BVH_BUILD_SAH_BINNED,
                                     nodes.data(), &count, order.data());
        if (err) { set_err(std::string("rt_build_bvh: ") + rt_build_bvh_last_error()); return err; }
        nodes.resize(count);
        std::vector<SortEntry> out(n);
        for (size_t i = 0; i < n; ++i) out[i] = in[order[i]];
        in.swap(out);
        return 0;
    }
    nodes = build_bvh(in, method);
    return 0;
}

int rth_build_bvh_entries(uint32_t n, const rt_v3* p, const rt_v3* r, int32_t method, rt_bvh_node* out_nodes,
                          uint32_t* out_node_count, uint32_t* out_order) {
    std::vector<SortEntry> in(n);
    for (uint32_t i = 0; i < n; ++i) { in[i].index = i; in[i].p = vr(p[i]); in[i].r = vr(r[i]); }
    std::vector<rt_bvh_node> nodes;
    const int err = build_entries(in, method, nodes);
    if (err) return err;
    memcpy(out_nodes, nodes.data(), nodes.size()*sizeof(rt_bvh_node));
    *out_node_count = (uint32_t)nodes.size();
    for (uint32_t i = 0; i < n; ++i) out_order[i] = in[i].index;
    return 0;
}

// create_bvh_for_mesh (RT/bvh.cpp:342-391, BVHStorage_Scalar)
uint32_t rth_create_mesh(rth_scene* s, uint32_t n, const rt_v3* tris, const rt_v3* normals, int32_t method) {
    std::vector<SortEntry> in(n);
    for (uint32_t i = 0; i < n; ++i) {
        V3 a = vr(tris[3*(size_t)i]), b = vr(tris[3*(size_t)i + 1]), c = vr(tris[3*(size_t)i + 2]);
        V3 mn = vmin(a, vmin(b, c)), mx = vmax(a, vmax(b, c));
        in[i].index = i;
        in[i].p = 0.5f*(mn + mx);
        in[i].r = 0.5f*(mx - mn);
    }
    Mesh m;
    if (build_entries(in, method, m.nodes)) return 0xFFFFFFFFu;
    m.indices.resize(n);
    m.tris.resize(3*(size_t)n);
    for (uint32_t i = 0; i < n; ++i) {
        m.indices[i] = in[i].index;
        for (int k = 0; k < 3; ++k) m.tris[3*(size_t)i + k] = tris[3*(size_t)in[i].index + k];
    }
    if (normals) { m.has_normals = true; m.normals.assign(normals, normals + 3*(size_t)n); }
    s->meshes.push_back(std::move(m));
    return (uint32_t)s->meshes.size() - 1;
}

int rth_load_obj_mesh(rth_scene* s, const char* path, int32_t method, uint32_t* out) {
    std::vector<char> file;
    if (!read_file(path, file)) { set_err(std::string("cannot read ") + path); return 0; }
    std::vector<rt_v3> tris, nrm;
    if (!parse_obj(file.data(), tris, nrm)) return 0;
    if (tris.empty()) { set_err("OBJ has no triangles"); return 0; }
    const uint32_t id = rth_create_mesh(s, (uint32_t)(tris.size()/3), tris.data(), nrm.empty() ? nullptr : nrm.data(), method);
    if (id == 0xFFFFFFFFu) return 0;               // the BVH build failed (rth_last_error says why)
    *out = id;
    return 1;
}

int rth_mesh_bvh_info(rth_scene* s, uint32_t mesh_id, rth_bvh_info* out) {
    if (mesh_id >= s->meshes.size()) return 0;
    bvh_info(s->meshes[mesh_id].nodes, out);
    return 1;
}
int rth_scene_bvh_info(rth_scene* s, rth_bvh_info* out) { bvh_info(s->bvh_nodes, out); return 1; }

void rth_set_sky(rth_scene* s, rt_v3 top, rt_v3 bot) { s->top_sky = top; s->bot_sky = bot; }

}  // extern "C"
int rth_load_environment_map_bytes(rth_scene* s, std::vector<char>& file);
extern "C" {

int rth_load_environment_map(rth_scene* s, const char* path) {              // RT/assets.cpp:620-665
    std::vector<char> file;
    if (!read_file(path, file)) { set_err(std::string("cannot read ") + path); return 0; }
    return rth_load_environment_map_bytes(s, file);
}

}  // extern "C"
static void build_sky_cdf(rth_scene* s);
int rth_load_environment_map_bytes(rth_scene* s, std::vector<char>& file) {
    uint32_t w, h;
    std::vector<rt_v3> px;
    if (!parse_hdr(file, &w, &h, px)) return 0;
    s->sky_w = w; s->sky_h = h; s->sky.swap(px);
    build_sky_cdf(s);
    return 1;
}

extern "C" int rth_set_environment_map(rth_scene* s, uint32_t w, uint32_t h, const rt_v3* pixels) {
    if (!s || !pixels || !w || !h) { set_err("rth_set_environment_map: empty map"); return 0; }
    s->sky_w = w; s->sky_h = h;
    s->sky.assign(pixels, pixels + (size_t)w*h);
    build_sky_cdf(s);
    return 1;
}

static void build_sky_cdf(rth_scene* s) {
    const uint32_t w = s->sky_w, h = s->sky_h;
    // luma CDF over 32x32 tiles: built exactly like the reference, and (like the
    // reference) never read by the integrator (RT/integrators.cpp:230-233).
    uint32_t tw = w / 32, th = h / 32;
    s->sky_cdf.assign((size_t)tw*th, 0.0f);
    if (tw && th) {
        float sum = 0.0f; size_t i = 0;
        for (uint32_t y = 0; y < h && i < s->sky_cdf.size(); y += th)
            for (uint32_t x = 0; x < w && i < s->sky_cdf.size(); x += tw, ++i) {
                float prev = i > 0 ? s->sky_cdf[i - 1] : 0.0f, cur = 0.0f;
                for (uint32_t yy = y; yy < std::min(y + th, h); ++yy)
                    for (uint32_t xx = x; xx < std::min(x + tw, w); ++xx) {
                        rt_v3 p = s->sky[(size_t)yy*w + xx];
                        cur += 0.299f*p.x + 0.587f*p.y + 0.114f*p.z;
                    }
                sum += cur;
                s->sky_cdf[i] = prev + cur;
            }
        float rcp = 1.0f / sum;
        for (auto& c : s->sky_cdf) c *= rcp;
    }
}

extern "C" {
int rth_create_scene_bvh(rth_scene* s) {                                      // RT/scene.cpp:173-242
    std::vector<SortEntry> in;
    for (size_t pi = 1; pi < s->primitives.size(); ++pi) {
        const rt_primitive& p = s->primitives[pi];
        V3 mn = v3(0.0f), mx = v3(0.0f);
        switch (p.type) {
            case RT_PRIMITIVE_SPHERE: mn = v3(-p.p[0]); mx = v3(p.p[0]); break;
            case RT_PRIMITIVE_BOX: mn = -v3(p.p[0], p.p[1], p.p[2]); mx = v3(p.p[0], p.p[1], p.p[2]); break;
            case RT_PRIMITIVE_MESH: {
                const rt_bvh_node& root = s->meshes[p.mesh_index].nodes[0];
                mn = vr(root.bv_p) - vr(root.bv_r); mx = vr(root.bv_p) + vr(root.bv_r);
            } break;
            default: continue;
        }
        const rt_m4x4& m = s->transforms[p.transform_index].forward;
        AABB b = inverted_infinity_aabb();
        b = grow(b, m_xform(m, v3(mn.x, mn.y, mn.z)));
        b = grow(b, m_xform(m, v3(mx.x, mn.y, mn.z)));
        b = grow(b, m_xform(m, v3(mn.x, mx.y, mn.z)));
        b = grow(b, m_xform(m, v3(mn.x, mn.y, mx.z)));
        b = grow(b, m_xform(m, v3(mx.x, mx.y, mn.z)));
        b = grow(b, m_xform(m, v3(mx.x, mn.y, mx.z)));
        b = grow(b, m_xform(m, v3(mn.x, mx.y, mx.z)));
        b = grow(b, m_xform(m, v3(mx.x, mx.y, mx.z)));
        SortEntry e;
        e.index = (uint32_t)pi;
        e.p = 0.5f*(b.min + b.max);
        e.r = 0.5f*(b.max - b.min);
        in.push_back(e);
    }
    if (build_entries(in, RTH_BVH_SAH_BINNED, s->bvh_nodes)) return 0;
    s->bvh_indices.resize(in.size());
    for (size_t i = 0; i < in.size(); ++i) s->bvh_indices[i] = in[i].index;
    return 1;
}

const rt_scene_desc* rth_scene_desc(rth_scene* s) {
    s->mesh_descs.resize(s->meshes.size());
    for (size_t i = 0; i < s->meshes.size(); ++i) {
        const Mesh& m = s->meshes[i];
        rt_mesh& d = s->mesh_descs[i];
        d.triangle_count = (uint32_t)m.indices.size();
        d.has_normals = m.has_normals ? 1u : 0u;
        d.triangles = m.tris.data();
        d.indices = m.indices.data();
        d.normals = m.has_normals ? m.normals.data() : nullptr;
        d.node_count = (uint32_t)m.nodes.size();
        d.nodes = m.nodes.data();
    }
    rt_scene_desc& d = s->desc;
    d.material_count = (uint32_t)s->materials.size(); d.materials = s->materials.data();
    d.primitive_count = (uint32_t)s->primitives.size(); d.primitives = s->primitives.data();
    d.plane_count = (uint32_t)s->planes.size(); d.planes = s->planes.data();
    d.transform_count = (uint32_t)s->transforms.size(); d.transforms = s->transforms.data();
    d.light_count = (uint32_t)s->lights.size(); d.lights = s->lights.data();
    d.mesh_count = (uint32_t)s->mesh_descs.size(); d.meshes = s->mesh_descs.data();
    d.bvh_node_count = (uint32_t)s->bvh_nodes.size(); d.bvh_nodes = s->bvh_nodes.data();
    d.bvh_index_count = (uint32_t)s->bvh_indices.size(); d.bvh_indices = s->bvh_indices.data();
    d.top_sky_color = s->top_sky; d.bot_sky_color = s->bot_sky;
    d.skydome_w = s->sky_w; d.skydome_h = s->sky_h;
    d.skydome = s->sky.empty() ? nullptr : s->sky.data();
    return &s->desc;
}

rt_m4x4inv rth_transform_identity(void) { return T_identity(); }
rt_m4x4inv rth_transform_translate(rt_v3 t) { return T_translate(vr(t)); }
rt_m4x4inv rth_transform_scale(rt_v3 s) { return T_scale(vr(s)); }
rt_m4x4inv rth_transform_rotate_x_axis(float a) { return T_rot_x(a); }
rt_m4x4inv rth_transform_rotate_y_axis(float a) { return T_rot_y(a); }
rt_m4x4inv rth_transform_rotate_z_axis(float a) { return T_rot_z(a); }
rt_m4x4inv rth_transform_mul(rt_m4x4inv a, rt_m4x4inv b) { return a*b; }

void rth_aim_camera(rt_camera* c, rt_v3 d) {                                 // RT/raytracer.cpp:26-40
    V3 z = noz(vr(d));
    V3 x = noz(cross(v3(0, 1, 0), z));
    V3 y = noz(cross(z, x));
    c->z = rv(z); c->x = rv(x); c->y = rv(y);
    float film_w = c->aspect_ratio, film_h = 1.0f;
    c->half_film_w = 0.5f*film_w;
    c->half_film_h = 0.5f*film_h;
    c->film_distance = film_h / tanf(c->vfov);
}
void rth_aim_camera_at(rt_camera* c, rt_v3 at) {                             // :42-48
    V3 cv = vr(at) - vr(c->p);
    V3 cd = normalize(cv);
    rth_aim_camera(c, rv(-cd));
    c->focus_distance = length(cv);
}
void rth_recompute_camera(rt_camera* c) {                                    // :50-59
    float film_w = c->aspect_ratio, film_h = 1.0f;
    c->half_film_w = 0.5f*film_w;
    c->half_film_h = 0.5f*film_h;
    c->film_distance = film_h / tanf(c->vfov);
}

void rth_default_settings(rt_settings* st, rth_post_settings* post) {       // :1430-1452
    memset(st, 0, sizeof(*st));
    st->next_event_estimation = 1;
    st->importance_sample_lights = 1;
    st->importance_sample_diffuse = 1;
    st->use_mis = 1;
    st->russian_roulette = 1;
    st->sampling_strategy = RT_SAMPLING_STRATIFIED;
    st->use_path_guide = 0;
    st->caustics = 1;
    st->lens_distortion = 1.0f;
    st->f_factor = 0.0f;
    st->diaphragm_edges = 6.0f;
    st->phi_shutter_max = 0.5f;
    st->vignette_strength = 0.25f;
    st->samples_per_pixel = 1;
    st->max_bounce_count = 12;
    st->integrator = RT_INTEGRATOR_ADVANCED;
    if (post) {
        memset(post, 0, sizeof(*post));
        post->tonemapping = 1;
        post->srgb_transform = 1;
        post->midpoint = 0.5f;
    }
}

// ---- reconstruction filters (RT/reconstruction_filters.cpp:8-121)
static float sinc_(float x) { return sinf(PI_32*x) / (PI_32*x); }
static float lanczos_(float x, float a) {
    x = fabsf(x);
    if (x < 0.0001f) return 1.0f;
    if (x <= a) return sinc_(x)*sinc_(x / a);
    return 0.0f;
}
static float gaussian_(float x, float alpha, float radius) {
    float re = (float)exp(-alpha*radius*radius);
    return fmax_(0.0f, expf(-alpha*x*x) - re);
}
static float mitchell_(float x) {
    const float B = 1.0f / 3.0f, C = 1.0f / 3.0f;
    x = fabsf(x);
    if (x > 1.0f) return (((-B - 6*C)*x*x*x + (6*B + 30*C)*x*x + (-12*B - 48*C)*x + (8*B + 24*C))*(1.0f / 6.0f));
    return (((12 - 9*B - 6*C)*x*x*x + (-18 + 12*B + 6*C)*x*x + (6 - 2*B))*(1.0f / 6.0f));
}

void rth_load_reconstruction_kernel(const char* name, rt_filter_cache* out) {   // RT/raytracer.cpp:164-185
    memset(out, 0, sizeof(*out));
    int kind = 0; uint32_t radius = 0;
    if (!strcmp(name, "Gaussian 3")) { kind = 1; radius = 3; }
    else if (!strcmp(name, "Gaussian 12")) { kind = 2; radius = 12; }
    else if (!strcmp(name, "Mitchell Netravali")) { kind = 3; radius = 2; }
    else if (!strcmp(name, "Lanczos 3")) { kind = 4; radius = 3; }
    else if (!strcmp(name, "Lanczos 4")) { kind = 5; radius = 4; }
    else if (!strcmp(name, "Lanczos 6")) { kind = 6; radius = 6; }
    else if (!strcmp(name, "Lanczos 12")) { kind = 7; radius = 12; }
    if (!kind) return;                     // "Box": no kernel, plain accumulate
    out->kernel_size = radius;
    out->cache_size = 256;
    for (uint32_t i = 0; i < 256; ++i) {
        float x = ((float)radius*(float)i) / (float)(256 - 1);
        float v = 0;
        switch (kind) {
            case 1: v = gaussian_(x, 3.0f, 3.0f); break;
            case 2: v = gaussian_(x, 0.03f, 12.0f); break;
            case 3: v = mitchell_(x); break;
            case 4: v = lanczos_(x, 3.0f); break;
            case 5: v = lanczos_(x, 4.0f); break;
            case 6: v = lanczos_(x, 6.0f); break;
            default: v = lanczos_(x, 12.0f); break;
        }
        out->cache[i] = v;
    }
}

uint32_t rth_generate_mesh(uint32_t target, uint32_t seed, rt_v3* out_tris, rt_v3* out_nrm) {
    std::vector<rt_v3> t, n;
    synth_mesh(target, seed, t, n);
    if (out_tris) memcpy(out_tris, t.data(), sizeof(rt_v3)*t.size());
    if (out_nrm) memcpy(out_nrm, n.data(), sizeof(rt_v3)*n.size());
    return (uint32_t)(t.size() / 3);
}

int rth_write_synthetic_obj(const char* path, uint32_t target, uint32_t seed) {
    std::vector<rt_v3> t, n;
    synth_mesh(target, seed, t, n);
    FILE* f = fopen(path, "wb");
    if (!f) { set_err(std::string("cannot write ") + path); return 0; }
    fprintf(f, "# synthetic mesh seed %u (%zu triangles)\n", seed, t.size()/3);
    for (auto& v : t) fprintf(f, "v %.9g %.9g %.9g\n", v.x, v.y, v.z);
    for (auto& v : n) fprintf(f, "vn %.9g %.9g %.9g\n", v.x, v.y, v.z);
    for (size_t i = 0; i < t.size()/3; ++i)
        fprintf(f, "f %zu//%zu %zu//%zu %zu//%zu\n", 3*i + 1, 3*i + 1, 3*i + 2, 3*i + 2, 3*i + 3, 3*i + 3);
    if (fclose(f) != 0) { set_err(std::string("cannot write ") + path); return 0; }
    return 1;
}

}  // extern "C"
std::vector<uint8_t> rth_synthetic_hdr_bytes(uint32_t w, uint32_t h, uint32_t seed) {
    std::vector<rt_v3> px = synth_sky(w, h, seed);
    std::vector<uint8_t> out;
    const char* hdr = "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n";
    out.insert(out.end(), hdr, hdr + strlen(hdr));
    char res[64];
    snprintf(res, sizeof(res), "-Y %u +X %u\n", h, w);
    out.insert(out.end(), res, res + strlen(res));
    std::vector<uint8_t> ch(4*(size_t)w);
    // "-Y": the first scanline in the file is image row h-1 (parse_hdr walks rows upward)
    for (uint32_t yy = 0; yy < h; ++yy) {
        uint32_t y = h - 1 - yy;
        for (uint32_t x = 0; x < w; ++x) {
            uint8_t e[4];
            encode_rgbe(px[(size_t)y*w + x], e);
            for (int c = 0; c < 4; ++c) ch[(size_t)c*w + x] = e[c];
        }
        out.push_back(2); out.push_back(2); out.push_back((uint8_t)(w >> 8)); out.push_back((uint8_t)(w & 255));
        for (int c = 0; c < 4; ++c) write_rle_channel(out, &ch[(size_t)c*w], w);
    }
    return out;
}

extern "C" {
int rth_write_synthetic_hdr(const char* path, uint32_t w, uint32_t h, uint32_t seed) {
    std::vector<uint8_t> out = rth_synthetic_hdr_bytes(w, h, seed);
    FILE* f = fopen(path, "wb");
    if (!f) { set_err(std::string("cannot write ") + path); return 0; }
    fwrite(out.data(), 1, out.size(), f);
    if (fclose(f) != 0) { set_err(std::string("cannot write ") + path); return 0; }
    return 1;
}

static float sigmoidal_contrast(float x, float contrast, float midpoint) {   // RT/raytracer.cpp:69-84
    float curve;
    if (x < midpoint) { float sc = (1.0f / midpoint)*x; curve = midpoint*(sc*sc); }
    else { float y = (1.0f / (1.0f - midpoint)); float sc = y - y*x; curve = 1.0f - (1.0f - midpoint)*(sc*sc); }
    return x*(1.0f - contrast) + curve*contrast;
}

void rth_resolve_bgra8(const rt_accumulation_buffer* a, const rth_post_settings* post, uint32_t* out) {
    size_t n = (size_t)a->w*a->h;
    for (size_t i = 0; i < n; ++i) {                                         // RT/raytracer.cpp:2111-2171
        const float* s = a->pixels + 4*i;
        V3 c = v3(0.0f);
        if (s[0] != s[0] || s[1] != s[1] || s[2] != s[2] || s[3] != s[3]) {
            c = v3(0, 255, 255);
        } else if (s[3] > 0.001f) {
            c = v3(s[0], s[1], s[2]) / s[3];
            c = vmax(c, v3(0.0f));
            if (post->exposure != 0.0f) c = c*powf(2, post->exposure);
            if (post->tonemapping) { c.x = 1.0f - expf(-c.x); c.y = 1.0f - expf(-c.y); c.z = 1.0f - expf(-c.z); }
            if (post->srgb_transform) {
                c.x = powf(c.x, 1.0f / 2.23333f); c.y = powf(c.y, 1.0f / 2.23333f); c.z = powf(c.z, 1.0f / 2.23333f);
            }
            if (post->contrast != 0.0f) {
                c.x = sigmoidal_contrast(c.x, post->contrast, post->midpoint);
                c.y = sigmoidal_contrast(c.y, post->contrast, post->midpoint);
                c.z = sigmoidal_contrast(c.z, post->contrast, post->midpoint);
            }
            c = c*255.0f;
            c = c + v3(0.5f);   // the reference adds 0.5 + TPDF blue-noise dither here
        } else if (s[3] < -0.01f) {
            c = v3(-255.0f*s[3], 0.0f, -255.0f*s[3]);
        }
        auto q = [](float x) { return (uint32_t)(uint8_t)(x < 0.0f ? 0.0f : (x > 255.0f ? 255.0f : x)); };
        out[i] = (255u << 24) | (q(c.x) << 16) | (q(c.y) << 8) | q(c.z);
    }
}

int rth_write_bitmap(const char* path, const uint32_t* px, uint32_t w, uint32_t h) {   // RT/assets.cpp:693-724
#pragma pack(push, 1)
    struct Hdr {
        uint16_t file_type; uint32_t file_size; uint16_t r1, r2; uint32_t offset; uint32_t size;
        int32_t width, height; uint16_t planes, bpp; uint32_t compression, size_of_bitmap;
        int32_t hres, vres; uint32_t colors_used, colors_important;
    } hd = {};
#pragma pack(pop)
    uint32_t psize = 4u*w*h;
    hd.file_type = 0x4D42; hd.file_size = (uint32_t)sizeof(hd) + psize; hd.offset = sizeof(hd);
    hd.size = sizeof(hd) - 14; hd.width = (int32_t)w; hd.height = -(int32_t)h; hd.planes = 1; hd.bpp = 32;
    hd.size_of_bitmap = psize; hd.hres = 4096; hd.vres = 4096;
    FILE* f = fopen(path, "wb");
    if (!f) { set_err(std::string("BMP WRITE ERROR: Failed to write output file ") + path); return 0; }
    fwrite(&hd, sizeof(hd), 1, f);
    fwrite(px, 4, (size_t)w*h, f);
    fclose(f);
    return 1;
}

int rth_read_bitmap(const char* path, uint32_t* px, uint32_t w, uint32_t h) {   // the layout write_bitmap writes
    FILE* f = fopen(path, "rb");
    if (!f) { set_err(std::string("cannot open ") + path); return 0; }
    unsigned char hd[54];
    int ok = fread(hd, 1, sizeof(hd), f) == sizeof(hd);
    uint32_t off = 0; int32_t bw = 0, bh = 0; uint16_t bpp = 0;
    if (ok) { memcpy(&off, hd + 10, 4); memcpy(&bw, hd + 18, 4); memcpy(&bh, hd + 22, 4); memcpy(&bpp, hd + 28, 2); }
    ok = ok && hd[0] == 'B' && hd[1] == 'M' && bpp == 32 && bw == (int32_t)w && bh == -(int32_t)h &&
         fseek(f, (long)off, SEEK_SET) == 0 && fread(px, 4, (size_t)w*h, f) == (size_t)w*h;
    fclose(f);
    if (!ok) set_err(std::string("not a top-down 32-bit bitmap of the expected size: ") + path);
    return ok;
}

}  // extern "C"
