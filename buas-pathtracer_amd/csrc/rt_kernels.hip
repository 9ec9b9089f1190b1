// rt_kernels.hip — gfx950 wavefront path tracer: kernels + the rt_abi.h C ABI.
//
// Reference hot path (RT/ = /root/reference/Raytracer/):
//   render_tile            RT/raytracer.cpp:366-495   -> k_generate (ray setup; splat of finished paths)
//   advanced_integrator    RT/integrators.cpp:581-821 -> k_shade (one bounce per launch)
//   intersect_scene        RT/intersection.cpp:606    -> k_trace (the extension queue)
//   intersect_shadow_ray   RT/intersection.cpp:600    -> k_trace (the previous iteration's shadow queue)
//   samplers / RNG         RT/samplers.{h,cpp}        -> rt_dmath.h + sample_1d/2d below
//   splat_filter           RT/raytracer.cpp:187-259   -> splat_sample records + k_resolve
//
// Wavefront loop: a pool of N in-flight paths lives in HBM as
// structure-of-arrays with a state byte per slot.  One iteration = generate ->
// trace -> shade -> bookkeep, each a separate kernel: trace takes this iteration's
// extension rays and the previous shade's shadow rays, generate first splats the
// paths the shade two iterations back finished (their last NEE terms came in the
// trace in between).
// generate / shade walk the pool in slot order; the two tracers
// consume compacted queues (extension rays, shadow rays) that those kernels
// append to with wave-aggregated atomics (__ballot + popcount + one atomic per
// wavefront).  Paths are regenerated into freed slots every iteration so the
// pool stays full.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <string>
#include <vector>
#include <chrono>
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <mutex>
#include <cerrno>

#include "rt_dmath.h"

using namespace rtd;

#define HIP_OK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { set_error(std::string(#x) + ": " + hipGetErrorString(e_)); return RT_ERROR_DEVICE; } } while (0)

namespace {
thread_local std::string g_error;
void set_error(const std::string& s) { g_error = s; }
uint32_t g_profiling = 0;       // stage mask: bit k = rt_kernel_stage k timed with HIP events
uint32_t g_pool_override = 0;
int g_splat_mode = RT_SPLAT_STREAM;
int g_env_sampling = 0;         // rt_set_env_sampling
int g_shard_mode = RT_SHARD_TILES;   // rt_set_shard_mode
}

// Tables embedded from data/ (extracted from the reference by tools/extract_tables.py).
extern "C" const unsigned char rt_dev_strata_tab[16384];
extern "C" const unsigned char rt_dev_bluenoise_tab[327680];
extern "C" const unsigned char rt_dev_dither_tab[8*256*256*3];

// ======================================================================
// Device scene
// ======================================================================
struct DevMesh { uint32_t tri_offset, node_offset, has_normals, pad; };

struct DevScene {
    const rt_material* materials;   // [material_count] + air at [material_count]
    uint32_t material_count;
    uint32_t air_id;
    const rt_primitive* prims;
    const rt_primitive* planes;
    const float4* plane_nd;         // the planes' p[0..3] (normal, distance) packed, padded to a multiple of 4 (the prologue's scalar loads)
    uint32_t plane_count;
    const M34* inv;                 // per transform: inverse (rows 0-2)
    const M34* fwd;                 // per transform: forward (rows 0-2)
    const uint32_t* lights;
    uint32_t light_count;
    const rt_bvh_node* bvh;         // traversal layout: {bv_p, bv_r.x}, {bv_r.yz, packed record, 0} (see pack_node)
    const rt_bvh_node* bvh_src;     // the caller's layout (records that do not pack)
    uint32_t bvh_root_rec;          // the top-level root's packed stack record
    const float4* top_seq;          // top level in the ray prologue: [8 octants][top_seq_len] x 2 float4, or null
    uint32_t top_seq_len;
    uint32_t mlist_max;             // mesh-list capacity, <= MLIST_MAX (RT_MLIST_MAX lowers it for tests)
    uint32_t listed_only;           // top_seq and no more mesh slots than mlist_max: no ray is MLIST_FULL
    uint32_t finite_boxes;          // every node box within 2^40 of the origin (finite_box_ray)
    const uint32_t* bvh_idx;
    const float4* leaf_rec;         // [bvh_index_count][LEAF_REC_Q]: everything a top-level leaf step needs
    uint32_t bvh_node_count;
    const DevMesh* meshes;
    const float4* tris;             // 3 float4 per triangle: a, b-a, c-a (BVH order, all meshes)
    const uint32_t* tri_orig;       // mesh-local original triangle index per BVH slot
    const float* normals;           // 9 floats per triangle, BVH slot order (same index as tris)
    const rt_bvh_node* mnodes;      // all mesh BVH nodes (child indices mesh-local), traversal layout
    const rt_bvh_node* mnodes_src;  // the same in the caller's layout
    const float4* mnodes4;          // mesh BVH4 nodes (MESH_BVH4), 8 float4 each, global indices
    // per BVH4 node: the boxes of the BVH2 node's two children (the level the BVH4 skips), 3 float4:
    // {pL.xyz, rL.x}, {rL.yz, pR.xy}, {pR.z, rR.xyz} -- read only when counting in the reference's units
    const float4* mid4;
    const float* sky;               // 3 floats per pixel
    uint32_t sky_w, sky_h;
    // environment-map sampling table (rt_set_env_sampling): per luma tile {alias threshold,
    // alias tile, density}, env_tx tiles per row of env_tw x env_th texels; null = no map
    const float4* env_tab;
    uint32_t env_n, env_tx, env_tw, env_th;
    V3 top_sky, bot_sky;
    const uint8_t* strata;          // g_strata_permutation_sets [256][64]
    const uint8_t* bluenoise;       // sobol | scrambling | ranking
    // The small tables above (materials, primitives, planes, transforms, lights, meshes)
    // packed into one blob that k_shade copies into LDS at start (scene_in_lds); 0 = too large.
    const float4* blob;
    uint32_t blob_q;                // float4 count (<= LDS_SCENE_Q)
    uint32_t off[7];                // byte offsets of the tables in the blob (BLOB_*)
};
// The 16 KB strata table is read at bounce 0 only (a few lookups per path): copying
// it into every block's LDS costs more than the L2 reads it saves, so it stays in HBM.
// The ray prologue's tables (top-level sequence, leaf records) stay in HBM too --
// scene_in_lds does not rebase them -- and its wave-uniform walk reads them with s_load
// through the scalar cache: no LDS round trip and no readfirstlane per value
// (ld_uniform's scalar load needs a global address).
enum { BLOB_MATERIALS, BLOB_PRIMS, BLOB_PLANES, BLOB_INV, BLOB_FWD, BLOB_LIGHTS, BLOB_MESHES, BLOB_COUNT };
constexpr uint32_t LDS_SCENE_Q = 2048;   // 32 KB
// The copy is the launch's dynamic LDS, sized to the blob (blob_q float4): a fixed
// 32 KB array held 256-thread blocks to 5 per CU whatever the scene's size.
extern __shared__ float4 lds_scene[];

// The scene seen through the LDS copy: every small table's pointer rebased onto
// `lds` (generic pointers, so the code that reads them is unchanged).  All
// threads of the block must call it.
// IN_LDS (the caller launched with the blob in LDS: DevScene::blob_q != 0): the rebased pointers
// are LDS pointers on every path, so the compiler emits ds_read for the table lookups.  Left to
// a run-time choice between the copy and HBM, the pointers are generic and every lookup is a
// FLAT load: a vector-memory instruction that also waits on the LDS counter.
template <bool IN_LDS = false>
RT_D DevScene scene_in_lds(const DevScene& sc, float4* lds) {
    if (!IN_LDS && !sc.blob_q) return sc;
    for (uint32_t i = threadIdx.x; i < sc.blob_q; i += blockDim.x) lds[i] = sc.blob[i];
    __syncthreads();
    DevScene s = sc;
    const char* b = reinterpret_cast<const char*>(lds);
    s.materials = reinterpret_cast<const rt_material*>(b + sc.off[BLOB_MATERIALS]);
    s.prims = reinterpret_cast<const rt_primitive*>(b + sc.off[BLOB_PRIMS]);
    s.planes = reinterpret_cast<const rt_primitive*>(b + sc.off[BLOB_PLANES]);
    s.inv = reinterpret_cast<const M34*>(b + sc.off[BLOB_INV]);
    s.fwd = reinterpret_cast<const M34*>(b + sc.off[BLOB_FWD]);
    s.lights = reinterpret_cast<const uint32_t*>(b + sc.off[BLOB_LIGHTS]);
    s.meshes = reinterpret_cast<const DevMesh*>(b + sc.off[BLOB_MESHES]);
    return s;
}

struct Ray { V3 o, d, inv_d; uint32_t neg; float max_t; uint32_t zero; };   // zero: axes with d == 0

RT_D Ray make_ray(V3 o, V3 d, float far_clip) {              // RT/intersection.h:13-24
    Ray r;
    r.o = o; r.d = d;
    r.inv_d = rcp3(d);
    r.neg = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    r.zero = (d.x == 0.0f ? 1u : 0u) | (d.y == 0.0f ? 2u : 0u) | (d.z == 0.0f ? 4u : 0u);
    r.max_t = far_clip;
    return r;
}

// ---------------------------------------------------------------- primitives
RT_D bool ray_plane(const Ray& ray, V3 n, float d, float& t) {       // RT/intersection.cpp:12-42
    float denom = dot(n, ray.d);
    if (denom < -EPSILON) {
        float tt = (d - dot(n, ray.o)) / denom;
        if ((tt >= EPSILON) && (tt < t)) { t = tt; return true; }
    }
    return false;
}
RT_D bool ray_sphere(const Ray& ray, float r, float& t) {           // :44-74
    V3 o = ray.o;
    float rsq = r*r;
    float b = dot(ray.d, o);
    float c = dot(o, o) - rsq;
    float discr = (b*b - c);
    if (discr >= 0) {
        float root = __builtin_sqrtf(discr);
        float tn = -b - root;
        float tf = -b + root;
        float tt = (tn >= 0.0f ? tn : tf);
        if ((tt >= EPSILON) && (t > tt)) { t = tt; return true; }
    }
    return false;
}
RT_D bool ray_box(const Ray& ray, V3 br, float& t) {               // :76-105
    V3 m = ray.inv_d;
    V3 n = mul(m, ray.o);
    V3 k = mul(vabs(m), br);
    V3 t1 = sub(neg(n), k);
    V3 t2 = add(neg(n), k);
    float tn = mx(mx(t1.x, t1.y), t1.z);
    float tf = mn(mn(t2.x, t2.y), t2.z);
    if (tn < tf) {
        float tt = (tn >= 0.0f ? tn : tf);
        if ((t > tt) && (tt >= EPSILON)) { t = tt; return true; }
    }
    return false;
}
// ray_intersect_bounding_volume (:107-133) split into the ray/box part (static)
// and the far-clip test against the current t, done when the node is popped.
//
// Degenerate-axis pruning (a performance change that leaves results intact):
// when a ray component is exactly 0, inv_d is +-inf and the reference's slab
// test yields NaN on that axis, which the ternary max/min then drop, so the
// axis is never tested and such a ray visits every node whose other slabs it
// crosses (~40k nodes of a 70k-triangle mesh for a ray grazing the floor: a
// 40 ms single-lane tail per launch).  Such a ray keeps that coordinate
// constant, so a node whose slab on that axis excludes the origin (by more
// than 1 % of the node's largest half extent, far above the barycentric
// round-off of the triangle test) contains nothing it can hit: it is skipped.
// Nodes that are kept get the reference's tn, so visit order, far-clip
// culling and tie-breaking are unchanged.  Applied inside mesh BVHs only:
// their leaves hold triangles, whose test is exact for such rays, while the
// top level holds box primitives whose ray_intersect_box (:76-105) has the
// same NaN quirk and reports hits the reference keeps (tests/test_gpu_parity.py
// checks axis-parallel rays against the unpruned oracle).
// FINITE: the caller guarantees no slab value is NaN (finite_box_ray below), so the
// reference's ternary max/min chains equal v_max3/v_min3 (a +-0 difference compares equal).
template <bool FINITE = false>
RT_D bool bv_static(const Ray& ray, V3 p, V3 r, float& tn_out) {
    V3 rel = sub(ray.o, p);
    V3 m = ray.inv_d;
    V3 n = mul(m, rel);
    V3 k = mul(vabs(m), r);
    V3 t1 = sub(neg(n), k);
    V3 t2 = add(neg(n), k);
    float tn, tf;
    if (FINITE) {
        tn = fmaxf(fmaxf(t1.x, t1.y), t1.z);
        tf = fminf(fminf(t2.x, t2.y), t2.z);
    } else {
        tn = mx(mx(t1.x, t1.y), t1.z);
        tf = mn(mn(t2.x, t2.y), t2.z);
    }
    tn_out = tn;
    bool hit = (tn < tf) && (tf > 0.0f);
    if (!FINITE && hit && ray.zero) {
        // margin: 1 % of the node's largest half extent (a triangle's barycentric error is
        // relative to its own size, which the box bounds) plus 1e-5 of its position
        const float margin = 0.01f*mx(r.x, mx(r.y, r.z)) + 1e-5f*mx(fabsf(p.x), mx(fabsf(p.y), fabsf(p.z)));
        if ((ray.zero & 1u) && fabsf(rel.x) > r.x + margin) hit = false;
        if ((ray.zero & 2u) && fabsf(rel.y) > r.y + margin) hit = false;
        if ((ray.zero & 4u) && fabsf(rel.z) > r.z + margin) hit = false;
    }
    return hit;
}
// Slab values stay finite when |1/d| <= 2^40, |o| <= 2^40 and every box of the scene
// lies within 2^40 of the origin (DevScene::finite_boxes): |o - p| * |1/d| < 2^81.
constexpr float FINITE_LIM = 1099511627776.0f;   // 2^40
RT_D bool finite_box_ray(V3 o, V3 inv_d) {
    return fabsf(inv_d.x) <= FINITE_LIM && fabsf(inv_d.y) <= FINITE_LIM && fabsf(inv_d.z) <= FINITE_LIM &&
           fabsf(o.x) <= FINITE_LIM && fabsf(o.y) <= FINITE_LIM && fabsf(o.z) <= FINITE_LIM;
}
RT_D bool ray_triangle(const Ray& ray, V3 a, V3 e1, V3 e2, float& t, float& ov, float& ow) {   // :135-182
    const float eps = 0.000000001f;
    V3 pvec = cross(ray.d, e2);
    float det = dot(e1, pvec);
    if (det > -eps && det < eps) return false;
    float inv_det = rcp_cr(det);
    V3 tvec = sub(ray.o, a);
    float v = dot(tvec, pvec)*inv_det;
    if (v < 0.0f || v > 1.0f) return false;
    V3 qvec = cross(tvec, e1);
    float w = dot(ray.d, qvec)*inv_det;
    if (w < 0.0f || v + w > 1.0f) return false;
    float tt = dot(e2, qvec)*inv_det;
    if ((tt < eps) || (t < tt)) return false;
    t = tt; ov = v; ow = w;
    return true;
}

RT_D M34 load_m34(const M34* p) { return *p; }
RT_D V3 ld3(const float4& f) { return {f.x, f.y, f.z}; }

RT_D void load_node(const rt_bvh_node* nodes, uint32_t i, V3& p, V3& r, uint32_t& lf, uint32_t& cnt, uint32_t& axis) {
    const float4* q = reinterpret_cast<const float4*>(nodes + i);
    float4 a = q[0], b = q[1];
    p = {a.x, a.y, a.z};
    r = {a.w, b.x, b.y};
    lf = __float_as_uint(b.z);
    uint32_t ca = __float_as_uint(b.w);
    cnt = ca & 0xFFFFu;
    axis = ca >> 16;
}
RT_D void load_child_boxes(const rt_bvh_node* nodes, uint32_t left, V3& p0, V3& r0, V3& p1, V3& r1) {
    const float4* q = reinterpret_cast<const float4*>(nodes + left);
    float4 a = q[0], b = q[1], c = q[2], d = q[3];
    p0 = {a.x, a.y, a.z}; r0 = {a.w, b.x, b.y};
    p1 = {c.x, c.y, c.z}; r1 = {c.w, d.x, d.y};
}

// A stack entry carries the node's own traversal record, so a pop needs no node
// load (the parent already loaded it to box-test it):
//   bit 31 = 0: bit 30 = leaf; leaf: bits 25-29 = count (1..31), bits 0-24 = first;
//               interior: bits 28-29 = split axis, bits 0-27 = left child
//   bit 31 = 1: bits 0-30 = node index (the record does not fit; the pop loads the node)
__host__ __device__ inline uint32_t pack_node(uint32_t idx, uint32_t lf, uint32_t cnt, uint32_t axis) {
    if (cnt) {
        if (cnt < 32u && lf < (1u << 25)) return (1u << 30) | (cnt << 25) | lf;
    } else if (axis < 4u && lf < (1u << 28)) {
        return (axis << 28) | lf;
    }
    return 0x80000000u | idx;
}
RT_D void unpack_node(const rt_bvh_node* nodes, uint32_t x, uint32_t& lf, uint32_t& cnt, uint32_t& ax) {
    const bool leaf = (x >> 30) & 1u;
    cnt = leaf ? (x >> 25) & 31u : 0u;
    lf = x & (leaf ? 0x1FFFFFFu : 0x0FFFFFFFu);
    ax = leaf ? 0u : (x >> 28) & 3u;
    if (x & 0x80000000u) {                                  // rare: the record did not fit
        V3 p, r;
        load_node(nodes, x & 0x7FFFFFFFu, p, r, lf, cnt, ax);
    }
}

// Top-level leaf record (one per bvh_indices slot, built at upload): the
// primitive's inverse transform, type and size, and for a mesh its offsets and
// root node, so a top-level leaf step is one round of independent loads.
//   q0-q2: inverse rows | q3: prim id, type, then
//   sphere/box: q3.zw = p[0], p[1]; q4.x = p[2]
//   mesh:       q3.zw = node_off, tri_off; q4 = root record, root bv_p.xyz; q5 = root bv_r.xyz
constexpr int LEAF_REC_Q = 6;
// q3.y: the primitive type in bits 0-7; LEAF_TRANSLATE: the inverse's 3x3 part is
// exactly the identity and its translation finite (spheres and unrotated boxes)
constexpr uint32_t LEAF_TRANSLATE = 0x100u;

// transform_ray (RT/intersection.cpp:403-409) into a leaf record's object space.  For a
// translation-only inverse the 3x4 products reduce to adding the translation, bit for
// bit, when every component of o and d is finite and non-zero (`plain`): x*1 = x,
// y*0 = +-0 and x + (+-0) = x for x != 0, and 0*t = +-0 for a finite t.  A wave with a
// lane that is not plain takes the full product for that lane.
RT_D bool plain_ray(V3 o, V3 d) {
    const V3 ao = vabs(o), ad = vabs(d);
    const float m = fminf(fminf(fminf(ao.x, ao.y), fminf(ao.z, ad.x)), fminf(ad.y, ad.z));
    const float sum = ((ao.x + ao.y) + (ao.z + ad.x)) + (ad.y + ad.z);   // NaN or inf (or overflow): not plain
    return m > 0.0f && sum < __builtin_inff();
}
RT_D void object_ray(float4 q0, float4 q1, float4 q2, bool translate, bool plain, V3 o, V3 d, V3& io, V3& id) {
    if (translate && plain) {
        io = {o.x + q0.w, o.y + q1.w, o.z + q2.w};
        id = d;
    } else {
        M34 inv;
        inv.e[0][0] = q0.x; inv.e[0][1] = q0.y; inv.e[0][2] = q0.z; inv.e[0][3] = q0.w;
        inv.e[1][0] = q1.x; inv.e[1][1] = q1.y; inv.e[1][2] = q1.z; inv.e[1][3] = q1.w;
        inv.e[2][0] = q2.x; inv.e[2][1] = q2.y; inv.e[2][2] = q2.z; inv.e[2][3] = q2.w;
        io = xform(inv, o, 1.0f);
        id = xform(inv, d, 0.0f);
    }
}

// ----------------------------------------------------------------------
// Scene traversal as a step machine.
//
// intersect_scene_internal (RT/intersection.cpp:411-598) restated as a
// sequence of small steps (one node, one leaf primitive or one mesh leaf per
// step) so that a persistent wave can refill lanes whose ray has finished
// instead of idling until the slowest lane's nested mesh traversal ends.
// The visit order is exactly the reference's: planes first, then the
// top-level BVH front-to-back by d_is_negative[split_axis]; each leaf's
// primitives in order, a mesh instance traversed completely (its own BVH,
// object-space ray) before the leaf's next primitive; far-clip culling of a
// node against the current t when the node is popped.  Children are box-
// tested when their parent is expanded and only hits are pushed together
// with their entry distance tn, which is exactly the reference's pop-time
// test (ray_intersect_bounding_volume, :107-133) split in two.
//
// Stack: per-lane, STACK_LDS entries in LDS ([level][lane], bank-conflict
// free), deeper levels spill to a per-thread global area.  Total depth 64 =
// the reference's node_stack[64] (:261, :445).
// ----------------------------------------------------------------------
constexpr int STACK_DEPTH = 64;
constexpr int STACK_LDS = 16;

struct Hit {
    float t;
    uint32_t code;      // RT_HIT_MISS | RT_HIT_PLANE_BIT|plane | primitive index
    uint32_t tri;       // global BVH-order triangle slot of the closest mesh hit
    float v, w;         // barycentrics of that triangle (uvw = (1-v-w, v, w))
};

// SL: the levels kept in LDS (STACK_LDS; the trace kernels' TRACE_STACK_LDS)
template <int SL>
struct StackT {
    uint2* lds;         // [SL][block] for this block
    uint2* spill;       // [STACK_DEPTH - SL][nthreads] global
    float2* bary;       // [block] the lane's closest-hit barycentrics (v, w), in LDS: out of the
                        // registers the traversal step holds (the listed extend kernel: 100 -> 96 VGPRs)
    uint32_t lane, block, gtid, nthreads;
    // LDS_ONLY: the caller knows every level it touches is below SL
    template <bool LDS_ONLY = false>
    RT_D void put(int level, uint32_t node, float tn) const {
        uint2 e = make_uint2(node, __float_as_uint(tn));
        if (LDS_ONLY || level < SL) lds[level*block + lane] = e;
        else spill[(size_t)(level - SL)*nthreads + gtid] = e;
    }
    template <bool LDS_ONLY = false>
    RT_D uint2 get(int level) const {
        return (LDS_ONLY || level < SL) ? lds[level*block + lane] : spill[(size_t)(level - SL)*nthreads + gtid];
    }
};
using Stack = StackT<STACK_LDS>;

enum { TM_TOP = 0, TM_LEAF = 1, TM_MESH = 2, TM_DONE = 3 };

// Each step is: pops (LDS only) until the lane holds a node that survives the
// far-clip test, ONE round of independent global loads for whatever the lane
// does next (a sibling pair of nodes, up to TRI_FETCH triangles of a leaf, or a
// top-level leaf record), then the arithmetic.  Lanes doing different kinds of
// work in the same step therefore share one memory latency.
constexpr uint32_t TRI_FETCH = 2;
// Mesh BVHs are traversed as BVH4: each interior node of the caller's BVH2 is
// merged with its interior children (built at upload, build_bvh4).  A node holds
// up to 4 children in SoA form, one 128-byte line:
//   F[0..2] = bv_p.x/y/z of children 0-3, F[3..5] = bv_r.x/y/z, F[6] = their packed
//   records (EMPTY4: no child), F[7].x = split axes: bits 0-1 the BVH2 node's,
//   2-3 its left child's (children 0,1), 4-5 its right child's (children 2,3).
// The children are visited in exactly the BVH2 depth-first order (the reference's
// front-to-back order by d_is_negative, RT/intersection.cpp:328-340); the BVH2
// level in between is skipped, i.e. its box test, which only culls what its
// children's own tests cull (their boxes lie inside it).  Halves the interior steps.
constexpr uint32_t EMPTY4 = 0xFFFFFFFFu;
// a stack entry that is no node: a skipped BVH2 level's far child, counted when popped (Traversal::rp,
// reference units only).  As an index form it would name node 0x7FFFFFFE, which no BVH has.
constexpr uint32_t REF_MARKER = 0xFFFFFFFEu;
constexpr int FETCH_Q = 8;                       // float4 per lane per step: one 128-byte BVH4 node

// The part of intersect_scene_internal (RT/intersection.cpp:411-598) that needs
// no BVH: the planes, brute force (:424-433), then the top-level root, which the
// traversal would pop first (its box test and the far-clip test against t).  It
// runs where the ray is made (k_generate / k_shade, all lanes busy), so the trace
// kernels only see rays that enter the BVH, already carrying t and 1/d.
//
// When the top level is small (DevScene::top_seq, built at upload), the prologue
// also walks it: the top-level BVH as one linear sequence per direction octant in
// the reference's front-to-back order (:509-517), where a node failing the pop-time
// test (box hit and tn < t, :107-133) jumps past its subtree.  Spheres and boxes
// are tested here; a mesh instance whose root box passes goes on the ray's mesh
// list (bvh_indices slots, 6 bits each, up to MLIST_MAX) and only rays with a
// non-empty list are queued.  The trace kernel then walks just those instances.
// Against the reference's interleaved order this only moves analytic tests ahead
// of mesh traversals: t only decreases and every test keeps its own comparison,
// so the closest hit is the same unless two surfaces meet at exactly equal t
// (an any-hit query is order-independent).  More than MLIST_MAX instances: the
// ray is queued with MLIST_FULL and the kernel re-walks the whole top level
// (re-testing an analytic primitive at equal t changes nothing: strict tests).
constexpr uint32_t MLIST_MAX = 4;
// a load whose address is the same in every active lane: an s_load through the scalar
// cache, its value in SGPRs
RT_D float4 ld_uniform(const float4* p) {
    // an LDS address here would be a bug (scene_in_lds rebased the table); trap rather
    // than read a wild global address
#ifdef __HIP_DEVICE_COMPILE__
    if (__builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)p)) __builtin_trap();
#endif
    const uint64_t a = (uint64_t)p;
    const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32);
    const __attribute__((address_space(4))) float* f = reinterpret_cast<const __attribute__((address_space(4))) float*>(u);
    return make_float4(f[0], f[1], f[2], f[3]);
}
// The same for 8 or 16 consecutive dwords: one s_load_dwordx8 / x16.  Scalar loads return out of order,
// so a wave waits for all of its outstanding ones (lgkmcnt(0)) before it uses any value: the prologue
// fetches what a step needs in one batch rather than one float4 per wait.  The empty asm takes the whole
// vector in SGPRs where it is loaded, so the compiler neither narrows it into per-field loads nor sinks
// those into the branches that use them (each would be a wait of its own again).
typedef float f32x8 __attribute__((ext_vector_type(8), aligned(16)));
typedef float f32x16 __attribute__((ext_vector_type(16), aligned(16)));
template <class V>
RT_D V ld_uniform_v(const float4* p) {
#ifdef __HIP_DEVICE_COMPILE__
    if (__builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)p)) __builtin_trap();
#endif
    const uint64_t a = (uint64_t)p;
    const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32);
    const V v = *reinterpret_cast<const __attribute__((address_space(4))) V*>(u);
    asm volatile("" :: "s"(v));
    return v;
}
RT_D float4 q4_of(const f32x16& v, int k) { return make_float4(v[4*k], v[4*k + 1], v[4*k + 2], v[4*k + 3]); }
RT_D float4 q4_of(const f32x8& v, int k) { return make_float4(v[4*k], v[4*k + 1], v[4*k + 2], v[4*k + 3]); }
constexpr uint32_t MLIST_FULL = 0xFFFFFFFFu;
// calls: the mesh instances the walk reaches -- the top-level leaf holding one passes its pop-time
// test, it is not the ignored light, and no plane, sphere or box has occluded a shadow query before
// it: the reference's intersect_mesh calls (RT/intersection.cpp:488, counted at :254) in this walk's
// order (rt_stats::traversal)
struct Prologue { float t; uint32_t code; bool occluded, bvh; V3 inv_d; uint32_t mlist, calls; };
RT_D Prologue ray_prologue(const DevScene& sc, V3 o, V3 d, float max_t, bool occ, uint32_t ignored) {
    Prologue r;
    Ray wr = make_ray(o, d, max_t);
    wr.zero = 0u;                                                  // no pruning on the world ray
    r.t = max_t; r.code = RT_HIT_MISS; r.occluded = false; r.bvh = false; r.inv_d = wr.inv_d; r.mlist = MLIST_FULL;
    r.calls = 0;
    // four planes per batch; a lane whose shadow ray a plane occluded tests no further plane (the
    // reference returns there, :424-433)
    for (uint32_t i = 0; i < sc.plane_count; i += 4) {
        const f32x16 pb = ld_uniform_v<f32x16>(sc.plane_nd + i);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const float4 pl = q4_of(pb, (int)k);
            if (i + k < sc.plane_count && !r.occluded && ray_plane(wr, {pl.x, pl.y, pl.z}, pl.w, r.t)) {
                r.code = RT_HIT_PLANE_BIT | (i + k);
                if (occ) r.occluded = true;
            }
        }
    }
    if (r.occluded || !sc.bvh_node_count) return r;
    if (!sc.top_seq) {                                             // large top level: the kernel walks it
        const float4* q = reinterpret_cast<const float4*>(sc.bvh);
        const float4 a = q[0], b = q[1];
        float tn;
        r.bvh = bv_static(wr, {a.x, a.y, a.z}, {a.w, b.x, b.y}, tn) && tn < r.t;
        return r;
    }
    // Wave-uniform walk: every lane follows octant 0's sequence, so entry and record
    // addresses are the same across the wave (one cache line per load, values moved to
    // SGPRs) and the lanes stay converged; each lane tests only the entries on its own
    // path (`next`).  Octant 0's order differs from the reference's front-to-back order
    // only in which of two surfaces at exactly equal t is kept (see above).
    const float4* seq = sc.top_seq;
    uint32_t list = 0, n = 0, next = 0;     // n: listed instances (bits 0-7) | instances reached << 8
    bool full = false;
    const uint32_t len = sc.top_seq_len;
    const bool plain = plain_ray(o, d);
    for (uint32_t i = 0; i < len; ++i) {
        const f32x8 e = ld_uniform_v<f32x8>(seq + 2*i);
        const float4 a = q4_of(e, 0), b = q4_of(e, 1);
        const uint32_t info = __float_as_uint(b.z), skip = __float_as_uint(b.w);
        bool pass = false;
        if (next == i) {
            float tn;
            pass = bv_static(wr, {a.x, a.y, a.z}, {a.w, b.x, b.y}, tn) && tn < r.t;
            next = pass ? ((info >> 31) ? skip : i + 1) : skip;
        }
        if (!(info >> 31) || __ballot(pass) == 0ull) continue;
        const uint32_t first = info & 0xFFFFFFu, end = first + ((info >> 24) & 127u);
        for (uint32_t j = first; j < end; ++j) {                   // the leaf's primitives in order
            const float4* q = sc.leaf_rec + (size_t)j*LEAF_REC_Q;
            const f32x16 qa = ld_uniform_v<f32x16>(q);                 // q0-q3
            const float4 q3 = q4_of(qa, 3);
            const uint32_t pi = __float_as_uint(q3.x), tword = __float_as_uint(q3.y), type = tword & 0xFFu;
            if (!pass || pi == ignored) continue;
            const float4 q0 = q4_of(qa, 0), q1 = q4_of(qa, 1), q2 = q4_of(qa, 2);
            V3 io, id;
            object_ray(q0, q1, q2, tword & LEAF_TRANSLATE, plain, o, d, io, id);   // transform_ray :403-409
            bool hit = false;
            if (type == RT_PRIMITIVE_SPHERE) {                     // needs no 1/d
                Ray ir; ir.o = io; ir.d = id;
                hit = ray_sphere(ir, q3.z, r.t);
            } else {
                const Ray ir = make_ray(io, id, 0.0f);
                if (type == RT_PRIMITIVE_MESH) {                   // the mesh root's pop-time test (:269-275)
                    const f32x8 qb = ld_uniform_v<f32x8>(q + 4);
                    const float4 q4 = q4_of(qb, 0), q5 = q4_of(qb, 1);
                    float tm;
                    n += 1u << 8;                                  // intersect_mesh called (:488)
                    if (bv_static(ir, {q4.y, q4.z, q4.w}, {q5.x, q5.y, q5.z}, tm) && tm < r.t) {
                        const uint32_t k = n & 0xFFu;
                        if (k < sc.mlist_max) list |= j << (6*k);
                        else full = true;
                        ++n;
                    }
                    continue;
                }
                if (type == RT_PRIMITIVE_BOX) hit = ray_box(ir, {q3.z, q3.w, ld_uniform(q + 4).x}, r.t);
            }
            if (hit) {
                r.code = pi;
                if (occ) { r.occluded = true; pass = false; next = 0xFFFFFFFFu; }
            }
        }
    }
    r.calls = n >> 8;
    if (r.occluded) return r;
    n &= 0xFFu;
    r.bvh = n > 0;
    r.mlist = full ? MLIST_FULL : (list | (n << 24));
    return r;
}

// What the traversal steps fetched, for the TraversalStats counts (rt_stats::traversal): each
// step adds one of these to its lane's Traversal::acc, a count field per kind.  ENTRY a mesh
// instance's top-level leaf record (its object-space ray and root box test: intersect_mesh
// entered); NODE a mesh BVH4 interior node; LEAF the first triangles of a mesh leaf (the leaf
// entered); TRIS any step that fetched triangles; TOP a top-level interior node or a sphere's /
// box's record (none in a listed-only walk).  Fields of B bits: 8 for the four kinds of a
// listed-only walk, 6 for the five otherwise.  HI holds each field's top bit: a lane whose field
// reached half its range is flushed (StepCounts) before it can take another MARGIN steps.
template <bool LST>
struct StepField {
    static constexpr uint32_t B = LST ? 8 : 6, M = (1u << B) - 1u;
    static constexpr uint32_t ENTRY = 1u, NODE = 1u << B, LEAF = 1u << 2*B, TRIS = 1u << 3*B,
                              TOP = LST ? 0u : 1u << 4*B;
    static constexpr uint32_t H = 1u << (B - 1);
    static constexpr uint32_t HI = H | H << B | H << 2*B | H << 3*B | (LST ? 0u : H << 4*B);
    static constexpr uint32_t MARGIN = (1u << (B - 1)) - 1u;     // steps a lane may take between checks
};

// TraversalStats counters of a partition: per ray kind (0 closest, 1 shadow) and shard, TV_* counts.
// TV_DRAIN: the fused drain's steps (entries + nodes + triangle fetches + top level), which the
// others include too: trace_steps leaves them out (rt_stats::trace_steps, the extend / connect launches')
// TV_REF_*: rt_scene_config::traversal_ref, the reference's own units (rt_stats::traversal_ref): BVH2
// nodes taken from the stack, interior nodes and leaves passing their pop-time test
enum { TV_ENTRIES, TV_NODES, TV_LEAVES, TV_TRIS, TV_TOP, TV_CALLS, TV_DRAIN, TV_REF_TRAV, TV_REF_NODE, TV_REF_LEAF,
       TV_N = 12 };
extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);
// A wave's step counts.  flush(acc), at a point every lane of the wave reaches, sums the lanes'
// Traversal::acc (StepField) over the wave with DPP reductions, two fields per reduction (64 x 255
// fits 16 bits), into the wave's totals, which stay in SGPRs, and clears it; check(acc) flushes
// once some lane has a field at half its range (k_trace, after each refill round: a ballot); k_drain,
// whose walks take one step per lane per iteration, flushes every H iterations instead (8 fewer
// VGPRs there than the ballot); commit: one lane adds the totals to the counters.
template <bool LST>
struct StepCounts {
    using F = StepField<LST>;
    uint32_t tot[5] = {0, 0, 0, 0, 0};                 // TV_ENTRIES .. TV_TOP
    RT_D void flush(uint32_t& acc) {
        constexpr uint32_t B = F::B, M = F::M;
        const uint32_t a = __ockl_wfred_add_u32((acc & M) | (((acc >> B) & M) << 16));              // entries | nodes
        const uint32_t b = __ockl_wfred_add_u32(((acc >> 2*B) & M) | (((acc >> 3*B) & M) << 16));  // leaves | tris
        tot[TV_ENTRIES] += a & 0xFFFFu; tot[TV_NODES] += a >> 16;
        tot[TV_LEAVES] += b & 0xFFFFu; tot[TV_TRIS] += b >> 16;
        if (!LST) tot[TV_TOP] += __ockl_wfred_add_u32(acc >> 4*B);
        acc = 0;
    }
    RT_D void check(uint32_t& acc) { if (__ballot((acc & F::HI) != 0u)) flush(acc); }
    // the reference-unit counts (Traversal::rc, rt_scene_config::traversal_ref), summed over the wave
    unsigned long long ref[3] = {0, 0, 0};
    RT_D void flush_ref(uint32_t (&rc)[3]) {
#pragma unroll
        for (int i = 0; i < 3; ++i) { ref[i] += __ockl_wfred_add_u32(rc[i]); rc[i] = 0; }
    }
    // drain: k_drain's counts, also added to TV_DRAIN as steps
    RT_D void commit(unsigned long long* trav, int kind, bool drain = false) const {
        if (__lane_id() != (uint32_t)(__ffsll((long long)__ballot(true)) - 1)) return;
#pragma unroll
        for (int i = 0; i < 5; ++i)
            if (tot[i]) atomicAdd(&trav[kind*TV_N + i], (unsigned long long)tot[i]);
        const unsigned long long st = (unsigned long long)tot[TV_ENTRIES] + tot[TV_NODES] + tot[TV_TRIS] + tot[TV_TOP];
        if (drain && st) atomicAdd(&trav[kind*TV_N + TV_DRAIN], st);
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (ref[i]) atomicAdd(&trav[kind*TV_N + TV_REF_TRAV + i], ref[i]);
    }
};

// REF: count the reference's TraversalStats units too (rt_scene_config::traversal_ref; top-level walks only)
template <bool OCC, bool LST = false, int SL = STACK_LDS, bool REF = false>
struct Traversal {
    static_assert(!(REF && LST), "reference units need the reference's top-level walk");
    using Stack = StackT<SL>;
    V3 wo, wd;          // world ray
    V3 co, cd, cinv;    // current ray (object space while in a mesh)
    uint32_t cflags;    // current ray: d < 0 per axis (bits 0-2) | d == 0 per axis (bits 3-5, mesh only)
                        // | bit 6: finite slabs (finite_box_ray and DevScene::finite_boxes)
    float t;
    uint32_t code, tri;
    uint32_t ignored;
    int sp, mode, mesh_base;
    uint32_t leaf_cur, leaf_end;        // TM_LEAF: range of bvh_indices slots still to test
    uint32_t leaf_list;                 // TM_LEAF from the prologue's mesh list: slots still to walk,
                                        // 6 bits each (leaf_cur/leaf_end then count the list)
    bool listed;
    uint32_t inst, node_off, tri_off;   // TM_MESH: the instance
    uint32_t cur_lf, cur_cnt, cur_ax;   // node held by the lane (cur_cnt: leaf size, 0 interior)
    bool has_cur, occluded, finite_world;
    // rt_scene_config::traversal_ref (REF; top-level walks only): the reference's
    // TraversalStats of the current mesh instance in its own units -- [0] BVH2 nodes taken from the stack,
    // [1] interior nodes and [2] leaves passing their pop-time test (RT/intersection.cpp:274-380) -- and
    // those committed: an instance's counts are committed when its walk ends, and dropped when a shadow
    // query ends inside it (the reference returns before adding them, :297-299)
    uint32_t rp[3] = {0, 0, 0}, rc[3] = {0, 0, 0};

    RT_D Ray cur_ray() const {
        Ray r; r.o = co; r.d = cd; r.inv_d = cinv; r.neg = cflags & 7u; r.zero = cflags >> 3; r.max_t = 0.0f;
        return r;
    }
    // Pruning stays off for the world ray: the top level holds box primitives, whose own
    // slab test (ray_intersect_box) inherits the NaN quirk and can report a hit far away.
    RT_D void set_world() {
        const Ray w = make_ray(wo, wd, 0.0f);
        co = wo; cd = wd; cinv = w.inv_d; cflags = w.neg | (finite_world ? 64u : 0u);
    }

    template <bool SH>
    RT_D void push(const Stack& st, uint32_t rec, float tn) { if (SH || sp < STACK_DEPTH) st.template put<SH>(sp++, rec, tn); }

    // children of an interior node from the fetched sibling pair F[0..3]
    template <bool SH, bool FIN>
    RT_D void push_children(const Stack& st, const float4* F) {
        const V3 p0 = {F[0].x, F[0].y, F[0].z}, r0 = {F[0].w, F[1].x, F[1].y};
        const V3 p1 = {F[2].x, F[2].y, F[2].z}, r1 = {F[2].w, F[3].x, F[3].y};
        const uint32_t e0 = __float_as_uint(F[1].z), e1 = __float_as_uint(F[3].z);   // precomputed records
        const Ray r = cur_ray();
        float tn0, tn1;
        const bool h0 = bv_static<FIN>(r, p0, r0, tn0);
        const bool h1 = bv_static<FIN>(r, p1, r1, tn1);
        // the reference pushes (left, left+1) or (left+1, left); the second is popped first
        const bool neg = ((cflags & 7u) >> cur_ax) & 1u;
        const uint32_t ea = neg ? e0 : e1, eb = neg ? e1 : e0;
        const float ta = neg ? tn0 : tn1, tb = neg ? tn1 : tn0;
        const bool ha = neg ? h0 : h1, hb = neg ? h1 : h0;
        if (ha) push<SH>(st, ea, ta);
        if (hb) push<SH>(st, eb, tb);
    }

    RT_D void init(const DevScene& sc, const Stack& st, V3 o, V3 d, float max_t, uint32_t ign) {
        wo = o; wd = d;
        finite_world = false;                                      // debug path: reference max/min chains
        set_world();
        t = max_t; code = RT_HIT_MISS; tri = 0; st.bary[st.lane] = make_float2(0.0f, 0.0f);
        ignored = ign; sp = 0; mode = TM_TOP; occluded = false; has_cur = false; listed = false;
        Ray wr = make_ray(o, d, max_t);
        wr.zero = 0u;                                              // no pruning on the world ray
        for (uint32_t i = 0; i < sc.plane_count; ++i) {            // planes, brute force (:424-433)
            const rt_primitive& pl = sc.planes[i];
            if (ray_plane(wr, {pl.p[0], pl.p[1], pl.p[2]}, pl.p[3], t)) {
                code = RT_HIT_PLANE_BIT | i;
                if (OCC) { occluded = true; mode = TM_DONE; return; }
            }
        }
        if (sc.bvh_node_count) {
            const float4* q = reinterpret_cast<const float4*>(sc.bvh);
            const float4 a = q[0], b = q[1];
            float tn;
            if (bv_static(wr, {a.x, a.y, a.z}, {a.w, b.x, b.y}, tn)) st.put(sp++, __float_as_uint(b.z), tn);
        }
    }

    // a queued ray: ray_prologue ran where it was made.  With a mesh list the ray walks
    // just those instances; with MLIST_FULL it enters the BVH at the root (whose pop-time
    // test is known to pass: -inf < t)
    RT_D void init_rec(const DevScene& sc, const Stack& st, V3 o, V3 d, V3 inv_d, float t0, uint32_t ign,
                       uint32_t mlist) {
        wo = o; wd = d; co = o; cd = d; cinv = inv_d;
        finite_world = sc.finite_boxes && finite_box_ray(o, inv_d);
        cflags = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u) | (finite_world ? 64u : 0u);
        t = t0; code = RT_HIT_MISS; tri = 0; st.bary[st.lane] = make_float2(0.0f, 0.0f);
        ignored = ign; sp = 0; occluded = false; has_cur = false;
        if (mlist == MLIST_FULL) {
            mode = TM_TOP; listed = false;
            st.put(sp++, sc.bvh_root_rec, __uint_as_float(0xFF800000u));
        } else {
            mode = TM_LEAF; listed = true;
            if (LST) leaf_list = mlist;                            // LST: the count stays in bits 24-31
            else { leaf_list = mlist & 0xFFFFFFu; leaf_cur = 0; leaf_end = mlist >> 24; }
        }
    }

    // pop until an entry above `base` survives the far-clip test (the reference's pop-time
    // ray_intersect_bounding_volume against the current t); false when none is left
    template <bool SH>
    RT_D bool pop(const Stack& st, const rt_bvh_node* nodes, int base) {
        while (sp > base) {
            const uint2 e = st.template get<SH>(--sp);
            if (REF && e.x == REF_MARKER) {              // a skipped BVH2 level's far child (push_children4)
                if (__uint_as_float(e.y) < t) { rp[0] += 2u; rp[1] += 1u; }
                continue;
            }
            if (__uint_as_float(e.y) < t) {
                unpack_node(nodes, e.x, cur_lf, cur_cnt, cur_ax);
                has_cur = true;
                return true;
            }
        }
        return false;
    }

    // children of a mesh BVH4 node F[0..7], pushed so they pop in the BVH2 depth-first order
    template <bool SH, bool FIN>
    RT_D void push_children4(const Stack& st, const float4* F, const float4* mid = nullptr) {
        const Ray r = cur_ray();
        const uint32_t meta = __float_as_uint(F[7].x), nb = cflags & 7u;
        const uint32_t g = (nb >> (meta & 3u)) & 1u;               // group visited first: 1 = the right pair
        const uint32_t fa = (nb >> ((meta >> 2) & 3u)) & 1u;       // left pair: child 1 first
        const uint32_t fb = (nb >> ((meta >> 4) & 3u)) & 1u;       // right pair: child 3 first
        const uint32_t rec[4] = {__float_as_uint(F[6].x), __float_as_uint(F[6].y), __float_as_uint(F[6].z), __float_as_uint(F[6].w)};
        float tn[4];
        bool h[4];
        h[0] = bv_static<FIN>(r, {F[0].x, F[1].x, F[2].x}, {F[3].x, F[4].x, F[5].x}, tn[0]) && rec[0] != EMPTY4;
        h[1] = bv_static<FIN>(r, {F[0].y, F[1].y, F[2].y}, {F[3].y, F[4].y, F[5].y}, tn[1]) && rec[1] != EMPTY4;
        h[2] = bv_static<FIN>(r, {F[0].z, F[1].z, F[2].z}, {F[3].z, F[4].z, F[5].z}, tn[2]) && rec[2] != EMPTY4;
        h[3] = bv_static<FIN>(r, {F[0].w, F[1].w, F[2].w}, {F[3].w, F[4].w, F[5].w}, tn[3]) && rec[3] != EMPTY4;
        // visit order: first pair (2g + its first, 2g + its second), then the other pair; push reversed
        const uint32_t f1 = g ? fb : fa, f2 = g ? fa : fb;
        const uint32_t v[4] = {2u*g + f1, 2u*g + 1u - f1, 2u*(1u - g) + f2, 2u*(1u - g) + 1u - f2};
        // Reference units (rt_scene_config::traversal_ref): this node passed its pop-time test and the
        // reference pops both its children; each child that is interior (its pair's second slot is
        // used) pops its own two when it passes -- the near one now (nothing changes t before the
        // reference pops it), the far one when a marker pushed below the near pair's entries is popped
        // (t then holds whatever the near subtree found).
        bool far_marker = false;
        float far_tn = 0.0f;
        if (REF) {
            rp[0] += 2u; rp[1] += 1u;
            const V3 pc[2] = {{mid[0].x, mid[0].y, mid[0].z}, {mid[1].z, mid[1].w, mid[2].x}};
            const V3 rr[2] = {{mid[0].w, mid[1].x, mid[1].y}, {mid[2].y, mid[2].z, mid[2].w}};
#pragma unroll
            for (uint32_t c = 0; c < 2; ++c) {
                if ((c == 0 ? rec[1] : rec[3]) == EMPTY4) continue;           // a leaf child: counted when popped
                float tc;
                const bool hc = bv_static<FIN>(r, pc[c], rr[c], tc);
                if (c == g) { if (hc && tc < t) { rp[0] += 2u; rp[1] += 1u; } }
                else if (hc) { far_marker = true; far_tn = tc; }
            }
        }
#pragma unroll
        for (int k = 3; k >= 0; --k) {
            const uint32_t i = v[k];
            const bool hi = i == 0 ? h[0] : i == 1 ? h[1] : i == 2 ? h[2] : h[3];
            const uint32_t ri = i == 0 ? rec[0] : i == 1 ? rec[1] : i == 2 ? rec[2] : rec[3];
            const float ti = i == 0 ? tn[0] : i == 1 ? tn[1] : i == 2 ? tn[2] : tn[3];
            if (hi) push<SH>(st, ri, ti);
            if (REF && k == 2 && far_marker) push<SH>(st, REF_MARKER, far_tn);
        }
    }

    // One traversal step; returns false once the query is finished (mode == TM_DONE).  What the
    // step fetched is added to `acc` (StepField, the lane's TraversalStats counts since the last flush).
    // A step pops before it pushes and pushes at most PUSH_MAX entries, so when no lane of
    // the wave is within PUSH_MAX levels of STACK_LDS the whole step stays in LDS.
    static constexpr int PUSH_MAX = REF ? 5 : 4;       // REF: a far-child marker beside the four children
    using SF = StepField<LST>;
    uint32_t acc = 0;                   // SF fields of the steps since the caller last flushed them
    RT_D bool step(const DevScene& sc, const Stack& st) {
        if (__ballot(sp > SL - PUSH_MAX || !(cflags & 64u)) == 0ull) return step_impl<true, true>(sc, st);
        return step_impl<false, false>(sc, st);
    }
    template <bool SH, bool FIN>
    RT_D bool step_impl(const DevScene& sc, const Stack& st) {
        bool fresh;
        const float4* src = step_begin<SH>(sc, st, fresh);
        if (!src) return false;
        // unconditional: every array the step reads is padded by FETCH_Q float4 at upload
        float4 F[FETCH_Q];
#pragma unroll
        for (int j = 0; j < FETCH_Q; ++j) F[j] = src[j];
        return step_end<SH, FIN>(sc, st, F, fresh);
    }
    // A step in two halves around its one round of loads (r05: a cooperative wave-wide fetch in
    // between lost 14-26 %, profiles/r05_coop_fetch_ab.txt; the split alone is neutral).
    // step_begin: the state changes that need no global memory; returns the FETCH_Q float4 the
    // step reads, or null once the query is finished (mode == TM_DONE).  fresh: a mesh node was
    // popped in this step.
    template <bool SH>
    RT_D const float4* step_begin(const DevScene& sc, const Stack& st, bool& fresh) {
        // 1. state changes that need no global memory
        const bool take = mode == TM_MESH && !has_cur;
        if (take && !pop<SH>(st, sc.mnodes_src + node_off, LST ? 0 : mesh_base)) {
            mode = TM_LEAF;                                        // instance finished
            if (REF) { rc[0] += rp[0]; rc[1] += rp[1]; rc[2] += rp[2]; rp[0] = rp[1] = rp[2] = 0u; }
            // LST: the next step is the end or a listed instance's leaf step, which sets the
            // object-space ray from wo / wd itself (nothing reads the world ray in between)
            if (!LST) set_world();
        }
        fresh = take && mode == TM_MESH;                          // a mesh node popped in this step
        if (mode == TM_LEAF && (LST ? (leaf_list >> 24) == 0u : leaf_cur == leaf_end)) {
            if (LST) { mode = TM_DONE; return nullptr; }         // the mesh list is the whole walk
            mode = TM_TOP;
        }
        if (!LST && mode == TM_TOP) {
            if (!has_cur && !pop<SH>(st, sc.bvh_src, 0)) { mode = TM_DONE; return nullptr; }
            if (cur_cnt) {                                         // top-level leaf: its primitives in order
                leaf_cur = cur_lf; leaf_end = cur_lf + cur_cnt; has_cur = false;
                mode = TM_LEAF;
            }
        }
        // 2. what the one round of loads reads
        if (mode == TM_LEAF)
            return sc.leaf_rec + (size_t)((LST || listed) ? (leaf_list & 63u) : leaf_cur)*LEAF_REC_Q;
        if (cur_cnt) return sc.tris + 3*(size_t)(tri_off + cur_lf);                    // mesh leaf
        if (LST || mode == TM_MESH) return sc.mnodes4 + 8*(size_t)cur_lf;              // mesh BVH4 node
        return reinterpret_cast<const float4*>(sc.bvh + cur_lf);                       // top level: the sibling pair
    }
    // step_end: the arithmetic on what the step fetched (F); returns false once the query is finished
    template <bool SH, bool FIN>
    RT_D bool step_end(const DevScene& sc, const Stack& st, const float4 (&F)[FETCH_Q], bool fresh) {
        // 3. arithmetic
        if (mode == TM_LEAF) {
            const uint32_t pi = __float_as_uint(F[3].x);
            if (LST) leaf_list = ((leaf_list >> 6) & 0x3FFFFu) | ((leaf_list & 0xFF000000u) - 0x01000000u);
            else { ++leaf_cur; leaf_list >>= 6; }
            if (pi == ignored) { if (!LST) acc += SF::TOP; return true; }
            const uint32_t type = __float_as_uint(F[3].y) & 0xFFu;
            M34 inv;
            inv.e[0][0] = F[0].x; inv.e[0][1] = F[0].y; inv.e[0][2] = F[0].z; inv.e[0][3] = F[0].w;
            inv.e[1][0] = F[1].x; inv.e[1][1] = F[1].y; inv.e[1][2] = F[1].z; inv.e[1][3] = F[1].w;
            inv.e[2][0] = F[2].x; inv.e[2][1] = F[2].y; inv.e[2][2] = F[2].z; inv.e[2][3] = F[2].w;
            const Ray ir = make_ray(xform(inv, wo, 1.0f), xform(inv, wd, 0.0f), 0.0f);   // transform_ray :403-409
            // LST: the prologue lists mesh instances only (spheres and boxes were tested there)
            if (LST || type == RT_PRIMITIVE_MESH) {               // intersect_mesh :243-401
                co = ir.o; cd = ir.d; cinv = ir.inv_d;
                // (reference units: no degenerate-axis pruning, so the walk visits the reference's nodes)
                cflags = ir.neg | (REF ? 0u : ir.zero << 3) | ((sc.finite_boxes && finite_box_ray(ir.o, ir.inv_d)) ? 64u : 0u);
                // the reference pops the root (:266-274) of a mesh that has a BVH (:259; leaf record q5.w)
                if (REF) { rp[0] = F[5].w != 0.0f ? 1u : 0u; rp[1] = 0u; rp[2] = 0u; }
                inst = pi; node_off = __float_as_uint(F[3].z); tri_off = __float_as_uint(F[3].w);
                if (!LST) mesh_base = sp;              // LST: the stack holds this mesh only
                const V3 rp = {F[4].y, F[4].z, F[4].w}, rr = {F[5].x, F[5].y, F[5].z};
                float tn;
                Ray rr_ = ir;
                if (REF) rr_.zero = 0u;                            // reference units: no pruning at the root either
                if (bv_static(rr_, rp, rr, tn)) push<SH>(st, __float_as_uint(F[4].x), tn);
                mode = TM_MESH;
                acc += SF::ENTRY;
                return true;
            }
            if (!LST) {
                bool hit = false;
                if (type == RT_PRIMITIVE_SPHERE) hit = ray_sphere(ir, F[3].z, t);
                else if (type == RT_PRIMITIVE_BOX) hit = ray_box(ir, {F[3].z, F[3].w, F[4].x}, t);
                if (hit) {
                    if (OCC) { occluded = true; mode = TM_DONE; if (!LST) acc += SF::TOP; return false; }
                    code = pi;
                }
            }
            if (!LST) acc += SF::TOP;
            return true;
        }
        if (cur_cnt) {                                             // mesh leaf: triangles in order
            acc += fresh ? (SF::LEAF | SF::TRIS) : SF::TRIS;
            if (REF && fresh) rp[2] += 1u;
            Ray r; r.o = co; r.d = cd;
            const uint32_t g0 = tri_off + cur_lf;
            float bv = 0.0f, bw = 0.0f;
            bool hit = false;
#pragma unroll
            for (uint32_t j = 0; j < TRI_FETCH; ++j)
                if (j < cur_cnt) {
                    float v, w;
                    if (ray_triangle(r, ld3(F[3*j]), ld3(F[3*j + 1]), ld3(F[3*j + 2]), t, v, w)) {
                        if (OCC) { occluded = true; mode = TM_DONE; return false; }
                        code = inst; tri = g0 + j; bv = v; bw = w; hit = true;   // t only decreases: closest so far
                    }
                }
            if (hit) st.bary[st.lane] = make_float2(bv, bw);
            if (cur_cnt > TRI_FETCH) { cur_lf += TRI_FETCH; cur_cnt -= TRI_FETCH; }
            else has_cur = false;
            return true;
        }
        has_cur = false;
        if (LST || mode == TM_MESH) {
            push_children4<SH, FIN>(st, F, REF ? sc.mid4 + 3*(size_t)cur_lf : nullptr);
            acc += SF::NODE;
            return true;
        }
        push_children<SH, FIN>(st, F);
        if (!LST) acc += SF::TOP;
        return true;
    }

    RT_D Hit result(const Stack& st) const {
        const float2 b = st.bary[st.lane];
        Hit h; h.t = t; h.code = OCC ? (occluded ? 0u : RT_HIT_MISS) : code; h.tri = tri; h.v = b.x; h.w = b.y;
        return h;
    }
};

// :NormalCalculation (RT/intersection.cpp:526-591)
RT_D void hit_geometry(const DevScene& sc, const Ray& ray, const Hit& h, V3& I, V3& N, uint32_t& material_id) {
    I = add(ray.o, smul(h.t, ray.d));
    V3 n = {0.0f, 0.0f, 0.0f};
    M34 inv;
    if (h.code & RT_HIT_PLANE_BIT) {
        const rt_primitive& pl = sc.planes[h.code & ~RT_HIT_PLANE_BIT];
        n = {pl.p[0], pl.p[1], pl.p[2]};
        inv = load_m34(&sc.inv[pl.transform_index]);
        material_id = pl.material_id;
    } else {
        const rt_primitive prim = sc.prims[h.code];
        inv = load_m34(&sc.inv[prim.transform_index]);
        material_id = prim.material_id;
        if (prim.type == RT_PRIMITIVE_MESH) {
            const DevMesh mesh = sc.meshes[prim.mesh_index];
            float u = 1.0f - h.v - h.w;
            if (mesh.has_normals) {
                const float* nt = sc.normals + 9*(size_t)h.tri;                 // BVH slot order
                n = add(add(smul(u, {nt[0], nt[1], nt[2]}), smul(h.v, {nt[3], nt[4], nt[5]})),
                        smul(h.w, {nt[6], nt[7], nt[8]}));
            } else {
                const float4* tp = sc.tris + 3*(size_t)h.tri;
                V3 e1 = normalize(ld3(tp[1]));
                V3 e2 = normalize(ld3(tp[2]));
                n = cross(e1, e2);
            }
        } else {
            V3 oo = xform(inv, ray.o, 1.0f);
            V3 od = xform(inv, ray.d, 0.0f);
            V3 os_p = add(oo, smul(h.t, od));
            if (prim.type == RT_PRIMITIVE_SPHERE) {
                n = os_p;
            } else {
                V3 rel = divv(os_p, {prim.p[0], prim.p[1], prim.p[2]});
                int li = 0;
                float le = fabsf(rel.x);
                if (fabsf(rel.y) > le) { li = 1; le = fabsf(rel.y); }
                if (fabsf(rel.z) > le) { li = 2; le = fabsf(rel.z); }
                float s = sign_of(comp(rel, li));
                n = {li == 0 ? s : 0.0f, li == 1 ? s : 0.0f, li == 2 ? s : 0.0f};
            }
        }
    }
    N = noz(xform_normal(inv, n));
}

// ======================================================================
// Samplers (RT/samplers.cpp:18-138)
// ======================================================================
enum { S_DirectLighting, S_IndirectLighting, S_LightSelection, S_Reflectance, S_DOF, S_AA, S_Roulette };

struct SamplerState { uint32_t x, y, index; int strategy; };

RT_D float blue_noise(const uint8_t* t, int pi, int pj, int si, int dim) {   // 256spp.cpp:14-34
    pi &= 127; pj &= 127; si &= 255; dim &= 255;
    int ranked = si ^ (int)t[65536 + 131072 + dim + (pi + pj*128)*8];
    int value = (int)t[dim + ranked*256];
    value = value ^ (int)t[65536 + (dim % 8) + (pi + pj*128)*8];
    return (float)value / 256.0f;
}

RT_D V2 sample_2d(const DevScene& sc, const SamplerState& s, Rng& rng, int dim, uint32_t bounce) {
    int strategy = s.strategy;
    if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE && s.index > 256) strategy = RT_SAMPLING_STRATIFIED;
    if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE && dim >= 4) strategy = RT_SAMPLING_STRATIFIED;
    float a, b, c, d;
    unilaterals(rng, a, b, c, d);
    (void)c; (void)d;
    V2 r;
    if (bounce == 0 && strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE) {
        float ex = (1.0f / 256.0f)*a, ey = (1.0f / 256.0f)*b;
        r.x = ex + blue_noise(sc.bluenoise, (int)s.x, (int)s.y, (int)s.index, 2*dim);
        r.y = ey + blue_noise(sc.bluenoise, (int)s.x, (int)s.y, (int)s.index, 2*dim + 1);
    } else if (bounce == 0 && strategy == RT_SAMPLING_STRATIFIED) {
        const float rx = 1.0f / 8.0f, ry = 1.0f / 8.0f;
        uint32_t off = (73856093u*(uint32_t)dim) ^ hash_coordinate2(s.x, s.y);
        uint32_t si = sc.strata[(off & 255u)*64u + (s.index % 64u)];
        float sx = (float)(si % 8u)*rx, sy = (float)(si / 8u)*ry;
        r.x = sx + a*rx; r.y = sy + b*ry;
    } else {
        r.x = a; r.y = b;
    }
    return r;
}

RT_D float sample_1d(const DevScene& sc, const SamplerState& s, Rng& rng, int dim, uint32_t bounce) {
    int strategy = s.strategy;
    if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE && s.index > 256) strategy = RT_SAMPLING_STRATIFIED;
    if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE && dim >= 4) strategy = RT_SAMPLING_STRATIFIED;
    float a, b, c, d;
    unilaterals(rng, a, b, c, d);
    (void)b; (void)c; (void)d;
    if (bounce == 0 && strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE) {
        return (1.0f / 256.0f)*a + blue_noise(sc.bluenoise, (int)s.x, (int)s.y, (int)s.index, 2*dim);
    } else if (bounce == 0 && strategy == RT_SAMPLING_STRATIFIED) {
        const float rc = 1.0f / 64.0f;
        uint32_t off = (73856093u*(uint32_t)dim) ^ hash_coordinate2(s.x, s.y);
        uint32_t si = sc.strata[(off & 255u)*64u + (s.index % 64u)];
        return (float)si*rc + a*rc;
    }
    return a;
}

// ======================================================================
// Integrator helpers (RT/integrators.cpp)
// ======================================================================
RT_D V3 random_in_unit_sphere(Rng& e) {                                   // :11-19
    V3 r;
    int guard = 0;   // bounded (a degenerate all-zero RandomSeries would spin forever)
    do {
        float a, b, c, d;
        unilaterals(e, a, b, c, d);
        r = {a*2.0f - 1.0f, b*2.0f - 1.0f, c*2.0f - 1.0f};
    } while (length_sq(r) >= 1.0f && ++guard < 4096);
    return r;
}
RT_D V3 oriented_around_normal(V3 v, V3 n) {                             // :58-75
    float sign = copy_sign(1.0f, n.z);
    float a = -rcp_cr(sign + n.z);                 // -1/x == -(1/x) exactly
    float b = n.x*n.y*a;
    V3 T = {1.0f + sign*n.x*n.x*a, sign*b, -sign*n.x};
    V3 B = {b, sign + n.y*n.y*a, -n.y};
    return add(add(smul(v.x, B), smul(v.y, n)), smul(v.z, T));
}
RT_D V3 map_to_hemisphere(V3 N, V2 rs) {                                 // :93-105
    float az = TAU_32*rs.x, y = rs.y;
    float s = __builtin_sqrtf(1.0f - y*y);
    // two calls, not d_sincosf: in the NEE light sample the fused form's two live results cost
    // k_shade 8 B of scratch at 64 VGPRs
    V3 h = {d_cosf(az)*s, y, d_sinf(az)*s};
    return oriented_around_normal(h, N);
}
RT_D V3 map_to_cosine_weighted_hemisphere(V3 N, V2 rs) {                 // :107-119
    float az = TAU_32*rs.x, y = rs.y;
    float s = __builtin_sqrtf(1.0f - y);
    float sa, ca;
    d_sincosf(az, sa, ca);                          // = d_sinf(az), d_cosf(az), bit for bit
    V3 h = {ca*s, __builtin_sqrtf(y), sa*s};
    return oriented_around_normal(h, N);
}
RT_D float fresnel_dielectric(float ci, float ei, float et, float eta, float& co) {   // :235-258
    float si = __builtin_sqrtf(mx(0.0f, 1.0f - ci*ci));
    float st = eta*si;
    float ct = __builtin_sqrtf(mx(0.0f, 1.0f - st*st));
    co = ct;
    if (st >= 1) return 1;
    float rpar = (((et*ci) - (ei*ct)) / ((et*ci) + (ei*ct)));
    float rperp = (((ei*ci) - (et*ct)) / ((ei*ci) + (et*ct)));
    return 0.5f * (rpar * rpar + rperp * rperp);
}
RT_D V3 sample_sky(const DevScene& sc, V3 d) {                           // :272-295
    if (sc.sky) {
        float rcp_pi = 1.0f / PI_32;
        float rcp_2pi = 0.5f / PI_32;
        float phi = d_atan2f(d.z, d.x);
        float theta = d_asinf(d.y);
        float u = 0.5f + rcp_2pi*phi;
        float v = 0.5f + rcp_pi*theta;
        uint32_t sx = (uint32_t)(int32_t)(u*(float)sc.sky_w) % sc.sky_w;
        uint32_t sy = (uint32_t)(int32_t)(v*(float)sc.sky_h) % sc.sky_h;
        const float* p = sc.sky + 3*((size_t)sy*sc.sky_w + sx);
        return {p[0], p[1], p[2]};
    }
    return lerp3(sc.bot_sky, sc.top_sky, fabsf(d.y));
}
// Environment-map sampling (rt_set_env_sampling; beyond the reference, whose CDF of
// RT/assets.cpp:620-665 is never read, RT/integrators.cpp:230-233).  The table has one
// entry per luma tile of load_environment_map's grid: {alias threshold, alias tile,
// density}, density = the tile's luma share x texels / tile texels (a pdf over the
// unit (u, v) square).  A sample is one 16-byte read: tile k = floor(e n) or its alias.
RT_D V3 env_direction(const DevScene& sc, float e, V2 s2) {
    const float fe = e*(float)sc.env_n;
    uint32_t k = (uint32_t)fe;
    if (k >= sc.env_n) k = sc.env_n - 1;
    const float frac = fe - (float)k;
    const float4 ent = sc.env_tab[k];
    const uint32_t tile = frac < ent.x ? k : __float_as_uint(ent.y);
    const uint32_t x0 = (tile % sc.env_tx)*sc.env_tw, y0 = (tile / sc.env_tx)*sc.env_th;
    const uint32_t cw = min(sc.env_tw, sc.sky_w - x0), ch = min(sc.env_th, sc.sky_h - y0);
    const float u = ((float)x0 + s2.x*(float)cw) / (float)sc.sky_w;
    const float v = ((float)y0 + s2.y*(float)ch) / (float)sc.sky_h;
    const float phi = (u - 0.5f)*(2.0f*PI_32), theta = (v - 0.5f)*PI_32;   // sample_sky's mapping inverted
    float st, ct, sp, cp;
    d_sincosf(theta, st, ct);
    d_sincosf(phi, sp, cp);
    return {ct*cp, st, ct*sp};
}
// sample_sky's texel for d, and the table tile it lies in
RT_D V3 sky_env(const DevScene& sc, V3 d, uint32_t& tile) {
    const float rcp_pi = 1.0f / PI_32;
    const float rcp_2pi = 0.5f / PI_32;
    const float u = 0.5f + rcp_2pi*d_atan2f(d.z, d.x);
    const float v = 0.5f + rcp_pi*d_asinf(d.y);
    const uint32_t sx = (uint32_t)(int32_t)(u*(float)sc.sky_w) % sc.sky_w;
    const uint32_t sy = (uint32_t)(int32_t)(v*(float)sc.sky_h) % sc.sky_h;
    tile = (sy / sc.env_th)*sc.env_tx + sx / sc.env_tw;
    const float* p = sc.sky + 3*((size_t)sy*sc.sky_w + sx);
    return {p[0], p[1], p[2]};
}
// solid-angle pdf of env_direction at d (in `tile`): density / (2 pi^2 cos theta)
RT_D float env_pdf(const DevScene& sc, uint32_t tile, V3 d) {
    const float c2 = 1.0f - d.y*d.y;
    if (!(c2 > 0.0f)) return 0.0f;
    return sc.env_tab[tile].z / ((2.0f*PI_32*PI_32)*__builtin_sqrtf(c2));
}
RT_D V3 evaluate_material(const rt_material& m, V3 p) {                 // :297-308
    if (m.flags & RT_MATERIAL_CHECKERS) {
        int32_t ch = (((int32_t)floorf(0.25f*p.x)) ^ ((int32_t)floorf(0.25f*p.z))) & 1;
        if (ch) return {m.checker_color.x, m.checker_color.y, m.checker_color.z};
    }
    return {m.albedo.x, m.albedo.y, m.albedo.z};
}
__host__ __device__ inline V3 rv3(const rt_v3& a) { return {a.x, a.y, a.z}; }
RT_D V3 translation(const M34& m) { return {m.e[0][3], m.e[1][3], m.e[2][3]}; }

// pick_random_light (:135-192) without scratch arrays: one pass for the sum,
// a second for the CDF walk (identical additions, identical rounding).
RT_D uint32_t pick_random_light(const DevScene& sc, const rt_settings& st, float rs, V3 I, float& out_p) {
    uint32_t n = sc.light_count;
    if (n == 0) return 0;
    if (st.importance_sample_lights) {
        float sum = 0.0f;
        for (uint32_t i = 0; i < n; ++i) {
            const rt_primitive light = sc.prims[sc.lights[i]];
            V3 lv = sub(translation(sc.fwd[light.transform_index]), I);
            float dsq = length_sq(lv);
            float l = max3(rv3(sc.materials[light.material_id].emission_color));
            float psa = light.type == RT_PRIMITIVE_SPHERE ? PI_32*light.p[0]*light.p[0] / dsq : 0.0f;
            sum += l*psa;
        }
        float e = sum*rs;
        float cdf = 0.0f, pdf = 0.0f;
        uint32_t li = 0;
        for (; li < n; ++li) {
            const rt_primitive light = sc.prims[sc.lights[li]];
            V3 lv = sub(translation(sc.fwd[light.transform_index]), I);
            float dsq = length_sq(lv);
            float l = max3(rv3(sc.materials[light.material_id].emission_color));
            float psa = light.type == RT_PRIMITIVE_SPHERE ? PI_32*light.p[0]*light.p[0] / dsq : 0.0f;
            pdf = l*psa;
            cdf = (li > 0 ? cdf : 0.0f) + pdf;
            if (!(cdf < e) || li == n - 1) break;
        }
        out_p = pdf / sum;
        return sc.lights[li];
    }
    out_p = rcp_cr((float)n);
    float f = rs*(float)n - EPSILON;
    uint32_t li = f <= 0.0f ? 0u : (uint32_t)f;
    if (li >= n) li = n - 1;
    return sc.lights[li];
}

// ======================================================================
// Path pool (SoA in HBM)
// ======================================================================
// Streaming access to the path pool, the queues and the sample records: each is read
// or written once per iteration (hundreds of MB per launch, no reuse before the next
// iteration), so they use non-temporal loads and stores and do not displace the BVH
// nodes and triangles the trace kernels keep re-reading from L2.
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef uint32_t nt_u4 __attribute__((ext_vector_type(4)));
typedef float nt_f2 __attribute__((ext_vector_type(2)));
typedef uint32_t nt_u2 __attribute__((ext_vector_type(2)));
RT_D float4 ldnt(const float4* p) { const nt_f4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(p)); return make_float4(v.x, v.y, v.z, v.w); }
RT_D uint4 ldnt(const uint4* p) { const nt_u4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_u4*>(p)); return make_uint4(v.x, v.y, v.z, v.w); }
RT_D float2 ldnt(const float2* p) { const nt_f2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f2*>(p)); return make_float2(v.x, v.y); }
RT_D float ldnt(const float* p) { return __builtin_nontemporal_load(p); }
RT_D uint2 ldnt(const uint2* p) { const nt_u2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_u2*>(p)); return make_uint2(v.x, v.y); }
RT_D uint32_t ldnt(const uint32_t* p) { return __builtin_nontemporal_load(p); }
RT_D void stnt(float4* p, float4 v) { const nt_f4 t = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(t, reinterpret_cast<nt_f4*>(p)); }
RT_D void stnt(uint4* p, uint4 v) { const nt_u4 t = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(t, reinterpret_cast<nt_u4*>(p)); }
RT_D void stnt(float2* p, float2 v) { const nt_f2 t = {v.x, v.y}; __builtin_nontemporal_store(t, reinterpret_cast<nt_f2*>(p)); }
RT_D void stnt(float* p, float v) { __builtin_nontemporal_store(v, p); }
RT_D void stnt(uint2* p, uint2 v) { const nt_u2 t = {v.x, v.y}; __builtin_nontemporal_store(t, reinterpret_cast<nt_u2*>(p)); }
RT_D void stnt(uint32_t* p, uint32_t v) { __builtin_nontemporal_store(v, p); }
// The path state is double-buffered: k_shade reads a wave's 64 slots of the current buffer
// and writes the paths that continue, compacted to the front of the same 64 slots of the
// other buffer (PathOut), and the paths that end into the finished array; the next
// k_generate fills the wave's remaining slots with new paths.  Every pool array is then
// written in whole runs (the survivors' prefix, the new paths' suffix) instead of at the
// scattered slots paths happened to free.  The host swaps the two buffers every iteration.
struct PathOut {
    float4 *ray_o, *ray_d, *thr, *L;
    float2* prev_n;
    uint4* rng;
    float4* hit;
    float* hit_w;
    uint16_t* mstack;
    uint8_t* state;
};
struct Pool {
    uint32_t n;
    float4* ray_o;       // o.xyz | w: the pixel, x | y << 16 (frames are at most 65535 a side)
    float4* ray_d;       // d.xyz | w: sample offset bits
    float4* thr;         // throughput.xyz | w: vignette
    float4* L;           // total_color.xyz | w: flags bits (bounce 0-7, specular 8, stack_at 9-15)
    // .x: the MIS pdf term of prev_N (RT/integrators.cpp:661-668, dot(prev_N, ray.d) / pi),
    // computed where the ray's direction is chosen (same operands, same bits), so prev_N
    // itself is never stored | .y: tile-list pixel index p (sample record = s*P + p)
    float2* prev_n;
    uint4*  rng;
    float4* hit;         // t | code | tri | v
    float*  hit_w;       // a mesh hit's w (written by k_trace with the hit; read for mesh hits only)
    uint16_t* mstack;    // [64][n]
    uint8_t*  state;     // S_FREE / S_TRACE / S_DONE / S_NEW (a traced camera ray) per slot
    float4*   ext_rec[2];// extension queues (ping-pong), REC_Q float4 per ray: {o, slot}, {d, t after planes}, {1/d, -}
    // The shadow queue.  k_shade writes a queued shadow ray's record and contribution at its own
    // slot as soon as the ray's prologue is done (so they are not held in registers across the next
    // bounce's prologue), the queue entry is just that slot, and the NEE term's destination goes to
    // sh_dst[slot] at the tail.  (k_drain_list reuses sh_slot for its list of live slots.)
    uint32_t* sh_slot;   // [Q] the slot holding the ray
    float4*   sh_rec;    // [N] REC_Q float4 per ray: {o, light id}, {d, max_t}, {1/d, mesh list}
    float4*   sh_c;      // [N] contribution.xyz
    uint32_t* sh_dst;    // [N] the NEE term's destination (survivor's nx slot or SH_FIN | entry)
    uint32_t  shard_cap; // queue entries per shard (queues are NSHARD shards of shard_cap)
    uint32_t* claim_base;// [blocks]: exclusive scan of the blocks' free slots (k_bookkeep: block_free) = first
                         // claim of the block
    PathOut nx;          // the other buffer: k_shade's survivors (the next k_trace adds their NEE terms)
    // finished paths, per wave of 64 slots compacted from the wave's first entry (k_shade; the next
    // k_trace adds a pending last NEE term, the k_generate after it splats them): {L, vignette}, {ray_d.w key,
    // tile-list pixel p}, ray_o.w pixel; fin_w[wave] of them.  free_w[wave]: the wave's slots past
    // its survivors (block_free sums a block's four).  The AA jitter is recomputed (sample_jitter).
    float4*   fin_L;
    uint2*    fin_k;
    uint32_t* fin_px;
    uint32_t* fin_w;
    // The finished arrays are double-buffered with the path buffers (r06): k_shade writes the set of its
    // iteration's parity, and the k_trace of the next iteration adds the last NEE terms of its paths
    // (their shadow rays ride in that launch), so they are splatted by the k_generate two iterations on,
    // which sees that set as its own again.  fin2_*: the other set (the previous k_shade's).
    float4*   fin2_L;
    uint2*    fin2_k;
    uint32_t* fin2_px;
    uint32_t* fin2_w;
    uint32_t* free_w;
    // This partition's sample records (the deterministic splats): pass s, tile-list pixel p at
    // ((s - rec_pass0) % rec_ring)*P + p.  A ring of rec_ring passes in the streaming splat
    // (k_resolve_tiles frees passes while the frame renders), the partition's whole pass range
    // in the exact splat (k_resolve).  Null: atomic splat.
    float4*  rec_rgbx;   // r, g, b, jitter_x
    float*   rec_jy;     // jitter_y
    uint32_t rec_pass0, rec_ring;
};

// Slot states.  Every per-iteration kernel except the tracers walks the pool in
// slot order (thread i = slot i): the SoA loads coalesce, and the queues it
// appends to come out as runs of consecutive slots (one run per wavefront).
enum : uint8_t { S_FREE = 0, S_TRACE = 1, S_DONE = 2, S_NEW = 3 };
// k_generate writes a new path as S_NEW without its throughput and total_color records (1, 0 and
// the bounce-0 flags), and k_shade / k_drain make them from the state, the vignette from the camera
// ray (new_path_records); 32 B per new path less to write.
constexpr int REC_Q = 3;     // float4 per queued ray record

constexpr uint32_t SH_FIN = 0x80000000u;   // Pool::sh_slot: the shadow ray's path is in the finished array

// Queues and fetch heads are sharded NSHARD ways (shard = blockIdx % NSHARD, the
// blocks that share an XCD), each counter on a 128-B line of its own: one word
// saturates at ~88 returning atomics/us, and a 2M-slot pool has 4096 blocks.
constexpr int NSHARD = 8;
static_assert(NSHARD <= 64 && (NSHARD & (NSHARD - 1)) == 0, "k_bookkeep sums the shards in one wave");
constexpr int NXCD = 8;                        // MI355X: workgroups are dealt round robin over 8 XCDs
constexpr int LINE_WORDS = 32;
struct Counters {
    uint32_t ext_count[2][NSHARD][LINE_WORDS];   // extension queue length per shard (ping-pong)
    uint32_t shadow_count[2][NSHARD][LINE_WORDS];   // shadow queue length per shard, by the path buffer parity of the
                                                    // k_shade that made it (the next iteration's k_trace traces it)
    uint32_t fetch[2][NSHARD][LINE_WORDS];       // persistent trace kernels: items handed out (extend, connect)
    uint32_t cast[2][NSHARD][LINE_WORDS];        // rays cast this iteration: [1] shadow (k_shade); [0] unused since r03 (k_bookkeep counts the camera rays from the claims)
    uint32_t alive[NSHARD][LINE_WORDS];          // paths k_shade continued (each casts a closest ray next iteration)
    uint32_t unsplat[NSHARD][LINE_WORDS];        // paths finished this iteration, splatted by the k_generate after next
    uint32_t unsplat_prev;                       // the previous iteration's (k_bookkeep): splatted by the next k_generate
    uint32_t gen_free;              // free slots counted by the last k_bookkeep = claims of the next k_generate
    uint32_t pending;               // paths queued for the next iteration (host termination test)
    uint32_t pending_splat;         // finished paths not yet splatted and shadow rays not yet traced (host termination test)
    uint32_t cancel;
    uint32_t done;                  // every sample claimed, traced and splatted (k_bookkeep); the launches
                                    // still queued behind it (drain mode) exit at once
    uint32_t fused;                 // nothing left to claim and few paths alive (k_bookkeep): the next
                                    // iteration launched with the drain kernels runs every remaining
                                    // path to its end in k_drain; its extend / shade / connect exit
    uint32_t drained;               // k_drain_list ran (it splatted the previous k_shade's finished paths)
    uint32_t drain_count[NSHARD][LINE_WORDS];   // k_drain_list: live slots per shard (in Pool::sh_slot)
    uint32_t drain_fetch[NSHARD][LINE_WORDS];   // k_drain: items handed out per shard
    // TraversalStats of the frame (rt_stats::traversal), per ray kind (0 closest, 1 shadow): TV_* counts,
    // one 128-byte line per shard (the block's or wave's shard adds to it; the host sums the shards)
    unsigned long long trav[NSHARD][2*TV_N];
    unsigned long long next_sample;
    unsigned long long total_samples;
    unsigned long long closest_rays;
    unsigned long long shadow_rays;
    unsigned long long traced_rays[2];   // handed to k_trace<false> / k_trace<true>
    // streaming splat (k_bookkeep plans, k_resolve_tiles consumes)
    unsigned long long claim_limit;      // samples below this may be claimed: the record ring's capacity
    unsigned long long start_sample;     // the partition's first sample
    uint32_t iter;                       // iterations bookkept so far
    uint32_t res_cursor;                 // passes below it are resolved (or planned for the next resolve)
    uint32_t res_from, res_to;           // the pass range the next k_resolve_tiles resolves (empty: none)
    unsigned long long hist[128];        // next_sample after the bookkeep of iteration i, at [i % 128]
};

struct FrameParams {
    uint32_t w, h, frame_count, total_frame_index;
    uint32_t tile_w, tile_h, tcx;
    // ceil(2^32 / tile_w), ceil(2^32 / tile_h), ceil(2^64 / pixels) (set_divisors): a coordinate's tile and a
    // sample number's pass by a multiply-high instead of the integer division expansion (div16, div_pixels)
    uint64_t tw_m, th_m, px_m;
    uint32_t pixels;                // P: pixels owned by this shard
    uint32_t ntiles;
    const uint32_t* tile_ids;       // owned tiles
    const uint32_t* tile_prefix;    // [ntiles+1] pixel prefix sums
    const uint32_t* pix_xy;         // [P]: x | y << 16 of tile-list pixel p (k_pixel_map)
    // explicit sample list mode (rt_trace_samples)
    const uint32_t* list_xy;
    const uint32_t* list_s;
    float* list_out;
    // camera (RT/raytracer.cpp:381-401)
    V3 cp, cx, cy, cz;
    float focus_distance, lens_radius, half_film_w, half_film_h, film_distance;
    // filter
    const float* lut;               // 512 floats
    int32_t kernel_size, cache_size;
    float4* accum;
    // deterministic splat: per-sample records, gathered by k_resolve
    float4* samp_rgbx;              // [spp*P]: r, g, b, jitter_x   (record = s*P + p)
    float*  samp_jy;                // [spp*P]: jitter_y
    const int32_t* tile_base;       // [tiles]: first tile-list pixel of an owned tile, -1 otherwise
    uint32_t spp;
};

// wave-aggregated queue append: one atomic per wavefront
RT_D uint32_t wave_append(uint32_t* counter, bool pred) {
    unsigned long long mask = __ballot(pred);
    if (mask == 0ull) return 0;
    uint32_t lane = __lane_id();
    uint32_t leader = (uint32_t)__ffsll((long long)mask) - 1u;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(mask));
    base = __shfl(base, (int)leader);
    unsigned long long lower = mask & ((1ull << lane) - 1ull);
    return base + (uint32_t)__popcll(lower);
}

// Workgroup-level exclusive rank of `pred` in thread order; *total = the block's
// count.  Every thread of the block must call it.  `scratch` is LDS of >= waves+1
// words; it is free again when the call returns.
template <int NT>
RT_D uint32_t block_rank(bool pred, uint32_t* scratch, uint32_t* total) {
    constexpr int NW = NT / 64;
    const uint32_t lane = __lane_id();
    const uint32_t wave = threadIdx.x / 64;
    const unsigned long long mask = __ballot(pred);
    if (lane == 0) scratch[wave] = (uint32_t)__popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < NW; ++w) { uint32_t c = scratch[w]; scratch[w] = t; t += c; }
        scratch[NW] = t;
    }
    __syncthreads();
    const uint32_t r = scratch[wave] + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
    *total = scratch[NW];
    __syncthreads();
    return r;
}

// Workgroup-aggregated append: one atomic per workgroup on the block's shard of
// the counter (the guide's single-word rate, ~88 returning atomics/us, made
// per-wavefront appends of a 2M-slot pool cost ~0.4 ms per launch).  Every
// thread of the block must call it.  Entries keep slot order within the block.
template <int NT>
RT_D uint32_t block_append(uint32_t* counter, bool pred, uint32_t* scratch) {
    constexpr int NW = NT / 64;
    const uint32_t lane = __lane_id();
    const uint32_t wave = threadIdx.x / 64;
    const unsigned long long mask = __ballot(pred);
    if (lane == 0) scratch[wave] = (uint32_t)__popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t total = 0;
        for (int w = 0; w < NW; ++w) { uint32_t c = scratch[w]; scratch[w] = total; total += c; }
        scratch[NW] = total ? atomicAdd(counter, total) : 0u;
    }
    __syncthreads();
    const uint32_t pos = scratch[NW] + scratch[wave] + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
    __syncthreads();     // scratch may be reused by the next append
    return pos;
}

// Adds the block's count of `pred` to a counter (one no-return atomic per block).
template <int NT>
RT_D void block_count(uint32_t* counter, bool pred, uint32_t* scratch) {
    uint32_t total;
    (void)block_rank<NT>(pred, scratch, &total);
    if (threadIdx.x == 0 && total) atomicAdd(counter, total);
}

// K block-wide tallies at once (k_drain_list; k_generate / k_shade until r05): one ballot per
// predicate, ONE barrier to publish the per-wave counts, then thread 0 scans the
// waves and adds each tally's block total to ctr[k] (a null ctr: total only), all K
// atomics in flight together; one barrier to publish the bases.  The
// separate block_count / block_append calls this replaces cost 3 barriers and a
// serialized atomic round trip each (13 % of a k_shade wave's time).
// pos[k] = the counter's old value + the thread's rank among the block's threads
// with pred[k] (an append position); total[k] = the block's count.
// scratch: LDS of (NT/64 + 2)*K words, not reused by the caller afterwards.
template <int NT, int K>
RT_D void block_tally(const bool (&pred)[K], uint32_t* const (&ctr)[K], uint32_t (&pos)[K], uint32_t (&total)[K],
                      uint32_t* scratch) {
    constexpr int NW = NT / 64;
    const uint32_t lane = __lane_id();
    const uint32_t wave = threadIdx.x / 64;
    const unsigned long long lt = (1ull << lane) - 1ull;
    unsigned long long mask[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        mask[k] = __ballot(pred[k]);
        if (lane == 0) scratch[wave*K + k] = (uint32_t)__popcll(mask[k]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {                 // static indices only: no pointer table in scratch
        uint32_t t[K], base[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            t[k] = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) { const uint32_t c = scratch[w*K + k]; scratch[w*K + k] = t[k]; t[k] += c; }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) base[k] = (ctr[k] && t[k]) ? atomicAdd(ctr[k], t[k]) : 0u;   // K in flight
#pragma unroll
        for (int k = 0; k < K; ++k) { scratch[NW*K + k] = base[k]; scratch[(NW + 1)*K + k] = t[k]; }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        pos[k] = scratch[NW*K + k] + scratch[wave*K + k] + (uint32_t)__popcll(mask[k] & lt);
        total[k] = scratch[(NW + 1)*K + k];
    }
}

// Samples still to be claimed now: up to the partition's end, and (streaming splat) no further than
// the record ring holds.
RT_D unsigned long long remaining_samples(const Counters* c) {
    const unsigned long long lim = c->claim_limit < c->total_samples ? c->claim_limit : c->total_samples;
    return lim > c->next_sample ? lim - c->next_sample : 0ull;
}

// ---- lens (RT/raytracer.cpp:86-123)
RT_D V2 transform_bokeh_sample(V2 o, float f, float n, float phi_shutter_max) {
    V2 ab = {(o.x*2.0f) - 1.0f, (o.y*2.0f) - 1.0f};
    V2 phir;
    if ((ab.x*ab.x) > (ab.y*ab.y)) {
        phir.x = (fabsf(ab.x) > 1e-8f) ? ((PI_32*0.25f)*(ab.y / ab.x)) : 0.0f;
        phir.y = ab.x;
    } else {
        phir.x = (fabsf(ab.y) > 1e-8f) ? ((PI_32*0.5f) - ((PI_32*0.25f)*(ab.x / ab.y))) : 0.0f;
        phir.y = ab.y;
    }
    phir.x += f*phi_shutter_max;
    if (f > 0.0f) {
        float k = floorf(((n*phir.x) + PI_32) / (2.0f*PI_32));
        phir.y *= d_powf(d_cosf(PI_32 / n) / d_cosf(phir.x - ((2.0f*(PI_32 / n))*k)), f);
    } else {
        phir.y *= 1.0f;
    }
    float sp, cp;
    d_sincosf(phir.x, sp, cp);
    return {cp*phir.y, sp*phir.y};
}
RT_D V2 brown_conrady(V2 uv, float amount, float woh) {
    uv.y /= woh;
    float bd1 = 0.1f*amount, bd2 = -0.025f*amount;
    float r2 = uv.x*uv.x + uv.y*uv.y;
    float f = 1.0f + r2*bd1 + r2*r2*bd2;
    uv.x *= f; uv.y *= f;
    uv.y *= woh;
    return uv;
}
RT_D void apply_lens_distortion(float amount, uint32_t w, uint32_t h, float& u, float& v) {
    float woh = (float)w / (float)h;
    V2 mn_ = brown_conrady({0.0f, 0.0f}, amount, woh);
    V2 mx_ = brown_conrady({1.0f, 1.0f}, amount, woh);
    V2 uv = brown_conrady({u, v}, amount, woh);
    if (amount > 0.0f) {
        uv.x = (uv.x - mn_.x) / (mn_.x + mx_.x);
        uv.y = (uv.y - mn_.y) / (mn_.y + mx_.y);
    }
    u = uv.x; v = uv.y;
}

RT_D uint32_t pack_flags(uint32_t bounce, uint32_t spec, uint32_t at) { return bounce | (spec << 8) | (at << 9); }

// x / d for x, d < 2^16 with m = ceil(2^32 / d): floor(x*m / 2^32) = floor(x / d + e) with
// 0 <= e < x / 2^32 < 1 / d, which cannot reach the next integer (Granlund & Montgomery 1994).
RT_D uint32_t div16(uint32_t x, uint64_t m) { return (uint32_t)(((uint64_t)x*m) >> 32); }
// k / P for k < 2^32, P < 2^32 with m = ceil(2^64 / P): the same bound with 2^64
RT_D uint32_t div_pixels(uint32_t k, uint64_t m) { return (uint32_t)__umul64hi((uint64_t)k, m); }
// a pixel's tile (RT/raytracer.cpp:551-560 numbering: row-major over tcx tiles per row)
RT_D uint32_t tile_of(const FrameParams& fp, uint32_t x, uint32_t y) { return div16(y, fp.th_m)*fp.tcx + div16(x, fp.tw_m); }

// ======================================================================
// Kernels
// ======================================================================
constexpr int BLOCK = 256;      // slot-ordered kernels (generate / shade)
// chunks in flight per partition in run_frame: 3 or 4 lose (the empty chunks after a partition's end
// cost more than the early chunks' host round trips: profiles/r05_host_ab.txt)
constexpr int NIF = 2;
constexpr int EV_SLOTS = 4*NIF;  // iterations in flight per partition in run_frame (NIF chunks of 4)

// The splat of a finished path (RT/raytracer.cpp:469-488): vignette (L . vig), then the
// 20-byte sample record k_resolve gathers (splat_filter :187-259 in reference order), or
// float atomics into the accumulator when the records do not fit.  Run by k_generate on
// the finished array k_shade wrote (key: ray_d.w, the sample pass or the list index;
// p: the tile-list pixel).
RT_D void splat_sample(const FrameParams& fp, const Pool& pool, V3 L, float vig, float2 j, uint32_t key, uint32_t p) {
    {
        V3 r = muls(L, vig);
        if (fp.list_xy) {
            float* o = fp.list_out + 5*(size_t)key;
            o[0] = r.x; o[1] = r.y; o[2] = r.z; o[3] = j.x; o[4] = j.y;
        } else if (pool.rec_rgbx) {
            // deterministic paths: store the sample; k_resolve_tiles / k_resolve gather it
            const uint32_t rel = key - pool.rec_pass0;
            const size_t rec = (size_t)(rel < pool.rec_ring ? rel : rel % pool.rec_ring)*fp.pixels + p;
            stnt(&pool.rec_rgbx[rec], make_float4(r.x, r.y, r.z, j.x));     // read again only by the resolve
            stnt(&pool.rec_jy[rec], j.y);
        } else if (fp.cache_size) {
            const uint32_t xy = fp.pix_xy[p];
            const int64_t x = xy & 0xFFFFu, y = xy >> 16;
            const int64_t ks = fp.kernel_size;
            const float kscale = (float)(fp.cache_size - 1) / (float)ks;
            int64_t x0 = x - ks, x1 = x + ks + 1, y0 = y - ks, y1 = y + ks + 1;
            int64_t xm = 0, ym = 0;
            if (x0 < 0) { xm = -x0; x0 = 0; }
            if (y0 < 0) { ym = -y0; y0 = 0; }
            if (x1 > (int64_t)fp.w) x1 = fp.w;
            if (y1 > (int64_t)fp.h) y1 = fp.h;
            for (int64_t sy = y0; sy < y1; ++sy) {
                int32_t jy = (int32_t)fabsf(0.5f + kscale*((float)(ym + (sy - y0) - ks) - j.y));
                float fy = fp.lut[jy];
                for (int64_t sx = x0; sx < x1; ++sx) {
                    int32_t jx = (int32_t)fabsf(0.5f + kscale*((float)(xm + (sx - x0) - ks) - j.x));
                    float f = fp.lut[jx]*fy;
                    float* dst = reinterpret_cast<float*>(fp.accum + (size_t)sy*fp.w + sx);
                    unsafeAtomicAdd(dst + 0, f*r.x);
                    unsafeAtomicAdd(dst + 1, f*r.y);
                    unsafeAtomicAdd(dst + 2, f*r.z);
                    unsafeAtomicAdd(dst + 3, f);
                }
            }
        } else {
            const uint32_t xy = fp.pix_xy[p];
            float* dst = reinterpret_cast<float*>(fp.accum + (size_t)(xy >> 16)*fp.w + (xy & 0xFFFFu));
            unsafeAtomicAdd(dst + 0, r.x);
            unsafeAtomicAdd(dst + 1, r.y);
            unsafeAtomicAdd(dst + 2, r.z);
            unsafeAtomicAdd(dst + 3, 1.0f);
        }
    }
}

// k_pixel_map — the coordinates of every pixel of the shard's tile list, in list
// order (tiles descending, raster inside a tile: RT/raytracer.cpp:555, :409-410),
// so k_generate maps a sample to its pixel with one coalesced load.  One block per tile.
__global__ void __launch_bounds__(256) k_pixel_map(FrameParams fp, uint32_t* out) {
    const uint32_t i = blockIdx.x;
    const uint32_t tile = fp.tile_ids[i], base = fp.tile_prefix[i], n = fp.tile_prefix[i + 1] - base;
    const uint32_t min_x = fp.tile_w*(tile % fp.tcx), min_y = fp.tile_h*(tile / fp.tcx);
    const uint32_t tw = min(fp.w, min_x + fp.tile_w) - min_x;
    for (uint32_t local = threadIdx.x; local < n; local += 256)
        out[base + local] = (min_x + local % tw) | ((min_y + local / tw) << 16);
}

// The vignette of a camera ray (RT/raytracer.cpp:451-453): k_generate stores it with the path, and
// k_shade / k_drain recompute it from the stored direction (same operations, same bits).
RT_D float camera_vignette(const FrameParams& fp, const rt_settings& st, V3 rd) {
    float vig = dot(rd, fp.cz);
    vig = vig*vig*vig*vig;
    return lerpf_(1.0f, vig, st.vignette_strength);
}
// The throughput and total_color records of an S_NEW path, as k_generate would have
// written them: throughput (1, 1, 1 | vignette), total_color (0, 0, 0 | bounce 0, specular)
RT_D void new_path_records(const FrameParams& fp, const rt_settings& st, float4 d4, float4& t4, float4& L4) {
    t4 = make_float4(1.0f, 1.0f, 1.0f, camera_vignette(fp, st, ld3(d4)));
    L4 = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(pack_flags(0, 1, 0)));
}

// The AA jitter of sample s of pixel (x, y): render_tile's first sampler draw (RT/raytracer.cpp:
// 431-435).  The sample's RandomSeries is seeded from its key and this draw comes first, so the
// jitter is a function of the key: the splat recomputes it instead of carrying it with the path.
RT_D V2 sample_jitter(const DevScene& sc, const rt_settings& st, const FrameParams& fp, uint32_t x, uint32_t y,
                      uint32_t s) {
    const uint32_t canonical = fp.frame_count + s;
    const uint32_t tile = tile_of(fp, x, y);
    Rng rng = random_seed(sample_seed(fp.total_frame_index, fp.frame_count, tile, y*fp.w + x, canonical));
    const SamplerState ss = {x, y, canonical, st.sampling_strategy};
    const V2 aa = sample_2d(sc, ss, rng, S_AA, 0);
    return {aa.x - 0.5f, aa.y - 0.5f};
}

// k_generate — render_tile's per-sample ray setup (RT/raytracer.cpp:409-463).  It reads only the
// sampler tables and the ray prologue's tables, which stay in HBM and are read through L2 and the
// scalar cache: a block needs no LDS copy of the scene, so it skips that copy, its barrier and its
// LDS footprint.
// SGPR budget: a wave holds ceil(sgpr/16)*16 + 16 of the SIMD's 800 SGPRs.  Left alone the compiler
// gives k_generate 102 (a 128-SGPR wave, as many as a trace wave); capped at 80 it needs 78 with no
// spills (96 per wave), so a generate wave finds room beside the trace waves sooner: a rank's share
// of 8 +1.4 %, C3 / C4 +0.1 / +0.2 % (profiles/r04_sgpr_ab.txt)
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_num_sgpr(80))) k_generate(DevScene sc_g, rt_settings st, FrameParams fp, Pool pool,
                                                        Counters* cnt, int cur) {
    const uint32_t slot = blockIdx.x*blockDim.x + threadIdx.x;
    const uint32_t lane = __lane_id(), wave = (slot >> 6) & (uint32_t)(BLOCK / 64 - 1);   // wave in the group
    const uint32_t wbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)(slot >> 6));
    // Each wave's survivors fill its first slots; the rest take new paths, claiming consecutive
    // sample numbers in slot order from the scan of the free counts k_bookkeep made (no atomics):
    // the block's first claim, the free slots of the block's earlier waves, the lane's rank.
    // The claim and the claimed sample's pixel are loaded first, so their round trips
    // overlap the splat's below instead of waiting behind its stores.
    const uint32_t first = 64u - pool.free_w[wbase];
    uint32_t before = 0;
    for (uint32_t w = 0; w < wave; ++w) before += pool.free_w[wbase - wave + w];
    const bool want = lane >= first;
    const uint32_t cbase = pool.claim_base[slot / BLOCK];
    const unsigned long long remaining = remaining_samples(cnt);
    const uint32_t claim = cbase + before + (lane - first);
    // No sample left for this block to claim (the frame's drain): its free slots go idle
    const bool none_left = (unsigned long long)cbase >= remaining;
    const bool active = !none_left && want && (unsigned long long)claim < remaining;
    const unsigned long long k = cnt->next_sample + claim;
    uint32_t x = 0, y = 0, s = 0, p = 0;
    if (active) {
        if (fp.list_xy) {
            x = fp.list_xy[2*k]; y = fp.list_xy[2*k + 1]; s = fp.list_s[k];
        } else {
            uint32_t pass;
            if (k < 0x100000000ull && fp.px_m) {             // a multiply-high when k fits 32 bits
                pass = div_pixels((uint32_t)k, fp.px_m);
                p = (uint32_t)k - pass*fp.pixels;
            } else {
                pass = (uint32_t)(k / fp.pixels);
                p = (uint32_t)(k % fp.pixels);
            }
            const uint32_t xy = fp.pix_xy[p];                // the tile list's pixel p (k_pixel_map)
            x = xy & 0xFFFFu; y = xy >> 16; s = pass;
        }
    }
    // The paths the k_shade two iterations back finished in this wave's slots (its finished array,
    // compacted): splat them.  Their last NEE contributions came in the k_trace in between.
    if (lane < pool.fin_w[wbase]) {
        const float4 fl = ldnt(&pool.fin_L[slot]);
        const uint2 fk = ldnt(&pool.fin_k[slot]);
        const uint32_t pixel = ldnt(&pool.fin_px[slot]);
        const uint32_t fs = fp.list_xy ? fp.list_s[fk.x] : fk.x;
        const V2 j = sample_jitter(sc_g, st, fp, pixel & 0xFFFFu, pixel >> 16, fs);
        splat_sample(fp, pool, ld3(fl), fl.w, make_float2(j.x, j.y), fk.x, fk.y);
    }
    if (none_left) {
        if (want) pool.state[slot] = S_FREE;
        return;
    }
    const DevScene& sc = sc_g;       // nothing generate reads lives in the LDS copy of the scene
    if (want && !active) pool.state[slot] = S_FREE;
    bool enqueue = false, cast = false;
    V3 nro = {0, 0, 0}, nrd = {0, 0, 0};
    Prologue pro = {};
    if (active) {
        uint32_t canonical = fp.frame_count + s;
        uint32_t tile = tile_of(fp, x, y);
        Rng rng = random_seed(sample_seed(fp.total_frame_index, fp.frame_count, tile, y*fp.w + x, canonical));
        // camera (RT/raytracer.cpp:381-401)
        float hfw = fp.half_film_w*fp.focus_distance;
        float hfh = fp.half_film_h*fp.focus_distance;
        float film_distance = fp.focus_distance*fp.film_distance;
        V3 film_center = sub(fp.cp, smul(film_distance, fp.cz));
        float pixel_w = 1.0f / (float)fp.w, pixel_h = 1.0f / (float)fp.h;
        float v = 1.0f - 2.0f*(float)y*pixel_h;
        float u = 1.0f - 2.0f*(float)x*pixel_w;
        apply_lens_distortion(st.lens_distortion, fp.w, fp.h, u, v);
        SamplerState ss = {x, y, canonical, st.sampling_strategy};
        V2 aa = sample_2d(sc, ss, rng, S_AA, 0);
        float jx = aa.x - 0.5f, jy = aa.y - 0.5f;
        V2 dof = sample_2d(sc, ss, rng, S_DOF, 0);
        dof = transform_bokeh_sample(dof, st.f_factor, st.diaphragm_edges, PI_32*st.phi_shutter_max);
        float djx = hfw*pixel_w*fp.lens_radius*dof.x;
        float djy = hfh*pixel_h*fp.lens_radius*dof.y;
        V3 film_p = film_center;
        film_p = add(film_p, smul((u + pixel_w*jx)*hfw, fp.cx));
        film_p = add(film_p, smul((v + pixel_h*jy)*hfh, fp.cy));
        V3 jcp = add(add(fp.cp, smul(djx, fp.cx)), smul(djy, fp.cy));
        V3 rd = normalize(sub(film_p, jcp));
        const float vig = camera_vignette(fp, st, rd);
        nro = jcp; nrd = rd;
        pool.ray_o[slot] = make_float4(jcp.x, jcp.y, jcp.z, __uint_as_float(x | (y << 16)));
        pool.ray_d[slot] = make_float4(rd.x, rd.y, rd.z, __uint_as_float(fp.list_xy ? (uint32_t)k : s));
        cast = st.max_bounce_count > 0;
        if (!cast) {
            pool.thr[slot] = make_float4(1.0f, 1.0f, 1.0f, vig);
            pool.L[slot] = make_float4(0.0f, 0.0f, 0.0f, !cast ? vig : __uint_as_float(pack_flags(0, 1, 0)));
        }
        pool.prev_n[slot] = make_float2(0.0f, __uint_as_float(p));
        pool.rng[slot] = make_uint4(rng.e0, rng.e1, rng.e2, rng.e3);
        // material_stack[0] = &air: level 0 is never stored; k_shade reads it as sc.air_id
        pool.state[slot] = cast ? S_NEW : S_DONE;   // max_bounce_count == 0: nothing to trace
        if (cast) {
            pro = ray_prologue(sc, jcp, rd, FLT_MAX_, false, 0u);
            pool.hit[slot] = make_float4(pro.t, __uint_as_float(pro.code), 0.0f, 0.0f);
            enqueue = pro.bvh;
        }
    }
    // new paths that enter the BVH go to the current extension queue: one returning atomic per wave,
    // no barrier (r05, as in k_shade's tail)
    const uint32_t shard = blockIdx.x % NSHARD;
    const unsigned long long emask = __ballot(enqueue);
    const uint32_t wsum = __ockl_wfred_add_u32(pro.calls);
    uint32_t got = 0;
    if (lane == 0 && emask) got = atomicAdd(&cnt->ext_count[cur][shard][0], (uint32_t)__popcll(emask));
    if (lane == 1 && wsum) __hip_atomic_fetch_add(&cnt->trav[shard][TV_CALLS], (unsigned long long)wsum, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t ebase = (uint32_t)__builtin_amdgcn_readlane((int)got, 0);
    if (enqueue) {
        float4* q = pool.ext_rec[cur] + REC_Q*((size_t)shard*pool.shard_cap + ebase +
                                               (uint32_t)__popcll(emask & ((1ull << lane) - 1ull)));
        q[0] = make_float4(nro.x, nro.y, nro.z, __uint_as_float(slot));
        q[1] = make_float4(nrd.x, nrd.y, nrd.z, pro.t);
        q[2] = make_float4(pro.inv_d.x, pro.inv_d.y, pro.inv_d.z, __uint_as_float(pro.mlist));
    }
}


// k_trace (below) — intersect_scene for every queued path (RT/intersection.cpp:606-610), then
// intersect_shadow_ray for every queued shadow ray (:600-604, RT/integrators.cpp:756); unoccluded
// NEE contributions are added to the path's total_color.
// Persistent waves: each wave grabs CHUNK_EXT / CHUNK_SH queue items with one atomic and
// refills lanes whose query has finished from that chunk (Aila & Laine 2009,
// for 64-wide waves), so lanes do not idle behind the wave's longest ray.
constexpr int TB = 256;                     // threads per persistent trace block
constexpr uint32_t CHUNK = 256;             // queue items a wave takes per fetch (k_drain)
// extension / shadow items: 128 (r05).  Only ~13 % of the closest and ~5 % of the shadow rays enter a
// BVH, so a launch has ~1 chunk of 256 per wave and its end waits on the waves holding the last ones; 128
// gives a rank's share of 8 +3.5 %, the full C3 / C4 frames within +-0.3 %; 96 or a chunk sized per launch
// for 2-3 fetches per wave less (profiles/r05_chunk_ab.txt).
constexpr uint32_t CHUNK_EXT = 128, CHUNK_SH = 128;
constexpr int STEPS_PER_REFILL = 8;         // trace steps between lane refills

// VGPR budget.  The block's LDS (a 16-entry stack + the hit barycentrics, 34.8 KB) allows 4
// blocks per CU, i.e. 4 trace waves per SIMD, whatever the registers.  The LDS is dynamic so
// that the compiler does not see that cap and keeps the listed builds in a 5-wave budget:
// 90 / 86 VGPRs without spills (r05: 96 before the step split), which leaves room for two 64-VGPR k_shade waves beside four
// trace waves instead of one (the 112-VGPR build).  The top-level builds keep the 4-wave
// budget (118 / 114 VGPRs; at 96 they spill).
#define RT_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(LST ? 5 : REF ? 3 : 4)))   // REF: the diagnostic reference-unit walk
constexpr int TRACE_STACK_LDS = STACK_LDS;
constexpr size_t TRACE_LDS = sizeof(uint2)*TRACE_STACK_LDS*TB + sizeof(float2)*TB;   // dynamic, per block
// LST: every queued ray carries a mesh list (the scene's top level is walked in the
// prologue and has no more mesh instances than MLIST_MAX, DevScene::listed_only), so
// the kernel is built without the top-level walk.
// One queue of a trace launch: persistent waves take CHUNK items per atomic from the queue's NSHARD
// shards (their own first, then the others) and refill lanes whose query has finished.  OCC = false:
// the extension queue (intersect_scene, the hit record into the path's slot); OCC = true: the shadow
// queue of the previous iteration's k_shade (intersect_shadow_ray; an unoccluded ray adds its NEE
// term to its path's total_color: a survivor's, now in this iteration's path buffer, or a finished
// path's entry of the other finished array, fin2).
template <bool OCC, bool LST, bool REF>
RT_D void trace_queue(const DevScene& sc, const Pool& pool, Counters* cnt, int cur, const StackT<TRACE_STACK_LDS>& st,
                      const uint32_t* qlen) {
    constexpr uint32_t chunk = OCC ? CHUNK_SH : CHUNK_EXT;
    // a wave drains its own shard first, then the others (a plain read of a head
    // skips exhausted shards without an atomic)
    uint32_t shard = blockIdx.x % NSHARD, tried = 0;
    const uint32_t lane = __lane_id();
    uint32_t chunk_next = 0, chunk_end = 0;
    bool exhausted = false, active = false;
    uint32_t item = 0;
    Traversal<OCC, LST, TRACE_STACK_LDS, REF> tr;
    StepCounts<LST> tally;                              // checked after every refill round
    static_assert(STEPS_PER_REFILL <= StepField<LST>::MARGIN, "StepCounts: a round's steps fit a field's upper half");
    auto finish = [&]() {
        if (OCC) {
            if (!tr.occluded) {
                const uint32_t slot = pool.sh_dst[item];
                const float4 c = ldnt(&pool.sh_c[item]);
                float4* const dst = (slot & SH_FIN) ? &pool.fin2_L[slot & ~SH_FIN] : &pool.L[slot];
                float4 L = ldnt(dst);
                L.x = L.x + c.x; L.y = L.y + c.y; L.z = L.z + c.z;   // total_color += ... (:768)
                stnt(dst, L);
            }
        } else if (tr.code != RT_HIT_MISS) {                  // a BVH hit; else k_shade's plane result stands
            const uint32_t slot = item;                       // the path's slot (from the record)
            const Hit h = tr.result(st);
            stnt(&pool.hit[slot], make_float4(h.t, __uint_as_float(h.code), __uint_as_float(h.tri), h.v));
            stnt(&pool.hit_w[slot], h.w);
        }
    };
    for (;;) {
        unsigned long long idle = __ballot(!active);
        while (idle && !exhausted) {
            if (chunk_next >= chunk_end) {
                const int leader = __ffsll((long long)__ballot(true)) - 1;
                bool got = false;
                while (tried < NSHARD) {
                    uint32_t* head = &cnt->fetch[OCC ? 1 : 0][shard][0];
                    const uint32_t len = qlen[shard];
                    uint32_t base = 0xFFFFFFFFu;
                    if (lane == (uint32_t)leader &&
                        __hip_atomic_load(head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < len)
                        base = atomicAdd(head, chunk);
                    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);   // wave-uniform: SGPRs
                    if (base < len) {
                        chunk_next = shard*pool.shard_cap + base;
                        chunk_end = shard*pool.shard_cap + min(base + chunk, len);
                        got = true;
                        break;
                    }
                    shard = (shard + 1) % NSHARD;
                    ++tried;
                }
                if (!got) { exhausted = true; break; }
            }
            const uint32_t avail = chunk_end - chunk_next;
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            if (!active && rank < avail) {
                item = chunk_next + rank;
                if (OCC) item = pool.sh_slot[item];               // the k_shade slot that staged the ray
                const float4* q = (OCC ? pool.sh_rec : pool.ext_rec[cur]) + REC_Q*(size_t)item;
                const float4 o = ldnt(&q[0]), d = ldnt(&q[1]), iv = ldnt(&q[2]);
                if (!OCC) item = __float_as_uint(o.w);            // the path's slot
                tr.init_rec(sc, st, ld3(o), ld3(d), ld3(iv), d.w, OCC ? __float_as_uint(o.w) : 0u, __float_as_uint(iv.w));
                if (tr.mode == TM_DONE) finish(); else active = true;
            }
            chunk_next += min((uint32_t)__popcll(idle), avail);
            idle = __ballot(!active);
        }
        if (__ballot(active) == 0ull) break;
        if (active) {
            for (int k = 0; k < STEPS_PER_REFILL; ++k) {
                if (!tr.step(sc, st)) { finish(); active = false; break; }
            }
        }
        tally.check(tr.acc);                            // every lane is here
    }
    tally.flush(tr.acc);
    if (REF) tally.flush_ref(tr.rc);
    tally.commit(cnt->trav[blockIdx.x % NSHARD], OCC ? 1 : 0);
}

// k_trace — one persistent launch per iteration for both queues (r06): intersect_scene for this
// iteration's extension queue (RT/intersection.cpp:606-610), then intersect_shadow_ray for the
// shadow queue the previous k_shade left (:600-604, RT/integrators.cpp:756).  Each wave finishes its
// extension items, then takes shadow items, so the shadow rays fill the extension queue's tail
// instead of a launch (and a tail) of their own; the finished paths they add to are splatted one
// iteration later for it (Pool::fin2).  The fused drain's iteration traces the shadow queue only.
// PH: bit 0 the extension queue, bit 1 the shadow queue -- 3 merged (rt_scene_config::shadow_launch), 1 and 2
// the separate launches (2 with a pool view whose L / fin2 are the survivors' and finished paths' of the
// same iteration and cur flipped, run_frame).  Each is its own instantiation: the separate ones keep the
// registers of one kind of query, and profiles tell the launches apart.
template <bool LST, bool REF, int PH>
__global__ void __launch_bounds__(TB) RT_TRACE_ATTR k_trace(DevScene sc, Pool pool, Counters* cnt, int cur, uint2* spill,
                                                              int fuse, uint32_t sh_pct) {
    // (no done check: once a partition is done its queues stay empty, and a check would put a dependent
    // load in front of every block)
    // trace waves are latency bound and issue little; shade waves sharing the SIMD are
    // issue bound: let a trace wave's next load go out first (r03b, priority 1: a rank's share of 8
    // +0.4 to +1.6 % in five pairs, the full frames within noise; profiles/r03b_ab.txt section 23)
    __builtin_amdgcn_s_setprio(1);
    extern __shared__ uint2 trace_lds[];   // TRACE_LDS bytes: the stack, then the barycentrics
    StackT<TRACE_STACK_LDS> st;
    st.lds = trace_lds; st.spill = spill; st.bary = reinterpret_cast<float2*>(trace_lds + TRACE_STACK_LDS*TB);
    st.lane = threadIdx.x; st.block = TB;
    st.gtid = blockIdx.x*TB + threadIdx.x; st.nthreads = gridDim.x*TB;
    // k_drain runs this iteration's extension rays once the drain is fused (uniform)
    const bool ext = (PH & 1) && !(fuse && cnt->fused);
    __shared__ uint32_t qlen[2][NSHARD];
    if (threadIdx.x < NSHARD) {
        if (PH & 1) qlen[0][threadIdx.x] = ext ? cnt->ext_count[cur][threadIdx.x][0] : 0u;
        if (PH & 2) qlen[1][threadIdx.x] = cnt->shadow_count[cur ^ 1][threadIdx.x][0];
    }
    __syncthreads();
    // the shadow queue after the extension items: sh_pct % of the blocks, spread evenly over the grid (and
    // the XCDs); all of them when there is no extension phase (the fused drain's iteration, whose k_drain
    // waits for it, and the separate shadow launch).  (Shadow items first: share of 8 -2 %, C3 / C4 +-0.5 %.)
    const bool sh = (PH & 2) && (!ext || (blockIdx.x*sh_pct) % 100u < sh_pct);
    if ((PH & 1) && ext) trace_queue<false, LST, REF>(sc, pool, cnt, cur, st, qlen[0]);
    if ((PH & 2) && sh) trace_queue<true, LST, REF>(sc, pool, cnt, cur, st, qlen[1]);
}

// k_shade — one bounce of advanced_integrator (RT/integrators.cpp:612-818)
// 8 waves per SIMD (64 VGPRs) for the default instantiation (scene in LDS, no environment NEE),
// which fits them without spills; the others need 66-67 and keep 7
#ifndef RT_SHADE_WAVES
#define RT_SHADE_WAVES 8            // tuning builds: -DRT_SHADE_WAVES=7
#endif
#define RT_SHADE_ATTR __attribute__((amdgpu_waves_per_eu((IN_LDS && !ENV) ? RT_SHADE_WAVES : 7)))
// One bounce of advanced_integrator (RT/integrators.cpp:612-815) for a path whose closest hit
// is h: emission / MIS, Beer absorption, Fresnel, reflect / refract / diffuse with NEE (the
// shadow ray is returned, not traced) and Russian roulette.  Shared by k_shade (one bounce per
// launch) and k_drain (a path's remaining bounces in one launch), so both compute the same bits.
// The material stack lives at pool.mstack[level*n + slot].  Returns true when the path ends.
template <bool ENV>
RT_D bool shade_bounce(const DevScene& sc, const rt_settings& st, const SamplerState& ss, const Pool& pool,
                       uint32_t slot, const Hit& h, V3& ro, V3& rd, V3& thr, V3& total, float& prev_pdf,
                       uint32_t& bounce, uint32_t& is_spec, int32_t& at, Rng& rng, bool& cast_shadow,
                       V3& sh_o, V3& sh_d, V3& sh_c, float& sh_t, uint32_t& sh_light) {
    bool done = false;
    if (h.code != RT_HIT_MISS) {
        V3 I, N;
        uint32_t surf_id;
        Ray ray; ray.o = ro; ray.d = rd;
        hit_geometry(sc, ray, h, I, N, surf_id);
        float t = h.t;
        float cos_i = -dot(rd, N);
        bool inside = (cos_i < 0.0f);
        uint32_t mi_id, mt_id;
        if (inside) {
            mi_id = surf_id;
            const int32_t lv = at - 1 > 0 ? at - 1 : 0;
            mt_id = lv ? pool.mstack[(size_t)lv*pool.n + slot] : sc.air_id;     // level 0 = air
            cos_i = -cos_i;
            N = neg(N);
        } else {
            mi_id = at ? pool.mstack[(size_t)at*pool.n + slot] : sc.air_id;
            mt_id = surf_id;
        }
        const rt_material mi = sc.materials[mi_id];
        const rt_material mt = sc.materials[mt_id];
        if (mi.is_participating_medium) {                                  // Beer :640-649
            V3 ab = {d_expf(-mi.absorb.x*t), d_expf(-mi.absorb.y*t), d_expf(-mi.absorb.z*t)};
            thr = mul(thr, ab);
        }
        if (mt.flags & RT_MATERIAL_EMISSIVE) {                             // :651-670
            bool allow = (!st.next_event_estimation ||
                          ((st.caustics || (bounce < 2)) && is_spec));
            if (allow) {
                total = add(total, mul(thr, rv3(mt.emission_color)));
            } else if (bounce > 0 && st.use_mis) {
                float ldsq = t*t;
                float light_pdf = ldsq / cos_i;
                float brdf_pdf = (st.importance_sample_diffuse ? prev_pdf : 1.0f / (2.0f*PI_32));
                float mis_pdf = light_pdf + brdf_pdf;
                total = add(total, mul(smul(rcp_cr(mis_pdf), thr), rv3(mt.emission_color)));
            }
            done = true;
        } else {
            float eta_i = mi.ior, eta_t = mt.ior;
            float eta = eta_i / eta_t;
            float cos_t;
            float refl = fresnel_dielectric(cos_i, eta_i, eta_t, eta, cos_t);
            float reflect_test = sample_1d(sc, ss, rng, S_Reflectance, bounce);
            refl = lerpf_(refl, 1.0f, mt.metallic);
            is_spec = 1;
            if (reflect_test < refl) {                                      // reflect :684-696
                V3 nd = reflect(rd, N);
                if (mt.roughness > 0.0f) {
                    V3 rs = random_in_unit_sphere(rng);
                    nd = normalize(add(smul(1.0f + EPSILON, nd), smul(mt.roughness, rs)));
                }
                ro = add(I, smul(EPSILON, nd)); rd = nd;
                thr = mul(thr, lerp3(v3s(1.0f), rv3(mt.albedo), mt.metallic));
            } else if (mt.is_participating_medium) {                       // refract :698-717
                if (inside) {
                    if (at > 0) --at;
                } else if (at < 63) {
                    ++at;
                    pool.mstack[(size_t)at*pool.n + slot] = (uint16_t)mt_id;   // moved with the path below
                }
                V3 fd = add(smul(eta, rd), muls(N, (eta*cos_i - cos_t)));
                ro = add(I, muls(fd, EPSILON)); rd = fd;
            } else {                                                        // diffuse :718-790
                is_spec = 0;
                V3 albedo = evaluate_material(mt, I);
                V3 brdf = smul(1.0f / PI_32, albedo);
                if (st.next_event_estimation && (sc.light_count > 0 || ENV)) {      // NEE :738-771
                    float lps = sample_1d(sc, ss, rng, S_LightSelection, bounce);
                    // ENV: the environment is picked with probability q (1 without lights)
                    const float q = sc.light_count > 0 ? 0.5f : 1.0f;
                    const bool pick_env = ENV && lps < q;
                    if (ENV) lps = pick_env ? lps / q : (lps - q) / (1.0f - q);
                    float lrp = 0.0f;
                    uint32_t lid = pick_env ? 0u : pick_random_light(sc, st, lps, I, lrp);
                    if (ENV) lrp = lrp*(1.0f - q);
                    V2 s2 = sample_2d(sc, ss, rng, S_DirectLighting, bounce);
                    if (pick_env) {
                        V3 Lv = env_direction(sc, lps, s2);
                        float ndl = dot(N, Lv);
                        if (ndl > 0.0f) {
                            uint32_t tile;
                            V3 Le = sky_env(sc, Lv, tile);
                            float pe = env_pdf(sc, tile, Lv);
                            if (pe > 0.0f) {
                                float bpdf = (st.importance_sample_diffuse ? ndl / PI_32 : 1.0f / (2.0f*PI_32));
                                float pdf = st.use_mis ? q*pe + bpdf : q*pe;
                                sh_c = mul(mul(muls(thr, ndl / pdf), brdf), Le);
                                sh_o = add(I, muls(Lv, EPSILON));
                                sh_d = Lv;
                                sh_t = FLT_MAX_;
                                sh_light = 0;                   // the null primitive: nothing ignored
                                cast_shadow = true;
                            }
                        }
                    } else {
                        // random_point_on_light (:199-228), sphere lights
                        const rt_primitive light = sc.prims[lid];
                        const M34 lf = load_m34(&sc.fwd[light.transform_index]);
                        V3 towards = normalize(sub(translation(lf), I));
                        if (light.type == RT_PRIMITIVE_SPHERE) {
                            float rad = light.p[0];
                            V3 Nl = map_to_hemisphere(neg(towards), s2);
                            V3 pw = xform(lf, muls(Nl, rad), 1.0f);
                            V3 Lv = sub(pw, I);
                            float dsq = length_sq(Lv);
                            float dist = __builtin_sqrtf(dsq);
                            Lv = divs(Lv, dist);
                            float A = 2.0f*PI_32*rad*rad;
                            float ndl = dot(N, Lv);
                            float nndl = -dot(Nl, Lv);
                            if (ndl > 0.0f && nndl > 0.0f) {
                                float sa = (nndl * A) / dsq;
                                float pdf;
                                if (st.use_mis) {
                                    float lpdf = rcp_cr(sa);
                                    float bpdf = (st.importance_sample_diffuse ? ndl / PI_32 : 1.0f / (2.0f*PI_32));
                                    pdf = lpdf + bpdf;
                                } else {
                                    pdf = rcp_cr(sa);
                                }
                                pdf *= lrp;
                                sh_c = mul(mul(muls(thr, dot(N, Lv) / pdf), brdf),
                                           rv3(sc.materials[light.material_id].emission_color));
                                sh_o = add(I, muls(Lv, EPSILON));
                                sh_d = Lv;
                                sh_t = dist - 2*EPSILON;
                                sh_light = lid;
                                cast_shadow = true;                 // traced below, lanes reconverged
                            }
                        }
                    }
                }
                V2 s2 = sample_2d(sc, ss, rng, S_IndirectLighting, bounce); // indirect :777-789
                V3 R;
                if (st.importance_sample_diffuse) {
                    R = map_to_cosine_weighted_hemisphere(N, s2);
                    thr = muls(thr, PI_32);
                } else {
                    R = map_to_hemisphere(N, s2);
                    thr = muls(thr, 2.0f*PI_32*dot(N, R));
                }
                thr = mul(thr, brdf);
                ro = add(I, muls(N, EPSILON)); rd = R;
            }
            if (st.russian_roulette && !is_spec) {                          // RR :801-811
                float p = clampf_(max3(thr), 0.1f, 0.9f);
                float e = sample_1d(sc, ss, rng, S_Roulette, bounce);
                if (e > p) done = true;
                else thr = muls(thr, rcp_cr(p));
            }
        }
        if (!done) {
            if (st.importance_sample_diffuse) prev_pdf = dot(N, rd) / PI_32;   // prev_N = N, and the new ray
            ++bounce;
            if (bounce >= st.max_bounce_count) done = true;
        }
    } else {
        if (ENV) {
            // a path leaving a diffuse vertex (which sampled the environment in its NEE):
            // balance heuristic against that pdf; without MIS the NEE alone carries it
            uint32_t tile;
            V3 Le = sky_env(sc, rd, tile);
            if (!is_spec) {
                float wgt = 0.0f;
                if (st.use_mis) {
                    const float q = sc.light_count > 0 ? 0.5f : 1.0f;
                    float pe = env_pdf(sc, tile, rd);
                    float bpdf = (st.importance_sample_diffuse ? prev_pdf : 1.0f / (2.0f*PI_32));
                    float den = q*pe + bpdf;
                    wgt = den > 0.0f ? bpdf / den : 0.0f;
                }
                Le = smul(wgt, Le);
            }
            total = add(total, mul(thr, Le));
        } else {
            total = add(total, mul(thr, sample_sky(sc, rd)));             // miss :812-815
        }
        done = true;
    }
    return done;
}

// ENV: rt_set_env_sampling on, the scene has an environment map and NEE is on
template <bool IN_LDS, bool ENV>
__global__ void __launch_bounds__(BLOCK) RT_SHADE_ATTR k_shade(DevScene sc_g, rt_settings st, FrameParams fp, Pool pool,
                                                 Counters* cnt, int cur, int sparse, int fuse) {
    if (fuse && cnt->fused) return;                 // k_drain runs this iteration's paths (uniform)
    const uint32_t slot = blockIdx.x*blockDim.x + threadIdx.x;
    // The slot's state and path record are loaded before the scene copy, whatever the
    // state: the three round trips (state, record, LDS blob) overlap instead of running
    // back to back.  A slot not traced this iteration (~1/6 of the pool) reads 120 B for nothing.
    // In the frame's drain (`sparse`: nothing left to claim, most slots idle) the record is read
    // only for the slots that hold a path, after their state; a partition already done exits.
    uint8_t state0 = S_FREE;
    float4 o4 = {}, d4 = {}, t4 = {}, L4 = {}, h4 = {};
    float2 pn2 = {};
    uint4 r4 = {};
    float hw = 0.0f;
    auto load_path = [&]() {
        o4 = ldnt(&pool.ray_o[slot]); d4 = ldnt(&pool.ray_d[slot]);
        t4 = ldnt(&pool.thr[slot]); L4 = ldnt(&pool.L[slot]); pn2 = ldnt(&pool.prev_n[slot]);
        h4 = ldnt(&pool.hit[slot]); r4 = ldnt(&pool.rng[slot]); hw = ldnt(&pool.hit_w[slot]);
    };
    if (sparse) {
        if (cnt->done) return;                                          // uniform: every block reads it
        if (slot < pool.n) {
            state0 = pool.state[slot];
            if (state0 != S_FREE) load_path();
        }
    } else if (slot < pool.n) {
        state0 = pool.state[slot];
        load_path();
    }
    if (state0 == S_NEW) {                              // a camera ray (k_generate)
        new_path_records(fp, st, d4, t4, L4);
        state0 = S_TRACE;
    }
    const DevScene sc = scene_in_lds<IN_LDS>(sc_g, lds_scene);
    const bool valid = slot < pool.n && state0 == S_TRACE;             // traced this iteration
    bool cont = false, done = false, shadow = false, cast_shadow = false, enq = false;
    Prologue spro = {}, cpro = {};
    V3 nro = {0, 0, 0}, nrd = {0, 0, 0};
    V3 sh_o = {0, 0, 0}, sh_d = {0, 0, 0}, sh_c = {0, 0, 0};
    float sh_t = 0.0f;
    uint32_t sh_light = 0;
    uint32_t nslot = 0;                                                // a survivor's slot in pool.nx
    // finished-array entries (see the tail): the slots k_generate made finished, then the paths
    // that end here
    const bool made_fin = slot < pool.n && state0 == S_DONE;
    const unsigned long long made_fin_mask = __ballot(made_fin);
    // pixel, sample key, vignette and tile-list pixel (`meta`): written out only at the end, so they
    // wait in LDS (the thread's own entry, no barrier) instead of registers across the bounce and
    // the prologues
    __shared__ uint4 stash[BLOCK];
    __shared__ uint8_t sh_calls[BLOCK];             // the shadow prologue's mesh instances reached
    if (valid || made_fin)
        stash[threadIdx.x] = make_uint4(__float_as_uint(o4.w), __float_as_uint(d4.w), __float_as_uint(t4.w),
                                        __float_as_uint(pn2.y));
    if (valid) {
        Rng rng = {r4.x, r4.y, r4.z, r4.w};
        V3 ro = ld3(o4), rd = ld3(d4);
        V3 thr = ld3(t4), total = ld3(L4);
        float prev_pdf = pn2.x;                      // dot(prev_N, rd) / PI_32 (Pool::prev_n)
        uint32_t flags = __float_as_uint(L4.w);
        uint32_t bounce = flags & 0xFFu, is_spec = (flags >> 8) & 1u;
        int32_t at = (int32_t)((flags >> 9) & 0x7Fu);
        uint32_t pixel = __float_as_uint(o4.w);
        uint32_t sample_off = __float_as_uint(d4.w);
        uint32_t px = pixel & 0xFFFFu, py = pixel >> 16;            // no integer division
        uint32_t canonical = fp.frame_count + (fp.list_xy ? fp.list_s[sample_off] : sample_off);
        SamplerState ss = {px, py, canonical, st.sampling_strategy};
        Hit h;
        h.t = h4.x; h.code = __float_as_uint(h4.y); h.tri = __float_as_uint(h4.z); h.v = h4.w; h.w = hw;
        done = shade_bounce<ENV>(sc, st, ss, pool, slot, h, ro, rd, thr, total, prev_pdf, bounce, is_spec, at, rng,
                                 cast_shadow, sh_o, sh_d, sh_c, sh_t, sh_light);
        // The survivor's state that the two prologues below do not change goes out now, so the
        // throughput, RNG and flags are not held in registers across them (total_color and the
        // hit record follow the prologues).  The wave's paths that continue go, in slot order, to
        // the front of its 64 slots in the other buffer (pool.nx): a ballot, no barrier.  The next
        // k_generate fills the rest.  A path that ends goes to the wave's finished array.
        cont = !done;
        const uint4 meta = stash[threadIdx.x];          // pixel, key, vignette, tile-list pixel
        {
            const unsigned long long smask = __ballot(cont);
            nslot = (slot & ~63u) + (uint32_t)__popcll(smask & ((1ull << __lane_id()) - 1ull));
        }
        if (cont) {
            stnt(&pool.nx.ray_o[nslot], make_float4(ro.x, ro.y, ro.z, __uint_as_float(meta.x)));
            stnt(&pool.nx.ray_d[nslot], make_float4(rd.x, rd.y, rd.z, __uint_as_float(meta.y)));
            stnt(&pool.nx.thr[nslot], make_float4(thr.x, thr.y, thr.z, __uint_as_float(meta.z)));
            stnt(&pool.nx.prev_n[nslot], make_float2(prev_pdf, __uint_as_float(meta.w)));
            stnt(&pool.nx.rng[nslot], make_uint4(rng.e0, rng.e1, rng.e2, rng.e3));
            pool.nx.state[nslot] = S_TRACE;
            // the material stack moves with the path (levels 1..at; level 0 is the implicit air)
            for (int32_t lv = 1; lv <= at; ++lv)
                pool.nx.mstack[(size_t)lv*pool.n + nslot] = pool.mstack[(size_t)lv*pool.n + slot];
        }
        const unsigned long long fm = made_fin_mask | __ballot(done);
        if (done) {                                        // everything but total_color
            const uint32_t fidx = (slot & ~63u) + (uint32_t)__popcll(fm & ((1ull << __lane_id()) - 1ull));
            stnt(&pool.fin_k[fidx], make_uint2(meta.y, meta.w));
            stnt(&pool.fin_px[fidx], meta.x);
        }
        const float vig = __uint_as_float(meta.z);
        const uint32_t nflags = pack_flags(bounce, is_spec, (uint32_t)at);
        if (cast_shadow) {
            // intersect_shadow_ray (:756): planes and the top level here; only rays that meet
            // a mesh are queued for the next iteration's k_trace.  Nothing else adds to total_color after the
            // NEE term in a bounce, so adding it here keeps the reference's order (:768).
            spro = ray_prologue(sc, sh_o, sh_d, sh_t, true, sh_light);
            sh_calls[threadIdx.x] = (uint8_t)spro.calls;   // counted at the tail, not held in a register
            shadow = !spro.occluded && spro.bvh;
            if (!spro.occluded && !spro.bvh) total = add(total, sh_c);
            if (shadow) {                                  // staged at the slot (Pool::sh_rec)
                float4* q = pool.sh_rec + REC_Q*(size_t)slot;
                stnt(&q[0], make_float4(sh_o.x, sh_o.y, sh_o.z, __uint_as_float(sh_light)));
                stnt(&q[1], make_float4(sh_d.x, sh_d.y, sh_d.z, sh_t));
                stnt(&q[2], make_float4(spro.inv_d.x, spro.inv_d.y, spro.inv_d.z, __uint_as_float(spro.mlist)));
                stnt(&pool.sh_c[slot], make_float4(sh_c.x, sh_c.y, sh_c.z, 0.0f));
            }
        }
        if (cont) stnt(&pool.nx.L[nslot], make_float4(total.x, total.y, total.z, __uint_as_float(nflags)));
        if (done) {
            const uint32_t fidx = (slot & ~63u) + (uint32_t)__popcll(fm & ((1ull << __lane_id()) - 1ull));
            stnt(&pool.fin_L[fidx], make_float4(total.x, total.y, total.z, vig));
        }
        nro = ro; nrd = rd;
        if (cont) {                                        // next bounce's intersect_scene: planes + top level here
            cpro = ray_prologue(sc, ro, rd, FLT_MAX_, false, 0u);
            enq = cpro.bvh;
            stnt(&pool.nx.hit[nslot], make_float4(cpro.t, __uint_as_float(cpro.code), 0.0f, 0.0f));
        }
    }
    const int nxt = cur ^ 1;
    const uint32_t shard = blockIdx.x % NSHARD;
    // The wave's paths that end here (or were made finished: max_bounce_count 0) go to the front of
    // its 64 entries of the finished array, which the next k_generate splats before it fills the
    // wave's slots past the survivors with new paths (the host's termination test waits for them).
    const bool fin = done || made_fin;
    const unsigned long long fmask = __ballot(fin);
    const uint32_t fidx = (slot & ~63u) + (uint32_t)__popcll(fmask & ((1ull << __lane_id()) - 1ull));
    if (made_fin) {                                 // L = 0 with the vignette in .w (k_generate)
        const uint4 fmeta = stash[threadIdx.x];
        stnt(&pool.fin_L[fidx], pool.L[slot]);
        stnt(&pool.fin_k[fidx], make_uint2(fmeta.y, fmeta.w));
        stnt(&pool.fin_px[fidx], fmeta.x);
    }
    const unsigned long long cmask = __ballot(cont);
    if (__lane_id() == 0) {
        pool.free_w[slot >> 6] = 64u - (uint32_t)__popcll(cmask);
        pool.fin_w[slot >> 6] = (uint32_t)__popcll(fmask);
    }
    // Each wave appends to its shard's queues with its own returning atomic (lanes 0 and 1: extension,
    // shadow; one instruction) and adds the other counters with no-return atomics: no barrier, so a wave
    // leaves without waiting for its block's slowest one (r05; the block tally's two barriers and its
    // thread-0 atomics before: C4 +2.2 % in five A/B pairs, C3 and a rank's share of 8 within +-0.4 %,
    // profiles/r05_wave_append_ab.txt).  Four times the atomics on a shard's queue counter (~16k per
    // launch at C3's pool) stay under the ~88 per us one word sustains.  k_bookkeep sums free_w.
    // Invariant: every lane of the wave reaches this block.  The atomics are issued from fixed lanes
    // (0..6) and the queue bases read back from lanes 0 and 1, so k_shade may only return where the
    // whole wave does: the three returns above test Counters flags every lane reads alike.
    {
        const unsigned long long emask = __ballot(enq), smask = __ballot(shadow), xmask = __ballot(cast_shadow);
        const uint32_t lane = __lane_id();
        const unsigned long long lt = (1ull << lane) - 1ull;
        uint32_t* ap = nullptr;
        uint32_t av = 0;
        if (lane == 0) { ap = &cnt->ext_count[nxt][shard][0]; av = (uint32_t)__popcll(emask); }
        if (lane == 1) { ap = &cnt->shadow_count[cur][shard][0]; av = (uint32_t)__popcll(smask); }
        uint32_t got = 0;
        if (av) got = atomicAdd(ap, av);
        // the other counters, no-return: alive, shadow rays cast, finished; the mesh instances reached
        uint32_t* np = nullptr;
        uint32_t nv = 0;
        if (lane == 2) { np = &cnt->alive[shard][0]; nv = (uint32_t)__popcll(cmask); }
        if (lane == 3) { np = &cnt->cast[1][shard][0]; nv = (uint32_t)__popcll(xmask); }
        if (lane == 4) { np = &cnt->unsplat[shard][0]; nv = (uint32_t)__popcll(fmask); }
        if (nv) __hip_atomic_fetch_add(np, nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t c = cpro.calls | ((cast_shadow ? (uint32_t)sh_calls[threadIdx.x] : 0u) << 16);
        const uint32_t wsum = __ockl_wfred_add_u32(c);
        unsigned long long* cp = nullptr;
        uint32_t cv = 0;
        if (lane == 5) { cp = &cnt->trav[shard][TV_CALLS]; cv = wsum & 0xFFFFu; }
        if (lane == 6) { cp = &cnt->trav[shard][TV_N + TV_CALLS]; cv = wsum >> 16; }
        if (cv) __hip_atomic_fetch_add(cp, (unsigned long long)cv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t ebase = (uint32_t)__builtin_amdgcn_readlane((int)got, 0);
        const uint32_t sbase = (uint32_t)__builtin_amdgcn_readlane((int)got, 1);
        if (enq) {
            float4* q = pool.ext_rec[nxt] + REC_Q*((size_t)shard*pool.shard_cap + ebase + (uint32_t)__popcll(emask & lt));
            stnt(&q[0], make_float4(nro.x, nro.y, nro.z, __uint_as_float(nslot)));
            stnt(&q[1], make_float4(nrd.x, nrd.y, nrd.z, cpro.t));
            stnt(&q[2], make_float4(cpro.inv_d.x, cpro.inv_d.y, cpro.inv_d.z, __uint_as_float(cpro.mlist)));
        }
        if (shadow) {
            pool.sh_slot[(size_t)shard*pool.shard_cap + sbase + (uint32_t)__popcll(smask & lt)] = slot;
            pool.sh_dst[slot] = cont ? nslot : (SH_FIN | fidx);
        }
    }
}



// The frame's drain, fused.  Once nothing is left to claim and few paths are alive, an iteration
// of separate launches costs about as long as its slowest ray whatever the number of paths (one
// extend launch lasts ~300 us for a query of ~300 steps), and a path of the last claims may need
// max_bounce_count more iterations.  So when k_bookkeep sets Counters::fused (see ResPlan::fuse),
// the next iteration launched with these kernels runs every remaining path to its end in one
// launch: k_drain_list gathers the live slots, then each k_drain lane takes a path and loops
// extend -> shade_bounce -> connect -> prologue of the next bounce until the path ends, then
// splats it.  Lanes take new paths as theirs end (at bounce boundaries: a wave syncs on its
// slowest traversal per bounce, not the whole launch per bounce).  The functions are the ones the
// separate kernels run (ray_prologue, Traversal, shade_bounce, splat_sample), so a path's
// result is the same bits; the order in which paths finish does not enter any result.
//
// k_drain_list (the fused iteration, after k_generate splatted the finished array of two iterations
// back and k_trace added the last NEE terms of the last k_shade's): it splats the last k_shade's
// finished paths (Pool::fin2, which the next k_generate would have splatted), the survivors of that
// k_shade (S_TRACE) go to Pool::sh_slot, sharded like the queues; both finished arrays are emptied,
// and the pool is retired: every wave's free count goes to 64, so a k_generate launched after the
// drain marks every slot of whichever buffer it gets S_FREE.
//
// Why the retirement (r06; the r05 every-4th-iteration carry lost the radiance of 13,120 samples
// of one claim batch on C4-small).  k_drain leaves the pool states as they were, and free_w keeps
// the counts of the k_shade before the drain.  The host enqueues iterations two chunks ahead; when
// an iteration after the drain did not carry the drain kernels (fuse = 0), its k_shade was not held
// back by Counters::fused: k_generate kept the first 64 - free_w slots of each wave of the other
// buffer (the stale inputs of that k_shade, still S_TRACE), k_shade shaded them a second time, and
// with k_bookkeep no longer resetting the counters once done, the connect and extend fetch heads
// stood past the re-runs' new queue entries: shadow rays went untraced and mesh hits unfound, and
// the re-runs splatted the poorer results over the finished records.  The default
// schedule never ran into it only because every iteration after the first fused one carried the drain
// kernels, whose fuse flag makes extend / shade / connect exit.  Now the drain leaves no live state
// behind, whatever the host's cadence: a k_generate after it marks every slot S_FREE and claims
// nothing (no sample is left), and the k_shade after that finds no path.  (A done check at the top of
// k_shade costs it an 8-byte spill at 64 VGPRs, and one at the top of k_generate a dependent load
// before its first: C3 -0.9 %, profiles/r06_vs_r05_ab.txt; the retired pool makes both unneeded.)
__global__ void __launch_bounds__(BLOCK) k_drain_list(DevScene sc, rt_settings st, FrameParams fp, Pool pool, Counters* cnt,
                                                      int splat_prev) {
    if (!cnt->fused || cnt->done) return;                              // uniform
    const uint32_t slot = blockIdx.x*blockDim.x + threadIdx.x;
    const uint8_t stv = slot < pool.n ? pool.state[slot] : S_FREE;
    const bool live = stv == S_TRACE || stv == S_NEW;
    const uint32_t wbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)(slot >> 6));
    if (splat_prev && slot < pool.n && __lane_id() < pool.fin2_w[wbase]) {   // as k_generate splats (fin2: its set)
        const float4 fl = ldnt(&pool.fin2_L[slot]);
        const uint2 fk = ldnt(&pool.fin2_k[slot]);
        const uint32_t pixel = ldnt(&pool.fin2_px[slot]);
        const uint32_t fs = fp.list_xy ? fp.list_s[fk.x] : fk.x;
        const V2 j = sample_jitter(sc, st, fp, pixel & 0xFFFFu, pixel >> 16, fs);
        splat_sample(fp, pool, ld3(fl), fl.w, make_float2(j.x, j.y), fk.x, fk.y);
    }
    if (slot < pool.n && (slot & 63u) == 0) {
        pool.fin_w[slot >> 6] = 0; pool.fin2_w[slot >> 6] = 0; pool.free_w[slot >> 6] = 64;
    }
    if (slot == 0) cnt->drained = 1;
    const uint32_t shard = blockIdx.x % NSHARD;
    __shared__ uint32_t tally[(BLOCK / 64 + 2)*1];
    const bool tp[1] = {live};
    uint32_t* const tc[1] = {&cnt->drain_count[shard][0]};
    uint32_t tpos[1], ttot[1];
    block_tally<BLOCK, 1>(tp, tc, tpos, ttot, tally);
    if (live) pool.sh_slot[(size_t)shard*pool.shard_cap + tpos[0]] = slot;
}

// k_drain — the rest of every live path (see above).  Persistent waves fetch CHUNK slots of
// the list per atomic, like k_trace.  Ray counts as the separate kernels make them: a closest
// ray per continuation, a shadow ray per NEE cast, "traced" for the rays that enter a BVH.
// One wave per block (DTB): a launch that finds the flag unset still has every block dispatched, and a
// ~220-VGPR wave finds room on one SIMD much sooner than a 256-thread block does on four at once beside
// the other partitions' kernels (those empty launches cost up to ~1 ms each in the iterations before
// the drain).
constexpr int DTB = 64;
template <bool LST, bool ENV, bool REF = false>
__global__ void __launch_bounds__(DTB) k_drain(DevScene sc, rt_settings st, FrameParams fp, Pool pool, Counters* cnt,
                                               uint2* spill) {
    if (!cnt->fused || cnt->done) return;                              // uniform
    __shared__ uint2 lds_stack[STACK_LDS*DTB];
    __shared__ float2 lds_bary[DTB];
    Stack stk;
    stk.lds = lds_stack; stk.spill = spill; stk.bary = lds_bary; stk.lane = threadIdx.x; stk.block = DTB;
    stk.gtid = blockIdx.x*DTB + threadIdx.x; stk.nthreads = gridDim.x*DTB;
    __shared__ uint32_t qlen[NSHARD];
    if (threadIdx.x < NSHARD) qlen[threadIdx.x] = cnt->drain_count[threadIdx.x][0];
    __syncthreads();
    uint32_t shard = blockIdx.x % NSHARD, tried = 0;
    const uint32_t lane = __lane_id();
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    uint32_t chunk_next = 0, chunk_end = 0;
    bool exhausted = false, active = false, fresh = false;
    uint32_t n_closest = 0, n_shadow = 0, n_traced = 0, n_traced_sh = 0, n_calls[2] = {0, 0};
    // the lane's path
    uint32_t slot = 0;
    V3 ro = {0, 0, 0}, rd = {0, 0, 0}, thr = {0, 0, 0}, total = {0, 0, 0};
    float prev_pdf = 0.0f, vig = 0.0f;
    uint32_t bounce = 0, is_spec = 0, pixel = 0, key = 0, p = 0;
    int32_t at = 0;
    Rng rng = {0, 0, 0, 0};
    Prologue pro = {};
    StepCounts<LST> tally[2];                       // closest, shadow
    for (;;) {
        // idle lanes take the next live slots
        unsigned long long idle = __ballot(!active);
        while (idle && !exhausted) {
            if (chunk_next >= chunk_end) {
                const int leader = __ffsll((long long)__ballot(true)) - 1;
                bool got = false;
                while (tried < NSHARD) {
                    uint32_t* head = &cnt->drain_fetch[shard][0];
                    const uint32_t len = qlen[shard];
                    uint32_t base = 0xFFFFFFFFu;
                    if (lane == (uint32_t)leader &&
                        __hip_atomic_load(head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < len)
                        base = atomicAdd(head, CHUNK);
                    base = __shfl(base, leader);
                    if (base < len) {
                        chunk_next = shard*pool.shard_cap + base;
                        chunk_end = shard*pool.shard_cap + min(base + CHUNK, len);
                        got = true;
                        break;
                    }
                    shard = (shard + 1) % NSHARD;
                    ++tried;
                }
                if (!got) { exhausted = true; break; }
            }
            const uint32_t avail = chunk_end - chunk_next;
            const uint32_t rank = (uint32_t)__popcll(idle & lt_mask);
            if (!active && rank < avail) {
                slot = pool.sh_slot[chunk_next + rank];
                const float4 o4 = ldnt(&pool.ray_o[slot]), d4 = ldnt(&pool.ray_d[slot]);
                float4 t4 = ldnt(&pool.thr[slot]), L4 = ldnt(&pool.L[slot]);
                const float2 pn2 = ldnt(&pool.prev_n[slot]);
                const uint4 r4 = ldnt(&pool.rng[slot]);
                if (pool.state[slot] == S_NEW) new_path_records(fp, st, d4, t4, L4);
                ro = ld3(o4); rd = ld3(d4); thr = ld3(t4); total = ld3(L4); vig = t4.w;
                prev_pdf = pn2.x; p = __float_as_uint(pn2.y);
                const uint32_t flags = __float_as_uint(L4.w);
                bounce = flags & 0xFFu; is_spec = (flags >> 8) & 1u; at = (int32_t)((flags >> 9) & 0x7Fu);
                pixel = __float_as_uint(o4.w); key = __float_as_uint(d4.w);
                rng = {r4.x, r4.y, r4.z, r4.w};
                active = true;
                fresh = true;
            }
            chunk_next += min((uint32_t)__popcll(idle), avail);
            idle = __ballot(!active);
        }
        if (__ballot(active) == 0ull) break;
        // the closest hit: the ray prologue (the same result k_shade / k_generate stored with the
        // path), then the BVH walk for a ray that meets a mesh
        if (active) pro = ray_prologue(sc, ro, rd, FLT_MAX_, false, 0u);
        // a fresh path's ray is counted already (k_bookkeep: alive / cast, and its queue entry; its
        // prologue's mesh instances by the k_shade / k_generate that made it)
        n_traced += (active && !fresh && pro.bvh) ? 1u : 0u;
        n_calls[0] += (active && !fresh) ? pro.calls : 0u;
        fresh = false;
        Hit h;
        h.t = pro.t; h.code = pro.code; h.tri = 0; h.v = 0.0f; h.w = 0.0f;
        {
            Traversal<false, LST, STACK_LDS, REF> tr;
            bool tracing = active && pro.bvh;
            if (tracing) {
                tr.init_rec(sc, stk, ro, rd, pro.inv_d, pro.t, 0u, pro.mlist);
                tracing = tr.mode != TM_DONE;
            }
            for (int k = 1; __ballot(tracing); ++k) {
                if (tracing && !tr.step(sc, stk)) tracing = false;
                if (k % StepField<LST>::H == 0) tally[0].flush(tr.acc);   // one step per lane per k
            }
            tally[0].flush(tr.acc);
            if (REF) tally[0].flush_ref(tr.rc);
            if (active && pro.bvh && tr.code != RT_HIT_MISS) h = tr.result(stk);
        }
        // one bounce
        bool done = false, cast_shadow = false;
        V3 sh_o = {0, 0, 0}, sh_d = {0, 0, 0}, sh_c = {0, 0, 0};
        float sh_t = 0.0f;
        uint32_t sh_light = 0;
        if (active) {
            const uint32_t canonical = fp.frame_count + (fp.list_xy ? fp.list_s[key] : key);
            const SamplerState ss = {pixel & 0xFFFFu, pixel >> 16, canonical, st.sampling_strategy};
            done = shade_bounce<ENV>(sc, st, ss, pool, slot, h, ro, rd, thr, total, prev_pdf, bounce, is_spec, at, rng,
                                     cast_shadow, sh_o, sh_d, sh_c, sh_t, sh_light);
        }
        // intersect_shadow_ray (:756): the prologue, then the BVH walk; the NEE term is added last
        // in the bounce, as k_trace adds it (:768)
        {
            Prologue spro = {};
            if (cast_shadow) spro = ray_prologue(sc, sh_o, sh_d, sh_t, true, sh_light);
            n_calls[1] += cast_shadow ? spro.calls : 0u;
            Traversal<true, LST, STACK_LDS, REF> tr;
            bool tracing = cast_shadow && !spro.occluded && spro.bvh;
            n_traced_sh += tracing ? 1u : 0u;
            if (tracing) {
                tr.init_rec(sc, stk, sh_o, sh_d, spro.inv_d, sh_t, sh_light, spro.mlist);
                tracing = tr.mode != TM_DONE;
            }
            for (int k = 1; __ballot(tracing); ++k) {
                if (tracing && !tr.step(sc, stk)) tracing = false;
                if (k % StepField<LST>::H == 0) tally[1].flush(tr.acc);   // one step per lane per k
            }
            tally[1].flush(tr.acc);
            if (REF) tally[1].flush_ref(tr.rc);
            if (cast_shadow && !spro.occluded && (!spro.bvh || !tr.occluded)) total = add(total, sh_c);
        }
        n_shadow += cast_shadow ? 1u : 0u;
        if (active && done) {
            const uint32_t s = fp.list_xy ? fp.list_s[key] : key;
            const V2 j = sample_jitter(sc, st, fp, pixel & 0xFFFFu, pixel >> 16, s);
            splat_sample(fp, pool, total, vig, make_float2(j.x, j.y), key, p);
            active = false;
        } else if (active) {
            ++n_closest;                                  // the next bounce's intersect_scene
        }
    }
    // the pool's material stacks were written at the path's slot (shade_bounce); nothing else of
    // the pool is read again.  Counts: one atomic per wave each.
    unsigned long long c[4] = {n_closest, n_shadow, n_traced, n_traced_sh};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (int m = 32; m; m >>= 1) c[k] += __shfl_xor(c[k], m);
    if (lane == 0) {
        if (c[0]) atomicAdd(&cnt->closest_rays, c[0]);
        if (c[1]) atomicAdd(&cnt->shadow_rays, c[1]);
        if (c[2]) atomicAdd(&cnt->traced_rays[0], c[2]);
        if (c[3]) atomicAdd(&cnt->traced_rays[1], c[3]);
    }
    unsigned long long* trav = cnt->trav[blockIdx.x % NSHARD];
    tally[0].commit(trav, 0, true);
    tally[1].commit(trav, 1, true);
    const uint32_t calls0 = __ockl_wfred_add_u32(n_calls[0]), calls1 = __ockl_wfred_add_u32(n_calls[1]);
    if (lane == 0) {
        if (calls0) atomicAdd(&trav[TV_CALLS], (unsigned long long)calls0);
        if (calls1) atomicAdd(&trav[TV_N + TV_CALLS], (unsigned long long)calls1);
    }
}

// k_resolve — splat_filter as a gather (RT/raytracer.cpp:187-259, :476-488).
// Every output pixel sums its neighbours' samples in exactly the order the
// reference's single-threaded renderer splats them: tiles in descending index
// (try_render_next_tile, :555), pixels in raster order inside a tile, samples
// in order (render_tile, :409-422).  The float additions are therefore the
// reference's, bit for bit, and need no atomics.
//
// A thread owns a column strip of RES_RY output pixels.  Every pixel's order is
// the one global order restricted to its (2r+1)^2 window, so the thread walks
// the union of its pixels' windows once in that order and adds each sample
// record to every pixel of the strip whose window holds it: a record is read
// once per strip instead of once per pixel ((RES_RY + 2r)(2r+1) reads for
// RES_RY pixels, 60 instead of 200 at r = 2).  The 64 lanes of a wave own 64
// adjacent columns, so at every step they read 64 adjacent records of one
// sample plane (record = s*P + p): the loads stay coalesced.
// Strip height: 8 rows when the shard owns at least RES_TALL_PIXELS pixels, else 4.  Taller
// strips read fewer records per pixel ((8 + 4)/8 against (4 + 4)/4 source rows) but make half
// as many threads: the full C3 frame resolves in 21.7 ms instead of 24.0 (frame +1.2 %, A/B
// twice), one rank's eighth in 9.8 ms instead of 5.5 (too few waves to cover the latency).
constexpr int RES_RY = 4, RES_RY_TALL = 8;
constexpr uint32_t RES_TALL_PIXELS = 1600000u;   // rt_scene_config::resolve_tall_pixels' default
constexpr int RES_U = 8;               // sample records loaded ahead per thread
constexpr int RES_BX = 64, RES_BY = 4;
template <int RY>
__global__ void __launch_bounds__(RES_BX*RES_BY) k_resolve(FrameParams fp) {
    __shared__ float lut[512];
    for (int i = threadIdx.x; i < 512; i += RES_BX*RES_BY) lut[i] = fp.cache_size ? fp.lut[i] : 0.0f;
    __syncthreads();
    const int X = blockIdx.x*RES_BX + (threadIdx.x % RES_BX);
    const int Y0 = (blockIdx.y*RES_BY + (threadIdx.x / RES_BX))*RY;
    const int W = (int)fp.w, H = (int)fp.h;
    if (X >= W || Y0 >= H) return;
    const int ks = fp.cache_size ? fp.kernel_size : 0;
    const float kscale = ks ? (float)(fp.cache_size - 1) / (float)ks : 0.0f;
    const int TW = (int)fp.tile_w, TH = (int)fp.tile_h;
    const int x0 = max(X - ks, 0), x1 = min(X + ks, W - 1);
    const int y0 = max(Y0 - ks, 0), y1 = min(Y0 + RY - 1 + ks, H - 1);
    float4 acc[RY];
#pragma unroll
    for (int r = 0; r < RY; ++r) acc[r] = (Y0 + r < H) ? fp.accum[(size_t)(Y0 + r)*W + X] : make_float4(0, 0, 0, 0);
    const size_t P = fp.pixels;
    const float dx = (float)(X);
    for (int ty = y1 / TH; ty >= y0 / TH; --ty) {
        for (int tx = x1 / TW; tx >= x0 / TW; --tx) {
            const int tile = ty*(int)fp.tcx + tx;
            const int base = fp.tile_base[tile];
            if (base < 0) continue;
            const int min_x = tx*TW, min_y = ty*TH;
            const int twid = min(W, min_x + TW) - min_x;
            const int ya = max(y0, min_y), yb = min(y1, min_y + TH - 1);
            const int xa = max(x0, min_x), xb = min(x1, min_x + TW - 1);
            for (int y = ya; y <= yb; ++y) {
                // strip pixels whose window holds row y: Y0 + r in [y - ks, y + ks]
                const int rlo = max(y - ks - Y0, 0), rhi = min(y + ks - Y0, RY - 1);
                for (int x = xa; x <= xb; ++x) {
                    const size_t p = (size_t)base + (size_t)(y - min_y)*twid + (size_t)(x - min_x);
                    if (ks) {
                        const float fdx = dx - (float)x;
                        auto splat = [&](const float4 c, const float jy) {
                            const float fx = lut[(int)fabsf(0.5f + kscale*(fdx - c.w))];
#pragma unroll
                            for (int r = 0; r < RY; ++r) {
                                if (r < rlo || r > rhi) continue;
                                const float dy = (float)(Y0 + r - y);
                                const float fy = lut[(int)fabsf(0.5f + kscale*(dy - jy))];
                                const float f = fx*fy;
                                acc[r].x = acc[r].x + f*c.x;
                                acc[r].y = acc[r].y + f*c.y;
                                acc[r].z = acc[r].z + f*c.z;
                                acc[r].w = acc[r].w + f;
                            }
                        };
                        // RES_U records in flight per thread: with few waves (a shard's frame)
                        // one load at a time would expose the full memory latency per sample
                        uint32_t s = 0;
                        for (; s + RES_U <= fp.spp; s += RES_U) {
                            float4 c[RES_U];
                            float jy[RES_U];
#pragma unroll
                            for (int u = 0; u < RES_U; ++u) {
                                const size_t rr = (size_t)(s + u)*P + p;
                                c[u] = fp.samp_rgbx[rr];
                                jy[u] = fp.samp_jy[rr];
                            }
#pragma unroll
                            for (int u = 0; u < RES_U; ++u) splat(c[u], jy[u]);
                        }
                        for (; s < fp.spp; ++s) {
                            const size_t rr = (size_t)s*P + p;
                            splat(fp.samp_rgbx[rr], fp.samp_jy[rr]);
                        }
                    } else {                                   // box filter: the pixel's own samples, (result, 1)
                        const int r = y - Y0;
                        if (r < 0 || r >= RY || x != X) continue;
                        for (uint32_t s = 0; s < fp.spp; ++s) {
                            const float4 c = fp.samp_rgbx[(size_t)s*P + p];
#pragma unroll
                            for (int q = 0; q < RY; ++q)
                                if (q == r) {
                                    acc[q].x = acc[q].x + c.x; acc[q].y = acc[q].y + c.y;
                                    acc[q].z = acc[q].z + c.z; acc[q].w = acc[q].w + 1.0f;
                                }
                        }
                    }
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RY; ++r)
        if (Y0 + r < H) fp.accum[(size_t)(Y0 + r)*W + X] = acc[r];
}

// k_resolve_tiles — splat_filter (RT/raytracer.cpp:187-259, :476-488) as a gather that
// reads every sample record from HBM once (the streaming splat, the default).
//
// A workgroup owns a 64 x 16 block of output pixels; a thread owns a column strip of
// TR_ROWS of them, accumulated in registers.  Per sample pass s of the planned range
// [res_from, res_to) the workgroup stages the records of the block's source region (the
// block plus the filter radius on every side, from the owned tiles only) into LDS with
// one coalesced load each, and every thread sums its strip's (2r+1)^2 windows out of LDS.
//
// Per output pixel the sum runs pass by pass, and inside a pass over the window rows and
// columns in ascending order, from the value the buffer held: deterministic, and the same
// however the passes are split between launches (an f32 load and store in between changes
// nothing).  It is not the reference's order (tiles descending, pixels, then samples,
// k_resolve), so it matches the reference's frame to float rounding, not bit for bit; the
// filter weight is the reference's LUT product fx*fy, accumulated with an FMA.  The box
// filter (cache_size 0) adds (L, 1) to the pixel's own sum in sample order, which IS the
// reference's order.
//
// Partition k resolves its own pass range into its own buffer (the caller's for k = 0),
// so partitions never write the same buffer; k_combine_partials adds them up at the end.
// Each pass's records are loaded at the start of that pass (r03b): 90 VGPRs, and the blocks find
// room beside the other partitions' kernels sooner than with the next pass loading into registers
// while this one is summed (120 VGPRs; C3 +0.2 %, C4 +0.6 %), at the cost of the load latency
// exposed once per pass.
constexpr int TR_W = 64, TR_H = 16, TR_THREADS = 256, TR_ROWS = TR_H / (TR_THREADS / TR_W);
__host__ __device__ constexpr int tr_stage_slots(int ks) { return ((TR_W + 2*ks)*(TR_H + 2*ks) + TR_THREADS - 1) / TR_THREADS; }
__host__ __device__ constexpr size_t tr_lds_bytes(int ks) {
    return (size_t)(TR_W + 2*ks)*(TR_H + 2*ks)*(16 + 4) + 512*4;
}
template <int KSMAX>
__global__ void __launch_bounds__(TR_THREADS) k_resolve_tiles(FrameParams fp, Pool pool, const Counters* cnt,
                                                               const uint32_t* blocks, float4* dst) {
    const uint32_t s0 = cnt->res_from, s1 = cnt->res_to;
    if (s0 >= s1) return;
    constexpr int NST = tr_stage_slots(KSMAX);
    extern __shared__ float4 tr_lds[];
    const int ks = fp.cache_size ? fp.kernel_size : 0;
    const int SW = TR_W + 2*ks, SH = TR_H + 2*ks, N = SW*SH;
    float4* srgb = tr_lds;                                          // [N] r, g, b, jitter_x
    float* sjy = reinterpret_cast<float*>(tr_lds + N);              // [N] jitter_y (NaN: not an owned sample)
    float* lut = sjy + N;                                           // [512]
    const int tid = threadIdx.x;
    const int W = (int)fp.w, H = (int)fp.h;
    const uint32_t blk = blocks[blockIdx.x];
    const int x0 = (int)(blk & 0xFFFFu)*TR_W, y0 = (int)(blk >> 16)*TR_H;
    const int xs0 = x0 - ks, ys0 = y0 - ks;
    for (int i = tid; i < 512; i += TR_THREADS) lut[i] = fp.cache_size ? fp.lut[i] : 0.0f;
    // the tile-list pixel of each staged source pixel (kept in registers for the stage loads)
    int myp[NST];
#pragma unroll
    for (int k = 0; k < NST; ++k) {
        const int i = tid + k*TR_THREADS;
        int pi = -1;
        const int sx = xs0 + i % SW, sy = ys0 + i / SW;
        if (i < N && sx >= 0 && sx < W && sy >= 0 && sy < H) {
            const int tx = sx / (int)fp.tile_w, ty = sy / (int)fp.tile_h;
            const int base = fp.tile_base[ty*(int)fp.tcx + tx];
            if (base >= 0) {
                const int min_x = tx*(int)fp.tile_w, min_y = ty*(int)fp.tile_h;
                const int twid = min(W, min_x + (int)fp.tile_w) - min_x;
                pi = base + (sy - min_y)*twid + (sx - min_x);
            }
        }
        myp[k] = pi;
    }
    const size_t P = fp.pixels;
    float4 pc[NST];
    float pj[NST];
    auto load_pass = [&](uint32_t s) {
        const uint32_t rel = s - pool.rec_pass0;
        const size_t base = (size_t)(rel < pool.rec_ring ? rel : rel % pool.rec_ring)*P;
#pragma unroll
        for (int k = 0; k < NST; ++k) {
            if (myp[k] >= 0) {
                pc[k] = ldnt(&pool.rec_rgbx[base + (size_t)myp[k]]);
                pj[k] = ldnt(&pool.rec_jy[base + (size_t)myp[k]]);
            } else {
                pc[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                pj[k] = __builtin_nanf("");
            }
        }
    };
    // this thread's output strip: column X, rows Y0 .. Y0 + TR_ROWS - 1
    const int X = x0 + tid % TR_W, Y0 = y0 + (tid / TR_W)*TR_ROWS;
    const bool col_in = X < W;
    float4 acc[TR_ROWS];
#pragma unroll
    for (int r = 0; r < TR_ROWS; ++r)
        acc[r] = (col_in && Y0 + r < H) ? dst[(size_t)(Y0 + r)*W + X] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const bool box = !fp.cache_size;
    const float kscale = ks ? (float)(fp.cache_size - 1) / (float)ks : 0.0f;
    const int xa = max(X - ks, 0), xb = min(X + ks, W - 1);
    const int ya = max(Y0 - ks, 0), yb = min(Y0 + TR_ROWS - 1 + ks, H - 1);
    for (uint32_t s = s0; s < s1; ++s) {
        load_pass(s);
        __syncthreads();                                    // the previous pass's sums are done with LDS
#pragma unroll
        for (int k = 0; k < NST; ++k) {
            const int i = tid + k*TR_THREADS;
            if (i < N) { srgb[i] = pc[k]; sjy[i] = pj[k]; }
        }
        __syncthreads();
        if (!col_in) continue;
        for (int sy = ya; sy <= yb; ++sy) {
            const int rlo = max(sy - ks - Y0, 0), rhi = min(sy + ks - Y0, TR_ROWS - 1);
            const int row = (sy - ys0)*SW - xs0;
            for (int sx = xa; sx <= xb; ++sx) {
                const float jy = sjy[row + sx];
                if (jy != jy) continue;                     // not a sample of this shard
                const float4 c = srgb[row + sx];
                if (box) {                                  // (result, 1) into the pixel itself
#pragma unroll
                    for (int r = 0; r < TR_ROWS; ++r)
                        if (r == sy - Y0) {
                            acc[r].x = acc[r].x + c.x; acc[r].y = acc[r].y + c.y;
                            acc[r].z = acc[r].z + c.z; acc[r].w = acc[r].w + 1.0f;
                        }
                    continue;
                }
                const float fx = lut[(int)fabsf(0.5f + kscale*((float)(X - sx) - c.w))];
#pragma unroll
                for (int r = 0; r < TR_ROWS; ++r) {
                    if (r < rlo || r > rhi) continue;
                    const float fy = lut[(int)fabsf(0.5f + kscale*((float)(Y0 + r - sy) - jy))];
                    const float f = fx*fy;
                    acc[r].x = fmaf(f, c.x, acc[r].x);
                    acc[r].y = fmaf(f, c.y, acc[r].y);
                    acc[r].z = fmaf(f, c.z, acc[r].z);
                    acc[r].w = acc[r].w + f;
                }
            }
        }
    }
    if (col_in) {
#pragma unroll
        for (int r = 0; r < TR_ROWS; ++r)
            if (Y0 + r < H) dst[(size_t)(Y0 + r)*W + X] = acc[r];
    }
}

// The partitions' buffers added to the caller's, in partition order (streaming splat).
__global__ void __launch_bounds__(256) k_combine_partials(float4* accum, const float4* const* parts, int nparts, size_t n) {
    for (size_t i = (size_t)blockIdx.x*256 + threadIdx.x; i < n; i += (size_t)gridDim.x*256) {
        float4 a = accum[i];
        for (int k = 0; k < nparts; ++k) {
            const float4 b = ldnt(&parts[k][i]);
            a.x = a.x + b.x; a.y = a.y + b.y; a.z = a.z + b.z; a.w = a.w + b.w;
        }
        accum[i] = a;
    }
}

// k_bookkeep — end of iteration (one workgroup): ray counts, counter roll-over,
// and the exclusive scan of the per-block free counts that gives every block of
// the next k_generate its first sample claim.  Phase BK_FIRST = before the first
// iteration (only the scan); BK_FINAL = after the partition's last iteration (only
// the resolve plan).
//
// Streaming splat: a path claimed by the k_generate of iteration j has made its last
// bounce by the k_shade of iteration j + max(max_bounce_count, 1) - 1 (one bounce per
// iteration), and its sample record is written by the next k_generate.  So once
// iteration i is bookkept, every sample claimed up to iteration i - life is in the
// record ring (life = max(max_bounce_count, 1)): hist[] holds the claim cursor per
// iteration.  With plan.mode set (the host launches k_resolve_tiles right after this
// kernel), the passes complete since the last plan become the next resolve's range
// once there are plan.chunk of them (or all that remain, BK_FINAL), and the claim
// limit moves to keep the ring from overwriting passes not yet resolved.
enum { BK_ITER = 0, BK_FIRST = 1, BK_FINAL = 2 };
// fuse: set Counters::fused once nothing is left to claim and at most this many paths are alive
// (0: never; see k_drain)
// cast0: max_bounce_count > 0, so every sample claimed this iteration casts a camera ray (k_bookkeep counts
// them from the claims; k_generate keeps no counter for them)
// merged: the shadow rays ride in the next iteration's trace launch (TraceMode): the previous k_shade's
// finished paths are splatted one iteration later, and the shadow queue of this iteration is still pending
struct ResPlan { uint32_t mode, P, pass1, ring, chunk, life, fuse, cast0, merged; };
// Two workgroup sizes, picked per frame by the partition's pool (BK_LARGE_POOL): a pool of 4M paths or
// more (a whole 1080p frame: 8.4M) takes the 512-thread build (92 VGPRs: 8 waves that find room beside
// the other partitions' kernels sooner), a smaller one (a rank's share of a multi-GPU frame: 3.3M) the
// 1024-thread build (62 VGPRs, 16 waves on one CU).  A/B (profiles/r03b_ab.txt section 14): 256 threads
// (156 VGPRs) gave the full C3 frame +0.5 to +0.9 % and C4 +1.2 to +1.5 % over 1024, but rank 0 of 8
// -1.9 to -2.8 %; with the 96-VGPR trace kernels 512 threads give C3 +1.5 to +2.2 % over 256 and C4 -0.1 to
// -1.0 % (profiles/r04_bookkeep_ab.txt).
constexpr int BK_THREADS_SMALL = 1024, BK_THREADS_LARGE = 512;
constexpr uint32_t BK_LARGE_POOL = 4u << 20;
// A k_shade block's slots past its survivors: its four waves' free_w in one 16-byte load.
static_assert(BLOCK == 256, "block_free: a k_shade block is four waves");
RT_D uint32_t block_free(const Pool& pool, uint32_t b) {
    const uint4 f = reinterpret_cast<const uint4*>(pool.free_w)[b];
    return f.x + f.y + f.z + f.w;
}
template <int BK_THREADS>
__global__ void __launch_bounds__(BK_THREADS) k_bookkeep(Counters* cnt, Pool pool, uint32_t nblocks, int cur, int phase,
                                                         ResPlan plan) {
    __shared__ uint32_t sc[BK_THREADS];
    __shared__ uint32_t carry;
    const uint32_t t = threadIdx.x;
    if (phase == BK_FINAL) {
        if (t == 0) {
            cnt->res_from = cnt->res_cursor;
            cnt->res_to = plan.pass1;
            cnt->res_cursor = plan.pass1;
        }
        return;
    }
    // The free counts' loads go out first, so they overlap the counter work below.
    // Up to BK_EMAX entries per thread (pools up to 32k blocks, 8.4M paths) are loaded at once into
    // registers, all in flight, and the claims are written from them; a loop covers larger pools.
    constexpr uint32_t BK_EMAX = 32*(1024 / BK_THREADS);
    const uint32_t E = (nblocks + BK_THREADS - 1) / BK_THREADS;
    const uint32_t lo = t*E, hi = min(lo + E, nblocks);
    uint32_t v[BK_EMAX];
    if (E <= BK_EMAX) {
#pragma unroll
        for (uint32_t j = 0; j < BK_EMAX; ++j) v[j] = lo + j < hi ? block_free(pool, lo + j) : 0u;
    }
    __shared__ uint32_t skip;
    if (t < 64) {
        // Lane k < NSHARD reads shard k's counters, all loads in flight, and the sums come from
        // shuffles.  (Thread 0 alone walking the shards, each load ordered behind the previous
        // shard's stores, took ~60 dependent round trips: 27 us alone, ~290 us beside the other
        // partitions' kernels, 10 % of a partition's iteration.)
        const bool it_phase = phase == BK_ITER;
        const uint32_t done_flag = it_phase ? cnt->done : 0u;
        // sq: the shadow queue this iteration's k_trace traced (the previous k_shade's); sp: the one this
        // iteration's k_shade left for the next k_trace
        uint32_t al = 0, c1 = 0, us = 0, eq = 0, sq = 0, sp = 0;
        if (it_phase && t < NSHARD) {
            al = cnt->alive[t][0];
            c1 = cnt->cast[1][t][0];
            us = cnt->unsplat[t][0];
            eq = cnt->ext_count[cur][t][0];
            sq = cnt->shadow_count[plan.merged ? cur ^ 1 : cur][t][0];
            sp = plan.merged ? cnt->shadow_count[cur][t][0] : 0u;
        }
        unsigned long long next = 0, total = 0, lim = 0, start = 0;
        uint32_t gfree = 0, it = 0, rcur = 0, us_prev = 0, drained = 0;
        if (t == 0 && it_phase) {
            next = cnt->next_sample; total = cnt->total_samples; lim = cnt->claim_limit;
            start = cnt->start_sample; gfree = cnt->gen_free; it = cnt->iter; rcur = cnt->res_cursor;
            us_prev = cnt->unsplat_prev; drained = cnt->drained;
        }
        // the claim cursor `life` iterations ago (loaded before any store to the counters)
        const unsigned long long done_cursor =
            (t == 0 && it_phase && plan.mode && it >= plan.life) ? cnt->hist[(it - plan.life) & 127u] : start;
        const bool sk = it_phase && done_flag;
        if (it_phase && !sk && t < NSHARD) {
            cnt->unsplat[t][0] = 0;
            cnt->cast[1][t][0] = 0;
            cnt->alive[t][0] = 0;
            cnt->ext_count[cur][t][0] = 0;
            cnt->shadow_count[plan.merged ? cur ^ 1 : cur][t][0] = 0;
            cnt->fetch[0][t][0] = 0;
            cnt->fetch[1][t][0] = 0;
        }
        uint32_t ext = al, sh = c1, pend = al, ps = us, tq = eq, ts = sq, spn = sp;
#pragma unroll
        for (int off = 1; off < NSHARD; off <<= 1) {
            ext += __shfl_xor(ext, off); sh += __shfl_xor(sh, off); pend += __shfl_xor(pend, off);
            ps += __shfl_xor(ps, off); tq += __shfl_xor(tq, off); ts += __shfl_xor(ts, off);
            spn += __shfl_xor(spn, off);
        }
        if (t == 0) {
            skip = sk;
            if (sk) {
                // done: the passes the bookkeep that found it complete could not plan (an iteration
                // without a resolve after it) are resolved after this one, on the device, instead of
                // waiting for the host's BK_FINAL
                const bool last = plan.mode && rcur < plan.pass1;
                cnt->res_from = last ? rcur : 0u;
                cnt->res_to = last ? plan.pass1 : 0u;
                if (last) cnt->res_cursor = plan.pass1;
            }
            if (it_phase && !sk) {
                const unsigned long long lm = lim < total ? lim : total;
                const unsigned long long rem = lm > next ? lm - next : 0ull;      // remaining_samples()
                const unsigned long long claimed = (unsigned long long)gfree < rem ? (unsigned long long)gfree : rem;
                next += claimed;
                cnt->next_sample = next;
                // the camera rays of this iteration's k_generate: one per claimed sample (every claim below
                // the remaining count becomes a path, k_generate) when max_bounce_count > 0
                cnt->closest_rays += ext + (plan.cast0 ? claimed : 0ull);
                cnt->shadow_rays += sh;
                cnt->traced_rays[0] += tq;
                cnt->traced_rays[1] += ts;
                cnt->pending = pend;
                // still to splat: this iteration's finished paths and the previous one's (the fused drain's
                // k_drain_list splatted those already), and the shadow rays the next k_trace traces for them
                const uint32_t prev = (drained || !plan.merged) ? 0u : us_prev;
                cnt->pending_splat = ps + prev + spn;
                cnt->unsplat_prev = ps;
                // nothing left to claim, trace or splat: every record is in the ring
                const bool complete = next >= total && pend == 0 && ps == 0 && prev == 0 && spn == 0;
                if (complete) cnt->done = 1;
                else if (plan.fuse && next >= total && pend <= plan.fuse) cnt->fused = 1;
                cnt->iter = it + 1;
                cnt->hist[it & 127u] = next;
                if (plan.mode) {
                    const uint32_t done_pass = complete ? plan.pass1 : (uint32_t)(done_cursor / plan.P);
                    const uint32_t from = rcur;
                    cnt->res_from = cnt->res_to = 0;
                    if (done_pass > from && (done_pass - from >= plan.chunk || done_pass >= plan.pass1)) {
                        cnt->res_from = from;
                        cnt->res_to = done_pass;
                        cnt->res_cursor = done_pass;
                        // the ring slots of [from, done_pass) are free once the resolve launched next has run
                        cnt->claim_limit = (unsigned long long)(done_pass + plan.ring)*plan.P;
                    }
                }
            }
            carry = 0;
        }
    }
    __syncthreads();
    if (skip) return;
    // exclusive scan of the free counts: thread t owns the contiguous entries [t*E, t*E + E), sums them,
    // then a wave scan by shuffles and one barrier for the 16 wave totals.
    // (A Hillis-Steele scan over 1024 threads took 20 barriers per 4096 entries: the single
    // workgroup ran 26 us alone and ~200 us beside the other partitions' kernels.)
    uint32_t sum = 0;
    if (E <= BK_EMAX) {
#pragma unroll
        for (uint32_t j = 0; j < BK_EMAX; ++j) sum += v[j];
    } else {
        for (uint32_t i = lo; i < hi; ++i) sum += block_free(pool, i);
    }
    const uint32_t lane = t & 63u, wave = t >> 6;
    uint32_t incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t u = __shfl_up(incl, off);
        if (lane >= (uint32_t)off) incl += u;
    }
    if (lane == 63) sc[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t w = 0; w < wave; ++w) before += sc[w];
    uint32_t run = before + incl - sum;
    if (E <= BK_EMAX) {
#pragma unroll
        for (uint32_t j = 0; j < BK_EMAX; ++j)
            if (lo + j < hi) { pool.claim_base[lo + j] = run; run += v[j]; }
    } else {
        for (uint32_t i = lo; i < hi; ++i) {
            const uint32_t x = block_free(pool, i);
            pool.claim_base[i] = run;
            run += x;
        }
    }
    if (t == BK_THREADS - 1) carry = run;
    __syncthreads();
    if (t == 0) cnt->gen_free = carry;
}

// debug / parity kernel: intersect_scene / intersect_shadow_ray for explicit rays,
// through the same Traversal step machine as k_trace (one ray per thread).
template <bool OCC>
__global__ void __launch_bounds__(128) k_debug_intersect(DevScene sc, const rt_ray_query* rays, rt_hit_record* out,
                                                         uint32_t n, uint2* spill) {
    __shared__ uint2 lds_stack[STACK_LDS*128];
    __shared__ float2 lds_bary[128];
    Stack st;
    st.lds = lds_stack; st.spill = spill; st.bary = lds_bary; st.lane = threadIdx.x; st.block = 128;
    st.gtid = blockIdx.x*128 + threadIdx.x; st.nthreads = gridDim.x*128;
    uint32_t i = blockIdx.x*blockDim.x + threadIdx.x;
    if (i >= n) return;
    rt_ray_query rq = rays[i];
    Traversal<OCC> tr;
    tr.init(sc, st, rv3(rq.o), rv3(rq.d), rq.max_t, rq.ignored_primitive);
    while (tr.mode != TM_DONE && tr.step(sc, st)) {}
    const Hit h = tr.result(st);
    rt_hit_record r;
    memset(&r, 0, sizeof(r));
    r.t = h.t;
    r.primitive = h.code;
    if (!OCC && h.code != RT_HIT_MISS) {
        Ray ray = make_ray(rv3(rq.o), rv3(rq.d), rq.max_t);
        V3 I, N; uint32_t mid;
        hit_geometry(sc, ray, h, I, N, mid);
        r.hit_p = {I.x, I.y, I.z};
        r.n = {N.x, N.y, N.z};
    }
    out[i] = r;
}

// k_post — the output pass (RT/raytracer.cpp:2103-2171): resolve, exposure,
// tonemap, sRGB, contrast, TPDF dither, BGRA8.  One pixel per thread; 16 B in,
// 4 B out (HBM-bound).  The dither texture (196 KB) stays in L2.
RT_D float post_clamp(float n, float a, float b) { return mx(a, mn(b, n)); }     // MathLib clamp
RT_D float sigmoidal_contrast(float x, float contrast, float midpoint) {        // :69-84
    float curve;
    if (x < midpoint) {
        float scale = (1.0f / midpoint)*x;
        curve = midpoint*(scale*scale);
    } else {
        float y = (1.0f / (1.0f - midpoint));
        float scale = y - y*x;
        curve = 1.0f - (1.0f - midpoint)*(scale*scale);
    }
    return lerpf_(x, curve, contrast);
}
RT_D float remap_tpdf(float x) {                                                // :125-132
    float orig = 2.0f*x - 1.0f;
    x = orig*(1.0f / __builtin_sqrtf(fabsf(orig)));   // rsqrtss there; correctly rounded here
    x = mx(-1.0f, x);
    x = x - sign_of(x);
    return x;
}
// rt_debug_verify_rcp: rcp_cr against the IEEE division, 16 inputs per thread.
__global__ void __launch_bounds__(256) k_verify_rcp(uint32_t base, unsigned long long* out) {
    const uint32_t t = blockIdx.x*256 + threadIdx.x, stride = gridDim.x*256;
    for (uint32_t i = 0; i < 16; ++i) {
        const uint32_t bits = base + t + i*stride;
        const float x = __uint_as_float(bits);
        const float a = rcp_cr(x), b = 1.0f / x;
        if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) {
            atomicAdd(out, 1ull);
            atomicMin(out + 1, (unsigned long long)bits);
        }
    }
}

__global__ void __launch_bounds__(256) k_post(const float4* px, uint32_t w, uint32_t h, rt_post_settings post,
                                              const uint8_t* noise, uint32_t* out) {
    const uint32_t x = blockIdx.x*64 + (threadIdx.x & 63), y = blockIdx.y*4 + (threadIdx.x >> 6);
    if (x >= w || y >= h) return;
    const size_t i = (size_t)y*w + x;
    const float4 s = px[i];
    V3 c = {0.0f, 0.0f, 0.0f};
    if ((s.x != s.x) || (s.y != s.y) || (s.z != s.z) || (s.w != s.w)) {
        c = {0.0f, 255.0f, 255.0f};
    } else if (s.w > 0.001f) {
        c = {s.x / s.w, s.y / s.w, s.z / s.w};
        c = {mx(c.x, 0.0f), mx(c.y, 0.0f), mx(c.z, 0.0f)};
        if (post.exposure != 0.0f) c = smul(d_powf(2.0f, post.exposure), c);
        if (post.tonemapping) c = {1.0f - d_expf(-c.x), 1.0f - d_expf(-c.y), 1.0f - d_expf(-c.z)};
        if (post.srgb_transform) {
            const float g = 1.0f / 2.23333f;
            c = {d_powf(c.x, g), d_powf(c.y, g), d_powf(c.z, g)};
        }
        if (post.contrast != 0.0f)
            c = {sigmoidal_contrast(c.x, post.contrast, post.midpoint), sigmoidal_contrast(c.y, post.contrast, post.midpoint),
                 sigmoidal_contrast(c.z, post.contrast, post.midpoint)};
        c = smul(255.0f, c);
        const uint8_t* d = noise + 3*((size_t)(y & 255u)*256 + (x & 255u));
        c.x = c.x + (0.5f + remap_tpdf((1.0f / 255.0f)*(float)d[0]));
        c.y = c.y + (0.5f + remap_tpdf((1.0f / 255.0f)*(float)d[1]));
        c.z = c.z + (0.5f + remap_tpdf((1.0f / 255.0f)*(float)d[2]));
    } else if (s.w < -0.01f) {
        c = {-255.0f*s.w, 0.0f, -255.0f*s.w};
    }
    const uint32_t r = (uint8_t)post_clamp(c.x, 0.0f, 255.0f);
    const uint32_t g = (uint8_t)post_clamp(c.y, 0.0f, 255.0f);
    const uint32_t b = (uint8_t)post_clamp(c.z, 0.0f, 255.0f);
    out[i] = (255u << 24) | (r << 16) | (g << 8) | b;
}

// ======================================================================
// Host side: rt_scene + C ABI
// ======================================================================
// A partition: one independent wavefront loop (its own path pool, queues,
// counters and traversal spill area) on its own stream.  run_frame splits the
// frame's samples between RT_PARTITIONS of them and interleaves their launches,
// so one partition's kernels fill the GPU while another's persistent trace
// kernel drains its last long rays (the per-launch tail).
constexpr int MAX_PARTITIONS = 8;
struct Partition {
    Pool pool = {};
    std::vector<void*> pool_allocs;
    Counters* cnt = nullptr;
    Counters* cnt_host = nullptr;       // pinned, [NIF + 1]: the counters after chunk c land in [c % NIF]; [NIF] stages the frame's initial counters
    hipEvent_t chunk_done[NIF] = {};
    uint2* spill = nullptr;             // traversal stack levels beyond STACK_LDS
    hipStream_t own_stream = nullptr;   // partitions > 0 (partition 0 runs on the caller's stream)
    hipEvent_t join = nullptr;
    hipEvent_t ev[EV_SLOTS * 2 * RT_KERNEL_COUNT] = {};
    hipEvent_t ev_final[2] = {};        // the partition's last k_resolve_tiles (streaming splat)
    bool events = false;
};

struct rt_scene {
    int device = 0;
    DevScene ds = {};
    std::vector<void*> allocs;
    // render-time state (grown on demand)
    Partition part[MAX_PARTITIONS];
    hipEvent_t start_ev = nullptr;
    uint32_t* d_tiles = nullptr;
    uint32_t* d_pixmap = nullptr;   // FrameParams::pix_xy
    size_t pixmap_cap = 0;
    size_t tiles_cap = 0;
    int32_t* d_tile_base = nullptr;
    size_t tile_base_cap = 0;
    uint32_t trace_grid = 0;        // persistent k_trace blocks (extend) for the largest pool (see run_frame)
    bool grid_by_pool = true;       // RT_TRACE_GRID_BY_POOL: a smaller pool's trace launch takes fewer blocks
    uint32_t drain_grid = 0;        // persistent k_drain blocks (<= trace_grid: the spill area)
    uint32_t drain_lanes_full = 0;  // k_drain lanes of a grid that fills the GPU (the fused-drain threshold's unit)
    uint32_t connect_grid = 0;      // the separate shadow launch's blocks (<= trace_grid: the spill area)
    uint32_t shadow_pct = 100;      // the k_trace blocks that also take the shadow queue, in % (RT_SHADOW_PCT)
    // traced shadow rays per traced extension ray in this scene's last frame (-1: none yet): the
    // shadow-launch policy's input (rt_scene_config::shadow_launch, AUTO)
    double shadow_share = -1.0;
    float4* d_samp = nullptr;       // per-sample records for the deterministic splat
    float* d_samp_jy = nullptr;
    size_t samp_cap = 0;
    float* d_lut = nullptr;
    float4* d_partials = nullptr;   // streaming splat: partitions 1.. accumulate here
    size_t partial_cap = 0;
    uint32_t* d_aux = nullptr;      // streaming splat: partial pointers, then k_resolve_tiles' blocks
    size_t aux_cap = 0;
    // The frame layout of the last rt_render_device (owned tiles, pixel map, tile bases, resolve
    // blocks): rebuilt and uploaded only when the frame size, tiling, shard or filter radius changes.
    struct Layout {
        bool valid = false;
        uint32_t w = 0, h = 0, tw = 0, th = 0, si = 0, sc = 0;
        std::vector<uint32_t> ids, prefix;
        uint64_t owned_px = 0;
        std::vector<int32_t> base;
        int blocks_ks = -1;                 // radius the resolve blocks were built for (-1: none)
        uint32_t nblocks = 0;
        const void* aux_partials = nullptr; // d_partials / npx the device pointer table holds
        size_t aux_npx = 0;
        int aux_parts = -1;
    } layout;
    volatile int cancel = 0;
    uint32_t bvh_depth = 0;
    uint32_t bvh_depth_ref = 0;         // stack entries a reference-unit walk (with markers) may hold
    rt_scene_config cfg = {};           // rt_scene_set_config; read at every frame, never the environment
};

namespace {

template <typename T>
int upload(rt_scene* s, const T* host, size_t count, const T** out) {
    *out = nullptr;
    if (!count) return RT_OK;
    void* p = nullptr;
    HIP_OK(hipMalloc(&p, sizeof(T)*count));
    s->allocs.push_back(p);
    HIP_OK(hipMemcpy(p, host, sizeof(T)*count, hipMemcpyHostToDevice));
    *out = static_cast<const T*>(p);
    return RT_OK;
}

// Device traversal layout of a node array: box unchanged, and in place of
// left_first / count / split_axis the node's packed stack record.
std::vector<rt_bvh_node> traversal_layout(const rt_bvh_node* nodes, uint32_t count) {
    std::vector<rt_bvh_node> out(nodes, nodes + count);
    for (uint32_t i = 0; i < count; ++i) {
        const uint32_t rec = pack_node(i, nodes[i].left_first, nodes[i].count, nodes[i].split_axis);
        memcpy(&out[i].left_first, &rec, 4);
        out[i].count = 0;
        out[i].split_axis = 0;
    }
    return out;
}

// The top level for ray_prologue: for each direction octant, the nodes in the
// reference's visit order (children by d_is_negative[split_axis], RT/intersection.cpp:
// 509-517) as {bv_p, bv_r.x}, {bv_r.yz, info, skip}: info = 0x80000000 | count << 24 |
// first for a leaf, 0 for an interior node; skip = the entry after the node's subtree.
// Empty when the top level is too large for the prologue's 6-bit mesh list.
std::vector<float4> top_sequences(const rt_bvh_node* nodes, uint32_t count, uint32_t index_count, uint32_t& len) {
    len = 0;
    if (!count || count > 255 || index_count > 63) return {};
    auto u2f = [](uint32_t u) { float f; memcpy(&f, &u, 4); return f; };
    std::vector<float4> out;
    for (uint32_t oct = 0; oct < 8; ++oct) {
        std::vector<float4> seq;
        bool ok = true;
        auto emit = [&](auto&& self, uint32_t n, uint32_t depth) -> void {
            if (!ok || n >= count || depth > 64) { ok = false; return; }
            const rt_bvh_node& nd = nodes[n];
            const size_t at = seq.size();
            seq.push_back(make_float4(nd.bv_p.x, nd.bv_p.y, nd.bv_p.z, nd.bv_r.x));
            seq.push_back(make_float4(nd.bv_r.y, nd.bv_r.z, 0.0f, 0.0f));
            if (nd.count) {
                if (nd.count > 127 || nd.left_first + nd.count > index_count) { ok = false; return; }
                seq[at + 1].z = u2f(0x80000000u | (nd.count << 24) | nd.left_first);
            } else if (nd.left_first == 0 || nd.left_first + 1 >= count || nd.split_axis > 2) {
                seq[at + 1].z = u2f(0x80000000u);                 // nothing below: an empty leaf
            } else {
                const bool neg = (oct >> nd.split_axis) & 1u;     // right child first when d < 0
                self(self, nd.left_first + (neg ? 1u : 0u), depth + 1);
                self(self, nd.left_first + (neg ? 0u : 1u), depth + 1);
            }
            seq[at + 1].w = u2f((uint32_t)(seq.size() / 2));
        };
        emit(emit, 0u, 0u);
        if (!ok) return {};
        len = (uint32_t)(seq.size() / 2);
        out.insert(out.end(), seq.begin(), seq.end());
    }
    return out;
}

// Mesh BVH4 (see RT_MESH_BVH4): node k for the BVH2 interior node i holds i's
// children, each replaced by its own two children when it is interior.  Interior
// records are global BVH4 indices (`base` + local); leaves keep the BVH2 packed
// record (or its index form, mesh-local).  `need` = an upper bound of the stack
// entries a traversal below this node can hold.  Returns the node's record.
// src (optional): the BVH2 node each BVH4 node was built from, by BVH4 index (mid4's boxes).
// levels: the BVH4 levels below and including this node (a reference-unit walk's markers, need_ref).
uint32_t build_bvh4(const rt_bvh_node* n, uint32_t count, uint32_t i, std::vector<float4>& out,
                    uint32_t& need, bool& ok, std::vector<uint32_t>* src = nullptr, uint32_t* levels = nullptr) {
    const uint32_t k = (uint32_t)(out.size() / 8);
    out.resize(out.size() + 8, make_float4(0, 0, 0, 0));
    if (src) { src->resize(k + 1); (*src)[k] = i; }
    uint32_t slot[4] = {EMPTY4, EMPTY4, EMPTY4, EMPTY4};
    uint32_t meta = n[i].split_axis & 3u;
    auto interior = [&](uint32_t c) { return n[c].count == 0 && n[c].left_first != 0 && n[c].left_first + 1 < count; };
    if (interior(i) || (i == 0 && n[0].count == 0 && n[0].left_first + 1 < count && n[0].left_first != 0)) {
        for (uint32_t g = 0; g < 2; ++g) {
            const uint32_t c = n[i].left_first + g;
            if (interior(c)) {
                slot[2*g] = n[c].left_first; slot[2*g + 1] = n[c].left_first + 1;
                meta |= (n[c].split_axis & 3u) << (2 + 2*g);
            } else {
                slot[2*g] = c;
            }
        }
    }
    float4 q[8];
    for (int j = 0; j < 8; ++j) q[j] = make_float4(0, 0, 0, 0);
    uint32_t nchild = 0, deeper = 0, lv = 0;
    for (int j = 0; j < 4; ++j) {
        uint32_t rec = EMPTY4;
        if (slot[j] != EMPTY4) {
            const uint32_t m = slot[j];
            const rt_bvh_node& c = n[m];
            (&q[0].x)[j] = c.bv_p.x; (&q[1].x)[j] = c.bv_p.y; (&q[2].x)[j] = c.bv_p.z;
            (&q[3].x)[j] = c.bv_r.x; (&q[4].x)[j] = c.bv_r.y; (&q[5].x)[j] = c.bv_r.z;
            ++nchild;
            if (interior(m)) {
                uint32_t cn = 0, cl = 0;
                rec = build_bvh4(n, count, m, out, cn, ok, src, &cl);
                deeper = std::max(deeper, cn);
                lv = std::max(lv, cl);
            } else {
                rec = pack_node(m, c.left_first, c.count, 0);
                if (!(rec & 0x80000000u) && !((rec >> 30) & 1u)) rec = 0x80000000u | m;   // never an interior form
            }
        }
        memcpy(&(&q[6].x)[j], &rec, 4);
    }
    memcpy(&q[7].x, &meta, 4);
    for (int j = 0; j < 8; ++j) out[8*(size_t)k + j] = q[j];
    need = (nchild ? nchild - 1 : 0) + deeper;
    if (levels) *levels = lv + 1;
    if (k >= (1u << 28)) ok = false;
    return k;                       // out holds every mesh's nodes: k is already the global index
}

uint32_t tree_depth(const rt_bvh_node* nodes, uint32_t count) {
    if (!count) return 0;
    uint32_t maxd = 0;
    std::vector<std::pair<uint32_t, uint32_t>> st{{0u, 1u}};
    while (!st.empty()) {
        auto [n, d] = st.back(); st.pop_back();
        maxd = std::max(maxd, d);
        if (n >= count) continue;
        const rt_bvh_node& nd = nodes[n];
        if (!nd.count && !(n == 0 && nd.left_first == 0)) {
            if (nd.left_first + 1 >= count) continue;
            st.push_back({nd.left_first, d + 1});
            st.push_back({nd.left_first + 1, d + 1});
        }
    }
    return maxd;
}

void free_pool(Partition& pt) {
    for (void* p : pt.pool_allocs) (void)hipFree(p);
    pt.pool_allocs.clear();
    pt.pool = Pool{};
}

void free_partition(Partition& pt) {
    free_pool(pt);
    if (pt.cnt) (void)hipFree(pt.cnt);
    if (pt.cnt_host) (void)hipHostFree(pt.cnt_host);
    if (pt.spill) (void)hipFree(pt.spill);
    if (pt.own_stream) (void)hipStreamDestroy(pt.own_stream);
    if (pt.join) (void)hipEventDestroy(pt.join);
    for (auto& e : pt.chunk_done) if (e) (void)hipEventDestroy(e);
    if (pt.events) {
        for (auto& e : pt.ev) (void)hipEventDestroy(e);
        for (auto& e : pt.ev_final) (void)hipEventDestroy(e);
    }
    pt = Partition{};
}

// counters, spill area, stream and events of partition k (allocated on first use)
int ensure_partition(rt_scene* s, int k) {
    Partition& pt = s->part[k];
    if (pt.cnt) return RT_OK;
    HIP_OK(hipMalloc(&pt.cnt, sizeof(Counters)));
    HIP_OK(hipHostMalloc(&pt.cnt_host, (NIF + 1)*sizeof(Counters)));
    for (auto& e : pt.chunk_done) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_OK(hipMalloc(&pt.spill, sizeof(uint2)*(size_t)(STACK_DEPTH - std::min(STACK_LDS, TRACE_STACK_LDS))*s->trace_grid*TB));
    if (k > 0) HIP_OK(hipStreamCreateWithFlags(&pt.own_stream, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&pt.join, hipEventDisableTiming));
    return RT_OK;
}

int ensure_pool(Partition& pt, uint32_t n) {
    if (pt.pool.n >= n) return RT_OK;
    free_pool(pt);
    Pool& p = pt.pool;
    auto alloc = [&](void** ptr, size_t bytes) -> int {
        HIP_OK(hipMalloc(ptr, bytes));
        pt.pool_allocs.push_back(*ptr);
        return RT_OK;
    };
    int e = 0;
    size_t N = n;
    const size_t nblocks = (N + BLOCK - 1) / BLOCK;
    const size_t cap = (nblocks + NSHARD - 1) / NSHARD * BLOCK;   // a block appends <= BLOCK entries per queue
    const size_t Q = cap*NSHARD;
    p.shard_cap = (uint32_t)cap;
    e |= alloc((void**)&p.claim_base, 4*nblocks);
    e |= alloc((void**)&p.fin_w, 4*(N / 64));
    e |= alloc((void**)&p.free_w, 4*(N / 64));
    e |= alloc((void**)&p.fin_L, 16*N);
    e |= alloc((void**)&p.fin_k, 8*N);
    e |= alloc((void**)&p.fin_px, 4*N);
    e |= alloc((void**)&p.fin2_w, 4*(N / 64));
    e |= alloc((void**)&p.fin2_L, 16*N);
    e |= alloc((void**)&p.fin2_k, 8*N);
    e |= alloc((void**)&p.fin2_px, 4*N);
    e |= alloc((void**)&p.nx.ray_o, 16*N);
    e |= alloc((void**)&p.nx.ray_d, 16*N);
    e |= alloc((void**)&p.nx.thr, 16*N);
    e |= alloc((void**)&p.nx.L, 16*N);
    e |= alloc((void**)&p.nx.prev_n, 8*N);
    e |= alloc((void**)&p.nx.rng, 16*N);
    e |= alloc((void**)&p.nx.hit, 16*N);
    e |= alloc((void**)&p.nx.hit_w, 4*N);
    e |= alloc((void**)&p.nx.mstack, 2*64*N);
    e |= alloc((void**)&p.nx.state, N);
    e |= alloc((void**)&p.ray_o, 16*N);
    e |= alloc((void**)&p.ray_d, 16*N);
    e |= alloc((void**)&p.thr, 16*N);
    e |= alloc((void**)&p.L, 16*N);
    e |= alloc((void**)&p.prev_n, 8*N);
    e |= alloc((void**)&p.rng, 16*N);
    e |= alloc((void**)&p.hit, 16*N);
    e |= alloc((void**)&p.hit_w, 4*N);
    e |= alloc((void**)&p.mstack, 2*64*N);
    e |= alloc((void**)&p.ext_rec[0], 16*REC_Q*Q);
    e |= alloc((void**)&p.ext_rec[1], 16*REC_Q*Q);
    e |= alloc((void**)&p.state, N);
    e |= alloc((void**)&p.sh_slot, 4*Q);
    e |= alloc((void**)&p.sh_rec, 16*REC_Q*N);
    e |= alloc((void**)&p.sh_c, 16*N);
    e |= alloc((void**)&p.sh_dst, 4*N);
    if (e) { free_pool(pt); return RT_ERROR_OUT_OF_MEMORY; }
    p.n = n;
    return RT_OK;
}

// The pool as the kernels of an iteration see it: buffer `par` current, the other one PathOut.
Pool pool_view(const Pool& p, int par) {
    if (!par) return p;
    Pool v = p;
    std::swap(v.ray_o, v.nx.ray_o); std::swap(v.ray_d, v.nx.ray_d); std::swap(v.thr, v.nx.thr);
    std::swap(v.L, v.nx.L); std::swap(v.prev_n, v.nx.prev_n);
    std::swap(v.rng, v.nx.rng); std::swap(v.hit, v.nx.hit); std::swap(v.hit_w, v.nx.hit_w);
    std::swap(v.mstack, v.nx.mstack); std::swap(v.state, v.nx.state);
    std::swap(v.fin_L, v.fin2_L); std::swap(v.fin_k, v.fin2_k); std::swap(v.fin_px, v.fin2_px); std::swap(v.fin_w, v.fin2_w);
    return v;
}

int check_inputs(const rt_settings* st, const rt_filter_cache* f) {
    if (!st || !f) { set_error("null settings/filter"); return RT_ERROR_INVALID; }
    if (st->integrator != RT_INTEGRATOR_ADVANCED) { set_error("only the Advanced Pathtracer integrator is on the device path"); return RT_ERROR_INVALID; }
    if (st->max_bounce_count > 63) { set_error("max_bounce_count > 63 overruns the 64-entry material stack"); return RT_ERROR_INVALID; }
    if (st->use_path_guide) { set_error("use_path_guide is dead code in the reference and unsupported"); return RT_ERROR_INVALID; }
    if (st->sampling_strategy < 0 || st->sampling_strategy > 2) { set_error("bad sampling_strategy"); return RT_ERROR_INVALID; }
    if (f->cache_size && (f->kernel_size == 0 || f->kernel_size > 32 || f->cache_size > 256)) { set_error("bad filter cache"); return RT_ERROR_INVALID; }
    return RT_OK;
}

// RT_DEBUG_TIMING=1: host-side timestamps of a frame's setup phases, to stderr.
inline double host_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline bool debug_timing() { static const bool on = getenv("RT_DEBUG_TIMING") != nullptr; return on; }

// Partitions and path pool of a frame of `total` samples (`passes` sample passes over the
// shard's pixels; 0 = an explicit sample list).  A larger pool amortizes each trace
// launch's tail (its slowest ray) over more rays, until the pool is so large that the
// frame is only a few pool fills and the final drain dominates: a fifth of the
// partition's samples, between 2^21 and 4 x 2^21 (~6.5 GB of path state and queues).  r01,
// C3 256 spp on one box: 1M 6552, 2M 8128, 4M 8613 / 8895, 6M 9058, 8M 9054 Mrays/s.
// With the compacted pool (r02) a larger pool costs less: rank 0 of 8 (16.6M samples per
// partition) 1M 53.9, 2M 44.6, 3M 42.7, 4M 43.1 ms; an eighth (2M) became a fifth (3.3M):
// 45.0 -> 43.4 ms (2 pairs), the full frame and rank 0 of 4 unchanged.  With the fused drain the
// full frame gains from 8M paths (6.3M 239.3 / 239.4, 8.4M 236.7 / 237.6, 10.5M 237.7 / 238.8, 12.6M
// 239.8 / 240.3 ms): the upper bound is 4 x 2^21 (rank 0 of 2 at 8.4M: 128.7 -> 128.8 / 129.2, unchanged).
struct FrameShape { int nparts; uint32_t pool_n; };
FrameShape frame_shape(const rt_scene* s, unsigned long long total, uint32_t passes) {
    FrameShape f;
    f.nparts = s->cfg.partitions > 0 ? std::min(MAX_PARTITIONS, (int)s->cfg.partitions) : 4;
    if (passes) f.nparts = std::max(1, std::min<int>(f.nparts, (int)passes));   // partitions own whole passes
    uint32_t pool_n = s->cfg.path_pool > 0 ? (uint32_t)s->cfg.path_pool : g_pool_override;
    if (!pool_n) {
        const unsigned long long want = total / (unsigned long long)f.nparts / 5ull;
        pool_n = (uint32_t)std::min<unsigned long long>(std::max<unsigned long long>(want, 1ull << 21), 4ull << 21);
    }
    // small frames: one partition, pool no larger than the work
    if ((unsigned long long)pool_n*f.nparts > total) f.nparts = 1;
    if ((unsigned long long)pool_n > total) pool_n = (uint32_t)std::max<unsigned long long>(total, 1ull);
    f.pool_n = (pool_n + BLOCK - 1) / BLOCK * BLOCK;
    return f;
}

// How a frame's samples reach the accumulation buffer (rt_set_splat_mode).
struct SplatCfg {
    int mode = RT_SPLAT_ATOMIC;         // rt_splat_mode; ATOMIC also for explicit sample lists
    uint32_t passes = 0;                // the frame's sample passes (of this shard)
    uint32_t pass_lo = 0;               // its first pass (RT_SHARD_PASSES: the shard's range)
    uint32_t ring = 0, chunk = 0;       // STREAM: record-ring passes per partition, passes per resolve
    float4* rec = nullptr;              // STREAM: nparts rings of ring*P; EXACT: spp*P, pass-major
    float* rec_jy = nullptr;
    const uint32_t* blocks = nullptr;   // STREAM: k_resolve_tiles' output blocks
    uint32_t nblocks = 0;
    int ksmax = 2;                      // STREAM: k_resolve_tiles instantiation
    size_t lds = 0;
    float4* partials = nullptr;         // STREAM: partitions 1.. accumulate here (w*h each)
    const float4* const* part_ptrs = nullptr;   // device array of the partials' addresses
};

void launch_resolve_tiles(const SplatCfg& sp, const FrameParams& fp, const Pool& pool, const Counters* cnt,
                          float4* dst, hipStream_t q) {
    switch (sp.ksmax) {
        case 2:  k_resolve_tiles<2><<<sp.nblocks, TR_THREADS, sp.lds, q>>>(fp, pool, cnt, sp.blocks, dst); break;
        case 4:  k_resolve_tiles<4><<<sp.nblocks, TR_THREADS, sp.lds, q>>>(fp, pool, cnt, sp.blocks, dst); break;
        default: k_resolve_tiles<12><<<sp.nblocks, TR_THREADS, sp.lds, q>>>(fp, pool, cnt, sp.blocks, dst); break;
    }
}

// The wavefront driver shared by rt_render_device and rt_trace_samples.
// The frame's samples [0, total) are split into contiguous ranges, one per
// partition (RT_PARTITIONS, default 4; whole sample passes each when the frame is
// rendered); each partition runs generate -> extend -> shade -> connect -> bookkeep
// on its own stream, and the host enqueues the partitions' iterations interleaved.
// Every sample is keyed by its own number (the RNG seed and the record slot), so the
// samples do not depend on the split.  The streaming splat resolves each partition's
// passes into its own buffer while the frame renders (k_resolve_tiles after the
// bookkeep of every chunk's last iteration), and the buffers are added at the end.
int run_frame(rt_scene* s, const rt_settings* st, FrameParams fp, unsigned long long total, hipStream_t stream,
              const SplatCfg& sp, rt_stats* stats, bool shard) {
    auto t0 = std::chrono::steady_clock::now();
    const bool listed = fp.list_xy != nullptr;
    const FrameShape shape = frame_shape(s, total, listed ? 0u : sp.passes);
    const int nparts = shape.nparts;
    const uint32_t pool_n = shape.pool_n;
    // k_bookkeep's workgroup size by the pool (BK_LARGE_POOL, see k_bookkeep)
    const bool bk_large = pool_n >= BK_LARGE_POOL;
    auto launch_bookkeep = [bk_large](Counters* c, const Pool& pl, uint32_t nblocks, int cur, int phase, ResPlan plan,
                                      hipStream_t q) {
        if (bk_large) k_bookkeep<BK_THREADS_LARGE><<<1, BK_THREADS_LARGE, 0, q>>>(c, pl, nblocks, cur, phase, plan);
        else k_bookkeep<BK_THREADS_SMALL><<<1, BK_THREADS_SMALL, 0, q>>>(c, pl, nblocks, cur, phase, plan);
    };
    const bool stream_splat = !listed && sp.mode == RT_SPLAT_STREAM;
    const size_t npx = (size_t)fp.w*fp.h;
    const uint32_t prof = g_profiling & ~(1u << RT_KERNEL_SPLAT);   // the splat runs inside k_generate
    const int diag = s->cfg.debug_traversal ? 1 : 0;
    if (!s->start_ev) HIP_OK(hipEventCreateWithFlags(&s->start_ev, hipEventDisableTiming));
    HIP_OK(hipEventRecord(s->start_ev, stream));
    struct Run { hipStream_t stream; uint32_t grid; uint64_t iters, chunks, consumed; int cur; bool live, drain, near;
                 unsigned long long seen_next; int final_buf;
                 uint64_t chunk_first[NIF]; int chunk_n[NIF]; uint32_t pass0, pass1, ring; float4* dst;
                 bool res_ev[EV_SLOTS]; };
    Run run[MAX_PARTITIONS] = {};
    double kms[RT_KERNEL_COUNT] = {};
    uint64_t klaunch[RT_KERNEL_COUNT] = {};
    const uint32_t life = std::max<uint32_t>(st->max_bounce_count, 1u);
    // live paths at which the drain is fused (k_drain): 2.5 times its grid's lanes, or a tenth of the
    // pool if more (r02 sweeps: rank 0 of 8, 3.3M-path pools: 1x the lanes 40.5 ms, 2.5x 39.3, 4.5x 40.0,
    // 9x 41.0; the full frame's 8.4M-path pools: 2.5x 235.8, 600k 234.1-235.2, 1M 234.2-234.3 ms);
    // rt_scene_config::fuse_paths another count (0 = never)
    const uint32_t fuse_paths = s->cfg.fuse_paths >= 0
        ? (uint32_t)std::min<int64_t>(s->cfg.fuse_paths, 0xFFFFFFFFll)
        : std::max(s->drain_lanes_full*5u/2u, pool_n / 10u);
    for (int k = 0; k < nparts; ++k) {
        int err = ensure_partition(s, k);
        if (!err) err = ensure_pool(s->part[k], pool_n);
        if (err) return err;
        Partition& pt = s->part[k];
        Run& r = run[k];
        r.stream = k ? pt.own_stream : stream;
        if (k) HIP_OK(hipStreamWaitEvent(r.stream, s->start_ev, 0));   // the caller's prior work (buffers, tables)
        const uint32_t N = pt.pool.n;
        r.grid = (N + BLOCK - 1) / BLOCK;
        r.live = true;
        Counters init = {};
        init.claim_limit = ~0ull;
        Pool& pool = pt.pool;
        pool.rec_rgbx = nullptr; pool.rec_jy = nullptr; pool.rec_pass0 = 0; pool.rec_ring = 1;
        if (listed) {
            init.next_sample = total*(unsigned long long)k / nparts;
            init.total_samples = total*(unsigned long long)(k + 1) / nparts;
        } else {
            r.pass0 = sp.pass_lo + (uint32_t)((unsigned long long)sp.passes*k / nparts);
            r.pass1 = sp.pass_lo + (uint32_t)((unsigned long long)sp.passes*(k + 1) / nparts);
            init.next_sample = (unsigned long long)r.pass0*fp.pixels;
            init.total_samples = (unsigned long long)r.pass1*fp.pixels;
            init.res_cursor = r.pass0;
            pool.rec_pass0 = r.pass0;
            if (sp.mode == RT_SPLAT_EXACT) {                   // the global pass-major layout, s*P + p
                pool.rec_rgbx = sp.rec + (size_t)r.pass0*fp.pixels;
                pool.rec_jy = sp.rec_jy + (size_t)r.pass0*fp.pixels;
                pool.rec_ring = std::max(1u, r.pass1 - r.pass0);
            } else if (stream_splat) {
                r.ring = std::min(sp.ring, std::max(1u, r.pass1 - r.pass0));
                pool.rec_rgbx = sp.rec + (size_t)k*sp.ring*fp.pixels;
                pool.rec_jy = sp.rec_jy + (size_t)k*sp.ring*fp.pixels;
                pool.rec_ring = r.ring;
                init.claim_limit = (unsigned long long)(r.pass0 + r.ring)*fp.pixels;
                r.dst = k ? sp.partials + (size_t)(k - 1)*npx : fp.accum;
                if (k) HIP_OK(hipMemsetAsync(r.dst, 0, sizeof(float4)*npx, r.stream));
            }
        }
        init.start_sample = init.next_sample;
        r.seen_next = init.next_sample;
        pt.cnt_host[NIF] = init;         // pinned: the copy is asynchronous (the frame ends before the next write)
        HIP_OK(hipMemcpyAsync(pt.cnt, pt.cnt_host + NIF, sizeof(Counters), hipMemcpyHostToDevice, r.stream));
        HIP_OK(hipMemsetAsync(pt.pool.state, S_FREE, N, r.stream));
        HIP_OK(hipMemsetAsync(pt.pool.fin_w, 0, 4ull*N / 64, r.stream));
        HIP_OK(hipMemsetAsync(pt.pool.fin2_w, 0, 4ull*N / 64, r.stream));
        HIP_OK(hipMemsetD32Async((hipDeviceptr_t)pt.pool.free_w, 64, N / 64, r.stream));
        launch_bookkeep(pt.cnt, pt.pool, r.grid, 0, BK_FIRST, ResPlan{}, r.stream);
        if (prof && !pt.events) {
            for (auto& e : pt.ev) HIP_OK(hipEventCreate(&e));
            for (auto& e : pt.ev_final) HIP_OK(hipEventCreate(&e));
            pt.events = true;
        }
    }
    // How the shadow rays are traced (rt_scene_config::shadow_launch).  Merged: in the next iteration's trace
    // launch, after its extension rays (one launch and one tail less per iteration; the finished paths are
    // splatted an iteration later).  Separate: a trace launch of their own after k_shade (r05's schedule).
    // Auto: merged for a rank's share of a multi-GPU frame and for small pools (under BK_LARGE_POOL), where
    // an iteration is short and its launches' tails weigh most; for a whole frame on one GPU, merged when
    // the scene's last frame traced at least SHADOW_SHARE_MERGED shadow rays per extension ray, else
    // separate (a scene's first frame: separate).  A/B (profiles/r06_shadow_launch_ab.txt,
    // r06_merged_whole_ab.txt), merged against separate: rank 0's C3 share of 8 32.8-33.0 ms against 34.1,
    // of 4 61.7-61.9 against 62.7, of 2 116.4-117.0 against 117.9-119.1; whole frames after the batched
    // prologue: C3 (0.26 shadow rays per extension ray) +0.7..+2.2 %, C2 (the same scene) +0.7..+2.3 %, C4
    // (0.11) -1.1..-3.0 %.
    constexpr double SHADOW_SHARE_MERGED = 0.15;
    // The trace launch's grid: the scene's (RT_TRACE_GRID_PCT of one full-occupancy wave of blocks) is sized for
    // a whole 1080p frame's pools; a small pool (under BK_LARGE_POOL: a rank's eighth of a multi-GPU frame,
    // 3.3M paths) queues fewer rays per launch and takes half of it, so the other partitions' kernels find the
    // rest of the GPU sooner.  Rank 0's C3 share of 8 (profiles/r06_grid_by_pool_ab.txt): 50 % of a wave
    // instead of 75 % +1.4..+3.3 %; then 37 % +0.4..+1.7 % and 31 % +0.1..+1.2 % over 50 %, 25 % -1.1..-2.0 %;
    // a grid by sqrt(pool / 8.4M) also gave a share of 4 (6.6M paths, 67 %) -0.6..0 %.
    const uint32_t tgrid = (s->grid_by_pool && pool_n < BK_LARGE_POOL) ? std::max(1u, s->trace_grid/2u) : s->trace_grid;
    const bool merged = s->cfg.shadow_launch == RT_SHADOW_LAUNCH_MERGED ||
                        (s->cfg.shadow_launch == RT_SHADOW_LAUNCH_AUTO &&
                         (shard || pool_n < BK_LARGE_POOL || s->shadow_share >= SHADOW_SHARE_MERGED));
    auto plan_of = [&](int k, uint32_t mode) {
        const Run& r = run[k];
        // merged: a path's record is written two iterations after its last bounce (its shadow ray rides in the
        // next k_trace, the k_generate after that splats it): life + 1
        return ResPlan{mode, fp.pixels, r.pass1, r.ring, sp.chunk, merged ? life + 1 : life, fuse_paths,
                       st->max_bounce_count > 0 ? 1u : 0u, merged ? 1u : 0u};
    };
    // Stage timing without extra host syncs: each iteration records begin/end
    // events into one of EV_SLOTS ring slots; a chunk's slots are read back when
    // the host has waited for that chunk anyway.
    auto ev = [&](int k, int slot, int kern, int end) -> hipEvent_t& {
        return s->part[k].ev[(slot*RT_KERNEL_COUNT + kern)*2 + end];
    };
    auto harvest = [&](int k, int b) {
        Run& r = run[k];
        if (!prof) return;
        for (int i = 0; i < r.chunk_n[b]; ++i) {
            const int slot = (int)((r.chunk_first[b] + i) % EV_SLOTS);
            for (int kern = 0; kern < RT_KERNEL_COUNT; ++kern) {
                // (the splat runs inside k_generate; merged, the shadow rays inside k_trace: no events of their own)
                if (!((prof >> kern) & 1u) || kern == RT_KERNEL_SPLAT || (merged && kern == RT_KERNEL_CONNECT)) continue;
                if (kern == RT_KERNEL_RESOLVE && !r.res_ev[slot]) continue;
                float ms = 0.0f;
                if (hipEventElapsedTime(&ms, ev(k, slot, kern, 0), ev(k, slot, kern, 1)) == hipSuccess) {
                    kms[kern] += ms; klaunch[kern] += 1;
                }
            }
        }
    };
    // environment-map NEE (rt_set_env_sampling): only with a map, its table and NEE
    // rt_scene_config::traversal_ref: the trace kernels walk the top level in the reference's order (no
    // prologue sequence: the prologue tests the planes and the root only) and count the reference's units
    const bool ref = s->cfg.traversal_ref > 0;
    DevScene ds = s->ds;
    if (ref) { ds.top_seq = nullptr; ds.top_seq_len = 0; ds.listed_only = 0; }
    const bool env = (s->cfg.env_sampling >= 0 ? s->cfg.env_sampling : g_env_sampling) && s->ds.env_tab &&
                     st->next_event_estimation;
    auto iterate = [&](int k, bool plan) {
        Partition& pt = s->part[k];
        Run& r = run[k];
        const hipStream_t q = r.stream;
        const int slot = (int)(r.iters % EV_SLOTS);
        auto b = [&](int kern) { if ((prof >> kern) & 1u) (void)hipEventRecord(ev(k, slot, kern, 0), q); };
        auto e = [&](int kern) { if ((prof >> kern) & 1u) (void)hipEventRecord(ev(k, slot, kern, 1), q); };
        const Pool pv = pool_view(pt.pool, r.cur);        // the path buffers swap every iteration
        // separate shadow launch: k_generate splats the previous k_shade's finished set (the view's fin2)
        Pool pg = pv;
        if (!merged) {
            std::swap(pg.fin_L, pg.fin2_L); std::swap(pg.fin_k, pg.fin2_k);
            std::swap(pg.fin_px, pg.fin2_px); std::swap(pg.fin_w, pg.fin2_w);
        }
        const int sparse = r.drain ? 1 : 0;
        // near the drain every iteration carries the fused-drain kernels; they run only in the
        // iteration after k_bookkeep set Counters::fused, whose extend / shade / connect then exit
        // (rt_scene_config::drain_every > 1: only every Nth iteration, a test of cadence independence)
        const uint32_t every = s->cfg.drain_every > 0 ? (uint32_t)s->cfg.drain_every : 1u;
        const int fuse = (r.near && fuse_paths && r.iters % every == every - 1) ? 1 : 0;
        b(RT_KERNEL_GENERATE);
        k_generate<<<r.grid, BLOCK, 0, q>>>(ds, *st, fp, pg, pt.cnt, r.cur);
        e(RT_KERNEL_GENERATE); b(RT_KERNEL_EXTEND);
        // the trace launch: this iteration's extension rays (merged: then the previous k_shade's shadow rays)
        auto trace = [&](auto ph, const Pool& tp, int tcur, uint32_t grid) {
            constexpr int PH = decltype(ph)::value;
            const uint32_t shp = s->shadow_pct;
            if (ds.listed_only) k_trace<true, false, PH><<<grid, TB, TRACE_LDS, q>>>(ds, tp, pt.cnt, tcur, pt.spill, fuse, shp);
            else if (ref) k_trace<false, true, PH><<<grid, TB, TRACE_LDS, q>>>(ds, tp, pt.cnt, tcur, pt.spill, fuse, shp);
            else k_trace<false, false, PH><<<grid, TB, TRACE_LDS, q>>>(ds, tp, pt.cnt, tcur, pt.spill, fuse, shp);
        };
        if (merged) trace(std::integral_constant<int, 3>{}, pv, r.cur, tgrid);
        else trace(std::integral_constant<int, 1>{}, pv, r.cur, tgrid);
        e(RT_KERNEL_EXTEND);
        if (fuse) {                      // the fused drain, after the shadow rays of the last k_shade are in
            k_drain_list<<<r.grid, BLOCK, 0, q>>>(ds, *st, fp, pv, pt.cnt, merged ? 1 : 0);
            if (ds.listed_only) {
                if (env) k_drain<true, true><<<s->drain_grid, DTB, 0, q>>>(ds, *st, fp, pv, pt.cnt, pt.spill);
                else k_drain<true, false><<<s->drain_grid, DTB, 0, q>>>(ds, *st, fp, pv, pt.cnt, pt.spill);
            } else if (ref) {
                if (env) k_drain<false, true, true><<<s->drain_grid, DTB, 0, q>>>(ds, *st, fp, pv, pt.cnt, pt.spill);
                else k_drain<false, false, true><<<s->drain_grid, DTB, 0, q>>>(ds, *st, fp, pv, pt.cnt, pt.spill);
            } else {
                if (env) k_drain<false, true><<<s->drain_grid, DTB, 0, q>>>(ds, *st, fp, pv, pt.cnt, pt.spill);
                else k_drain<false, false><<<s->drain_grid, DTB, 0, q>>>(ds, *st, fp, pv, pt.cnt, pt.spill);
            }
        }
        b(RT_KERNEL_SHADE);
        if (env) {
            if (ds.blob_q) k_shade<true, true><<<r.grid, BLOCK, 16*ds.blob_q, q>>>(ds, *st, fp, pv, pt.cnt, r.cur, sparse, fuse);
            else k_shade<false, true><<<r.grid, BLOCK, 0, q>>>(ds, *st, fp, pv, pt.cnt, r.cur, sparse, fuse);
        } else if (ds.blob_q) {
            k_shade<true, false><<<r.grid, BLOCK, 16*ds.blob_q, q>>>(ds, *st, fp, pv, pt.cnt, r.cur, sparse, fuse);
        } else {
            k_shade<false, false><<<r.grid, BLOCK, 0, q>>>(ds, *st, fp, pv, pt.cnt, r.cur, sparse, fuse);
        }
        e(RT_KERNEL_SHADE);
        if (!merged) {
            // separate: this k_shade's shadow rays now; their NEE terms go to the survivors in the other
            // buffer and to this iteration's finished set, and the queue is the one of this parity
            Pool pc = pv;
            pc.L = pv.nx.L;
            pc.fin2_L = pv.fin_L;
            b(RT_KERNEL_CONNECT);
            trace(std::integral_constant<int, 2>{}, pc, r.cur ^ 1, s->connect_grid);
            e(RT_KERNEL_CONNECT);
        }
        // in the drain every iteration plans a resolve: the one after the bookkeep that finds the
        // partition complete resolves its last passes at once, without waiting for the host
        const bool res = stream_splat && (plan || r.drain);
        launch_bookkeep(pt.cnt, pv, r.grid, r.cur, BK_ITER, plan_of(k, res ? 1u : 0u), q);
        r.res_ev[slot] = res && ((prof >> RT_KERNEL_RESOLVE) & 1u);
        if (res) {                       // the passes the bookkeep found complete, if enough of them
            b(RT_KERNEL_RESOLVE);
            launch_resolve_tiles(sp, fp, pv, pt.cnt, r.dst, q);
            e(RT_KERNEL_RESOLVE);
        }
        ++r.iters;
        r.cur ^= 1;
    };
    // A chunk: 4 iterations (1 in a partition's first 3 chunks), then the counters into
    // the pinned buffer of the chunk's parity and an event.  Every live partition keeps
    // NIF = two chunks in flight, so while the host reads one chunk's counters the next one
    // already runs and the partitions never drain between host checks.
    auto enqueue_chunk = [&](int k) -> int {
        Partition& pt = s->part[k];
        Run& r = run[k];
        const int b = (int)(r.chunks % NIF);
        r.chunk_first[b] = r.iters;
        r.chunk_n[b] = r.chunks < 3 ? 1 : 4;
        for (int i = 0; i < r.chunk_n[b]; ++i) iterate(k, i == r.chunk_n[b] - 1);
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpyAsync(pt.cnt_host + b, pt.cnt, sizeof(Counters), hipMemcpyDeviceToHost, r.stream));
        HIP_OK(hipEventRecord(pt.chunk_done[b], r.stream));
        ++r.chunks;
        return RT_OK;
    };
    // A partition whose samples are all splatted resolves whatever passes are left.
    auto finish = [&](int k) -> int {
        if (!stream_splat) return RT_OK;
        Partition& pt = s->part[k];
        Run& r = run[k];
        launch_bookkeep(pt.cnt, pt.pool, r.grid, r.cur, BK_FINAL, plan_of(k, 2u), r.stream);
        const bool t = (prof >> RT_KERNEL_RESOLVE) & 1u;
        if (t) HIP_OK(hipEventRecord(pt.ev_final[0], r.stream));
        launch_resolve_tiles(sp, fp, pt.pool, pt.cnt, r.dst, r.stream);
        if (t) HIP_OK(hipEventRecord(pt.ev_final[1], r.stream));
        HIP_OK(hipGetLastError());
        return RT_OK;
    };
    s->cancel = 0;
    const double t_setup = debug_timing() ? host_ms() : 0.0;
    for (int c = 0; c < NIF; ++c)
        for (int k = 0; k < nparts; ++k) {
            int err = enqueue_chunk(k);
            if (err) return err;
        }
    if (debug_timing())
        fprintf(stderr, "[rt timing] run_frame: partitions set up %.3f ms, first chunks enqueued %.3f ms\n",
                t_setup - std::chrono::duration<double, std::milli>(t0.time_since_epoch()).count(), host_ms() - t_setup);
    uint64_t rounds = 0;
    std::string host_log;                        // RT_DEBUG_TIMING: the host's waits and enqueues
    for (int live = nparts; live > 0; ++rounds) {
        for (int k = 0; k < nparts; ++k) {
            Run& r = run[k];
            if (!r.live) continue;
            const int b = (int)(r.consumed % NIF);
            const double tw0 = debug_timing() ? host_ms() : 0.0;
            HIP_OK(hipEventSynchronize(s->part[k].chunk_done[b]));
            if (debug_timing()) {
                char buf[96];
                snprintf(buf, sizeof buf, " p%d:c%llu@%.3f+%.3f", k, (unsigned long long)r.consumed,
                         tw0 - t_setup, host_ms() - tw0);
                host_log += buf;
            }
            harvest(k, b);
            ++r.consumed;
            const Counters& c = s->part[k].cnt_host[b];
            if (c.next_sample >= c.total_samples) r.drain = true;     // the chunks enqueued from now on
            // the claims of a few more chunks reach the end: from now on the iterations carry the
            // fused-drain kernels (two chunks are in flight when the host sees a chunk's counters)
            if (c.next_sample + NIF*(c.next_sample - r.seen_next) >= c.total_samples) r.near = true;
            r.seen_next = c.next_sample;
            if (c.next_sample >= c.total_samples && c.pending == 0 && c.pending_splat == 0) {
                r.live = false; r.final_buf = b; --live;       // its chunk still in flight finds nothing to do
                int err = finish(k);
                if (err) return err;
            } else {
                int err = enqueue_chunk(k);
                if (err) return err;
            }
        }
        if (debug_timing()) {
            char buf[48];
            snprintf(buf, sizeof buf, " |%.3f\n", host_ms() - t_setup);
            host_log += buf;
        }
        if (s->cancel || rounds > 1000000) {
            // Every partition may still have two chunks in flight that write the pool, the sample
            // records or (atomic splat) the caller's accumulation buffer: wait for them before the
            // error returns, so the caller may reuse its memory at once.
            for (int k = 0; k < nparts; ++k) (void)hipStreamSynchronize(run[k].stream);
            if (s->cancel) { set_error("render cancelled"); return RT_ERROR_CANCELLED; }
            set_error("wavefront loop did not converge");
            return RT_ERROR_DEVICE;
        }
    }
    if (debug_timing()) fprintf(stderr, "[rt timing] host rounds (partition:chunk@wait start+wait ms | round end):\n%s", host_log.c_str());
    for (int k = 1; k < nparts; ++k) {                     // the caller's stream continues after every partition
        HIP_OK(hipEventRecord(s->part[k].join, run[k].stream));
        HIP_OK(hipStreamWaitEvent(stream, s->part[k].join, 0));
    }
    if (stream_splat && nparts > 1) {
        k_combine_partials<<<(uint32_t)std::min<size_t>((npx + 255) / 256, 8192), 256, 0, stream>>>(
            fp.accum, sp.part_ptrs, nparts - 1, npx);
        HIP_OK(hipGetLastError());
    }
    if (stream_splat && ((prof >> RT_KERNEL_RESOLVE) & 1u)) {
        HIP_OK(hipStreamSynchronize(stream));
        for (int k = 0; k < nparts; ++k) {
            float ms = 0.0f;
            if (hipEventElapsedTime(&ms, s->part[k].ev_final[0], s->part[k].ev_final[1]) == hipSuccess) {
                kms[RT_KERNEL_RESOLVE] += ms; klaunch[RT_KERNEL_RESOLVE] += 1;
            }
        }
    }
    Counters sum = {};
    unsigned long long tv[2*TV_N] = {};
    uint64_t iters = 0;
    for (int k = 0; k < nparts; ++k) {
        const Counters& c = s->part[k].cnt_host[run[k].final_buf];
        sum.closest_rays += c.closest_rays;
        sum.shadow_rays += c.shadow_rays;
        sum.traced_rays[0] += c.traced_rays[0];
        sum.traced_rays[1] += c.traced_rays[1];
        for (int sh = 0; sh < NSHARD; ++sh)
            for (int i = 0; i < 2*TV_N; ++i) tv[i] += c.trav[sh][i];
        iters = std::max(iters, run[k].iters);
    }
    if (sum.traced_rays[0]) s->shadow_share = (double)sum.traced_rays[1] / (double)sum.traced_rays[0];
    // TraversalStats per kind (rt_stats::traversal, rt_abi.h)
    rt_traversal_stats ts[2] = {};
    uint64_t steps[2] = {};
    for (int a = 0; a < 2; ++a) {
        const unsigned long long* v = tv + a*TV_N;
        // the prologue's walk reaches the instances (ray_prologue); a scene whose top level is too large
        // for the prologue has it walked by the trace kernels, whose entries are then the calls
        ts[a].mesh_intersection_count = (s->ds.top_seq && !ref) ? v[TV_CALLS] : v[TV_ENTRIES];
        ts[a].mesh_bvh_traversals = v[TV_ENTRIES] + v[TV_NODES] + v[TV_TRIS];
        ts[a].mesh_node_traversals = v[TV_NODES];
        ts[a].mesh_leaf_traversals = v[TV_LEAVES];
        steps[a] = ts[a].mesh_bvh_traversals + v[TV_TOP] - v[TV_DRAIN];   // the extend / connect launches'
    }
    if (diag)                                       // rt_scene_config::debug_traversal
        for (int a = 0; a < 2; ++a)
            fprintf(stderr, "[rt] %s queries: %llu mesh instances reached, %llu entered, %llu mesh steps (%llu BVH4 "
                    "nodes, %llu leaves entered), %llu trace steps\n", a ? "shadow" : "closest",
                    (unsigned long long)ts[a].mesh_intersection_count, tv[a*TV_N + TV_ENTRIES],
                    (unsigned long long)ts[a].mesh_bvh_traversals,
                    (unsigned long long)ts[a].mesh_node_traversals, (unsigned long long)ts[a].mesh_leaf_traversals,
                    (unsigned long long)steps[a]);
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->closest_hit_rays = sum.closest_rays;
        stats->shadow_rays = sum.shadow_rays;
        stats->samples = total;
        stats->iterations = iters;
        stats->shadow_launch = merged ? RT_SHADOW_LAUNCH_MERGED : RT_SHADOW_LAUNCH_SEPARATE;
        stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (int k = 0; k < RT_KERNEL_COUNT; ++k) { stats->kernel_ms[k] = kms[k]; stats->kernel_launches[k] = klaunch[k]; }
        stats->traced_rays[0] = sum.traced_rays[0];
        stats->traced_rays[1] = sum.traced_rays[1];
        for (int a = 0; a < 2; ++a) {
            stats->traversal[a] = ts[a];
            stats->trace_steps[a] = steps[a];
            if (ref) {                                  // the reference's units (rt_scene_config::traversal_ref)
                const unsigned long long* v = tv + a*TV_N;
                stats->traversal_ref[a].mesh_intersection_count = v[TV_ENTRIES];
                stats->traversal_ref[a].mesh_bvh_traversals = v[TV_REF_TRAV];
                stats->traversal_ref[a].mesh_node_traversals = v[TV_REF_NODE];
                stats->traversal_ref[a].mesh_leaf_traversals = v[TV_REF_LEAF];
            }
        }
    }
    return RT_OK;
}

// FrameParams' multiply-high divisors (div16, div_pixels); tile sides and pixels are non-zero
void set_divisors(FrameParams& fp) {
    fp.tw_m = ((1ull << 32) + fp.tile_w - 1) / fp.tile_w;
    fp.th_m = ((1ull << 32) + fp.tile_h - 1) / fp.tile_h;
    // ceil(2^64 / P) = floor((2^64 - 1) / P) + 1 for P > 1; 2^64 does not fit, so P <= 1 keeps m = 0 and
    // k_generate divides
    fp.px_m = fp.pixels > 1 ? (~0ull / fp.pixels) + 1ull : 0ull;
}

void fill_camera(FrameParams& fp, const rt_camera* c) {
    fp.cp = rv3(c->p); fp.cx = rv3(c->x); fp.cy = rv3(c->y); fp.cz = rv3(c->z);
    fp.focus_distance = c->focus_distance;
    fp.lens_radius = c->lens_radius;
    fp.half_film_w = c->half_film_w;
    fp.half_film_h = c->half_film_h;
    fp.film_distance = c->film_distance;
}

int bind_device(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        set_error("no HIP device visible: the MI355X path has no CPU fallback");
        return RT_ERROR_NO_DEVICE;
    }
    if (device < 0 || device >= count) { set_error("device index out of range"); return RT_ERROR_INVALID; }
    HIP_OK(hipSetDevice(device));
    return RT_OK;
}

// The environment-map sampling table (rt_set_env_sampling, env_direction).  Tiles are
// load_environment_map's grid (RT/assets.cpp:620-665): tile_w = w / 32, tile_h = h / 32,
// row-major, a tile's luma (0.299 r + 0.587 g + 0.114 b, RT/common.h:142-145) summed in texel
// order.  A tile is drawn with probability luma / total through an alias table (Vose's
// method); its density over the unit (u, v) square is that probability x texels / tile texels.
// No table (false) for maps under 32 x 32 texels, negative luma or no light at all.
bool build_env_table(uint32_t w, uint32_t h, const rt_v3* px, std::vector<float4>& tab,
                     uint32_t& tx, uint32_t& tw, uint32_t& th) {
    if (!px || w < 32 || h < 32) return false;
    tw = w / 32; th = h / 32;
    tx = (w + tw - 1) / tw;
    const uint32_t ty = (h + th - 1) / th, n = tx*ty;
    std::vector<float> lum(n), scaled(n), prob(n, 1.0f);
    std::vector<uint32_t> alias(n);
    float sum = 0.0f;
    for (uint32_t t = 0; t < n; ++t) {
        const uint32_t x0 = (t % tx)*tw, y0 = (t / tx)*th;
        const uint32_t x1 = std::min(x0 + tw, w), y1 = std::min(y0 + th, h);
        float cur = 0.0f;
        for (uint32_t y = y0; y < y1; ++y)
            for (uint32_t x = x0; x < x1; ++x) {
                const rt_v3& c = px[(size_t)y*w + x];
                cur += 0.299f*c.x + 0.587f*c.y + 0.114f*c.z;
            }
        if (!(cur >= 0.0f)) return false;
        lum[t] = cur;
        sum += cur;
    }
    if (!(sum > 0.0f) || !std::isfinite(sum)) return false;
    const float rcp = 1.0f / sum;
    tab.assign(n, make_float4(0, 0, 0, 0));
    std::vector<uint32_t> small, large;
    for (uint32_t t = 0; t < n; ++t) {
        const uint32_t x0 = (t % tx)*tw, y0 = (t / tx)*th;
        const uint32_t cw = std::min(x0 + tw, w) - x0, ch = std::min(y0 + th, h) - y0;
        const float p = lum[t]*rcp;
        tab[t].z = p*((float)((uint64_t)w*h) / (float)(cw*ch));
        scaled[t] = p*(float)n;
        alias[t] = t;
        (scaled[t] < 1.0f ? small : large).push_back(t);
    }
    while (!small.empty() && !large.empty()) {
        const uint32_t l = small.back(), g = large.back();
        small.pop_back(); large.pop_back();
        prob[l] = scaled[l];
        alias[l] = g;
        scaled[g] = (scaled[g] + scaled[l]) - 1.0f;
        (scaled[g] < 1.0f ? small : large).push_back(g);
    }
    for (uint32_t t = 0; t < n; ++t) {
        tab[t].x = prob[t];
        uint32_t a = alias[t];
        memcpy(&tab[t].y, &a, 4);
    }
    return true;
}

rt_scene_config default_config() {
    rt_scene_config c;
    memset(&c, 0, sizeof(c));
    c.splat_mode = RT_CONFIG_INHERIT;
    c.shard_mode = RT_CONFIG_INHERIT;
    c.env_sampling = RT_CONFIG_INHERIT;
    c.fuse_paths = -1;
    c.sample_budget_gb = -1.0;
    return c;
}

int check_config(const rt_scene_config* c) {
    const char* bad = nullptr;
    if (c->splat_mode != RT_CONFIG_INHERIT && (c->splat_mode < RT_SPLAT_STREAM || c->splat_mode > RT_SPLAT_ATOMIC)) bad = "splat_mode";
    else if (c->shard_mode != RT_CONFIG_INHERIT && c->shard_mode != RT_SHARD_TILES && c->shard_mode != RT_SHARD_PASSES) bad = "shard_mode";
    else if (c->env_sampling != RT_CONFIG_INHERIT && c->env_sampling != 0 && c->env_sampling != 1) bad = "env_sampling";
    else if (c->partitions < 0 || c->partitions > MAX_PARTITIONS) bad = "partitions (0..8)";
    else if (c->path_pool < 0 || c->path_pool > (1ll << 30)) bad = "path_pool (0..2^30)";
    else if (c->fuse_paths < -1) bad = "fuse_paths";
    else if (c->splat_chunk < 0 || c->splat_ring < 0) bad = "splat_chunk / splat_ring";
    else if (!(c->sample_budget_gb == c->sample_budget_gb)) bad = "sample_budget_gb";
    else if (c->resolve_tall_pixels < 0) bad = "resolve_tall_pixels";
    else if (c->traversal_ref != 0 && c->traversal_ref != 1) bad = "traversal_ref";
    else if (c->drain_every < 0 || c->drain_every > 1024) bad = "drain_every (0..1024)";
    else if (c->shadow_launch < RT_SHADOW_LAUNCH_AUTO || c->shadow_launch > RT_SHADOW_LAUNCH_MERGED) bad = "shadow_launch";
    if (bad) { set_error(std::string("rt_scene_config: bad ") + bad); return RT_ERROR_INVALID; }
    return RT_OK;
}

// An integer override `name` from the environment: true and `out` set when present and a whole
// number in [lo, hi]; a malformed or out-of-range value sets the error (naming `who` and the
// variable) and clears `ok`.
bool env_int(const char* who, const char* name, long long lo, long long hi, long long& out, bool& ok) {
    const char* e = getenv(name);
    if (!e) return false;
    char* end = nullptr;
    errno = 0;
    const long long v = strtoll(e, &end, 0);
    if (!*e || *end || errno || v < lo || v > hi) {
        set_error(std::string(who) + ": bad " + name + "=" + e);
        ok = false;
        return false;
    }
    out = v;
    return true;
}

// The test-override environment variables, applied once at rt_scene_upload (never per frame).
// A value that is not a whole number (RT_SPLAT=exact) is an error, not a silent 0: false, with
// the variable named in the error text.
bool config_from_env(rt_scene_config& c) {
    bool ok = true;
    auto num = [&](const char* name, long long lo, long long hi, long long& out) {
        return env_int("rt_scene_upload", name, lo, hi, out, ok);
    };
    long long v = 0;
    if (num("RT_SPLAT", RT_SPLAT_STREAM, RT_SPLAT_ATOMIC, v)) c.splat_mode = (int32_t)v;
    if (num("RT_PARTITIONS", 1, MAX_PARTITIONS, v)) c.partitions = (int32_t)v;
    if (num("RT_FUSE_PATHS", 0, 0xFFFFFFFFll, v)) c.fuse_paths = v;
    if (num("RT_SPLAT_CHUNK", 1, 1 << 20, v)) c.splat_chunk = (int32_t)v;
    if (num("RT_SPLAT_RING", 1, 1 << 20, v)) c.splat_ring = (int32_t)v;
    if (const char* e = getenv("RT_SAMPLE_BUDGET_GB")) {
        char* end = nullptr;
        const double g = strtod(e, &end);
        if (!*e || *end || !(g >= 0.0)) { set_error(std::string("rt_scene_upload: bad RT_SAMPLE_BUDGET_GB=") + e); ok = false; }
        else c.sample_budget_gb = g;
    }
    if (num("RT_RES_TALL_PIXELS", 0, 1ll << 40, v)) c.resolve_tall_pixels = v;
    if (num("RT_DEBUG_TRAVERSAL", 0, 1, v)) c.debug_traversal = (int32_t)v;
    if (num("RT_TRAVERSAL_REF", 0, 1, v)) c.traversal_ref = (int32_t)v;
    if (num("RT_DRAIN_EVERY", 0, 1024, v)) c.drain_every = (int32_t)v;
    if (num("RT_SHADOW_LAUNCH", RT_SHADOW_LAUNCH_AUTO, RT_SHADOW_LAUNCH_MERGED, v)) c.shadow_launch = (int32_t)v;
    return ok;
}

}  // namespace

extern "C" {

int rt_scene_default_config(rt_scene_config* out) {
    if (!out) { set_error("null argument"); return RT_ERROR_INVALID; }
    *out = default_config();
    return RT_OK;
}

int rt_scene_get_config(const rt_scene* s, rt_scene_config* out) {
    if (!s || !out) { set_error("null argument"); return RT_ERROR_INVALID; }
    *out = s->cfg;
    return RT_OK;
}

int rt_scene_set_config(rt_scene* s, const rt_scene_config* c) {
    if (!s || !c) { set_error("null argument"); return RT_ERROR_INVALID; }
    int err = check_config(c);
    if (err) return err;
    if (c->traversal_ref && s->bvh_depth_ref + 2 > STACK_DEPTH) {
        set_error("rt_scene_config: traversal_ref needs more than the 64-entry traversal stack for this BVH");
        return RT_ERROR_INVALID;
    }
    s->cfg = *c;
    memset(s->cfg.reserved, 0, sizeof(s->cfg.reserved));
    return RT_OK;
}

int rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_error(void) { return g_error.c_str(); }

int rt_device_count(int* out) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    if (out) *out = n;
    return RT_OK;
}

int rt_set_profiling(int enable) { g_profiling = enable ? (1u << RT_KERNEL_COUNT) - 1u : 0u; return RT_OK; }
int rt_set_profiling_stages(uint32_t mask) { g_profiling = mask & ((1u << RT_KERNEL_COUNT) - 1u); return RT_OK; }
int rt_set_path_pool(uint32_t paths) { g_pool_override = paths; return RT_OK; }
int rt_set_env_sampling(int mode) {
    if (mode != 0 && mode != 1) { set_error("rt_set_env_sampling: mode must be 0 or 1"); return RT_ERROR_INVALID; }
    g_env_sampling = mode;
    return RT_OK;
}

int rt_set_shard_mode(int mode) {
    if (mode != RT_SHARD_TILES && mode != RT_SHARD_PASSES) { set_error("bad shard mode"); return RT_ERROR_INVALID; }
    g_shard_mode = mode;
    return RT_OK;
}

int rt_set_splat_mode(int mode) {
    if (mode < RT_SPLAT_STREAM || mode > RT_SPLAT_ATOMIC) { set_error("bad splat mode"); return RT_ERROR_INVALID; }
    g_splat_mode = mode;
    return RT_OK;
}

int rt_scene_upload(const rt_scene_desc* d, int device, rt_scene** out) {
    if (!d || !out) { set_error("null argument"); return RT_ERROR_INVALID; }
    *out = nullptr;
    int err = bind_device(device);
    if (err) return err;
    if (d->material_count == 0 || d->material_count >= 0xFFFFu) { set_error("material count must be in [1, 65534]"); return RT_ERROR_INVALID; }
    rt_scene* s = new rt_scene();
    s->device = device;
    s->cfg = default_config();
    if (!config_from_env(s->cfg)) { delete s; return RT_ERROR_INVALID; }
    if ((err = check_config(&s->cfg))) { delete s; return err; }
    DevScene& ds = s->ds;
    auto fail = [&](int e) { rt_scene_free(s); return e; };
    // materials + the integrator's local `air` (RT/integrators.cpp:597-599)
    std::vector<rt_material> mats(d->materials, d->materials + d->material_count);
    rt_material air = {};
    air.ior = 1.0f;
    air.is_participating_medium = 1;
    mats.push_back(air);
    ds.material_count = d->material_count;
    ds.air_id = d->material_count;
    if ((err = upload(s, mats.data(), mats.size(), &ds.materials))) return fail(err);
    for (uint32_t i = 0; i < d->primitive_count; ++i) {
        const rt_primitive& p = d->primitives[i];
        if (p.transform_index >= d->transform_count || p.material_id >= d->material_count ||
            (p.type == RT_PRIMITIVE_MESH && p.mesh_index >= d->mesh_count)) {
            set_error("primitive references out of range"); return fail(RT_ERROR_INVALID);
        }
    }
    for (uint32_t i = 0; i < d->plane_count; ++i)
        if (d->planes[i].transform_index >= d->transform_count || d->planes[i].material_id >= d->material_count) {
            set_error("plane references out of range"); return fail(RT_ERROR_INVALID);
        }
    for (uint32_t i = 0; i < d->light_count; ++i)
        if (d->lights[i] >= d->primitive_count) { set_error("light id out of range"); return fail(RT_ERROR_INVALID); }
    if ((err = upload(s, d->primitives, d->primitive_count, &ds.prims))) return fail(err);
    if ((err = upload(s, d->planes, d->plane_count, &ds.planes))) return fail(err);
    {   // the prologue's plane table: p[0..3] per plane, four per scalar load
        std::vector<float4> nd((d->plane_count + 3u) / 4u * 4u + 4u, make_float4(0, 0, 0, 0));
        for (uint32_t i = 0; i < d->plane_count; ++i)
            nd[i] = make_float4(d->planes[i].p[0], d->planes[i].p[1], d->planes[i].p[2], d->planes[i].p[3]);
        if ((err = upload(s, nd.data(), nd.size(), &ds.plane_nd))) return fail(err);
    }
    ds.plane_count = d->plane_count;
    std::vector<M34> inv(d->transform_count), fwd(d->transform_count);
    for (uint32_t i = 0; i < d->transform_count; ++i)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) { inv[i].e[r][c] = d->transforms[i].inverse.e[r][c]; fwd[i].e[r][c] = d->transforms[i].forward.e[r][c]; }
    if ((err = upload(s, inv.data(), inv.size(), &ds.inv))) return fail(err);
    if ((err = upload(s, fwd.data(), fwd.size(), &ds.fwd))) return fail(err);
    if ((err = upload(s, d->lights, d->light_count, &ds.lights))) return fail(err);
    ds.light_count = d->light_count;
    uint32_t top_depth = tree_depth(d->bvh_nodes, d->bvh_node_count);
    for (uint32_t i = 0; i < d->bvh_index_count; ++i)
        if (d->bvh_indices[i] >= d->primitive_count) { set_error("bvh index out of range"); return fail(RT_ERROR_INVALID); }
    // node, triangle and leaf-record arrays get FETCH_Q float4 of padding: a traversal
    // step loads FETCH_Q float4 unconditionally
    std::vector<rt_bvh_node> top_nodes(d->bvh_nodes, d->bvh_nodes + d->bvh_node_count);
    top_nodes.resize(top_nodes.size() + (FETCH_Q*16 + 31)/32, rt_bvh_node{});
    if ((err = upload(s, top_nodes.data(), top_nodes.size(), &ds.bvh_src))) return fail(err);
    {
        std::vector<rt_bvh_node> tl = traversal_layout(top_nodes.data(), (uint32_t)top_nodes.size());
        ds.bvh_root_rec = tl[0].left_first;
        if ((err = upload(s, tl.data(), tl.size(), &ds.bvh))) return fail(err);
    }
    if ((err = upload(s, d->bvh_indices, d->bvh_index_count, &ds.bvh_idx))) return fail(err);
    {
        bool env_ok = true;
        long long top = 1, mlist = MLIST_MAX;
        env_int("rt_scene_upload", "RT_TOP_PROLOGUE", 0, 1, top, env_ok);   // 0: the trace kernels walk the top level
        env_int("rt_scene_upload", "RT_MLIST_MAX", 0, MLIST_MAX, mlist, env_ok);
        if (!env_ok) return fail(RT_ERROR_INVALID);
        std::vector<float4> seq;
        uint32_t len = 0;
        if (top) seq = top_sequences(d->bvh_nodes, d->bvh_node_count, d->bvh_index_count, len);
        ds.top_seq = nullptr; ds.top_seq_len = 0; ds.mlist_max = (uint32_t)mlist;
        if (!seq.empty()) {
            if ((err = upload(s, seq.data(), seq.size(), &ds.top_seq))) return fail(err);
            ds.top_seq_len = len;
        }
        uint32_t mesh_slots = 0;
        for (uint32_t j = 0; j < d->bvh_index_count; ++j)
            mesh_slots += d->primitives[d->bvh_indices[j]].type == RT_PRIMITIVE_MESH ? 1u : 0u;
        ds.listed_only = (ds.top_seq && mesh_slots <= ds.mlist_max) ? 1u : 0u;
    }
    ds.bvh_node_count = d->bvh_node_count;
    // meshes: concatenate, triangles as (a, b-a, c-a) float4 triples
    std::vector<DevMesh> meshes(d->mesh_count);
    std::vector<float4> tris;
    std::vector<uint32_t> orig;
    std::vector<float> normals;
    std::vector<rt_bvh_node> mnodes;
    uint32_t mesh_depth = 0;
    std::vector<float4> mnodes4;
    std::vector<uint32_t> root4(d->mesh_count, 0u);
    std::vector<uint32_t> src4;                 // BVH4 node -> its BVH2 node (mesh-local)
    std::vector<uint32_t> mesh4(1, 0u);         // BVH4 nodes before mesh m's
    uint32_t mesh_depth_ref = 0;                // mesh_depth with a reference-unit walk's markers
    for (uint32_t m = 0; m < d->mesh_count; ++m) {
        const rt_mesh& M = d->meshes[m];
        meshes[m].tri_offset = (uint32_t)orig.size();
        meshes[m].node_offset = (uint32_t)mnodes.size();
        meshes[m].has_normals = (M.has_normals && M.normals) ? 1u : 0u;
        for (uint32_t i = 0; i < M.node_count; ++i) {
            const rt_bvh_node& nd = M.nodes[i];
            if (nd.count ? (nd.left_first + nd.count > M.triangle_count) : (nd.left_first + 1 >= M.node_count && !(i == 0 && nd.left_first == 0))) {
                set_error("mesh BVH node out of range"); return fail(RT_ERROR_INVALID);
            }
        }
        if (M.node_count) {
            const rt_bvh_node& r0 = M.nodes[0];
            if (r0.count) {
                root4[m] = pack_node(0u, r0.left_first, r0.count, 0u);
                mesh_depth = std::max(mesh_depth, 1u);
            } else {
                bool ok = true;
                uint32_t need = 0, levels = 0;
                root4[m] = build_bvh4(M.nodes, M.node_count, 0u, mnodes4, need, ok, &src4, &levels);
                if (!ok) { set_error("mesh BVH too large for the BVH4 records"); return fail(RT_ERROR_INVALID); }
                mesh_depth = std::max(mesh_depth, need + 1);
                mesh_depth_ref = std::max(mesh_depth_ref, need + 1 + levels);
            }
        }
        for (uint32_t t = 0; t < M.triangle_count; ++t) {
            const rt_v3* v = M.triangles + 3*(size_t)t;
            tris.push_back(make_float4(v[0].x, v[0].y, v[0].z, 0.0f));
            tris.push_back(make_float4(v[1].x - v[0].x, v[1].y - v[0].y, v[1].z - v[0].z, 0.0f));
            tris.push_back(make_float4(v[2].x - v[0].x, v[2].y - v[0].y, v[2].z - v[0].z, 0.0f));
            if (M.indices[t] >= M.triangle_count) { set_error("mesh index out of range"); return fail(RT_ERROR_INVALID); }
            orig.push_back(M.indices[t]);
        }
        // vertex normals gathered into BVH slot order (the reference looks them up by the
        // original index, get_normals(mesh)[indices[slot]], RT/intersection.cpp:574-578):
        // the hit's slot then addresses them directly
        for (uint32_t t = 0; t < M.triangle_count; ++t)
            for (int k = 0; k < 3; ++k) {
                rt_v3 nn = meshes[m].has_normals ? M.normals[3*(size_t)M.indices[t] + k] : rt_v3{0, 0, 0};
                normals.push_back(nn.x); normals.push_back(nn.y); normals.push_back(nn.z);
            }
        mnodes.insert(mnodes.end(), M.nodes, M.nodes + M.node_count);
        mesh4.push_back((uint32_t)(mnodes4.size() / 8));
    }
    {   // finite_box_ray's scene condition: every box within 2^40 of the origin
        auto within = [](const rt_bvh_node* n, size_t count) {
            for (size_t i = 0; i < count; ++i) {
                const float c[3] = {n[i].bv_p.x, n[i].bv_p.y, n[i].bv_p.z}, r[3] = {n[i].bv_r.x, n[i].bv_r.y, n[i].bv_r.z};
                for (int k = 0; k < 3; ++k)
                    if (!(std::fabs(c[k]) + std::fabs(r[k]) <= 1099511627776.0f)) return false;   // NaN fails too
            }
            return true;
        };
        ds.finite_boxes = (within(d->bvh_nodes, d->bvh_node_count) && within(mnodes.data(), mnodes.size())) ? 1u : 0u;
    }
    if (top_depth + mesh_depth + 2 > STACK_DEPTH) {
        set_error("BVH too deep for the 64-entry traversal stack (RT/intersection.cpp:445)");
        return fail(RT_ERROR_INVALID);
    }
    s->bvh_depth = top_depth + mesh_depth;
    s->bvh_depth_ref = top_depth + std::max(mesh_depth, mesh_depth_ref);
    if (s->cfg.traversal_ref && s->bvh_depth_ref + 2 > STACK_DEPTH) {       // RT_TRAVERSAL_REF
        set_error("rt_scene_upload: traversal_ref needs more than the 64-entry traversal stack for this BVH");
        return fail(RT_ERROR_INVALID);
    }
    {   // top-level leaf records, in bvh_indices order
        auto u2f = [](uint32_t u) { float f; memcpy(&f, &u, 4); return f; };
        std::vector<float4> rec((size_t)d->bvh_index_count*LEAF_REC_Q, make_float4(0, 0, 0, 0));
        for (uint32_t j = 0; j < d->bvh_index_count; ++j) {
            const uint32_t pi = d->bvh_indices[j];
            const rt_primitive& p = d->primitives[pi];
            float4* q = rec.data() + (size_t)j*LEAF_REC_Q;
            const M34& iv = inv[p.transform_index];
            for (int r = 0; r < 3; ++r) q[r] = make_float4(iv.e[r][0], iv.e[r][1], iv.e[r][2], iv.e[r][3]);
            if (p.type == RT_PRIMITIVE_MESH) {
                const rt_mesh& M = d->meshes[p.mesh_index];
                rt_bvh_node rn = {};
                if (M.node_count) rn = M.nodes[0];
                const uint32_t root = root4[p.mesh_index];
                q[3] = make_float4(u2f(pi), u2f(p.type), u2f(meshes[p.mesh_index].node_offset), u2f(meshes[p.mesh_index].tri_offset));
                q[4] = make_float4(u2f(root), rn.bv_p.x, rn.bv_p.y, rn.bv_p.z);
                // q5.w: the mesh has a BVH.  Without one the reference tests none of its triangles
                // (intersect_mesh, RT/intersection.cpp:259: `if (bvh)`): the root box is made empty
                // (half sides -1: no slab test passes), and the reference-unit walk counts no root pop
                if (M.node_count) q[5] = make_float4(rn.bv_r.x, rn.bv_r.y, rn.bv_r.z, 1.0f);
                else q[5] = make_float4(-1.0f, -1.0f, -1.0f, 0.0f);
            } else {
                bool translate = std::isfinite(iv.e[0][3]) && std::isfinite(iv.e[1][3]) && std::isfinite(iv.e[2][3]);
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) translate = translate && iv.e[r][c] == (r == c ? 1.0f : 0.0f);
                q[3] = make_float4(u2f(pi), u2f(p.type | (translate ? LEAF_TRANSLATE : 0u)), p.p[0], p.p[1]);
                q[4] = make_float4(p.p[2], 0.0f, 0.0f, 0.0f);
            }
        }
        rec.resize(rec.size() + FETCH_Q, make_float4(0, 0, 0, 0));
        if ((err = upload(s, rec.data(), rec.size(), &ds.leaf_rec))) return fail(err);
    }
    if ((err = upload(s, meshes.data(), meshes.size(), &ds.meshes))) return fail(err);
    tris.resize(tris.size() + FETCH_Q, make_float4(0, 0, 0, 0));
    if ((err = upload(s, tris.data(), tris.size(), &ds.tris))) return fail(err);
    if ((err = upload(s, orig.data(), orig.size(), &ds.tri_orig))) return fail(err);
    if ((err = upload(s, normals.data(), normals.size(), &ds.normals))) return fail(err);
    mnodes.resize(mnodes.size() + (FETCH_Q*16 + 31)/32, rt_bvh_node{});
    if ((err = upload(s, mnodes.data(), mnodes.size(), &ds.mnodes_src))) return fail(err);
    {
        // records are mesh-local: the index form carries the node's index within its mesh
        std::vector<rt_bvh_node> tl(mnodes.size());
        for (uint32_t m = 0; m < d->mesh_count; ++m) {
            const uint32_t off = meshes[m].node_offset, n = d->meshes[m].node_count;
            std::vector<rt_bvh_node> one = traversal_layout(mnodes.data() + off, n);
            std::copy(one.begin(), one.end(), tl.begin() + off);
        }
        if ((err = upload(s, tl.data(), tl.size(), &ds.mnodes))) return fail(err);
    }
    ds.mnodes4 = nullptr;
    {   // every interior record of the concatenated BVH4s addresses a node that exists
        const uint32_t n4 = (uint32_t)(mnodes4.size() / 8);
        bool bad = false;
        for (uint32_t m = 0; m < d->mesh_count; ++m)
            bad |= root4[m] < (1u << 28) && root4[m] >= n4 && d->meshes[m].node_count && !d->meshes[m].nodes[0].count;
        for (size_t k = 0; k < n4 && !bad; ++k)
            for (int j = 0; j < 4; ++j) {
                uint32_t r;
                memcpy(&r, &(&mnodes4[8*k + 6].x)[j], 4);
                bad |= r != EMPTY4 && r < (1u << 28) && r >= n4;
            }
        if (bad) { set_error("internal: mesh BVH4 record out of range"); return fail(RT_ERROR_INVALID); }
    }
    ds.mid4 = nullptr;
    if (!mnodes4.empty()) {
        // mid4: per BVH4 node, the boxes of its BVH2 node's two children (the skipped level)
        std::vector<float4> mid(3*(mnodes4.size() / 8), make_float4(0, 0, 0, 0));
        for (uint32_t m = 0; m < d->mesh_count; ++m) {
            const rt_mesh& M = d->meshes[m];
            for (uint32_t k = mesh4[m]; k < mesh4[m + 1]; ++k) {
                const uint32_t i = src4[k], l = M.nodes[i].left_first;
                if (M.nodes[i].count || l + 1 >= M.node_count) continue;
                const rt_bvh_node& L = M.nodes[l];
                const rt_bvh_node& R = M.nodes[l + 1];
                mid[3*k] = make_float4(L.bv_p.x, L.bv_p.y, L.bv_p.z, L.bv_r.x);
                mid[3*k + 1] = make_float4(L.bv_r.y, L.bv_r.z, R.bv_p.x, R.bv_p.y);
                mid[3*k + 2] = make_float4(R.bv_p.z, R.bv_r.x, R.bv_r.y, R.bv_r.z);
            }
        }
        if ((err = upload(s, mid.data(), mid.size(), &ds.mid4))) return fail(err);
        mnodes4.resize(mnodes4.size() + FETCH_Q, make_float4(0, 0, 0, 0));
        if ((err = upload(s, mnodes4.data(), mnodes4.size(), &ds.mnodes4))) return fail(err);
    }
    if (d->skydome && d->skydome_w && d->skydome_h) {
        if ((err = upload(s, reinterpret_cast<const float*>(d->skydome), 3*(size_t)d->skydome_w*d->skydome_h, &ds.sky))) return fail(err);
        ds.sky_w = d->skydome_w; ds.sky_h = d->skydome_h;
        std::vector<float4> et;
        if (build_env_table(d->skydome_w, d->skydome_h, d->skydome, et, ds.env_tx, ds.env_tw, ds.env_th)) {
            if ((err = upload(s, et.data(), et.size(), &ds.env_tab))) return fail(err);
            ds.env_n = (uint32_t)et.size();
        }
    }
    ds.top_sky = rv3(d->top_sky_color);
    ds.bot_sky = rv3(d->bot_sky_color);
    if ((err = upload(s, rt_dev_strata_tab, sizeof(rt_dev_strata_tab), &ds.strata))) return fail(err);
    if ((err = upload(s, rt_dev_bluenoise_tab, sizeof(rt_dev_bluenoise_tab), &ds.bluenoise))) return fail(err);
    {   // the LDS blob (scene_in_lds): the small tables, 16-byte aligned, when they fit
        std::vector<uint8_t> blob;
        auto put = [&](int which, const void* p, size_t bytes) {
            ds.off[which] = (uint32_t)blob.size();
            if (bytes) blob.insert(blob.end(), (const uint8_t*)p, (const uint8_t*)p + bytes);
            blob.resize((blob.size() + 15) & ~(size_t)15, 0);
        };
        put(BLOB_MATERIALS, mats.data(), mats.size()*sizeof(rt_material));
        put(BLOB_PRIMS, d->primitives, (size_t)d->primitive_count*sizeof(rt_primitive));
        put(BLOB_PLANES, d->planes, (size_t)d->plane_count*sizeof(rt_primitive));
        put(BLOB_INV, inv.data(), inv.size()*sizeof(M34));
        put(BLOB_FWD, fwd.data(), fwd.size()*sizeof(M34));
        put(BLOB_LIGHTS, d->lights, (size_t)d->light_count*sizeof(uint32_t));
        // the prologue reads the top-level sequences and leaf records from HBM through the scalar
        // cache, and the strata table stays in HBM (both read through L2): not copied into LDS
        put(BLOB_MESHES, meshes.data(), meshes.size()*sizeof(DevMesh));
        bool env_ok = true;
        long long lds_scene = 1;                                 // 0: the kernels read the tables from HBM
        env_int("rt_scene_upload", "RT_LDS_SCENE", 0, 1, lds_scene, env_ok);
        if (!env_ok) return fail(RT_ERROR_INVALID);
        ds.blob = nullptr; ds.blob_q = 0;
        if (blob.size() <= 16*(size_t)LDS_SCENE_Q && lds_scene) {
            std::vector<float4> q(blob.size() / 16);
            memcpy(q.data(), blob.data(), blob.size());
            if ((err = upload(s, q.data(), q.size(), &ds.blob))) return fail(err);
            ds.blob_q = (uint32_t)q.size();
        }
        if (debug_timing())
            fprintf(stderr, "[rt timing] rt_scene_upload: scene tables %zu B (%s LDS; materials %zu, primitives %u, planes %u, "
                    "transforms %zu, lights %u, meshes %zu)\n", blob.size(), ds.blob_q ? "in" : "not in", mats.size(),
                    d->primitive_count, d->plane_count, inv.size(), d->light_count, meshes.size());
    }
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) != hipSuccess) { set_error("hipGetDeviceProperties"); return fail(RT_ERROR_DEVICE); }
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_trace<false, false, 3>, TB, TRACE_LDS) != hipSuccess || per_cu < 1) per_cu = 1;
        s->trace_grid = (uint32_t)(prop.multiProcessorCount*per_cu);
        // Persistent trace blocks: 75 % of one full-occupancy wave of blocks (RT_TRACE_GRID_PCT).
        // Four partitions run their trace launches side by side; a full grid per launch left
        // less room for the other partitions' generate / shade blocks.  C3 A/B, 5 alternating
        // pairs: 75 % +1.5 %, 60 % +0.9 %, 50 % +1.5 % (2 pairs), 150 % -0.8 %.  The spill
        // area is sized from the result.
        bool env_ok = true;
        long long grid_pct = 75, connect_pct = 25, drain_pct = 100, shadow_pct = 33;
        env_int("rt_scene_upload", "RT_TRACE_GRID_PCT", 1, 1000, grid_pct, env_ok);
        env_int("rt_scene_upload", "RT_CONNECT_GRID_PCT", 1, 1000, connect_pct, env_ok);
        env_int("rt_scene_upload", "RT_SHADOW_PCT", 1, 100, shadow_pct, env_ok);
        s->shadow_pct = (uint32_t)shadow_pct;
        env_int("rt_scene_upload", "RT_DRAIN_GRID_PCT", 1, 100, drain_pct, env_ok);
        long long by_pool = 1;
        env_int("rt_scene_upload", "RT_TRACE_GRID_BY_POOL", 0, 1, by_pool, env_ok);
        s->grid_by_pool = by_pool != 0;
        if (!env_ok) return fail(RT_ERROR_INVALID);
        const uint32_t full = s->trace_grid;
        s->trace_grid = std::max(1u, (uint32_t)((unsigned long long)full*(unsigned)grid_pct / 100ull));
        // The separate shadow launch carries a quarter of the extension rays (~0.8 per lane of a 75 % grid):
        // a 25 % grid does them as fast and leaves the registers to the other partitions' kernels
        // (C3: +0.6 %, 2 pairs; 40 / 55 % between).  Merged into the trace launch, a third of its blocks
        // take them (RT_SHADOW_PCT; all blocks: C4 -1 %, the share of 8 -0.3 %, profiles/r06_shadow_launch_ab.txt).
        s->connect_grid = std::min(s->trace_grid,
                                   std::max(1u, (uint32_t)((unsigned long long)full*(unsigned)connect_pct / 100ull)));
        int drain_cu = 0;     // k_drain holds ~220 VGPRs: 2 waves per SIMD; its grid is what fits at once
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&drain_cu, k_drain<false, false>, DTB, 0) != hipSuccess || drain_cu < 1)
            drain_cu = 1;
        // (lanes <= the trace grid's: the spill area is sized for those)
        s->drain_grid = std::min(s->trace_grid*(uint32_t)(TB / DTB), (uint32_t)(prop.multiProcessorCount*drain_cu));
        s->drain_lanes_full = s->drain_grid*DTB;
        s->drain_grid = std::max(1u, (uint32_t)((unsigned long long)s->drain_grid*(unsigned long long)drain_pct / 100ull));
    }
    if (ensure_partition(s, 0)) return fail(RT_ERROR_OUT_OF_MEMORY);
    if (hipMalloc(&s->d_lut, 512*sizeof(float)) != hipSuccess) { set_error("hipMalloc lut"); return fail(RT_ERROR_OUT_OF_MEMORY); }
    *out = s;
    return RT_OK;
}

int rt_scene_free(rt_scene* s) {
    if (!s) return RT_OK;
    (void)hipSetDevice(s->device);
    for (void* p : s->allocs) (void)hipFree(p);
    for (auto& pt : s->part) free_partition(pt);
    if (s->start_ev) (void)hipEventDestroy(s->start_ev);
    if (s->d_tiles) (void)hipFree(s->d_tiles);
    if (s->d_pixmap) (void)hipFree(s->d_pixmap);
    if (s->d_tile_base) (void)hipFree(s->d_tile_base);
    if (s->d_samp) (void)hipFree(s->d_samp);
    if (s->d_samp_jy) (void)hipFree(s->d_samp_jy);
    if (s->d_lut) (void)hipFree(s->d_lut);
    if (s->d_partials) (void)hipFree(s->d_partials);
    if (s->d_aux) (void)hipFree(s->d_aux);
    delete s;
    return RT_OK;
}

int rt_cancel(rt_scene* s) { if (s) s->cancel = 1; return RT_OK; }

int rt_postprocess_device(int device, const float* d_pixels, uint32_t w, uint32_t h, const rt_post_settings* post,
                          uint32_t total_frame_index, uint32_t* d_bgra, void* hip_stream) {
    if (!d_pixels || !post || !d_bgra || !w || !h) { set_error("null argument"); return RT_ERROR_INVALID; }
    int err = bind_device(device);
    if (err) return err;
    static std::mutex mu;
    static std::vector<uint8_t*> tabs;                 // per device: the 8 dither textures (1.5 MB)
    const uint8_t* tab = nullptr;
    {
        std::lock_guard<std::mutex> lock(mu);
        if ((int)tabs.size() <= device) tabs.resize(device + 1, nullptr);
        if (!tabs[device]) {
            HIP_OK(hipMalloc(&tabs[device], sizeof(rt_dev_dither_tab)));
            HIP_OK(hipMemcpy(tabs[device], rt_dev_dither_tab, sizeof(rt_dev_dither_tab), hipMemcpyHostToDevice));
        }
        tab = tabs[device];
    }
    hipStream_t stream = static_cast<hipStream_t>(hip_stream);
    const dim3 grid((w + 63) / 64, (h + 3) / 4);
    k_post<<<grid, 256, 0, stream>>>(reinterpret_cast<const float4*>(d_pixels), w, h, *post,
                                     tab + (size_t)(total_frame_index % 8u)*256*256*3, d_bgra);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(stream));
    return RT_OK;
}

int rt_postprocess(int device, const rt_accumulation_buffer* accum, const rt_post_settings* post,
                   uint32_t total_frame_index, uint32_t* out_bgra) {
    if (!accum || !accum->pixels || !post || !out_bgra || !accum->w || !accum->h) { set_error("null argument"); return RT_ERROR_INVALID; }
    int err = bind_device(device);
    if (err) return err;
    const size_t n = (size_t)accum->w*accum->h;
    float* d_px = nullptr;
    uint32_t* d_out = nullptr;
    HIP_OK(hipMalloc(&d_px, 16*n));
    if (hipMalloc(&d_out, 4*n) != hipSuccess) { (void)hipFree(d_px); set_error("hipMalloc"); return RT_ERROR_OUT_OF_MEMORY; }
    err = RT_OK;
    if (hipMemcpy(d_px, accum->pixels, 16*n, hipMemcpyHostToDevice) != hipSuccess) { set_error("hipMemcpy"); err = RT_ERROR_DEVICE; }
    if (!err) err = rt_postprocess_device(device, d_px, accum->w, accum->h, post, total_frame_index, d_out, nullptr);
    if (!err && hipMemcpy(out_bgra, d_out, 4*n, hipMemcpyDeviceToHost) != hipSuccess) { set_error("hipMemcpy"); err = RT_ERROR_DEVICE; }
    (void)hipFree(d_px);
    (void)hipFree(d_out);
    return err;
}

int rt_render_device(rt_scene* s, const rt_camera* camera, const rt_settings* st,
                     const rt_filter_cache* filter, const rt_tile_set* tiles,
                     uint32_t total_frame_index, uint32_t w, uint32_t h, uint32_t frame_count,
                     float* d_pixels, void* hip_stream, rt_stats* stats) {
    if (!s || !camera || !tiles || !d_pixels || !w || !h) { set_error("null argument"); return RT_ERROR_INVALID; }
    int err = check_inputs(st, filter);
    if (err) return err;
    if (!tiles->tile_w || !tiles->tile_h || !tiles->shard_count || tiles->shard_index >= tiles->shard_count) {
        set_error("bad tile set"); return RT_ERROR_INVALID;
    }
    const double t_entry = debug_timing() ? host_ms() : 0.0;
    HIP_OK(hipSetDevice(s->device));
    hipStream_t stream = (hipStream_t)hip_stream;
    FrameParams fp = {};
    fp.w = w; fp.h = h; fp.frame_count = frame_count; fp.total_frame_index = total_frame_index;
    fp.tile_w = tiles->tile_w; fp.tile_h = tiles->tile_h;
    fp.tcx = (w + tiles->tile_w - 1) / tiles->tile_w;
    uint32_t tcy = (h + tiles->tile_h - 1) / tiles->tile_h;
    if (w > 65535 || h > 65535) { set_error("frame larger than 65535 pixels a side"); return RT_ERROR_INVALID; }
    // RT_SHARD_PASSES: every tile, and the shard's range of sample passes (below)
    const int shard_mode = s->cfg.shard_mode >= 0 ? s->cfg.shard_mode : g_shard_mode;
    const bool by_pass = shard_mode == RT_SHARD_PASSES && tiles->shard_count > 1;
    const uint32_t tsi = by_pass ? 0u : tiles->shard_index, tsc = by_pass ? 1u : tiles->shard_count;
    auto& L = s->layout;
    const bool same = L.valid && L.w == w && L.h == h && L.tw == tiles->tile_w && L.th == tiles->tile_h &&
                      L.si == tsi && L.sc == tsc;
    if (!same) {
        // owned tiles: t % shard_count == shard_index, descending like the reference's queue (:555)
        L.valid = false;
        L.ids.clear(); L.prefix.assign(1, 0); L.owned_px = 0;
        for (uint32_t t = fp.tcx*tcy; t-- > 0;) {
            if (t % tsc != tsi) continue;
            uint32_t min_x = tiles->tile_w*(t % fp.tcx), min_y = tiles->tile_h*(t / fp.tcx);
            uint32_t tw = std::min(w, min_x + tiles->tile_w) - min_x, th = std::min(h, min_y + tiles->tile_h) - min_y;
            L.ids.push_back(t);
            L.owned_px += (uint64_t)tw*th;
            L.prefix.push_back((uint32_t)std::min<uint64_t>(L.owned_px, 0xFFFFFFFFull));
        }
    }
    const std::vector<uint32_t>& ids = L.ids;
    const std::vector<uint32_t>& prefix = L.prefix;
    if (ids.empty()) { if (stats) memset(stats, 0, sizeof(*stats)); return RT_OK; }
    if (L.owned_px >= 0x80000000ull) {      // tile_base / pixel indices are 31-bit
        set_error("shard of 2^31 or more pixels: use more shards"); return RT_ERROR_INVALID;
    }
    fp.ntiles = (uint32_t)ids.size();
    fp.pixels = prefix.back();
    const size_t ntile_all = (size_t)fp.tcx*tcy;
    if (!same) {
        size_t need = ids.size() + prefix.size();
        if (s->tiles_cap < need) {
            if (s->d_tiles) (void)hipFree(s->d_tiles);
            s->d_tiles = nullptr;
            HIP_OK(hipMalloc(&s->d_tiles, need*sizeof(uint32_t)));
            s->tiles_cap = need;
        }
        std::vector<uint32_t> packed(ids);
        packed.insert(packed.end(), prefix.begin(), prefix.end());
        HIP_OK(hipMemcpy(s->d_tiles, packed.data(), packed.size()*sizeof(uint32_t), hipMemcpyHostToDevice));
        if (s->pixmap_cap < fp.pixels) {
            if (s->d_pixmap) (void)hipFree(s->d_pixmap);
            s->d_pixmap = nullptr; s->pixmap_cap = 0;
            HIP_OK(hipMalloc(&s->d_pixmap, sizeof(uint32_t)*(size_t)fp.pixels));
            s->pixmap_cap = fp.pixels;
        }
        L.base.assign(ntile_all, -1);
        for (size_t i = 0; i < ids.size(); ++i) L.base[ids[i]] = (int32_t)prefix[i];
        if (s->tile_base_cap < ntile_all) {
            if (s->d_tile_base) (void)hipFree(s->d_tile_base);
            s->d_tile_base = nullptr;
            HIP_OK(hipMalloc(&s->d_tile_base, sizeof(int32_t)*ntile_all));
            s->tile_base_cap = ntile_all;
        }
        HIP_OK(hipMemcpy(s->d_tile_base, L.base.data(), sizeof(int32_t)*ntile_all, hipMemcpyHostToDevice));
    }
    HIP_OK(hipMemcpyAsync(s->d_lut, filter->cache, 512*sizeof(float), hipMemcpyHostToDevice, stream));
    fp.tile_ids = s->d_tiles;
    fp.tile_prefix = s->d_tiles + ids.size();
    if (!same) {
        k_pixel_map<<<fp.ntiles, 256, 0, stream>>>(fp, s->d_pixmap);
        HIP_OK(hipGetLastError());
        L.w = w; L.h = h; L.tw = tiles->tile_w; L.th = tiles->tile_h; L.si = tsi; L.sc = tsc;
        L.blocks_ks = -1;
        L.valid = true;
    }
    fp.pix_xy = s->d_pixmap;
    set_divisors(fp);
    fill_camera(fp, camera);
    fp.lut = s->d_lut;
    fp.kernel_size = (int32_t)filter->kernel_size;
    fp.cache_size = (int32_t)filter->cache_size;
    fp.accum = reinterpret_cast<float4*>(d_pixels);
    const uint32_t spp_all = st->samples_per_pixel;
    const uint32_t pass_lo = by_pass ? (uint32_t)((unsigned long long)spp_all*tiles->shard_index / tiles->shard_count) : 0u;
    const uint32_t pass_hi = by_pass ? (uint32_t)((unsigned long long)spp_all*(tiles->shard_index + 1) / tiles->shard_count)
                                     : spp_all;
    unsigned long long total = (unsigned long long)fp.pixels*(pass_hi - pass_lo);
    if (total == 0) { if (stats) memset(stats, 0, sizeof(*stats)); return RT_OK; }
    // The splat (rt_set_splat_mode).  Both deterministic modes keep a 20-byte record per
    // sample in HBM: STREAM a ring of `ring` passes per partition (k_resolve_tiles frees
    // passes as the frame renders), EXACT the whole frame (k_resolve at the end, the
    // reference's order).  The budget is the free memory (plus the records already held)
    // less 16 GB for the partitions' path pools.  EXACT falls back to STREAM over budget or
    // past the filter radius k_resolve_tiles stages (12); STREAM to ATOMIC only if even
    // one pass per partition does not fit.
    const uint32_t spp = pass_hi - pass_lo;                       // this shard's passes
    const int ks = fp.cache_size ? fp.kernel_size : 0;
    const FrameShape shape = frame_shape(s, total, spp);
    int want_mode = s->cfg.splat_mode >= 0 ? s->cfg.splat_mode : g_splat_mode;
    // k_resolve gathers passes 0..spp-1 of one record array: a pass shard never takes the exact splat
    if (by_pass && want_mode == RT_SPLAT_EXACT) want_mode = RT_SPLAT_STREAM;
    // the splat for a record budget (bytes): the mode, and for STREAM the ring and chunk
    auto plan_splat = [&](double budget, SplatCfg& sp, size_t& need_rec) {
        sp = SplatCfg{};
        sp.passes = spp;
        sp.pass_lo = pass_lo;
        sp.mode = want_mode;
        need_rec = 0;
        if (sp.mode == RT_SPLAT_EXACT && (double)total*20.0 > budget) sp.mode = RT_SPLAT_STREAM;
        // past the radius k_resolve_tiles stages: the exact gather, or atomics for a pass shard (whose
        // records would be placed at pass_lo*P in an array sized for its own passes) or over budget
        if (sp.mode == RT_SPLAT_STREAM && ks > 12)
            sp.mode = (!by_pass && (double)total*20.0 <= budget) ? RT_SPLAT_EXACT : RT_SPLAT_ATOMIC;
        if (sp.mode == RT_SPLAT_STREAM) {
            // a resolve every ~32M samples, and at least four per partition (a small shard, e.g. one
            // rank's eighth of a frame, would otherwise resolve all its passes after its drain); the
            // ring holds the passes not yet resolved: the chunk, the claims of the iterations between
            // a sample's claim and its record (the life of a path, max_bounce_count iterations, plus
            // one: its last NEE term rides in the next k_trace), at most a pool fill each, and slack.
            // (r05 sized it at 5 pool fills: C4's shorter paths claim ~0.4 of the pool per iteration,
            // so its claims waited on the ring: a ring of 60 passes gave C4 1080p +1.9 %,
            // profiles/r06_ring_ab.txt)
            const uint32_t per_part = (spp + shape.nparts - 1) / shape.nparts;
            sp.chunk = (uint32_t)std::min<unsigned long long>(std::max<unsigned long long>((32ull << 20) / fp.pixels, 1ull),
                                                               std::max(1u, per_part / 4));
            if (s->cfg.splat_chunk > 0) sp.chunk = (uint32_t)s->cfg.splat_chunk;
            const unsigned long long fills = std::max<uint32_t>(st->max_bounce_count, 1u) + 1ull;
            const unsigned long long lag = (fills*shape.pool_n + fp.pixels - 1) / fp.pixels;
            sp.ring = (uint32_t)std::min<unsigned long long>(sp.chunk + lag + 2ull, per_part);
            if (s->cfg.splat_ring > 0) sp.ring = (uint32_t)s->cfg.splat_ring;
            sp.chunk = std::min(sp.chunk, sp.ring);                   // the planner needs chunk <= ring
            while (sp.ring > 1 && 20.0*(double)shape.nparts*sp.ring*fp.pixels > budget) {
                sp.ring = std::max(1u, sp.ring / 2);
                sp.chunk = std::min(sp.chunk, sp.ring);
            }
            need_rec = (size_t)shape.nparts*sp.ring*fp.pixels;
            if (20.0*(double)need_rec > budget) { sp.mode = RT_SPLAT_ATOMIC; need_rec = 0; }
        }
        if (sp.mode == RT_SPLAT_EXACT) need_rec = (size_t)total;
    };
    // The records held already need no budget: the free-memory query runs only when they must grow.
    SplatCfg sp;
    size_t need_rec = 0;
    const bool fixed_budget = s->cfg.sample_budget_gb >= 0.0;
    plan_splat(fixed_budget ? s->cfg.sample_budget_gb*1e9 : 20.0*(double)s->samp_cap, sp, need_rec);
    if (!fixed_budget && (sp.mode != want_mode || need_rec > s->samp_cap)) {
        size_t free_b = 0, total_b = 0;
        HIP_OK(hipMemGetInfo(&free_b, &total_b));
        plan_splat((double)free_b + 20.0*(double)s->samp_cap - 16e9, sp, need_rec);
    }
    if (sp.mode != RT_SPLAT_ATOMIC && s->samp_cap < need_rec) {
        if (s->d_samp) (void)hipFree(s->d_samp);
        if (s->d_samp_jy) (void)hipFree(s->d_samp_jy);
        s->d_samp = nullptr; s->d_samp_jy = nullptr; s->samp_cap = 0;
        if (hipMalloc(&s->d_samp, sizeof(float4)*need_rec) != hipSuccess ||
            hipMalloc(&s->d_samp_jy, sizeof(float)*need_rec) != hipSuccess) {
            (void)hipGetLastError();
            if (s->d_samp) (void)hipFree(s->d_samp);
            s->d_samp = nullptr; s->d_samp_jy = nullptr;
            sp.mode = RT_SPLAT_ATOMIC;                                 // out of memory
        } else {
            s->samp_cap = need_rec;
        }
    }
    if (sp.mode != RT_SPLAT_ATOMIC) {
        fp.samp_rgbx = s->d_samp;
        fp.samp_jy = s->d_samp_jy;
        fp.tile_base = s->d_tile_base;
        fp.spp = spp;
        sp.rec = s->d_samp;
        sp.rec_jy = s->d_samp_jy;
        if (sp.mode == RT_SPLAT_STREAM) {
            sp.ksmax = ks <= 2 ? 2 : ks <= 4 ? 4 : 12;
            sp.lds = tr_lds_bytes(sp.ksmax);
            const size_t npx = (size_t)w*h;
            const size_t parts = (size_t)std::max(shape.nparts - 1, 0);
            if (parts && s->partial_cap < parts*npx) {
                if (s->d_partials) (void)hipFree(s->d_partials);
                s->d_partials = nullptr; s->partial_cap = 0;
                HIP_OK(hipMalloc(&s->d_partials, sizeof(float4)*parts*npx));
                s->partial_cap = parts*npx;
            }
            sp.partials = s->d_partials;
            if (L.blocks_ks != ks) {
                // output blocks whose source region (the block + the filter radius) meets an owned tile
                std::vector<uint32_t> blocks;
                const uint32_t nbx = (w + TR_W - 1) / TR_W, nby = (h + TR_H - 1) / TR_H;
                for (uint32_t by = 0; by < nby; ++by)
                    for (uint32_t bx = 0; bx < nbx; ++bx) {
                        const int rx0 = std::max<int>((int)(bx*TR_W) - ks, 0), rx1 = std::min<int>((int)(bx*TR_W + TR_W - 1) + ks, (int)w - 1);
                        const int ry0 = std::max<int>((int)(by*TR_H) - ks, 0), ry1 = std::min<int>((int)(by*TR_H + TR_H - 1) + ks, (int)h - 1);
                        bool any = false;
                        for (int ty = ry0 / (int)fp.tile_h; ty <= ry1 / (int)fp.tile_h && !any; ++ty)
                            for (int tx = rx0 / (int)fp.tile_w; tx <= rx1 / (int)fp.tile_w && !any; ++tx)
                                any = L.base[(size_t)ty*fp.tcx + tx] >= 0;
                        if (any) blocks.push_back(bx | (by << 16));
                    }
                // XCD-aware order.  Blocks are dealt round robin over the 8 XCDs (b and b + 8 share one, each
                // with its own L2: MI355X_MICROARCH.md), so the list gives each XCD one contiguous run of the
                // blocks in column-major order: an XCD resolves its blocks top to bottom, and the filter-radius
                // rows a block stages above its own were read into that L2 by the block before it.  The sums
                // do not depend on the order (each pixel belongs to one block).
                {
                    std::vector<uint32_t> colmajor(blocks);
                    std::stable_sort(colmajor.begin(), colmajor.end(), [](uint32_t a, uint32_t b) {
                        return (a & 0xFFFFu) != (b & 0xFFFFu) ? (a & 0xFFFFu) < (b & 0xFFFFu) : (a >> 16) < (b >> 16);
                    });
                    // run x holds column-major positions [n*x/8, n*(x+1)/8); its k-th block goes to list
                    // position 8k + x (in the last round, when the runs differ by one, in order)
                    const size_t n = colmajor.size();
                    std::vector<size_t> start(NXCD + 1);
                    for (int x = 0; x <= NXCD; ++x) start[x] = n*(size_t)x / NXCD;
                    blocks.clear();
                    for (size_t k = 0; blocks.size() < n; ++k)
                        for (int x = 0; x < NXCD; ++x)
                            if (start[x] + k < start[x + 1]) blocks.push_back(colmajor[start[x] + k]);
                }
                const size_t aux = blocks.size() + 2*MAX_PARTITIONS;       // the pointer table, then the blocks
                if (s->aux_cap < aux) {
                    if (s->d_aux) (void)hipFree(s->d_aux);
                    s->d_aux = nullptr; s->aux_cap = 0;
                    HIP_OK(hipMalloc(&s->d_aux, sizeof(uint32_t)*aux));
                    s->aux_cap = aux;
                    L.aux_parts = -1;
                }
                HIP_OK(hipMemcpy(s->d_aux + 2*MAX_PARTITIONS, blocks.data(), sizeof(uint32_t)*blocks.size(), hipMemcpyHostToDevice));
                L.nblocks = (uint32_t)blocks.size();
                L.blocks_ks = ks;
            }
            if (L.aux_parts != (int)parts || L.aux_partials != s->d_partials || L.aux_npx != npx) {
                std::vector<const float4*> part_ptrs;
                for (size_t k = 0; k < parts; ++k) part_ptrs.push_back(s->d_partials + k*npx);
                if (parts) HIP_OK(hipMemcpy(s->d_aux, part_ptrs.data(), sizeof(float4*)*parts, hipMemcpyHostToDevice));
                L.aux_parts = (int)parts; L.aux_partials = s->d_partials; L.aux_npx = npx;
            }
            sp.nblocks = L.nblocks;
            sp.blocks = s->d_aux + 2*MAX_PARTITIONS;
            sp.part_ptrs = reinterpret_cast<const float4* const*>(s->d_aux);
            static bool attr_set = false;
            if (!attr_set) {                      // k_resolve_tiles<12> stages up to 72 KB
                HIP_OK(hipFuncSetAttribute((const void*)k_resolve_tiles<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tr_lds_bytes(2)));
                HIP_OK(hipFuncSetAttribute((const void*)k_resolve_tiles<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tr_lds_bytes(4)));
                HIP_OK(hipFuncSetAttribute((const void*)k_resolve_tiles<12>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tr_lds_bytes(12)));
                attr_set = true;
            }
        }
    }
    if (debug_timing()) fprintf(stderr, "[rt timing] rt_render_device: layout + splat plan %.3f ms\n", host_ms() - t_entry);
    err = run_frame(s, st, fp, total, stream, sp, stats, tiles->shard_count > 1);
    if (debug_timing()) fprintf(stderr, "[rt timing] rt_render_device: frame done %.3f ms after entry\n", host_ms() - t_entry);
    if (err || sp.mode != RT_SPLAT_EXACT) {
        if (!err) HIP_OK(hipStreamSynchronize(stream));      // the frame (and its last resolve, combine) is done
        if (stats && !err) stats->splat_mode = sp.mode;
        return err;
    }
    auto t0 = std::chrono::steady_clock::now();
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool prof_resolve = (g_profiling >> RT_KERNEL_RESOLVE) & 1u;
    if (prof_resolve) { HIP_OK(hipEventCreate(&e0)); HIP_OK(hipEventCreate(&e1)); HIP_OK(hipEventRecord(e0, stream)); }
    const uint64_t tall_px = s->cfg.resolve_tall_pixels > 0 ? (uint64_t)s->cfg.resolve_tall_pixels : RES_TALL_PIXELS;
    const bool tall = fp.pixels >= tall_px;
    const int rry = tall ? RES_RY_TALL : RES_RY;
    dim3 rgrid((w + RES_BX - 1) / RES_BX, (h + RES_BY*rry - 1) / (RES_BY*rry));
    if (tall) k_resolve<RES_RY_TALL><<<rgrid, RES_BX*RES_BY, 0, stream>>>(fp);
    else k_resolve<RES_RY><<<rgrid, RES_BX*RES_BY, 0, stream>>>(fp);
    HIP_OK(hipGetLastError());
    if (prof_resolve) HIP_OK(hipEventRecord(e1, stream));
    HIP_OK(hipStreamSynchronize(stream));
    if (stats) {
        stats->splat_mode = sp.mode;
        stats->seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (prof_resolve) {
            float ms = 0.0f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            stats->kernel_ms[RT_KERNEL_RESOLVE] += ms;
            stats->kernel_launches[RT_KERNEL_RESOLVE] += 1;
        }
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return RT_OK;
}

int rt_render(rt_scene* s, const rt_camera* camera, const rt_settings* st, const rt_filter_cache* filter,
              const rt_tile_set* tiles, uint32_t total_frame_index, rt_accumulation_buffer* accum, rt_stats* stats) {
    if (!s || !accum || !accum->pixels) { set_error("null argument"); return RT_ERROR_INVALID; }
    HIP_OK(hipSetDevice(s->device));
    size_t bytes = (size_t)accum->w*accum->h*4*sizeof(float);
    float* d = nullptr;
    HIP_OK(hipMalloc(&d, bytes));
    int err = RT_OK;
    if (hipMemcpy(d, accum->pixels, bytes, hipMemcpyHostToDevice) != hipSuccess) { set_error("copy in"); err = RT_ERROR_DEVICE; }
    if (!err) err = rt_render_device(s, camera, st, filter, tiles, total_frame_index, accum->w, accum->h,
                                     accum->frame_count, d, nullptr, stats);
    if (!err && hipMemcpy(accum->pixels, d, bytes, hipMemcpyDeviceToHost) != hipSuccess) { set_error("copy out"); err = RT_ERROR_DEVICE; }
    (void)hipFree(d);
    return err;
}

int rt_render_picture(rt_scene* s, const rt_camera* camera, const rt_settings* st, const rt_filter_cache* filter,
                      const rt_tile_set* tiles, uint32_t total_frame_index, uint32_t w, uint32_t h,
                      const rt_post_settings* post, uint32_t* out_bgra, rt_stats* stats) {
    if (!s || !post || !out_bgra || !w || !h) { set_error("null argument"); return RT_ERROR_INVALID; }
    HIP_OK(hipSetDevice(s->device));
    const size_t n = (size_t)w*h;
    float* d_px = nullptr;
    uint32_t* d_out = nullptr;
    HIP_OK(hipMalloc(&d_px, 16*n));
    if (hipMalloc(&d_out, 4*n) != hipSuccess) { (void)hipFree(d_px); set_error("hipMalloc"); return RT_ERROR_OUT_OF_MEMORY; }
    int err = RT_OK;
    if (hipMemset(d_px, 0, 16*n) != hipSuccess) { set_error("hipMemset"); err = RT_ERROR_DEVICE; }
    // discard_current_render + reset: a fresh buffer, frame_count 0 (RT/raytracer.cpp:2037-2041, :711-719)
    if (!err) err = rt_render_device(s, camera, st, filter, tiles, total_frame_index, w, h, 0u, d_px, nullptr, stats);
    // the frame completes with settings and camera unchanged, so render_all_tiles has moved
    // total_frame_index on (:720-724) before the output pass picks its dither texture (:2108)
    if (!err) err = rt_postprocess_device(s->device, d_px, w, h, post, total_frame_index + 1u, d_out, nullptr);
    if (!err && hipMemcpy(out_bgra, d_out, 4*n, hipMemcpyDeviceToHost) != hipSuccess) { set_error("copy out"); err = RT_ERROR_DEVICE; }
    (void)hipFree(d_px);
    (void)hipFree(d_out);
    return err;
}

int rt_trace_samples(rt_scene* s, const rt_camera* camera, const rt_settings* st,
                     uint32_t w, uint32_t h, uint32_t tile_w, uint32_t tile_h,
                     uint32_t frame_count, uint32_t total_frame_index,
                     uint32_t count, const uint32_t* pixel_xy, const uint32_t* sample_offset,
                     float* out, rt_stats* stats) {
    rt_filter_cache box = {};
    int err = check_inputs(st, &box);
    if (err) return err;
    if (!s || !camera || !pixel_xy || !sample_offset || !out || !w || !h || !tile_w || !tile_h) { set_error("null argument"); return RT_ERROR_INVALID; }
    if (!count) return RT_OK;
    if (w > 65535 || h > 65535) { set_error("frame larger than 65535 pixels a side"); return RT_ERROR_INVALID; }
    for (uint32_t i = 0; i < count; ++i)
        if (pixel_xy[2*i] >= w || pixel_xy[2*i + 1] >= h) { set_error("sample pixel out of range"); return RT_ERROR_INVALID; }
    HIP_OK(hipSetDevice(s->device));
    uint32_t* d_xy = nullptr; uint32_t* d_s = nullptr; float* d_out = nullptr;
    HIP_OK(hipMalloc(&d_xy, 8*(size_t)count));
    HIP_OK(hipMalloc(&d_s, 4*(size_t)count));
    HIP_OK(hipMalloc(&d_out, 20*(size_t)count));
    HIP_OK(hipMemcpy(d_xy, pixel_xy, 8*(size_t)count, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_s, sample_offset, 4*(size_t)count, hipMemcpyHostToDevice));
    FrameParams fp = {};
    fp.w = w; fp.h = h; fp.frame_count = frame_count; fp.total_frame_index = total_frame_index;
    fp.tile_w = tile_w; fp.tile_h = tile_h; fp.tcx = (w + tile_w - 1) / tile_w;
    fp.list_xy = d_xy; fp.list_s = d_s; fp.list_out = d_out;
    set_divisors(fp);
    fill_camera(fp, camera);
    err = run_frame(s, st, fp, count, nullptr, SplatCfg{}, stats, false);
    if (!err && hipMemcpy(out, d_out, 20*(size_t)count, hipMemcpyDeviceToHost) != hipSuccess) { set_error("copy out"); err = RT_ERROR_DEVICE; }
    (void)hipFree(d_xy); (void)hipFree(d_s); (void)hipFree(d_out);
    return err;
}

int rt_debug_mesh_bvh4(const rt_bvh_node* nodes, uint32_t node_count, float* out, uint32_t out_cap_nodes,
                       uint32_t* out_nodes, uint32_t* out_root_record) {
    if (!nodes || !node_count || !out_nodes || !out_root_record) { set_error("null argument"); return RT_ERROR_INVALID; }
    std::vector<float4> q;
    uint32_t root;
    if (nodes[0].count) {
        root = pack_node(0u, nodes[0].left_first, nodes[0].count, 0u);
    } else {
        bool ok = true;
        uint32_t need = 0;
        root = build_bvh4(nodes, node_count, 0u, q, need, ok);
        if (!ok) { set_error("BVH too large for the BVH4 records"); return RT_ERROR_INVALID; }
    }
    *out_nodes = (uint32_t)(q.size() / 8);
    *out_root_record = root;
    if (out && out_cap_nodes >= *out_nodes) memcpy(out, q.data(), q.size()*sizeof(float4));
    return (out && out_cap_nodes < *out_nodes) ? RT_ERROR_INVALID : RT_OK;
}

int rt_debug_top_sequences(const rt_bvh_node* nodes, uint32_t node_count, uint32_t index_count,
                           float* out, uint32_t out_cap_entries, uint32_t* out_len) {
    if (!nodes || !out_len) { set_error("null argument"); return RT_ERROR_INVALID; }
    uint32_t len = 0;
    std::vector<float4> q = top_sequences(nodes, node_count, index_count, len);
    *out_len = len;
    if (q.empty()) { set_error("top level too large for the prologue"); return RT_ERROR_INVALID; }
    if (out && out_cap_entries >= 8*len) memcpy(out, q.data(), q.size()*sizeof(float4));
    return (out && out_cap_entries < 8*len) ? RT_ERROR_INVALID : RT_OK;
}

int rt_debug_verify_rcp(int device, uint64_t* out_mismatches, uint32_t* out_first_bits) {
    if (!out_mismatches || !out_first_bits) { set_error("null argument"); return RT_ERROR_INVALID; }
    int err = bind_device(device);
    if (err) return err;
    unsigned long long* d = nullptr;
    HIP_OK(hipMalloc(&d, 2*sizeof(unsigned long long)));
    const unsigned long long init[2] = {0ull, 0xFFFFFFFFull};
    HIP_OK(hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice));
    for (uint32_t chunk = 0; chunk < 16; ++chunk)                 // 2^28 inputs per launch
        k_verify_rcp<<<(1u << 28) / (256*16), 256>>>(chunk << 28, d);
    HIP_OK(hipGetLastError());
    unsigned long long h[2];
    HIP_OK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    *out_mismatches = h[0];
    *out_first_bits = (uint32_t)h[1];
    return RT_OK;
}

int rt_debug_intersect(rt_scene* s, uint32_t count, const rt_ray_query* rays, int occlusion, rt_hit_record* out) {
    if (!s || !rays || !out) { set_error("null argument"); return RT_ERROR_INVALID; }
    if (!count) return RT_OK;
    HIP_OK(hipSetDevice(s->device));
    rt_ray_query* d_r = nullptr; rt_hit_record* d_o = nullptr;
    HIP_OK(hipMalloc(&d_r, sizeof(rt_ray_query)*count));
    HIP_OK(hipMalloc(&d_o, sizeof(rt_hit_record)*count));
    HIP_OK(hipMemcpy(d_r, rays, sizeof(rt_ray_query)*count, hipMemcpyHostToDevice));
    uint2* d_sp = nullptr;
    const uint32_t dgrid = (count + 127) / 128;
    HIP_OK(hipMalloc(&d_sp, sizeof(uint2)*(size_t)(STACK_DEPTH - STACK_LDS)*dgrid*128));
    if (occlusion) k_debug_intersect<true><<<dgrid, 128>>>(s->ds, d_r, d_o, count, d_sp);
    else k_debug_intersect<false><<<dgrid, 128>>>(s->ds, d_r, d_o, count, d_sp);
    HIP_OK(hipGetLastError());
    HIP_OK(hipDeviceSynchronize());
    (void)hipFree(d_sp);
    HIP_OK(hipMemcpy(out, d_o, sizeof(rt_hit_record)*count, hipMemcpyDeviceToHost));
    (void)hipFree(d_r); (void)hipFree(d_o);
    return RT_OK;
}

}  // extern "C"
