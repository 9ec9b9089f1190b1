/*
 * rt_abi.h — C ABI of the MI355X wavefront path tracer (drop-in for the
 * reference's tile renderer hot path).
 *
 * The reference (TheSandvichMaker/BUAS-Pathtracer) renders a frame as
 *   render_all_tiles (RT/raytracer.cpp:692)
 *     -> worker threads -> try_render_next_tile (:551)
 *       -> render_tile (:366) -> per pixel, per sample:
 *            scene->settings.integrator->f(&state)   (:467, advanced_integrator
 *                                                     RT/integrators.cpp:581-821)
 *            splat_filter(...)                       (:187-259)
 * into an AccumulationBuffer{w,h,frame_count,V4* pixels} (RT/Raytracer.h:44-48).
 *
 * Per-sample function pointers are far too fine-grained for a GPU, so this
 * ABI replaces the path at frame / tile-set granularity:
 * rt_render() consumes the same Scene / Material / Camera / SceneSettings /
 * FilterCache data (flattened to plain arrays: pointers become indices) and
 * fills the same float4 accumulation buffer.
 *
 * Everything here is plain C: POD structs, pointers and sizes, no C++ or
 * torch types.  Every function returns an int status (RT_OK == 0); on error
 * rt_last_error() returns a thread-local message.
 *
 * RT/ = /root/reference/Raytracer/,  MathLib/ = /root/reference/MathLib/.
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 8

/* ---------------------------------------------------------------- status */
enum rt_status {
    RT_OK                 = 0,
    RT_ERROR_INVALID      = 1,  /* bad argument / unsupported setting      */
    RT_ERROR_DEVICE       = 2,  /* HIP runtime failure                     */
    RT_ERROR_OUT_OF_MEMORY= 3,
    RT_ERROR_CANCELLED    = 4,  /* rt_cancel() hit during rt_render()      */
    RT_ERROR_NO_DEVICE    = 5,  /* no MI355X visible: the product path never
                                   falls back to a CPU implementation      */
};

/* ------------------------------------------------------------ math types */
typedef struct rt_v3 { float x, y, z; } rt_v3;                 /* MathLib/math_types.h:12-17 */
typedef struct rt_m4x4 { float e[4][4]; } rt_m4x4;             /* MathLib/math_types.h:43-45 */
typedef struct rt_m4x4inv { rt_m4x4 forward, inverse; } rt_m4x4inv; /* :47-50 */

/* ----------------------------------------------------------- scene model */
enum rt_material_flag {                                        /* RT/scene.h:9-13 */
    RT_MATERIAL_MIRROR   = 0x1,
    RT_MATERIAL_CHECKERS = 0x2,
    RT_MATERIAL_EMISSIVE = 0x4,
};

typedef struct rt_material {                                   /* RT/scene.h:15-29 (68 B) */
    uint32_t flags;
    rt_v3    albedo;
    rt_v3    checker_color;
    rt_v3    emission_color;
    float    ior;
    float    metallic;
    float    roughness;
    int32_t  is_participating_medium;
    rt_v3    absorb;                                           /* Medium::absorb */
} rt_material;

enum rt_primitive_type {                                       /* RT/primitives.h:3-10 */
    RT_PRIMITIVE_NONE   = 0,
    RT_PRIMITIVE_PLANE  = 1,
    RT_PRIMITIVE_SPHERE = 2,
    RT_PRIMITIVE_BOX    = 3,
    RT_PRIMITIVE_MESH   = 4,
};

typedef struct rt_primitive {                                  /* RT/primitives.h:92-106 */
    uint32_t transform_index;  /* Primitive::transform -> index into transforms[] */
    uint32_t material_id;      /* MaterialID */
    uint32_t type;             /* rt_primitive_type */
    uint32_t mesh_index;       /* RT_PRIMITIVE_MESH: index into meshes[] */
    float    p[4];             /* plane: n.xyz, d | sphere: r | box: r.xyz */
} rt_primitive;

typedef struct rt_bvh_node {                                   /* RT/bvh.h:31-37 (32 B) */
    rt_v3    bv_p;             /* centre      */
    rt_v3    bv_r;             /* half extent */
    uint32_t left_first;       /* interior: left child (right = +1); leaf: first index */
    uint16_t count;            /* > 0 => leaf */
    uint16_t split_axis;
} rt_bvh_node;

typedef struct rt_mesh {               /* RT/primitives.h:58-67 + MeshBVH RT/bvh.h:52-58 */
    uint32_t            triangle_count;
    uint32_t            has_normals;
    const rt_v3*        triangles;  /* MeshBVH::triangles: BVH order, a,b,c per triangle */
    const uint32_t*     indices;    /* MeshBVH::indices: BVH slot -> original triangle  */
    const rt_v3*        normals;    /* get_normals(mesh): ORIGINAL order, 3 per triangle */
    uint32_t            node_count;
    const rt_bvh_node*  nodes;      /* BVHStorage_Scalar layout (node 1 is padding)      */
} rt_mesh;

typedef struct rt_scene_desc {                                 /* RT/scene.h:92-120 */
    uint32_t            material_count;   const rt_material*  materials;  /* [0] null material  */
    uint32_t            primitive_count;  const rt_primitive* primitives; /* [0] null primitive */
    uint32_t            plane_count;      const rt_primitive* planes;     /* Scene::planes      */
    uint32_t            transform_count;  const rt_m4x4inv*   transforms;
    uint32_t            light_count;      const uint32_t*     lights;     /* PrimitiveIDs       */
    uint32_t            mesh_count;       const rt_mesh*      meshes;
    uint32_t            bvh_node_count;   const rt_bvh_node*  bvh_nodes;  /* Scene::bvh         */
    uint32_t            bvh_index_count;  const uint32_t*     bvh_indices;
    rt_v3               top_sky_color;
    rt_v3               bot_sky_color;
    uint32_t            skydome_w, skydome_h;
    const rt_v3*        skydome;          /* EnvironmentMap pixels (Image_V3), NULL = sky colours */
} rt_scene_desc;

typedef struct rt_camera {                                     /* RT/scene.h:31-46 */
    rt_v3 p, x, y, z;
    float vfov;
    float aspect_ratio;
    float lens_radius;
    float focus_distance;
    float film_distance;
    float half_film_w;
    float half_film_h;
} rt_camera;

enum rt_sampling_strategy {                                    /* RT/samplers.h:110-117 */
    RT_SAMPLING_UNIFORM              = 0,
    RT_SAMPLING_OPTIMIZED_BLUE_NOISE = 1,
    RT_SAMPLING_STRATIFIED           = 2,
};

enum rt_integrator {                                           /* g_integrators RT/integrators.cpp:823 */
    RT_INTEGRATOR_ADVANCED = 0,   /* "Advanced Pathtracer" — the only one on the hot path */
};

typedef struct rt_settings {                                   /* RT/scene.h:64-82 */
    int32_t  next_event_estimation;
    int32_t  importance_sample_lights;
    int32_t  importance_sample_diffuse;
    int32_t  use_mis;
    int32_t  russian_roulette;
    int32_t  caustics;
    int32_t  sampling_strategy;     /* rt_sampling_strategy */
    int32_t  use_path_guide;        /* must be 0 (dead code in the reference) */
    float    vignette_strength;
    float    lens_distortion;
    float    f_factor;
    float    diaphragm_edges;
    float    phi_shutter_max;
    uint32_t samples_per_pixel;
    uint32_t max_bounce_count;      /* <= 63: the material stack holds 64 entries */
    int32_t  integrator;            /* rt_integrator (SceneSettings::integrator) */
} rt_settings;

typedef struct rt_filter_cache {                               /* FilterCache RT/Raytracer.h:34-40 */
    uint32_t kernel_size;           /* filter radius in pixels; 0 => box (plain accumulate) */
    uint32_t cache_size;            /* 256 when a kernel is loaded, 0 for the box filter    */
    float    cache[512];            /* load_reconstruction_kernel RT/raytracer.cpp:164-185 */
} rt_filter_cache;

typedef struct rt_accumulation_buffer {                        /* RT/Raytracer.h:44-48 */
    uint32_t w, h;
    uint32_t frame_count;
    float*   pixels;                /* w*h float4 (xyz = weighted radiance, w = weight) */
} rt_accumulation_buffer;

typedef struct rt_post_settings {   /* PostProcessSettings RT/scene.h:84-90 */
    float   exposure;               /* stops: colour *= 2^exposure when != 0 */
    int32_t tonemapping;            /* 1 - exp(-x) */
    int32_t srgb_transform;         /* x^(1/2.23333) */
    float   midpoint;               /* sigmoidal_contrast (RT/raytracer.cpp:69-84) */
    float   contrast;
} rt_post_settings;

typedef struct rt_tile_set {        /* WorkQueue tiling RT/Raytracer.h:70-91 + sharding */
    uint32_t tile_w, tile_h;        /* 64x64 in the reference (RT/raytracer.cpp:1657) */
    uint32_t shard_index;           /* this GPU renders tiles t with t % shard_count == shard_index */
    uint32_t shard_count;
} rt_tile_set;

enum rt_rng_mode {
    /* One xorshift RandomSeries per sample, seeded from
     * (total_frame_index, frame_count, tile_index, pixel, sample): the draw
     * order inside a sample is exactly the reference's.  The GPU path. */
    RT_RNG_PER_SAMPLE  = 0,
    /* One RandomSeries per 64x64 tile consumed serially in pixel/sample order,
     * exactly RT/raytracer.cpp:588-593 (CPU oracle only). */
    RT_RNG_TILE_STREAM = 1,
};

enum rt_kernel_id {                 /* wavefront stages, for rt_stats::kernel_ms */
    RT_KERNEL_GENERATE = 0,         /* camera rays (render_tile ray setup)               */
    RT_KERNEL_EXTEND   = 1,         /* closest hit (intersect_scene)                     */
    RT_KERNEL_SHADE    = 2,         /* one bounce of advanced_integrator                 */
    RT_KERNEL_CONNECT  = 3,         /* shadow rays (intersect_shadow_ray)                */
    RT_KERNEL_SPLAT    = 4,         /* finished samples -> records (or atomic splat)     */
    RT_KERNEL_RESOLVE  = 5,         /* splat_filter as a gather in reference order       */
    RT_KERNEL_COUNT    = 6,
};

/* The reference's TraversalStats (RT/intersection.h:33-40): render_all_tiles hands them to its
 * caller and zeroes them every frame (RT/raytracer.cpp:727-731); intersect_mesh counts them
 * (RT/intersection.cpp:254, :378-380).  Here they are counted on the device, per frame, in this
 * library's own walk, whose order and layout differ from the reference's in two documented ways
 * (DESIGN.md section 3):
 *   - the top level is walked in one fixed order with the planes, spheres and boxes tested before
 *     any mesh BVH (the hits are the reference's), so t at a top-level node does not yet include
 *     the mesh hits the reference's front-to-back walk would have found;
 *   - mesh BVHs are BVH4s (each BVH2 interior node merged with its interior children), and a child
 *     is box-tested when its parent is expanded instead of when it is popped.
 * A shadow query that a mesh occludes is counted like any other (the reference returns before its
 * traversal counts are added, RT/intersection.cpp:297-299).
 * So these values are NOT comparable to the reference's own TraversalStats for the same frame (C3:
 * mesh_bvh_traversals 3.6 G BVH4 steps against the reference's 10.4 G BVH2 pops); tests pin them
 * against the oracle's restatement of this library's walk (tests/test_gpu_fullscale.py). */
typedef struct rt_traversal_stats {
    /* intersect_mesh calls (RT/intersection.cpp:488, counted at :254): mesh instances a query's
       top-level walk reaches -- the top-level leaf holding the instance passes its pop-time test
       (:454), the instance is not the query's ignored light (:466), and no plane, sphere or box has
       occluded a shadow query before it */
    uint64_t mesh_intersection_count;
    /* mesh BVH steps: each one round of 8 x 16-byte loads per lane -- an instance's entry (its
       object-space ray, RT/intersection.cpp:472, and its root box test), a BVH4 interior node, or up
       to two triangles of a leaf.  (Reference: BVH2 nodes taken from the stack, :274.) */
    uint64_t mesh_bvh_traversals;
    /* BVH4 interior nodes expanded: taken from the stack with their far-clip test passed.
       (Reference: BVH2 interior nodes that pass their pop-time test, :358.) */
    uint64_t mesh_node_traversals;
    /* mesh BVH leaves entered: taken from the stack with their far-clip test passed -- the
       reference's definition (:279); the BVH4 has the BVH2's leaves */
    uint64_t mesh_leaf_traversals;
} rt_traversal_stats;

typedef struct rt_stats {
    uint64_t closest_hit_rays;      /* intersect_scene calls (RT/integrators.cpp:615)      */
    uint64_t shadow_rays;           /* intersect_shadow_ray calls (RT/integrators.cpp:756) */
    uint64_t samples;               /* camera samples integrated                            */
    uint64_t iterations;            /* wavefront iterations (GPU) / 0 (CPU)                 */
    double   seconds;               /* wall time of the render call                         */
    /* filled only while rt_set_profiling(1): HIP-event time per stage, summed over
       launches, measured on the stream the stage kernels run on */
    double   kernel_ms[RT_KERNEL_COUNT];
    uint64_t kernel_launches[RT_KERNEL_COUNT];
    /* rays handed to the trace kernels (closest, shadow): the rest were settled by
       the planes / top-level root test where they were made (GPU only) */
    uint64_t traced_rays[2];
    int32_t  splat_mode;            /* rt_splat_mode the frame used (rt_render / rt_render_device) */
    int32_t  shadow_launch;         /* (ABI 8) rt_shadow_launch the frame used: SEPARATE or MERGED */
    /* TraversalStats of the frame (above) per query kind: [0] closest-hit (intersect_scene),
       [1] shadow (intersect_shadow_ray); the reference's totals are the sums of the two */
    rt_traversal_stats traversal[2];
    /* trace steps per kind of the extend / connect kernels (top-level steps included; r05: the fused
       drain's steps, which the TraversalStats above include, are left out, so that the steps match the
       launches bench.py times): the fetch rounds of 128 B per lane the traversal roofline counts */
    uint64_t trace_steps[2];
    /* (ABI 7) The reference's own TraversalStats units, filled only when rt_scene_config::traversal_ref
       is set (zero otherwise): per query kind, intersect_mesh calls and the BVH2 counts of the
       reference's walk -- nodes taken from the stack (RT/intersection.cpp:274), interior nodes (:358)
       and leaves (:279) passing their pop-time test -- with its top-level order and its early return
       (a shadow query that a mesh occludes adds no traversal counts, :297-299).  These are the numbers
       the reference's UI prints (RT/raytracer.cpp:2050-2056); tests/test_gpu_fullscale.py holds them to
       the oracle's reference walk of the same frame. */
    rt_traversal_stats traversal_ref[2];
} rt_stats;

typedef struct rt_ray_query {       /* debug/parity entry: one ray for rt_debug_intersect */
    rt_v3    o, d;
    float    max_t;
    uint32_t ignored_primitive;     /* 0 for closest hit; light id for shadow rays */
} rt_ray_query;

typedef struct rt_hit_record {
    float    t;
    uint32_t primitive;             /* primitive index, or RT_HIT_PLANE_BIT|plane index; 0xFFFFFFFF = miss */
    rt_v3    hit_p;
    rt_v3    n;
} rt_hit_record;

#define RT_HIT_MISS       0xFFFFFFFFu
#define RT_HIT_PLANE_BIT  0x80000000u

/* ------------------------------------------------------------ functions */
typedef struct rt_scene rt_scene;   /* device-resident scene (opaque) */

int         rt_abi_version(void);
const char* rt_last_error(void);
int         rt_device_count(int* out_count);

/* Upload a flattened scene to `device` (create_scene_bvh must have run on
 * the host: RT/scene.cpp:173-242).  The device copy is owned by *out. */
int rt_scene_upload(const rt_scene_desc* desc, int device, rt_scene** out);
int rt_scene_free(rt_scene* scene);

/* Render one progressive frame: the equivalent of render_all_tiles releasing
 * its workers over every tile of `tiles` (RT/raytracer.cpp:692-757), with
 * accum->frame_count as the canonical sample base (RT/raytracer.cpp:427-428).
 * accum->pixels is HOST memory; samples are ADDED to it (the caller resets it
 * exactly as reset() does, RT/raytracer.cpp:511-515). */
int rt_render(rt_scene* scene, const rt_camera* camera, const rt_settings* settings,
              const rt_filter_cache* filter, const rt_tile_set* tiles,
              uint32_t total_frame_index, rt_accumulation_buffer* accum, rt_stats* stats);

/* Same, but d_pixels is a DEVICE pointer (w*h float4 on the scene's device)
 * and `hip_stream` (hipStream_t, may be NULL) is the stream the work is
 * ordered on.  Returns after the frame has completed on the device. */
int rt_render_device(rt_scene* scene, const rt_camera* camera, const rt_settings* settings,
                     const rt_filter_cache* filter, const rt_tile_set* tiles,
                     uint32_t total_frame_index, uint32_t w, uint32_t h, uint32_t frame_count,
                     float* d_pixels, void* hip_stream, rt_stats* stats);

/* The frame of the reference's "Take picture" (RT/raytracer.cpp:2031-2048, :2089-2176):
 * renders total_frame_index's frame of settings->samples_per_pixel samples per pixel
 * into a fresh device buffer (frame_count 0), then runs the output pass on the device
 * (rt_postprocess_device) with the dither texture of total_frame_index + 1 -- the frame
 * completing advances the index before the output pass reads it (:720-724, :2108) -- and
 * copies the BGRA8 picture (w*h u32, host) out.  write_bitmap is the caller's. */
int rt_render_picture(rt_scene* scene, const rt_camera* camera, const rt_settings* settings,
                      const rt_filter_cache* filter, const rt_tile_set* tiles, uint32_t total_frame_index,
                      uint32_t w, uint32_t h, const rt_post_settings* post, uint32_t* out_bgra, rt_stats* stats);

/* Parity entry: integrate an explicit list of samples (pixel x,y + sample
 * offset s, canonical index = frame_count + s) with RT_RNG_PER_SAMPLE and
 * return, per sample, {r, g, b, jitter_x, jitter_y} (radiance after
 * vignetting, the value splat_filter receives).  Host pointers. */
int rt_trace_samples(rt_scene* scene, const rt_camera* camera, const rt_settings* settings,
                     uint32_t w, uint32_t h, uint32_t tile_w, uint32_t tile_h,
                     uint32_t frame_count, uint32_t total_frame_index,
                     uint32_t count, const uint32_t* pixel_xy, const uint32_t* sample_offset,
                     float* out_rgbjj, rt_stats* stats);

/* Parity entry: intersect_scene (closest hit, occlusion = 0) or
 * intersect_shadow_ray (occlusion = 1) for `count` rays (RT/intersection.cpp:600-610). */
int rt_debug_intersect(rt_scene* scene, uint32_t count, const rt_ray_query* rays,
                       int occlusion, rt_hit_record* out);

/* Verification entries for the device layouts built at rt_scene_upload (host only,
 * no device needed).  rt_debug_mesh_bvh4: the BVH4 a mesh BVH2 (the caller's
 * BVHNode array, RT/bvh.h:31-37) is traversed as, 8 x float4 per node (SoA
 * children: p.x[4] p.y[4] p.z[4] r.x[4] r.y[4] r.z[4], packed records[4], split
 * axes); interior records are node indices, leaf records bit 30 | count << 25 |
 * first, 0xFFFFFFFF no child.  rt_debug_top_sequences: the top level as the ray
 * prologue walks it, per direction octant (bit k = d[k] < 0) node_count entries of
 * 2 x float4 {bv_p, bv_r.x}, {bv_r.yz, leaf info (0x80000000 | count << 24 | first,
 * 0 interior), skip (the entry after the subtree)}.  Both return RT_ERROR_INVALID
 * when the tree does not fit the layout, and write the counts they need. */
int rt_debug_mesh_bvh4(const rt_bvh_node* nodes, uint32_t node_count, float* out, uint32_t out_cap_nodes,
                       uint32_t* out_nodes, uint32_t* out_root_record);
int rt_debug_top_sequences(const rt_bvh_node* nodes, uint32_t node_count, uint32_t index_count,
                           float* out, uint32_t out_cap_entries, uint32_t* out_len);

/* Exhaustive check of the kernels' fast reciprocal (3 instructions instead of the
 * division expansion) against the correctly rounded IEEE 1.0f / x on `device`: every
 * one of the 2^32 bit patterns (NaNs compare equal as NaNs).  Writes the number of
 * mismatching inputs and the smallest mismatching bit pattern (0xFFFFFFFF: none). */
int rt_debug_verify_rcp(int device, uint64_t* out_mismatches, uint32_t* out_first_bits);

/* The output pass of RT/raytracer.cpp:2103-2171 on the device: per pixel resolve
 * (xyz / w), exposure, 1-exp(-x) tonemap, sRGB power, sigmoidal contrast, x255,
 * TPDF dither from the reference's LDR_RGB1 blue-noise texture number
 * total_frame_index % 8 (RT/assets.cpp:63-113), clamp, BGRA8 pack; NaN pixels
 * become (0,255,255), negative weights magenta.  d_pixels (w*h float4) and d_bgra
 * (w*h u32) are DEVICE pointers on `device`; `hip_stream` may be NULL.
 * remap_tpdf's rsqrtss (an approximation whose bits differ between CPU models)
 * is computed as 1/sqrt, correctly rounded. */
int rt_postprocess_device(int device, const float* d_pixels, uint32_t w, uint32_t h,
                          const rt_post_settings* post, uint32_t total_frame_index,
                          uint32_t* d_bgra, void* hip_stream);

/* Same, from and to host memory (accum->pixels in, out_bgra w*h u32 out). */
int rt_postprocess(int device, const rt_accumulation_buffer* accum, const rt_post_settings* post,
                   uint32_t total_frame_index, uint32_t* out_bgra);

/* The reference's top-down BVH builders on the device (RT/bvh.cpp:222-326 with
 * partition_midpoint :53-61 or partition_sah_binned :138-213, the partition of :26-51):
 * one launch per tree level, one workgroup per node.  Bit-identical to the sequential
 * recursion: out_nodes holds the reference's BVHNode array (root 0, node 1 padding,
 * children pairs in its order; capacity 2n + 2 nodes), out_order[i] the entry index at
 * position i of the partitioned entry array (BVHSortEntry::index).  Entries are the
 * centre p and half extent r of each primitive's or triangle's box (BVHSortEntry,
 * RT/bvh.h:25-29).  Host pointers; returns an rt_status (text: rt_build_bvh_last_error). */
enum rt_bvh_build_method {
    RT_BVH_BUILD_MIDPOINT   = 0,    /* BVH_MidpointSplit */
    RT_BVH_BUILD_SAH_BINNED = 1,    /* BVH_SAHBinned (16 bins) */
};
int rt_build_bvh(int device, uint32_t n, const rt_v3* p, const rt_v3* r, int method,
                 rt_bvh_node* out_nodes, uint32_t* out_node_count, uint32_t* out_order);
const char* rt_build_bvh_last_error(void);

/* Record per-stage HIP-event timings into rt_stats::kernel_ms (off by default). */
int rt_set_profiling(int enable);
/* The same for a subset of stages: bit k = stage k of rt_kernel_stage (other stages
 * record no events, so their launches are not slowed by the markers). */
int rt_set_profiling_stages(uint32_t mask);

/* Size of the in-flight path pool per partition (paths resident in HBM); 0 = default:
 * a fifth of the partition's samples, clamped to [2^21, 4 x 2^21]. */
int rt_set_path_pool(uint32_t paths);

/* How samples reach the accumulation buffer (splat_filter, RT/raytracer.cpp:187-259).
 *   RT_SPLAT_STREAM (default): each sample's 20-byte record goes to a ring of sample passes
 *     in HBM; k_resolve_tiles gathers completed passes into the buffer while the frame still
 *     renders, reading every record once.  Deterministic (the same bits whatever the timing
 *     or the split of passes between launches); equal to the reference's frame up to float
 *     summation order.
 *   RT_SPLAT_EXACT: records of the whole frame, then one gather in the reference's
 *     single-threaded order (tiles descending, pixels, samples): bit-identical to the
 *     reference order.  Over the HBM budget it renders as RT_SPLAT_STREAM.
 *   RT_SPLAT_ATOMIC: float atomics into the buffer (order-dependent last bits).
 * The mode a frame used is reported in rt_stats::splat_mode. */
enum rt_splat_mode {
    RT_SPLAT_STREAM = 0,
    RT_SPLAT_EXACT  = 1,
    RT_SPLAT_ATOMIC = 2,
};
int rt_set_splat_mode(int mode);

/* What rt_tile_set::shard_index / shard_count split a frame by (multi-GPU: one shard per rank,
 * the ranks' frames summed).  Either way every sample keeps its own key (frame, tile, pixel,
 * sample), so the shards' frames sum to the single-GPU frame up to float summation order.
 *   RT_SHARD_TILES (default): tile t belongs to shard t % shard_count (the reference's tile
 *     queue, RT/raytracer.cpp:551-560, dealt out round robin).
 *   RT_SHARD_PASSES: every tile, sample passes [spp*i/n, spp*(i+1)/n) of shard i of n: each
 *     shard sees the whole image, so the shards' costs match whatever the content.  The
 *     exact splat (RT_SPLAT_EXACT) is not split this way: such frames use RT_SPLAT_STREAM. */
enum rt_shard_mode {
    RT_SHARD_TILES  = 0,
    RT_SHARD_PASSES = 1,
};
int rt_set_shard_mode(int mode);

/* Environment-map importance sampling for next event estimation; 0 (default) = off.
 * The reference builds a luma CDF over 32 x 32 tiles of the environment map
 * (load_environment_map, RT/assets.cpp:620-665) but never samples it
 * (sample_environment_map is a stub, RT/integrators.cpp:230-233), so mode 0 is the
 * reference's estimator.  Mode 1, for scenes with an environment map and with
 * next_event_estimation on: a diffuse vertex's NEE picks the environment with probability
 * 1/2 (1 when the scene has no lights; a sphere light is then picked as before, its
 * probability halved), draws a tile with probability proportional to its luma (an alias
 * table built from the same tile sums at rt_scene_upload) and a uniform point in it, and
 * casts an unbounded shadow ray.  A path that leaves a diffuse vertex and escapes is
 * weighted against that pdf by the balance heuristic (use_mis; without MIS the
 * environment reaches diffuse vertices through the NEE only, as lights do in the
 * reference).  The estimate's expectation is unchanged; its noise is not the reference's.
 * No effect for scenes without an environment map (or one under 32 x 32 texels). */
int rt_set_env_sampling(int mode);

/* discard_current_render (RT/raytracer.cpp:686-690): polled between wavefront
 * iterations; the render in flight returns RT_ERROR_CANCELLED. */
int rt_cancel(rt_scene* scene);

/* Per-scene configuration of the wavefront schedule and the splat (none of it changes a
 * sample's bits; splat_mode and partitions change the float summation order of a pixel).
 * Two scenes in one process may differ.  rt_scene_upload starts a scene from
 * rt_scene_default_config(), then applies the test-override environment variables once
 * (RT_SPLAT, RT_PARTITIONS, RT_FUSE_PATHS, RT_SPLAT_CHUNK, RT_SPLAT_RING,
 * RT_SAMPLE_BUDGET_GB, RT_RES_TALL_PIXELS, RT_DEBUG_TRAVERSAL, RT_DRAIN_EVERY, RT_SHADOW_LAUNCH);
 * nothing reads the
 * environment per frame.  A field at RT_CONFIG_INHERIT follows the process-wide setter
 * above at each frame (rt_set_splat_mode / rt_set_shard_mode / rt_set_env_sampling /
 * rt_set_path_pool), so callers of those setters see no change. */
#define RT_CONFIG_INHERIT (-1)
/* rt_scene_config::shadow_launch (ABI 8): the shadow rays of an iteration's k_shade are traced in a launch
 * of their own right after it (SEPARATE), or in the next iteration's trace launch after its extension rays
 * (MERGED: one launch and one tail less per iteration; a finished path is splatted an iteration later).
 * AUTO: merged for a shard of a multi-rank frame (rt_tile_set::shard_count > 1), for path pools under
 * 4M paths (small frames), and for a whole frame on one GPU when the scene's previous frame traced at least
 * 0.15 shadow rays per extension ray (rt_stats::traced_rays); else separate -- a scene's first whole frame
 * is separate. */
typedef enum rt_shadow_launch {
    RT_SHADOW_LAUNCH_AUTO = 0,
    RT_SHADOW_LAUNCH_SEPARATE = 1,
    RT_SHADOW_LAUNCH_MERGED = 2
} rt_shadow_launch;
typedef struct rt_scene_config {
    int32_t  splat_mode;            /* rt_splat_mode, or RT_CONFIG_INHERIT                          */
    int32_t  shard_mode;            /* rt_shard_mode, or RT_CONFIG_INHERIT                          */
    int32_t  env_sampling;          /* 0 / 1, or RT_CONFIG_INHERIT                                  */
    int32_t  partitions;            /* concurrent partitions (streams) per frame, 1..8; 0 = auto (4) */
    int64_t  path_pool;             /* in-flight paths per partition; 0 = rt_set_path_pool / auto    */
    int64_t  fuse_paths;            /* fused drain below this many live paths; -1 = auto, 0 = never */
    int32_t  splat_chunk;           /* streaming splat: passes per resolve; 0 = auto                 */
    int32_t  splat_ring;            /* streaming splat: record-ring passes per partition; 0 = auto   */
    double   sample_budget_gb;      /* HBM for sample records; < 0 = auto (free HBM less 16 GB)      */
    int64_t  resolve_tall_pixels;   /* exact splat: 8-row gather strips from this many pixels; 0 = auto */
    int32_t  debug_traversal;       /* 1: each frame's TraversalStats and trace steps to stderr      */
    int32_t  traversal_ref;         /* 1: also count rt_stats::traversal_ref (the reference's units);
                                       the trace kernels then walk the top level in the reference's
                                       order (slower: no prologue mesh lists) -- a diagnostic mode  */
    int32_t  drain_every;           /* (ABI 8) fused-drain kernels ride on every Nth iteration once the
                                       host expects the drain (N >= 1; 0 = auto: every iteration).  A
                                       schedule knob for the tests: frames are identical for every N */
    int32_t  shadow_launch;         /* (ABI 8) rt_shadow_launch: where the NEE shadow rays are traced.
                                       Frames are identical for every value */
    int32_t  reserved[4];
} rt_scene_config;
int rt_scene_default_config(rt_scene_config* out);
int rt_scene_get_config(const rt_scene* scene, rt_scene_config* out);
int rt_scene_set_config(rt_scene* scene, const rt_scene_config* config);

#ifdef __cplusplus
}
#endif

#endif /* RT_ABI_H */
