/*
 * oracle.h — CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 *
 * This library is the parity oracle and the CPU baseline.  It is NOT part of
 * the product: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / the timed CPU leg.
 *
 * It restates, in plain C11 + pthreads, the reference's
 *   render_tile            RT/raytracer.cpp:366-495
 *   advanced_integrator    RT/integrators.cpp:581-821
 *   intersect_scene[_internal] / intersect_shadow_ray   RT/intersection.cpp:411-610
 *   samplers + RNG         RT/samplers.h:3-108, RT/samplers.cpp:18-138
 *   splat_filter           RT/raytracer.cpp:187-259
 *   try_render_next_tile seeding  RT/raytracer.cpp:588-593
 * with deterministic transcendental functions (Cephes single-precision
 * algorithms, restated in the same operation order as the HIP kernels) and
 * -ffp-contract=off, so that in RT_RNG_PER_SAMPLE mode it is bit-comparable
 * with the GPU path.  RT_RNG_TILE_STREAM reproduces the reference's
 * per-tile RandomSeries consumption order.
 *
 * Parity pinning: see DESIGN.md §Oracle (reference KATs from
 * UnitTests/main.cpp:733-786, committed golden vectors under tests/golden/).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include "../include/rt_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Full frame, like rt_render.  threads <= 1 splats straight into `accum` in the
 * reference's single-thread order (tiles total-1 .. 0); threads > 1 renders
 * tiles in parallel into private tile buffers merged in that same order, so
 * the result is independent of the thread count. */
int oracle_render(const rt_scene_desc* scene, const rt_camera* camera, const rt_settings* settings,
                  const rt_filter_cache* filter, const rt_tile_set* tiles,
                  uint32_t total_frame_index, int rng_mode, int threads,
                  rt_accumulation_buffer* accum, rt_stats* stats);

/* Render only the tiles listed in tile_list (bounded CPU-baseline sample). */
int oracle_render_tiles(const rt_scene_desc* scene, const rt_camera* camera, const rt_settings* settings,
                        const rt_filter_cache* filter, uint32_t tile_w, uint32_t tile_h,
                        uint32_t total_frame_index, int rng_mode, int threads,
                        uint32_t tile_list_count, const uint32_t* tile_list,
                        rt_accumulation_buffer* accum, rt_stats* stats);

/* Same contract as rt_trace_samples (RT_RNG_PER_SAMPLE). */
int oracle_trace_samples(const rt_scene_desc* scene, const rt_camera* camera, const rt_settings* settings,
                         uint32_t w, uint32_t h, uint32_t tile_w, uint32_t tile_h,
                         uint32_t frame_count, uint32_t total_frame_index,
                         uint32_t count, const uint32_t* pixel_xy, const uint32_t* sample_offset,
                         float* out_rgbjj, rt_stats* stats);

/* Same contract as rt_debug_intersect. */
int oracle_debug_intersect(const rt_scene_desc* scene, uint32_t count, const rt_ray_query* rays,
                           int occlusion, rt_hit_record* out);

/* The output pass (RT/raytracer.cpp:2103-2171): resolve, exposure, tonemap, sRGB,
 * contrast, TPDF dither (LDR_RGB1 texture total_frame_index % 8), BGRA8.  remap_tpdf's
 * rsqrtss is 1/sqrtf here (and on the GPU); transcendentals follow oracle_set_math_mode. */
void oracle_postprocess(const rt_accumulation_buffer* accum, const rt_post_settings* post,
                        uint32_t total_frame_index, uint32_t* out_bgra);

/* ---- known-answer helpers (unit tests / golden vectors) ---------------- */
uint32_t oracle_wang_hash(uint32_t key);
uint32_t oracle_sample_seed(uint32_t total_frame_index, uint32_t frame_count, uint32_t tile_index,
                            uint32_t pixel_id, uint32_t canonical_sample_index);
/* random_seed(seed) then `count` random_unilaterals() calls -> out[4*count] */
void     oracle_rng_unilaterals(uint32_t seed, uint32_t count, float* out);
/* get_next_sample_2d for (x,y,index,dim,bounce) with a fresh random_seed(seed) */
void     oracle_sample_2d(uint32_t seed, int strategy, uint32_t x, uint32_t y, uint32_t index,
                          int dimension, uint32_t bounce, float* out2);
float    oracle_sample_1d(uint32_t seed, int strategy, uint32_t x, uint32_t y, uint32_t index,
                          int dimension, uint32_t bounce);
/* ray_intersect_plane / ray_intersect_sphere exactly as RT/intersection.cpp:12-74 */
int      oracle_ray_intersect_plane(const float* o, const float* d, const float* n, float dist, float* inout_t);
int      oracle_ray_intersect_sphere(const float* o, const float* d, float r, float* inout_t);
/* deterministic transcendentals shared (as a spec) with the HIP kernels */
float    oracle_sinf(float x);
float    oracle_cosf(float x);
float    oracle_expf(float x);
float    oracle_logf(float x);
float    oracle_atan2f(float y, float x);
float    oracle_asinf(float x);
/* 0 = deterministic spec transcendentals (default), 1 = C library (pins vs the reference) */
void     oracle_set_math_mode(int libm);
/* 1 = environment-map sampling in the NEE, as rt_set_env_sampling (include/rt_abi.h); 0 = off */
void     oracle_set_env_sampling(int mode);
/* rt_stats::traversal of the oracle's renders is the reference's own TraversalStats (BVH2 pops,
 * its front-to-back walk; RT/intersection.cpp:254, :378-380).  The GPU library counts its own walk
 * (rt_abi.h).  oracle_gpu_walk_stats(1, ...) additionally restates that walk in every query of the
 * following renders (the prologue's order, mlist_max = RT_MLIST_MAX of the GPU run, top_prologue = 0
 * as RT_TOP_PROLOGUE=0) and resets the sums; oracle_gpu_walk_result gives them per kind (closest-hit,
 * then shadow), five each: mesh instances reached (the GPU's mesh_intersection_count), mesh instances
 * entered by the trace kernels, leaves entered (mesh_leaf_traversals), BVH4 interior nodes expanded
 * (mesh_node_traversals), triangle steps (mesh_bvh_traversals = entered + nodes + triangle steps). */
void     oracle_gpu_walk_stats(int on, uint32_t mlist_max, int top_prologue);
void     oracle_gpu_walk_result(uint64_t out[10]);
/* Mitchell–Netravali and friends (RT/reconstruction_filters.cpp:8-95) + LUT */
int      oracle_load_filter(const char* name, rt_filter_cache* out);

#ifdef __cplusplus
}
#endif
#endif
