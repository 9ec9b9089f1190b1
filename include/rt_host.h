/*
 * rt_host.h — host-side scene model of the MI355X path tracer (C ABI).
 *
 * Mirrors the reference's host code that feeds the hot path, so a caller of
 * the reference finds the same operations:
 *   add_material / add_diffuse_material / add_translucent_material /
 *   add_emissive_material / add_plane / add_sphere / add_box / add_mesh /
 *   create_scene_bvh                                     RT/scene.cpp:9-242
 *   create_bvh / create_bvh_for_mesh (midpoint, SAH, binned SAH)
 *                                                        RT/bvh.cpp:6-426
 *   transform_* (M4x4Inv)                                MathLib/my_math.h:1009-1069
 *   aim_camera / aim_camera_at / recompute_camera        RT/raytracer.cpp:26-59
 *   init_scene defaults                                  RT/raytracer.cpp:1424-1453
 *   load_reconstruction_kernel + g_filters               RT/raytracer.cpp:164-185,
 *                                                        RT/reconstruction_filters.cpp
 *   parse_obj / parse_hdr / load_environment_map / write_bitmap
 *                                                        RT/assets.cpp:187-724
 *   post-process (resolve, exposure, tonemap, sRGB, contrast, BGRA8)
 *                                                        RT/raytracer.cpp:2103-2173
 *   scene presets (g_scenes)                             RT/raytracer.cpp:795-1422
 * and flattens the result into an rt_scene_desc (rt_abi.h) for rt_scene_upload.
 *
 * Assets the reference ships but that are absent here (dragon_mcguire.obj and
 * three .hdr files, /root/reference/.MISSING_LARGE_BLOBS) are replaced by
 * seeded synthetic generators (rth_generate_mesh, rth_write_synthetic_hdr).
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include "rt_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rth_scene rth_scene;

enum rth_bvh_method {                          /* BVHConstructionMethod RT/bvh.h:7-11 */
    RTH_BVH_MIDPOINT_SPLIT = 0,
    RTH_BVH_SAH_BINNED     = 1,
    RTH_BVH_SAH_FULL       = 2,
};

typedef struct rth_post_settings {             /* PostProcessSettings RT/scene.h:84-90 */
    float   exposure;
    int32_t tonemapping;
    int32_t srgb_transform;
    float   midpoint;
    float   contrast;
} rth_post_settings;

typedef struct rth_bvh_info {
    uint32_t node_count;
    uint32_t leaf_count;
    uint32_t max_depth;
    uint32_t max_leaf_size;
} rth_bvh_info;

const char* rth_last_error(void);

/* clear_scene + init_scene's null material / null primitive (RT/raytracer.cpp:1426-1427) */
rth_scene* rth_scene_create(void);
void       rth_scene_destroy(rth_scene* scene);

uint32_t rth_add_material(rth_scene* s, const rt_material* m);
uint32_t rth_add_diffuse_material(rth_scene* s, rt_v3 diffuse_color, float ior, float roughness,
                                  int32_t checkers, rt_v3 checker_color);
uint32_t rth_add_translucent_material(rth_scene* s, rt_v3 absorb, float ior, float roughness);
uint32_t rth_add_emissive_material(rth_scene* s, rt_v3 emission_color);

/* transform == NULL means the shared identity transform */
uint32_t rth_add_plane(rth_scene* s, uint32_t material_id, rt_v3 n, float d);
uint32_t rth_add_sphere(rth_scene* s, uint32_t material_id, float r, const rt_m4x4inv* transform);
uint32_t rth_add_box(rth_scene* s, uint32_t material_id, rt_v3 r, const rt_m4x4inv* transform);
uint32_t rth_add_mesh(rth_scene* s, uint32_t material_id, uint32_t mesh_id, const rt_m4x4inv* transform);

/* Meshes: triangles a,b,c (3*count v3), optional per-vertex normals (3*count v3).
 * Builds the mesh BVH with `method` (BVHStorage_Scalar layout).  Returns mesh id. */
uint32_t rth_create_mesh(rth_scene* s, uint32_t triangle_count, const rt_v3* triangles,
                         const rt_v3* normals, int32_t method);
/* parse_obj (CounterClockwise winding) + create_bvh_for_mesh; returns 0 on failure */
int      rth_load_obj_mesh(rth_scene* s, const char* path, int32_t method, uint32_t* out_mesh_id);
int      rth_mesh_bvh_info(rth_scene* s, uint32_t mesh_id, rth_bvh_info* out);
int      rth_scene_bvh_info(rth_scene* s, rth_bvh_info* out);

void     rth_set_sky(rth_scene* s, rt_v3 top, rt_v3 bot);
/* load_environment_map: parse_hdr + luma CDF (the CDF is built, as in the reference) */
int      rth_load_environment_map(rth_scene* s, const char* hdr_path);
/* The same from pixels in memory (w*h, row 0 = the bottom row sample_sky reads at v = 0) */
int      rth_set_environment_map(rth_scene* s, uint32_t w, uint32_t h, const rt_v3* pixels);

/* Build the BVHs of rth_create_mesh / rth_create_scene_bvh on `device` with rt_build_bvh
 * (midpoint and binned SAH; bit-identical to the host builder); -1 (the default): on the host.
 * rth_build_bvh_entries: the builder on raw BVHSortEntry boxes (centre p, half extent r),
 * with the same outputs as rt_build_bvh; uses the device when one was set.  Returns an
 * rt_status. */
void     rth_set_bvh_device(int device);
int      rth_build_bvh_entries(uint32_t n, const rt_v3* p, const rt_v3* r, int32_t method,
                               rt_bvh_node* out_nodes, uint32_t* out_node_count, uint32_t* out_order);

/* create_scene_bvh (binned SAH over primitives 1..n) */
int      rth_create_scene_bvh(rth_scene* s);
/* Flattened view, valid until the scene is modified or destroyed. */
const rt_scene_desc* rth_scene_desc(rth_scene* s);

/* transforms (MathLib/my_math.h:1009-1069) */
rt_m4x4inv rth_transform_identity(void);
rt_m4x4inv rth_transform_translate(rt_v3 t);
rt_m4x4inv rth_transform_scale(rt_v3 s);
rt_m4x4inv rth_transform_rotate_x_axis(float angle);
rt_m4x4inv rth_transform_rotate_y_axis(float angle);
rt_m4x4inv rth_transform_rotate_z_axis(float angle);
rt_m4x4inv rth_transform_mul(rt_m4x4inv a, rt_m4x4inv b);

/* camera (RT/raytracer.cpp:26-59) */
void rth_aim_camera(rt_camera* c, rt_v3 camera_d);
void rth_aim_camera_at(rt_camera* c, rt_v3 at);
void rth_recompute_camera(rt_camera* c);

/* init_scene defaults (RT/raytracer.cpp:1430-1452) */
void rth_default_settings(rt_settings* out, rth_post_settings* post);
/* load_reconstruction_kernel(find_filter(name)); unknown names give Box */
void rth_load_reconstruction_kernel(const char* name, rt_filter_cache* out);

/* Presets: "week_6", "cornell_box", "dragon", "nested_dielectrics", "c1".."c5",
 * plus the other g_scenes entries.  Fills the scene (BVH built), camera,
 * settings, filter and post settings exactly like load_scene (RT/raytracer.cpp:1455-1470). */
int rth_load_preset(const char* name, uint32_t w, uint32_t h, const char* asset_dir,
                    rth_scene** out_scene, rt_camera* camera, rt_settings* settings,
                    rt_filter_cache* filter, rth_post_settings* post);

/* Synthetic assets (deterministic, seeded) standing in for the missing blobs. */
uint32_t rth_generate_mesh(uint32_t target_triangles, uint32_t seed, rt_v3* out_triangles,
                           rt_v3* out_normals);          /* returns triangle count; pass NULL to size */
int      rth_write_synthetic_obj(const char* path, uint32_t target_triangles, uint32_t seed);
int      rth_write_synthetic_hdr(const char* path, uint32_t w, uint32_t h, uint32_t seed);

/* Host preview of the output pass (RT/raytracer.cpp:2103-2173 with a flat 0.5 in place of
 * the blue-noise TPDF dither; the picture path uses the device pass, rt_postprocess*), and
 * write_bitmap (RT/assets.cpp:693-724): top-down 32-bit BGRA.  rth_read_bitmap reads such a
 * file back (tests). */
void rth_resolve_bgra8(const rt_accumulation_buffer* accum, const rth_post_settings* post, uint32_t* out_bgra);
int  rth_write_bitmap(const char* path, const uint32_t* bgra, uint32_t w, uint32_t h);
int  rth_read_bitmap(const char* path, uint32_t* bgra, uint32_t w, uint32_t h);

/* Render-to-bitmap entry point ("Take picture", RT/raytracer.cpp:2031-2048, 2089-2185):
 * renders `spp` samples per pixel of frame `total_frame_index` on `device` into a fresh
 * accumulation buffer, runs the reference's output pass with its TPDF dither on the device
 * (rt_render_picture) and writes the BMP.  stats_out may be NULL. */
int rth_take_picture(rth_scene* s, const rt_camera* camera, const rt_settings* settings,
                     const rt_filter_cache* filter, const rth_post_settings* post,
                     uint32_t w, uint32_t h, uint32_t spp, uint32_t total_frame_index, int device,
                     const char* bmp_path, rt_stats* stats_out);

#ifdef __cplusplus
}
#endif
#endif
