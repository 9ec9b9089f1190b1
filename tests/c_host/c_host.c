/*
 * c_host.c — a plain C host of librt_mi355x.so, written the way INTEGRATION.md §3's adapter
 * drops the library into the reference's host: build the scene with the host scene model
 * (the reference's add_* / create_scene_bvh, RT/scene.cpp:9-242), flatten it into the
 * host's OWN arrays and rt_scene_desc field by field (Primitive::transform pointer ->
 * index, MeshBVH -> rt_mesh, BVHNode as is), upload it, and render through rt_render
 * where render_all_tiles released its workers (RT/raytracer.cpp:692-757), then take the
 * picture (rt_render_picture + write_bitmap, RT/raytracer.cpp:2031-2185).
 *
 *   c_host <w> <h> <out.bin> [bmp]
 *
 * Writes <out.bin>: w*h float4 of the accumulation buffer (rt_render, exact splat), then
 * w*h u32 of the picture (rt_render_picture of frame 0), then the two ray counts (u64).
 * Exit status: 0, or the rt_status of the first failing call (5 = no MI355X visible).
 * tests/test_c_host.py compares the output with the CPU oracle.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_abi.h"
#include "rt_host.h"

static int fail(const char* what, int err) {
    fprintf(stderr, "c_host: %s failed (%d): %s\n", what, err, rt_last_error());
    return err;
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: c_host <w> <h> <out.bin> [bmp]\n"); return 1; }
    const uint32_t w = (uint32_t)atoi(argv[1]), h = (uint32_t)atoi(argv[2]);
    if (rt_abi_version() != RT_ABI_VERSION) { fprintf(stderr, "c_host: ABI version mismatch\n"); return 1; }

    /* the reference's load_scene(g_scenes["Week 6"]) with the C1 settings (RT/raytracer.cpp:926-978) */
    rth_scene* hs = NULL;
    rt_camera cam;
    rt_settings st;
    rt_filter_cache fc;
    rth_post_settings post;
    if (!rth_load_preset("c1", w, h, NULL, &hs, &cam, &st, &fc, &post)) { fprintf(stderr, "c_host: preset\n"); return 1; }
    const rt_scene_desc* src = rth_scene_desc(hs);

    /* flatten into the host's own arrays, as the adapter does from the reference's Scene */
    rt_material* mats = malloc(sizeof(rt_material)*src->material_count);
    rt_primitive* prims = malloc(sizeof(rt_primitive)*src->primitive_count);
    rt_primitive* planes = malloc(sizeof(rt_primitive)*(src->plane_count ? src->plane_count : 1));
    rt_m4x4inv* xforms = malloc(sizeof(rt_m4x4inv)*src->transform_count);
    uint32_t* lights = malloc(sizeof(uint32_t)*(src->light_count ? src->light_count : 1));
    rt_bvh_node* nodes = malloc(sizeof(rt_bvh_node)*src->bvh_node_count);
    uint32_t* indices = malloc(sizeof(uint32_t)*src->bvh_index_count);
    for (uint32_t i = 0; i < src->material_count; ++i) {          /* RT/scene.h:15-29, field by field */
        const rt_material* m = &src->materials[i];
        rt_material* d = &mats[i];
        d->flags = m->flags; d->albedo = m->albedo; d->checker_color = m->checker_color;
        d->emission_color = m->emission_color; d->ior = m->ior; d->metallic = m->metallic;
        d->roughness = m->roughness; d->is_participating_medium = m->is_participating_medium; d->absorb = m->absorb;
    }
    for (uint32_t i = 0; i < src->primitive_count; ++i) {         /* transform pointer -> index */
        const rt_primitive* p = &src->primitives[i];
        rt_primitive q;
        memset(&q, 0, sizeof(q));
        q.transform_index = p->transform_index; q.material_id = p->material_id; q.type = p->type;
        q.mesh_index = p->mesh_index;
        if (p->type == RT_PRIMITIVE_SPHERE) q.p[0] = p->p[0];
        if (p->type == RT_PRIMITIVE_BOX) { q.p[0] = p->p[0]; q.p[1] = p->p[1]; q.p[2] = p->p[2]; }
        prims[i] = q;
    }
    for (uint32_t i = 0; i < src->plane_count; ++i) {
        const rt_primitive* p = &src->planes[i];
        rt_primitive q;
        memset(&q, 0, sizeof(q));
        q.material_id = p->material_id; q.type = RT_PRIMITIVE_PLANE;
        q.p[0] = p->p[0]; q.p[1] = p->p[1]; q.p[2] = p->p[2]; q.p[3] = p->p[3];   /* n.xyz, d */
        planes[i] = q;
    }
    memcpy(xforms, src->transforms, sizeof(rt_m4x4inv)*src->transform_count);   /* M4x4Inv: same layout */
    memcpy(lights, src->lights, sizeof(uint32_t)*src->light_count);
    memcpy(nodes, src->bvh_nodes, sizeof(rt_bvh_node)*src->bvh_node_count);     /* BVHNode: same 32 B layout */
    memcpy(indices, src->bvh_indices, sizeof(uint32_t)*src->bvh_index_count);

    rt_scene_desc desc;
    memset(&desc, 0, sizeof(desc));
    desc.material_count = src->material_count;   desc.materials = mats;
    desc.primitive_count = src->primitive_count; desc.primitives = prims;
    desc.plane_count = src->plane_count;         desc.planes = planes;
    desc.transform_count = src->transform_count; desc.transforms = xforms;
    desc.light_count = src->light_count;         desc.lights = lights;
    desc.mesh_count = 0;                         desc.meshes = NULL;      /* Week 6 has no meshes */
    desc.bvh_node_count = src->bvh_node_count;   desc.bvh_nodes = nodes;
    desc.bvh_index_count = src->bvh_index_count; desc.bvh_indices = indices;
    desc.top_sky_color = src->top_sky_color;     desc.bot_sky_color = src->bot_sky_color;
    desc.skydome_w = 0; desc.skydome_h = 0;      desc.skydome = NULL;

    int count = 0, err = rt_device_count(&count);
    if (err || count < 1) return fail("rt_device_count", err ? err : RT_ERROR_NO_DEVICE);
    rt_scene* dev = NULL;
    if ((err = rt_scene_upload(&desc, 0, &dev))) return fail("rt_scene_upload", err);

    /* render_all_tiles -> rt_render into the host's AccumulationBuffer (reset to zero first) */
    float* px = calloc((size_t)w*h*4, sizeof(float));
    rt_accumulation_buffer acc = {w, h, 0, px};
    rt_tile_set tiles = {64, 64, 0, 1};
    rt_stats stats;
    if ((err = rt_set_splat_mode(RT_SPLAT_EXACT))) return fail("rt_set_splat_mode", err);
    if ((err = rt_render(dev, &cam, &st, &fc, &tiles, 0, &acc, &stats))) return fail("rt_render", err);

    /* "Take picture": frame 0 rendered afresh, output pass on the device, write_bitmap */
    rt_post_settings pp = {post.exposure, post.tonemapping, post.srgb_transform, post.midpoint, post.contrast};
    uint32_t* bgra = malloc(sizeof(uint32_t)*(size_t)w*h);
    rt_stats pstats;
    if ((err = rt_render_picture(dev, &cam, &st, &fc, &tiles, 0, w, h, &pp, bgra, &pstats))) return fail("rt_render_picture", err);
    if (argc > 4 && !rth_write_bitmap(argv[4], bgra, w, h)) { fprintf(stderr, "c_host: %s\n", rth_last_error()); return 1; }

    FILE* f = fopen(argv[3], "wb");
    if (!f) { fprintf(stderr, "c_host: cannot write %s\n", argv[3]); return 1; }
    fwrite(px, sizeof(float), (size_t)w*h*4, f);
    fwrite(bgra, sizeof(uint32_t), (size_t)w*h, f);
    fwrite(&stats.closest_hit_rays, sizeof(uint64_t), 1, f);
    fwrite(&stats.shadow_rays, sizeof(uint64_t), 1, f);
    /* render_all_tiles' out_stats (RT/raytracer.cpp:727-730): the reference's TraversalStats are the
       sums of the two query kinds */
    {
        const rt_traversal_stats* k = stats.traversal;
        const uint64_t t[4] = {k[0].mesh_intersection_count + k[1].mesh_intersection_count,
                               k[0].mesh_bvh_traversals + k[1].mesh_bvh_traversals,
                               k[0].mesh_node_traversals + k[1].mesh_node_traversals,
                               k[0].mesh_leaf_traversals + k[1].mesh_leaf_traversals};
        fwrite(t, sizeof(uint64_t), 4, f);
    }
    fclose(f);
    printf("c_host: %ux%u, %llu samples, %llu + %llu rays\n", w, h, (unsigned long long)stats.samples,
           (unsigned long long)stats.closest_hit_rays, (unsigned long long)stats.shadow_rays);

    rt_scene_free(dev);
    rth_scene_destroy(hs);
    free(px); free(bgra); free(mats); free(prims); free(planes); free(xforms); free(lights); free(nodes); free(indices);
    return 0;
}
