/*
 * akr_hip.h — C-ABI drop-in boundary of the MI355X (gfx950) ray-scene intersection and
 * unidirectional path-tracing backend for AkariRender.
 *
 * Plain pointers and sizes only; no C++ or torch types cross this boundary.  Every export
 * returns an int status (0 = ok) and never throws or aborts across the ABI; the message of the
 * last failure on a context is available from akr_hip_last_error().  The C++ host adapter
 * (akarirender-1_amd/csrc/akari_hip.hpp) turns a non-zero status into std::runtime_error, the
 * reference's AKR_ASSERT_THROW convention (src/akari/common/panic.h:52-57).
 *
 * What each entry point replaces in the reference (paths relative to the reference root):
 *
 *  akr_hip_upload_mesh       MeshInstance<C> views built by AkariMesh::compile
 *                            (src/akari/core/nodes/mesh.cpp:47-61; layout kernel/instance.h:30-35)
 *  akr_hip_upload_textures   ConstantTexture / ImageTexture  (src/akari/kernel/texture.h:30-66)
 *  akr_hip_upload_materials  Material<C> closed Variant     (src/akari/kernel/material.h:205-298)
 *  akr_hip_upload_lights     AreaLight list + Distribution1D built in SceneNode::compile
 *                            (src/akari/core/nodes/scene.cpp:51-92; common/distribution.h:46-102)
 *  akr_hip_build_accel       BVHAccelerator<C>::build / Scene<C>::commit
 *                            (src/akari/kernel/bvh-accelerator.h:673-678; kernel/scene.cpp:64-81)
 *  akr_hip_trace (any_hit=0) BVHAccelerator<C>::intersect  (bvh-accelerator.h:679-681, 488-518)
 *  akr_hip_trace (any_hit=1) BVHAccelerator<C>::occlude    (bvh-accelerator.h:682, 519-547)
 *  akr_hip_set_camera        PerspectiveCameraNode::compile + PerspectiveCamera::preprocess
 *                            (src/akari/core/nodes/camera.cpp:26-52; kernel/camera.h:45-59)
 *  akr_hip_render            gpu::PathTracer<C>::render / cpu::PathTracer<C>::render
 *                            (kernel/integrators/gpu/cuda/integrator.cpp:137-424,
 *                             kernel/integrators/cpu/integrator.cpp:89-142), called from
 *                             SceneNode::render (src/akari/core/nodes/scene.cpp:137-150)
 *  akr_hip_kernel_stats      print_kernel_stats (src/akari/kernel/cuda/launch.cpp:92-118)
 *
 * Semantics are those of the reference CPU path (no radiance clamp unless ray_clamp > 0,
 * max_depth from the parameters, NEE only, LCG sampler seeded x + y*W per pixel).
 *
 * Threading and ordering: a context is bound to one device.  Its traces and renders share the
 * context's work counters, traversal overflow stacks and queues, so every trace / render call on a
 * context is ordered after the previous one on the device (an event the next call's stream waits
 * on), whatever streams the caller passes; calls from several host threads on one context must
 * still be serialised by the caller.  Different contexts are independent.
 */
#ifndef AKR_HIP_H
#define AKR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: akr_trace_counts gained deep_rays[3]; akr_pixel_probe / akr_hip_pixel_probe added
 * 3: akr_trace_counts gained leaf_tests[3] */
#define AKR_HIP_API_VERSION 3

typedef struct akr_hip_ctx akr_hip_ctx;

/* Ray<C> (common/math.h:183-199): origin, tmin, direction, tmax.  32 bytes. */
typedef struct akr_ray {
    float o[3];
    float tmin;
    float d[3];
    float tmax;
} akr_ray;

/* Intersection<C> (kernel/scene.h:40-49).  Miss: t = +inf, geom_id = prim_id = -1. 32 bytes. */
typedef struct akr_hit {
    float t;
    float u, v;        /* barycentrics (b1, b2) of the Moller-Trumbore test, instance.h:57-68 */
    int32_t geom_id;   /* index of the mesh in upload order */
    int32_t prim_id;   /* triangle index inside that mesh */
    int32_t _pad[3];
} akr_hit;

enum { AKR_TEX_CONSTANT = 0, AKR_TEX_IMAGE = 1 };
typedef struct akr_texture {
    int32_t type;      /* AKR_TEX_CONSTANT: value[] used; AKR_TEX_IMAGE: image index */
    float value[3];
    int32_t image;
    int32_t _pad[3];
} akr_texture;

enum { AKR_MAT_DIFFUSE = 0, AKR_MAT_GLOSSY = 1, AKR_MAT_EMISSIVE = 2, AKR_MAT_MIX = 3 };
typedef struct akr_material {
    int32_t type;
    int32_t color;      /* texture index: Diffuse/Glossy/Emissive colour */
    int32_t roughness;  /* texture index: Glossy roughness (x channel, squared -> alpha) */
    int32_t fraction;   /* texture index: Mix fraction (x channel) */
    int32_t first;      /* material index: Mix material_A */
    int32_t second;     /* material index: Mix material_B */
    int32_t double_sided; /* Emissive */
    int32_t _pad;
} akr_material;

/* One emissive triangle (AreaLight, kernel/light.h:47-71). */
typedef struct akr_area_light {
    int32_t geom_id;
    int32_t prim_id;
} akr_area_light;

/* PerspectiveCameraNode fields (core/nodes/camera.cpp:26-52). */
typedef struct akr_camera {
    float position[3];
    float rotation_deg[3];
    double fov_deg;
    int32_t resolution[2];
    int32_t _pad[2];
} akr_camera;

/* Path node fields (core/nodes/integrator.cpp:50-84).  ray_clamp <= 0 disables the clamp
 * (reference CPU semantics); > 0 clamps each sample to [0, ray_clamp] (GPU semantics).
 * flags: AKR_PT_EXACT_CULL = traverse with the reference's intersectAABB bit for bit (it keeps
 * boxes that lie behind the ray origin); default is the standard slab test, same hits. */
#define AKR_PT_EXACT_CULL 1
typedef struct akr_pt_params {
    int32_t spp;
    int32_t max_depth;
    float ray_clamp;
    int32_t flags;
} akr_pt_params;

/* Ambient-occlusion integrator parameters (cpu::AmbientOcclusion, kernel/integrators/cpu/
 * integrator.h:35-45; AOIntegratorNode defaults spp 16, occlude +inf, core/nodes/integrator.cpp:26-49). */
typedef struct akr_ao_params {
    int32_t spp;
    float occlude;  /* a closest hit of the AO ray with t < occlude occludes it */
    int32_t flags;  /* AKR_PT_EXACT_CULL */
    int32_t _pad;
} akr_ao_params;

/* Pixel rectangle [x0, x1) x [y0, y1). */
typedef struct akr_rect {
    int32_t x0, y0, x1, y1;
} akr_rect;

typedef struct akr_build_params {
    int32_t max_leaf_size;  /* <= 8 */
    int32_t n_bins;         /* SAH bins per axis (reference: 32, bvh-accelerator.h:104) */
    float traversal_cost;   /* SAH cost of a traversal step (default 1) */
    float intersect_cost;   /* SAH cost of a triangle test (default 4: measured best for the wide
                             * traversal, where a leaf visit also pays its exact-box test) */
    int32_t n_threads;      /* 0 = hardware concurrency */
    int32_t builder;        /* AKR_BUILDER_SAH (host binned SAH, default), _LBVH (GPU) or _SBVH (host) */
    float spatial_budget;   /* SBVH: extra references allowed, as a fraction of the triangles
                             * (0 = default 0.5) */
    int32_t wide_collapse;  /* the traversal's 4-wide view: AKR_COLLAPSE_SAH (0,
                             * default) or AKR_COLLAPSE_BALANCED */
} akr_build_params;
#define AKR_COLLAPSE_SAH 0       /* treelets of up to 3 BVH2 nodes chosen for the fewest expected visits */
#define AKR_COLLAPSE_BALANCED 1  /* a wide node folds in only its own internal children */
#define AKR_BUILDER_SAH 0
#define AKR_BUILDER_LBVH 1  /* GPU Morton/Karras build: much faster, lower tree quality */
#define AKR_BUILDER_SBVH 2  /* host SBVH: the reference's spatial splits (bvh-accelerator.h:125-475) */

typedef struct akr_accel_info {
    uint64_t n_nodes;       /* 64-byte BVH2 nodes, node 0 is the virtual root */
    uint64_t n_tris;        /* 48-byte leaf-ordered triangle records */
    int32_t max_depth;
    int32_t max_leaf;
    double build_ms;
    double sah_cost;
} akr_accel_info;

typedef struct akr_kernel_stat {
    char name[48];
    uint64_t launches;
    double total_ms;
    double min_ms;
    double max_ms;
} akr_kernel_stat;

/* Traversal counters (filled when option "count_tests" is 1). */
typedef struct akr_trace_counts {
    uint64_t rays;
    uint64_t box_tests;
    uint64_t tri_tests;
    uint64_t closest_rays;
    uint64_t shadow_rays;
    uint64_t per_mode[3][3]; /* [closest, any-hit, shadow] x [rays, box_tests, tri_tests] */
    /* SIMD lane slots per mode: [traversal-loop lane-iterations (64 per wave-iteration), of which
     * lanes holding a ray, triangle-loop lane-iterations, node visits]; visits / slots[0] and
     * tri_tests / slots[2] are lane utilisations. */
    uint64_t lane_slots[3][4];
    /* rays per mode whose traversal stack grew past the LDS-resident entries into the global
     * overflow area (the deep-stack path, kernels.hip stack_pop / wide_order_push) */
    uint64_t deep_rays[3];
    /* leaf records fetched per mode (each an exact leaf-box test; with the node visits, the
     * dependent fetch rounds of a traversal) */
    uint64_t leaf_tests[3];
} akr_trace_counts;

/* Test-only per-pixel fingerprint of the last render's sample loop (option "pixel_probe" = 1),
 * one record per film slot in packed tile order (as akr_hip_render_device): the LCG state after the
 * pixel's last sample (its draw count encodes every path length, kernel/sampler.h:54-67), and the
 * closest-hit and shadow traces of all its samples (pathtracer.h:69-91, 133-164).  The seed is
 * recorded by every render form; the ray counts by the wavefront form and by the counting build of
 * the persistent kernels (option "count_tests"), flagged in `flags`. */
#define AKR_PROBE_SEED 1u
#define AKR_PROBE_RAYS 2u
typedef struct akr_pixel_probe {
    uint32_t seed;
    uint32_t closest_rays;   /* camera + extension rays traced (none at depth == max_depth) */
    uint32_t shadow_rays;    /* NEE shadow rays traced */
    uint32_t flags;          /* AKR_PROBE_SEED | AKR_PROBE_RAYS: which fields were recorded */
} akr_pixel_probe;

int akr_hip_api_version(void);
int akr_hip_device_count(int *n);

int akr_hip_create(int device, akr_hip_ctx **out);
int akr_hip_destroy(akr_hip_ctx *ctx);
const char *akr_hip_last_error(const akr_hip_ctx *ctx);
/* Options: "stats" (per-kernel HIP-event timing: 0 off, 1 every kernel, 2 trace_closest only), "count_tests" (traversal counters),
 * "count_lines" (with count_tests: k_path marks the 128-B lines it reads, see akr_hip_path_profile),
 * "exact_cull", "wide", "lean", "shadow_grid_pct", "rays_per_lane" (tuning / A-B).
 * Render forms and their tuning (all give the same bits): "path" (0 wavefront,
 * 1 persistent kernel, 2 auto), "path_auto_pixels", "path_auto_complex";
 * the persistent form: "path_spec" (k_path_spec: 1 always, 0 never, 2 auto), "path_defer" (k_path_defer:
 * 1 forced, 0 k_path forced, 2 auto), the auto rule's "path_tail_ppl10" and "path_tail_steps" and its
 * overrides "path_spec_pixels", "path_defer_pixels", "path_defer_min_tris"; k_path_spec's "path_spec_depth",
 * "path_spec_fetch", "path_spec_fetch_pixels";
 * "path_tab", "path_mix", "path_min_wait", "path_grid_pct", "path_prio";
 * the cost order: "path_order", "path_order_min_spp", "path_order_share_pixels", "path_order_share_min_spp",
 * "path_order_shift", "path_order_pair", "path_order_classes", "path_order_cap", "path_order_sub",
 * "path_order_pilot_spp", "wave_order" (the wavefront's camera rays in cost order).
 * "verify" (default 1): in-band film check after every render.  Test only: "pixel_probe" (record
 * akr_pixel_probe per slot), "fault_test" (raise the hang guard's fault word once), "ray_steps",
 * "serial_shadow", "any_far_first". */
int akr_hip_set_option(akr_hip_ctx *ctx, const char *key, int64_t value);

int akr_hip_upload_mesh(akr_hip_ctx *ctx, const float *vertices, uint64_t n_vertices,
                        const int32_t *indices, const float *normals, const float *texcoords,
                        const int32_t *material_indices, uint64_t n_triangles,
                        const int32_t *material_slots, int32_t n_slots, int32_t *geom_id);
int akr_hip_upload_images(akr_hip_ctx *ctx, const float *rgba, const int32_t *widths,
                          const int32_t *heights, int32_t n_images);
int akr_hip_upload_textures(akr_hip_ctx *ctx, const akr_texture *textures, int32_t n);
int akr_hip_upload_materials(akr_hip_ctx *ctx, const akr_material *materials, int32_t n);
int akr_hip_upload_lights(akr_hip_ctx *ctx, const akr_area_light *lights, int32_t n,
                          const float *power);
int akr_hip_build_accel(akr_hip_ctx *ctx, const akr_build_params *params);
/* Adopt a BVH2 built elsewhere (the arrays akr_hip_accel_export writes: akr_bvh_node[n_nodes],
 * akr_bvh_tri[n_tris]) for the uploaded meshes, instead of building one: the same wide view and
 * device copy follow.  The tree is validated first (akr_bvh_validate); results are those of the
 * context that built it, bit for bit.  Lets the ranks of a node build the scene's BVH once. */
int akr_hip_import_accel(akr_hip_ctx *ctx, const void *nodes, uint64_t n_nodes, const void *tris,
                         uint64_t n_tris, int32_t n_threads);
int akr_hip_accel_info(akr_hip_ctx *ctx, akr_accel_info *info);
int akr_hip_accel_export(akr_hip_ctx *ctx, void *nodes, uint64_t node_bytes, void *tris,
                         uint64_t tri_bytes);
int akr_hip_set_camera(akr_hip_ctx *ctx, const akr_camera *camera);

/* Batched trace, host buffers in and out, synchronous. */
int akr_hip_trace(akr_hip_ctx *ctx, const akr_ray *rays, uint64_t n, akr_hit *hits, int any_hit);
/* Batched trace on device buffers (akr_ray[n] -> akr_hit[n]) on `stream` (hipStream_t, may be 0). */
int akr_hip_trace_device(akr_hip_ctx *ctx, const void *d_rays, uint64_t n, void *d_hits,
                         int any_hit, void *stream);

/* Render the pixels of `tiles` (clipped to the camera resolution) and ACCUMULATE into host
 * full-frame buffers radiance[W*H*3] (sum of L) and weight[W*H] (sample count), the reference
 * Film's Pixel{radiance, weight} (core/film.h:31-35).  Synchronous. */
int akr_hip_render(akr_hip_ctx *ctx, const akr_pt_params *params, const akr_rect *tiles,
                   int32_t n_tiles, float *radiance, float *weight);
/* cpu::AmbientOcclusion::render (kernel/integrators/cpu/integrator.cpp:40-87) — replaces
 * AOIntegrator::render (core/nodes/integrator.cpp:33-38) for the pixels of `tiles`: per sample,
 * L = 1 if the camera ray hits and the cosine-sampled ray about the geometric normal from the hit
 * point has no closest hit with t < occlude, else 0; accumulated like akr_hip_render.  Reuses the
 * path tracer's raygen / closest-hit trace; with occlude = +inf the AO ray is an occlusion query
 * (shadow-mode trace), otherwise a closest-hit trace whose t is compared.  Synchronous. */
int akr_hip_render_ao(akr_hip_ctx *ctx, const akr_ao_params *params, const akr_rect *tiles,
                      int32_t n_tiles, float *radiance, float *weight);
/* Multi-GPU render from one host process (SURVEY.md §8b akr_hip_render_node): tile j goes to
 * ctxs[j % n_ctx] (one context per device, each holding the same scene and camera), the contexts
 * render concurrently on one host thread each, and their films are gathered on ctxs[0]'s device
 * (device-to-device / xGMI peer copies) and merged there into the frame in context order, which is
 * added to the host buffers — the same pixels as akr_hip_render on one context, bit for bit.
 * (Multi-process runs over RCCL use akr_hip_render_device + akari_amd/dist.py instead.)
 * On failure the message is on ctxs[0]. */
int akr_hip_render_node(akr_hip_ctx *const *ctxs, int32_t n_ctx, const akr_pt_params *params,
                        const akr_rect *tiles, int32_t n_tiles, float *radiance, float *weight);
/* Same, but writes (overwrites) device buffers in packed tile order: pixel k of the tile list
 * (tiles in order, row-major inside a tile) -> radiance[3k..3k+2], weight[k].  Returns the
 * pixel count in *n_pixels.  The work is enqueued on `stream`; with option "verify" on (the
 * default) the call then WAITS on the host for the render and its in-band check (every slot holds
 * spp samples, and no persistent wave stopped on its hang guard) before it returns, so the check
 * can fail this call.  With "verify" 0 the call returns once the work is enqueued (fully
 * asynchronous); a hang-guard fault is then reported by the context's next render or
 * akr_hip_synchronize. */
int akr_hip_render_device(akr_hip_ctx *ctx, const akr_pt_params *params, const akr_rect *tiles,
                          int32_t n_tiles, float *d_radiance, float *d_weight, void *stream,
                          uint64_t *n_pixels);

/* Host-only BVH build (no device needed): the same builder akr_hip_build_accel runs, for tools
 * and CPU-side checks.  Arrays are owned by the handle; free with akr_bvh_host_free. */
typedef struct akr_bvh_host akr_bvh_host;
int akr_bvh_host_build(const float *vertices, uint64_t n_vertices, const int32_t *indices,
                       uint64_t n_triangles, const akr_build_params *params, akr_bvh_host **out,
                       akr_accel_info *info);
const void *akr_bvh_host_nodes(const akr_bvh_host *h);
const void *akr_bvh_host_tris(const akr_bvh_host *h);
void akr_bvh_host_free(akr_bvh_host *h);
/* The 4-wide quantized view the traversal kernels walk (akr_bvh4_node / akr_bvh_leaf), built from
 * the handle's BVH2 on first call; pointers stay valid until akr_bvh_host_free. */
int akr_bvh_host_wide(akr_bvh_host *h, uint64_t *n_nodes, uint64_t *n_leaves, uint32_t *root_ref);
/* Host check of a BVH2 before it is adopted (no device): a tree from the virtual root, references and
 * leaf ranges in range, triangle ids < n_scene_tris, depth <= AKR_BVH_MAX_DEPTH.  0 = valid. */
int akr_bvh_validate(const void *nodes, uint64_t n_nodes, const void *tris, uint64_t n_tris,
                     uint64_t n_scene_tris, int32_t *max_depth);
const void *akr_bvh_host_wide_nodes(const akr_bvh_host *h);
const void *akr_bvh_host_wide_leaves(const akr_bvh_host *h);

int akr_hip_kernel_stats(akr_hip_ctx *ctx, akr_kernel_stat *out, int32_t max_n, int32_t *n);
int akr_hip_trace_counts(akr_hip_ctx *ctx, akr_trace_counts *out);

/* Diagnostic (option count_tests): phase profile of the persistent path kernel's last counted
 * launches, summed over waves, wall-clock ticks at 100 MHz: out[0..10] = waves, outer iterations,
 * processing phases, traversal-loop iterations, ticks processing / traversing / in leaves / in
 * total, the longest wave's ticks, lanes processed, ticks of processing spent on finished rays'
 * results (shading), k_path_spec's speculative samples started / dropped, and the time split of the
 * traversal and leaf phases: ticks issuing their loads, waiting for them, working after them, then
 * k_path's processing split: the park, the sample end with splat / pixel fetch / camera ray, and the
 * unpark with the new rays' start, and the shading's wait for the hit's record (out[19..22]),
 * then the leaf phases entered with a leaf held and the lanes holding one, summed (out[23..24]), then
 * the distinct 128-B lines of the wide nodes, the leaf blob and the shading records that the last
 * k_path render with "count_lines" read (out[25..27]).
 * Not part of the reference interface. */
int akr_hip_path_profile(akr_hip_ctx *ctx, uint64_t *out, int32_t n);
int akr_hip_reset_stats(akr_hip_ctx *ctx);
/* The last akr_hip_render's lanes per pixel (always 1) and sample passes launched (diagnostic). */
int akr_hip_render_info(akr_hip_ctx *ctx, int32_t *lanes, int32_t *passes);
/* Which form ran the last path render (all give the same bits): the wavefront
 * kernels (north_star's layout: raygen -> closest -> shade -> shadow -> splat launches), the
 * persistent path kernel, its deferred-NEE form or its speculative-sample
 * form; *ordered = 1 when
 * the persistent kernel fetched pixels in pilot-cost order.  AKR_FORM_NONE: nothing rendered. */
#define AKR_FORM_NONE (-1)
#define AKR_FORM_WAVEFRONT 0
#define AKR_FORM_PATH 2
#define AKR_FORM_PATH_DEFER 3
#define AKR_FORM_PATH_SPEC 4
int akr_hip_render_form(akr_hip_ctx *ctx, int32_t *form, int32_t *ordered);
/* The inputs of the last persistent render's form choice: its pixels per resident
 * lane x 1000, and the cost-ordering pilot's camera rays and their summed traversal steps; -1 when the
 * choice did not read the pilot (a forced form, no cost order, or a render too large for a tail form). */
int akr_hip_render_form_inputs(akr_hip_ctx *ctx, int64_t *pixels_per_lane_x1000, int64_t *pilot_rays,
                               int64_t *pilot_steps);
int akr_hip_synchronize(akr_hip_ctx *ctx);
/* Copies the first n records of the last render's pixel probe (see akr_pixel_probe); fails when
 * the last render ran without option "pixel_probe" or has fewer slots. */
int akr_hip_pixel_probe(akr_hip_ctx *ctx, akr_pixel_probe *out, uint64_t n);
/* Diagnostic: with option "ray_steps" set, each standalone trace (akr_hip_trace /
 * akr_hip_trace_device) runs the counting kernel and records, per ray, the traversal-loop
 * iterations it was active for plus its triangle tests (0xFFFFFFFF: traced by the exact BVH2
 * fallback); this copies the first n of the last trace to host memory. */
int akr_hip_ray_steps(akr_hip_ctx *ctx, uint32_t *out, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif /* AKR_HIP_H */
