/*
 * akr_oracle.h — CPU restatement of AkariRender's ray-scene intersection and unidirectional
 * path tracer (TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker; never linked into the product library).
 *
 * Parity status: the reference itself cannot be compiled or run here (denied by the
 * environment), and its own tests pin nothing on this path.  The restatement is
 * pinned by (a) known-answer vectors derived in closed form from the reference source
 * (LCG, Distribution1D, Moller-Trumbore, camera), (b) the reference's own test
 * tests/test-math.cpp:49-58 (Frame round trip), (c) the reference's own fixtures
 * (resources/data/cornell_box/CornellBox-Original.obj.mesh and ref.png, loose statistical
 * check only: ref.png's render settings are unknown).  Pixel-level parity against the reference
 * binary is therefore "partially pinned" — see DESIGN.md §5.
 */
#ifndef AKR_ORACLE_H
#define AKR_ORACLE_H
#include <stdint.h>
#include "../include/akr_hip.h"
#include "../include/akr_bvh_format.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Flattened render scene: every mesh concatenated (global triangle id = mesh base + prim). */
typedef struct orc_scene {
    const float *vertices;      /* 3 * n_vertices */
    uint64_t n_vertices;
    const int32_t *indices;     /* 3 * n_tris, global vertex indices */
    const float *normals;       /* 9 * n_tris (per face-vertex, core/mesh.cpp:69-70) */
    const float *texcoords;     /* 6 * n_tris */
    const int32_t *matid;       /* n_tris, global material index or -1 */
    uint64_t n_tris;
    const akr_material *materials;
    int32_t n_materials;
    const akr_texture *textures;
    int32_t n_textures;
    const float *images;        /* concatenated RGBA f32 texels */
    const int64_t *image_offset;/* float offset of each image */
    const int32_t *image_w;
    const int32_t *image_h;
    int32_t n_images;
    const uint32_t *light_gid;  /* n_lights global triangle ids */
    const float *light_power;   /* n_lights */
    int32_t n_lights;
    const akr_bvh_node *nodes;
    uint64_t n_nodes;
    const akr_bvh_tri *tris;
    uint64_t n_bvh_tris;
    akr_camera camera;
} orc_scene;

typedef struct orc_hit {
    float t, u, v;
    uint32_t gid; /* 0xFFFFFFFF on miss */
} orc_hit;

typedef struct orc_render_stats {
    uint64_t camera_rays;
    uint64_t extension_rays;
    uint64_t shadow_rays;
    uint64_t box_tests;
    uint64_t tri_tests;
} orc_render_stats;

int orc_version(void);
/* LCGSampler (kernel/sampler.h:54-67): n next1d() draws from `seed`; returns the final state. */
uint32_t orc_lcg(uint32_t seed, int32_t n, float *out);
/* PCG32 (kernel/sampler.h:28-53) next1d() draws after set_sample_index(seed). */
void orc_pcg(uint64_t seed, int64_t n, float *out);
/* PerspectiveCamera::generate_ray (kernel/camera.h:67-86) with the camera-node transform
 * (core/nodes/camera.cpp:32-38); consumes 4 LCG draws per ray from *seed (canonical order). */
int orc_camera_ray(const akr_camera *cam, int32_t x, int32_t y, uint32_t *seed, akr_ray *out);
/* r2c and c2w 4x4 matrices (row major) as computed by the reference (camera.h:45-59). */
void orc_camera_matrices(const akr_camera *cam, float *r2c16, float *c2w16);
/* Distribution1D (common/distribution.h:46-102): sample_discrete for each u. */
void orc_distribution_sample(const float *func, int32_t n, const float *u, int32_t m,
                             int32_t *idx, float *pdf);
/* Frame (common/math.h:201-225): local_to_world then world_to_local of w in frame(n). */
void orc_frame_roundtrip(const float *n3, const float *w3, float *local_to_world3, float *back3);
/* Cosine-hemisphere / concentric disk warps (kernel/sampling.h:32-53). */
void orc_cosine_hemisphere(const float *u2, int32_t n, float *out3);

/* Closest-hit (any_hit = 0) or occlusion (any_hit = 1) over the scene BVH with the reference
 * traversal (bvh-accelerator.h:488-547); tight = 0 is the reference's intersectAABB bit for bit,
 * tight = 1 also rejects boxes behind the origin (the device default); n_threads <= 0 -> all. */
int orc_trace(const orc_scene *s, const akr_ray *rays, uint64_t n, orc_hit *hits, int any_hit,
              int32_t tight, int32_t n_threads, uint64_t *box_tests, uint64_t *tri_tests);
/* Builder-independent brute force over every triangle in global-id order. */
int orc_trace_brute(const orc_scene *s, const akr_ray *rays, uint64_t n, orc_hit *hits,
                    int any_hit, int32_t n_threads);
/* cpu::PathTracer::render (kernel/integrators/cpu/integrator.cpp:89-142) over the pixels of
 * `tiles`, 16x16 work tiles on n_threads workers with an atomic work counter
 * (core/parallel.cpp:44-129); accumulates into full-frame radiance[W*H*3], weight[W*H]. */
int orc_render(const orc_scene *s, const akr_pt_params *p, const akr_rect *tiles, int32_t n_tiles,
               float *radiance, float *weight, int32_t n_threads, orc_render_stats *stats);
/* orc_render plus a per-pixel fingerprint of the sample loop into the frame-indexed probe[W*H]
 * (pixels outside the tiles untouched): the sampler state after the pixel's last sample (its draw
 * count encodes every path length and BSDF-pdf rejection), the closest-hit traces below
 * max(1, max_depth) and the shadow traces, summed over the pixel's samples
 * (pathtracer.h:69-91, 133-164; cpu/integrator.cpp:124-134). */
int orc_render_probe(const orc_scene *s, const akr_pt_params *p, const akr_rect *tiles, int32_t n_tiles,
                     float *radiance, float *weight, int32_t n_threads, orc_render_stats *stats,
                     akr_pixel_probe *probe);
/* cpu::AmbientOcclusion::render (kernel/integrators/cpu/integrator.cpp:40-87) over the pixels of
 * `tiles`, same work split; L is 1 when the cosine-sampled ray from the camera hit (frame of the
 * geometric normal, tmin Eps) has no closest hit with t < occlude, 0 otherwise or on a camera miss.
 * AO rays are counted as stats->shadow_rays. */
int orc_render_ao(const orc_scene *s, const akr_ao_params *p, const akr_rect *tiles, int32_t n_tiles,
                  float *radiance, float *weight, int32_t n_threads, orc_render_stats *stats);

#ifdef __cplusplus
}
#endif
#endif
