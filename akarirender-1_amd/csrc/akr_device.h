// akr_device.h — device-resident scene, queue and launch-argument layouts (HBM).
//
// HBM layout:
//   BVH:   akr_bvh_node[n_nodes] (64 B, DFS order) + leaf-ordered akr_bvh_tri[n] (48 B)
//   shade: per triangle (global id order) 3 x float4 corner positions, 9 normals, 6 texcoords,
//          material id — read once per hit, never by traversal
//   paths: SoA per path slot: seed (u32), beta (float4), L (float4), film (float4 = rgb + weight)
//   queues (per bounce, ping-pong): ray float4[2], slot u32; hits float4 (t, u, v, gid bits);
//          shadow queue ray float4[2] + (colour.xyz, slot bits) float4
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "../../include/akr_hip.h"
#include "../../include/akr_bvh_format.h"

namespace akr {

constexpr int kBlock = 256;           // threads per workgroup (4 waves)
constexpr int kStackLds = 16;         // LDS-resident traversal stack entries per ray
constexpr int kStackMax = 64;         // >= AKR_BVH_MAX_DEPTH
constexpr uint32_t kNoHit = 0xFFFFFFFFu;

struct LightDev {          // AreaLight (kernel/light.h:47-57): triangle + emission texture
    float v[9];
    float tc[6];
    int32_t color_tex;
    int32_t _pad[2];
};

struct SceneDev {
    const akr_bvh_node *nodes;
    const float4 *tris;            // akr_bvh_tri as 3 x float4
    const float4 *corner;          // 3 per triangle: positions of the three vertices
    const float *normals;          // 9 per triangle
    const float *texcoords;        // 6 per triangle
    const int32_t *matid;          // per triangle, global material or -1
    const akr_material *mats;
    const akr_texture *texs;
    const float *images;
    const int64_t *image_off;
    const int32_t *image_w;
    const int32_t *image_h;
    const LightDev *lights;
    const float *light_cdf;        // n_lights + 1
    const float *light_func;       // n_lights
    float light_func_int;
    int32_t n_lights;
    const uint32_t *mesh_base;     // n_meshes + 1 prefix of triangle counts
    int32_t n_meshes;
};

struct CameraDev {
    float r2c[16];
    float c2w[16];
    int32_t width, height;
};

struct TraceCounters {             // reduced per wave, one atomic per wave
    unsigned long long rays, box, tri;
};

struct TraceArgs {
    SceneDev sc;
    const float4 *rays;            // 2 per ray
    const uint32_t *count;         // device count (queue) or nullptr -> n
    uint32_t n;
    float4 *hits;                  // closest: (t, u, v, gid bits)
    akr_hit *abi_hits;             // optional: write akr_hit instead
    // shadow epilogue: colour.xyz + slot bits in .w; L accumulated per slot when unoccluded
    const float4 *shadow_color;
    float4 *L;
    uint32_t *stack_ovf;           // 2 u32 per entry (ref, t bits) beyond the LDS stack
    uint32_t ovf_threads;          // threads covered by stack_ovf
    TraceCounters *counters;       // [3]: closest, any, shadow
};

struct ShadeArgs {
    SceneDev sc;
    const float4 *ray_in;
    const uint32_t *slot_in;
    const float4 *hit_in;
    const uint32_t *count_in;
    float4 *ray_out;
    uint32_t *slot_out;
    uint32_t *count_out;
    float4 *shadow_ray;
    float4 *shadow_color;
    uint32_t *shadow_count;
    uint32_t *seed;
    float4 *beta;
    float4 *L;
    int32_t depth;
    int32_t max_depth;
    uint32_t capacity;
};

struct RaygenArgs {
    CameraDev cam;
    const uint32_t *pixel;         // per slot: x | y << 16
    uint32_t n;
    uint32_t *seed;
    float4 *beta;
    float4 *L;
    float4 *ray_out;
    uint32_t *slot_out;
    uint32_t *count_out;
    int32_t first_pass;
};

struct SplatArgs {
    const float4 *L;
    float4 *film;
    uint32_t n;
    float ray_clamp;
};

}  // namespace akr
