// akr_device.h — device-resident scene, queue and launch-argument layouts (HBM).
//
// HBM layout:
//   BVH:    akr_bvh_node[n_nodes] (64 B, DFS order) + leaf-ordered akr_bvh_tri[n] (48 B)
//   shade:  one 80-B record per triangle (global id order): v0|matid, v1|n0.x, v2|n0.y,
//           n0.z n1, n2|pad — one gather per hit; texcoords (6 f32) only for textured scenes
//   paths:  per slot (pixel of the tile list): seed u32, L float4, film float4 (rgb, weight)
//   queues: per bounce (ping-pong) ray float4[2] (o|tmin, d|tmax), state float4 (beta|seed),
//           slot u32 — path state travels with the ray, so shade reads and writes it coalesced;
//           hits float4 (t, u, v, gid bits); shadow queue ray float4[2] + (colour|slot) float4
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "../../include/akr_hip.h"
#include "../../include/akr_bvh_format.h"

// Device code sees the scene record's pointers as global memory (address space 1), so loads through
// them are global_load even inside an out-of-line function, where the compiler cannot infer it
// (flat loads also count against lgkmcnt and tie LDS waits to outstanding memory loads).
#if defined(__HIP_DEVICE_COMPILE__)
#define AKR_GLOBAL __attribute__((address_space(1)))
#else
#define AKR_GLOBAL
#endif

namespace akr {

constexpr int kBlock = 256;           // threads per workgroup (4 waves)
#ifndef AKR_TRACE_BLOCK
#define AKR_TRACE_BLOCK 256
#endif
constexpr int kTraceBlock = AKR_TRACE_BLOCK;  // threads per traversal workgroup (the LDS stack's row)
#ifndef AKR_STACK_LDS
#define AKR_STACK_LDS 15
#endif
#ifndef AKR_REFILL_MIN
#define AKR_REFILL_MIN 32
#endif
constexpr int kStackLds = AKR_STACK_LDS;  // LDS-resident traversal stack entries per ray (8 B each; 15 fill the LDS left by the path kernels' park area)
constexpr int kStackMax = 96;         // >= 3 pushes x 32 wide levels (BVH2 depth <= 64)
constexpr uint32_t kNoHit = 0xFFFFFFFFu;
constexpr int kRefillMin = AKR_REFILL_MIN;  // refill a wave's idle lanes once at least this many are idle
#ifndef AKR_REFILL_MIN_ANY
#define AKR_REFILL_MIN_ANY AKR_REFILL_MIN
#endif
constexpr int kRefillMinAny = AKR_REFILL_MIN_ANY;  // the same for occlusion (any-hit / shadow) traces
#ifndef AKR_WHILE_EXIT_ANY
#define AKR_WHILE_EXIT_ANY AKR_WHILE_EXIT
#endif
#ifndef AKR_WHILE_EXIT
#define AKR_WHILE_EXIT 12  // 16 before the r21 one-pop loop; 8 / 12 / 16 / 24 re-swept on it: profiles/r21_while_exit_ab.log
#endif
constexpr uint64_t kMaxWideNodes = 1ull << 26;  // 64-B wide nodes addressed by a 32-bit byte offset (visit_wide_lean)
constexpr int kWhileExit = AKR_WHILE_EXIT;  // traversal phase ends when <= this many lanes still search
#ifndef AKR_WHILE_EXIT_PATH
#define AKR_WHILE_EXIT_PATH 16  // k_path: 4.034-4.064 against 4.060-4.078 ms per spp at 12, 20 slower (profiles/r24/path_exit_ab.log)
#endif
constexpr int kWhileExitPath = AKR_WHILE_EXIT_PATH;  // the same for k_path alone (the other persistent forms keep kWhileExit)
#ifndef AKR_WHILE_EXIT_SPEC
#define AKR_WHILE_EXIT_SPEC AKR_WHILE_EXIT
#endif
constexpr int kWhileExitSpec = AKR_WHILE_EXIT_SPEC;  // the same for k_path_spec
constexpr int kWhileExitAny = AKR_WHILE_EXIT_ANY;  // the same for occlusion traces
#ifndef AKR_WORK_SHARDS
#define AKR_WORK_SHARDS 8
#endif
constexpr uint32_t kWorkShards = AKR_WORK_SHARDS;  // dynamic-fetch counters per trace launch (>= one per XCD)
constexpr uint32_t kWorkStride = 32;  // u32 between counters: each on its own 128-B line
constexpr uint32_t kWorkWords = kWorkShards * kWorkStride;
constexpr uint32_t kTraceWords = kWorkWords;  // per trace launch

// First queue index of shard k of [0, n) (k = kWorkShards gives n).
__host__ __device__ inline uint32_t shard_begin(uint32_t n, uint32_t k) {
    return (uint32_t)(((uint64_t)n * k) / kWorkShards);
}

// AreaLight (kernel/light.h:47-71): triangle, texcoords, emission, and the per-light constants of
// AreaLight::sample / Scene::select_light precomputed on the host with the device's f32 operations
// (cross, normalize, length, one division): one 96-B record per NEE sample, no dependent loads.
struct LightDev {
    float v[9];            // corners
    float tc[6];           // corner texcoords
    int32_t color_img;     // -1: constant emission Le; else the (image) texture index
    float Le[3];           // constant emission
    float area_half;       // length(cross(v1 - v0, v2 - v0)) * 0.5
    float lng[3];          // normalize(cross(v1 - v0, v2 - v0))
    float sel_pdf;         // light_func[i] / (light_func_int * n_lights) (scene.h:79-90)
};

// akr_material with its constant textures resolved (Texture::evaluate of a ConstantTexture is its
// value): one 48-B record per material lookup; *_img >= 0 names an image texture to evaluate.
struct MatDev {
    int32_t type, double_sided, first, second;
    float color[3];
    int32_t color_img;
    float rough;
    int32_t rough_img;
    float frac;
    int32_t frac_img;
};
static_assert(sizeof(LightDev) == 96, "LightDev: six float4");

struct ShadeTri {          // Triangle<C> data of one global triangle id (shape.h:26-42)
    float4 a;              // v0.xyz, material id (int bits, -1 = none)
    float4 b;              // v1.xyz, n0.x
    float4 c;              // v2.xyz, n0.y
    float4 d;              // n0.z, n1.xyz
    float4 e;              // n2.xyz, 0
};

// Device copy of a texture (akr_texture + its image's size and offset): one 32-B record per
// lookup, so an image texel is two dependent loads instead of four.
struct TexDev {
    int32_t type;                  // AKR_TEX_CONSTANT / AKR_TEX_IMAGE
    float value[3];                // constant colour
    int32_t w, h;                  // image size
    int64_t off;                   // image's first float in SceneDev::images
};

struct SceneDev {
    const AKR_GLOBAL ShadeTri *tri;     // per global triangle id
    const AKR_GLOBAL float *texcoords;  // 6 per triangle (read only when has_image_tex)
    int32_t has_image_tex;
    const AKR_GLOBAL MatDev *mats;
    const AKR_GLOBAL TexDev *texs;
    const AKR_GLOBAL float *images;
    const AKR_GLOBAL LightDev *lights;
    const AKR_GLOBAL float *light_cdf;  // n_lights + 1
    int32_t n_lights;
    int32_t n_mats;
};

struct CameraDev {
    float r2c[16];
    float c2w[16];
    int32_t width, height;
};

struct TraceCounters {             // reduced per wave, one atomic per wave
    unsigned long long rays, box, tri;
    unsigned long long slots_trav, slots_leaf, slots_tri;  // lane-iterations: traversal loop, busy in it, tri loop
    unsigned long long visits;                             // internal-node visits
    unsigned long long deep;                               // rays whose stack went past kStackLds
    unsigned long long leaves;                             // leaf records fetched (exact leaf-box tests)
};

struct TraceArgs {                 // kept small: fewer SGPRs, higher residency
    const akr_bvh_node *nodes;
    const float4 *tris;            // akr_bvh_tri as 3 x float4
    const float4 *rays;            // 2 per ray
    const uint32_t *count;         // device count (queue) or nullptr -> n
    uint32_t n;
    uint32_t ovf_threads;          // threads covered by stack_ovf
    uint32_t *work;                // kWorkShards dynamic-fetch counters, kWorkStride apart (zeroed before)
    float4 *hits;                  // closest: (t, u, v, gid bits)
    akr_hit *abi_hits;             // optional: write akr_hit instead
    const uint32_t *mesh_base;     // for abi_hits: n_meshes + 1 prefix of triangle counts
    int32_t n_meshes;
    const float4 *shadow_color;    // shadow epilogue: colour.xyz + slot bits in .w
    float4 *L;                     //   L[slot] += colour when unoccluded
    uint2 *stack_ovf;              // (ref, t bits) entries beyond the LDS stack
    const float4 *wide_nodes;      // akr_bvh4_node as 4 x float4
    const float4 *wide_leaves;     // leaf blob: per leaf [lo.xyz hi.x | hi.yz first count] + its triangles
                                   // (3 x float4 each); wide leaf refs hold the float4 offset
    uint32_t wide_root;            // wide reference of the real root
    uint32_t lean;                 // 1: lean slot tests allowed (wide view's frames bounded by 2^40)
    uint32_t any_far_first;        // 1: shadow (boolean occlusion) rays visit the far slots first (order-free)
    TraceCounters *counters;       // [3]: closest, any, shadow
    uint32_t *ray_steps;           // COUNT builds, diagnostic: per ray, traversal iterations + triangle tests
    uint32_t step_cap;             // COUNT builds with ray_steps: a ray stops after this many steps (0: none;
                                   // the cost-ordered fetch's pilot, whose hits nobody reads)
};

struct ShadeArgs {
    SceneDev sc;
    const float4 *ray_in;
    const float4 *state_in;        // beta.xyz, seed bits
    const uint32_t *slot_in;
    const float4 *hit_in;
    const uint32_t *count_in;
    float4 *ray_out;
    float4 *state_out;
    uint32_t *slot_out;
    uint32_t *count_out;
    float4 *shadow_ray;
    float4 *shadow_color;
    uint32_t *shadow_count;
    uint32_t *seed;                // per slot: written when the path ends this bounce
    float4 *L;
    uint4 *probe;                  // optional, per slot (akr_pixel_probe): .y closest-hit / .z shadow rays
    int32_t depth;
    int32_t max_depth;
    int32_t last;                  // no extension ray is traced after this bounce
};

// One AO bounce (cpu/integrator.cpp:46-56) for every queued camera hit: appends the AO ray to
// ray_out (+ colour (1,1,1, slot) for a shadow-mode trace, or the slot for a closest-hit trace).
struct AoShadeArgs {
    const ShadeTri *tri;
    const float4 *hit_in;
    const uint32_t *slot_in;
    const float4 *state_in;        // seed bits in .w
    const uint32_t *count_in;
    uint32_t *seed;                // per slot: the sampler state after the sample
    float4 *ray_out;
    float4 *color_out;             // shadow-mode queue: (1, 1, 1, slot bits), or nullptr
    uint32_t *slot_out;            // closest-hit queue: slot, or nullptr
    uint32_t *count_out;
};

// After a closest-hit AO trace: L[slot] += 1 unless the hit has t < occlude.
struct AoResolveArgs {
    const float4 *hits;            // (t, u, v, gid bits) per queue entry
    const uint32_t *slot;
    const uint32_t *count;
    float4 *L;
    float occlude;
};

struct RaygenArgs {
    CameraDev cam;
    const uint32_t *pixel;         // per slot: x | y << 16
    uint32_t n;
    uint32_t *seed;
    float4 *L;
    float4 *ray_out;
    float4 *state_out;
    uint32_t *slot_out;
    uint32_t *count_out;
    int32_t first_pass;
    uint4 *probe;                  // optional, per slot (akr_pixel_probe): .y counts the camera ray
    const uint32_t *order;         // optional: queue position -> slot (the cost order)
    uint32_t slot_base;            // without `order`: queue position i holds slot slot_base + i
};

struct SplatArgs {
    float4 *L;
    float4 *film;
    uint32_t n;
    float ray_clamp;
    const uint32_t *order;         // optional: slot of entry i (the cost order) ...
    uint32_t slot_base;            // ... else slot_base + i
};

// k_path counting build: per-wave phase profile (wall clock, 100 MHz), summed over waves
struct PathProfile {
    unsigned long long waves;      // waves that ran
    unsigned long long outer;      // outer iterations
    unsigned long long procs;      // processing phases (A)
    unsigned long long trav_iters; // traversal-loop iterations (B)
    unsigned long long t_proc, t_trav, t_leaf, t_total;  // ticks in A, B, C, and the whole wave
    unsigned long long t_max;      // longest wave (atomicMax)
    unsigned long long lanes_proc; // waiting lanes processed, summed over phases
    unsigned long long t_shade;    // ticks of A spent on finished rays' results (shading, shadow hand-over)
    unsigned long long spec_started, spec_aborted;  // k_path_spec: speculative samples started / dropped
    // time split of B and C (ticks, wave-uniform clocks summed per wave): load issue, the explicit
    // wait for the loads, the dependent work after them
    unsigned long long tv_issue, tv_wait, tv_comp, tl_issue, tl_wait, tl_comp;
    // time split of A (k_path): the park, the finished rays' results (t_shade above), the sample end
    // with the splat, pixel fetch and camera ray, and the unpark with the new rays' start
    unsigned long long tp_park, tp_next, tp_begin;
    unsigned long long tp_load;    // of t_shade: until the hit's shading record is loaded
    unsigned long long leaf_phases, leaf_holders;  // leaf phases with a leaf held, lanes holding one (summed per wave)
};

// Persistent path kernel (k_path): the whole sample loop of every pixel of the tile list.
struct PathArgs {
    TraceArgs t;                   // BVH, wide view, overflow stacks, counters
    SceneDev sc;
    CameraDev cam;
    const uint32_t *pixel;         // per slot: x | y << 16
    float4 *film;                  // per slot: (rgb sums, weight), written when the pixel's samples are done
    uint32_t *work;                // kWorkShards pixel-fetch counters, kWorkStride apart (zeroed before)
    uint32_t n_pix, spp;
    int32_t max_depth;
    float ray_clamp;
    uint32_t min_wait;             // a wave processes its waiting lanes once min_wait / 64 of its live lanes wait
    PathProfile *prof;             // counting build only
    float4 *contrib;               // k_path_defer: per lane, [18][lanes]: 16 NEE contributions awaiting their
                                   // shadow result (parity * 8 + bounce), then the waiting extension ray
    uint32_t mix;                  // k_path_defer: scrambled pixel order within each XCD shard
    const uint32_t *order;         // optional: fetch index -> slot (cost-ordered fetch)
    uint32_t order_mode;           // with `order`: FETCH_LINEAR (costliest first) or FETCH_PAIR (kernels.hip)
    uint32_t prio;                 // 0, or: waves fetching in the first prio/256 of a shard raise their priority
    uint4 *probe;                  // optional, per slot (akr_pixel_probe): final sampler state; the counting
                                   // build adds the pixel's closest-hit and shadow rays
    uint32_t *fault;               // mapped host word: set when a wave stops on the hang guard (k_path_defer)
    uint32_t fault_test;           // test only: k_path_defer raises `fault` once at the end of the launch
    uint32_t spec_depth;           // k_path_spec: levels of the speculation tree (samples beyond the head)
    const uint32_t *gate;          // optional: the launch exits at once unless *gate == gate_want (two
    uint32_t gate_want;            //   candidate forms launched back to back, k_pick_form chose one)
    uint32_t probe_clock;          // diagnostic (counting build, option "pixel_probe" 2): the probe's flags
                                   // carry the pixel's completion time, (wall clock >> 4) << 8 | flags
    uint32_t *lines;               // counting build, k_path, option "count_lines": bitmap of the 128-B lines
    uint32_t lines_span[4];        // read; bit ranges [span[r], span[r + 1]) of the wide nodes, the leaf blob
                                   // and the shading records
};

}  // namespace akr
