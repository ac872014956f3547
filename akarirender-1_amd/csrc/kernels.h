// kernels.h — host-side launchers of the gfx950 kernels (kernels.hip).
#pragma once
#include "akr_device.h"

namespace akr {

// TRACE_PILOT: closest-hit traversal that records only each ray's step count (a.ray_steps, capped at
// a.step_cap) for the cost-ordered fetch's pilot: no hits, no counters
enum : int { TRACE_CLOSEST = 0, TRACE_ANY = 1, TRACE_SHADOW = 2, TRACE_PILOT = 3 };

// tight = standard slab test (default); !tight = the reference's intersectAABB, bit for bit
void launch_trace(int mode, bool count, bool tight, bool wide, const TraceArgs &a, uint32_t grid, hipStream_t st);
int trace_blocks_per_cu(int mode);
void launch_raygen(const RaygenArgs &a, hipStream_t st);
void launch_shade(const ShadeArgs &a, uint32_t max_items, hipStream_t st);
void launch_splat(const SplatArgs &a, uint32_t max_items, hipStream_t st);
void launch_pick_form(const unsigned long long *sum, unsigned long long thresh, uint32_t *gate, hipStream_t st);
void launch_store_word(const uint32_t *src, uint32_t *dst, hipStream_t st);
void launch_ao_shade(const AoShadeArgs &a, uint32_t max_items, hipStream_t st);
void launch_ao_resolve(const AoResolveArgs &a, uint32_t max_items, hipStream_t st);
// persistent path kernel forms
enum : int { PATH_PLAIN = 0, PATH_DEFER = 1, PATH_SPEC = 2 };
void launch_path(bool count, int kind, bool tab, const PathArgs &a, uint32_t grid, hipStream_t st);
int path_blocks_per_cu(int kind, bool tab);
bool path_tab_fits(int32_t n_mats, int32_t n_lights);
void launch_check_weights(const float4 *film, uint32_t n, float expect, uint32_t *bad, hipStream_t st);
void launch_merge_film(const float4 *film, const uint32_t *pixel, const uint32_t *order, uint32_t n, int32_t width,
                       float *rad, float *w, hipStream_t st);
void launch_unpack(const float4 *film, uint32_t n, float *rad, float *w, hipStream_t st);
void launch_expand_pixels(const uint4 *tiles, uint32_t n_tiles, uint32_t n, uint32_t *pixel, hipStream_t st);
void launch_probe_seed(const uint32_t *seed, uint32_t n, uint4 *probe, hipStream_t st);
void launch_probe_cost(const uint4 *probe, uint32_t n, uint32_t *cost, hipStream_t st);
// cost-ordered pixel fetch: pilot camera rays, sort keys, and the stable key sort (lbvh.hip, rocPRIM)
// 5-bit cost classes (31 = the costliest, with the rays the pilot does not trace): with the shard's 3 bits
// the key is one byte, so the radix sort is a single 8-bit pass (12-bit classes took 17 kernel launches,
// ~0.11 ms; the pilot's 64-step cap at the default shift 2 needs 17 classes)
constexpr uint32_t kOrderClassBits = 5, kOrderClassMask = (1u << kOrderClassBits) - 1u;
void launch_pilot_rays(const CameraDev &cam, const uint32_t *pixel, uint32_t n, uint32_t sub, float4 *rays,
                       hipStream_t st);
void launch_order_keys(const uint32_t *steps, uint32_t n, uint32_t shift, uint32_t cmax, uint32_t sub, uint32_t *key,
                       uint32_t *idx, hipStream_t st, unsigned long long *sum = nullptr);
size_t pixel_order_tmp_bytes(uint32_t n);
void sort_pixel_order(void *tmp, size_t tmp_bytes, const uint32_t *key_in, uint32_t *key_out, const uint32_t *idx_in,
                      uint32_t *idx_out, uint32_t n, hipStream_t st);

}  // namespace akr
