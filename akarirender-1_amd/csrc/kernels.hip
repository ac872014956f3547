// kernels.hip — hand-written gfx950 kernels of the wavefront path tracer.
//
//   k_trace<MODE,...>  BVH2 traversal, one ray per lane, LDS-resident stack, persistent waves that
//                      refill idle lanes from the queue (TBVHAccelerator::intersect / occlude,
//                      bvh-accelerator.h:488-547)
//   k_raygen           camera rays for every path slot (pathtracer.h:61-64, camera.h:67-86)
//   k_shade            hit -> emission / BSDF sample / NEE light sample, wave-ballot compaction
//                      of live paths and shadow rays (pathtracer.h:69-132, 137-162)
//   k_splat            Tile::add_sample per pixel, in sample order (core/film.h:66-70)
//
// Numerics: f32 with the reference's operation order (akr_math.h); the library is built with
// -ffp-contract=off and correctly rounded division/sqrt.
#include "akr_device.h"
#include "akr_math.h"
#include "kernels.h"

namespace akr {

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __uint_as_float(u); }

// intersectAABB (bvh-accelerator.h:89-103); returns -1 on a miss.  The reference accepts every
// box whose slab interval is non-empty and starts before tmax — including boxes that lie wholly
// BEHIND the origin (exit m1 < tmin).  TIGHT additionally requires t <= m1 (the standard slab
// test): it culls only boxes that cannot contain a hit with t > tmin, so it changes which nodes
// are visited, never which triangle is the closest hit.
template <bool TIGHT, bool FAST = false>
__device__ __forceinline__ float box_test(float lox, float hix, float loy, float hiy, float loz, float hiz, V3 o,
                                          V3 invd, float tmin, float tmax) {
    float t0x = (lox - o.x) * invd.x, t1x = (hix - o.x) * invd.x;
    float t0y = (loy - o.y) * invd.y, t1y = (hiy - o.y) * invd.y;
    float t0z = (loz - o.z) * invd.z, t1z = (hiz - o.z) * invd.z;
    float m0, m1, t;
    if (FAST) {
        // Only for rays whose origin and 1/d are finite and non-zero (fast_box_ok): then no slab
        // value is NaN, and the hardware min/max (v_min3/v_max3) select the same values as the
        // reference's std::min/max ternaries — they can differ only in the sign of a zero, which
        // no comparison below can see.
        m0 = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
        m1 = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
        t = fmaxf(tmin, m0);
    } else {
        m0 = rmax(rmax(rmin(t0x, t1x), rmin(t0y, t1y)), rmin(t0z, t1z));
        m1 = rmin(rmin(rmax(t0x, t1x), rmax(t0y, t1y)), rmax(t0z, t1z));
        t = rmax(tmin, m0);
    }
    bool hit = m0 <= m1 && !(t >= tmax);
    if (TIGHT) hit = hit && t <= m1;
    return hit ? t : -1.0f;
}

// A ray whose slab values can never be NaN: finite origin, finite non-zero 1/d components, non-NaN
// tmin/tmax
// (0 * inf arises only from an infinite 1/d or an infinite/NaN origin; box bounds are finite or
// the +-inf of an empty box, which a finite non-zero 1/d maps to +-inf, never NaN).
__device__ __forceinline__ bool fast_box_ok(V3 o, V3 invd, float tmin, float tmax) {
    return isfinite(o.x) && isfinite(o.y) && isfinite(o.z) && isfinite(invd.x) && isfinite(invd.y) &&
           isfinite(invd.z) && invd.x != 0.0f && invd.y != 0.0f && invd.z != 0.0f && !isnan(tmin) && !isnan(tmax);
}

// MeshInstance::intersect (instance.h:42-80), Moller-Trumbore on a leaf record (v0, e1, e2).
__device__ __forceinline__ bool mt(V3 o, V3 d, float tmin, float tmax, float4 a, float4 b, float4 c, float best,
                                   float &tout, float &uout, float &vout) {
    V3 v0{a.x, a.y, a.z}, e1{b.x, b.y, b.z}, e2{c.x, c.y, c.z};
    V3 h = cross(d, e2);
    float det = dot(e1, h);
    if (det > -1e-6f && det < 1e-6f) return false;
    float f = 1.0f / det;
    V3 s = sub(o, v0);
    float u = f * dot(s, h);
    if (u < 0.0f || u > 1.0f) return false;
    V3 q = cross(s, e1);
    float v = f * dot(d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    float t = f * dot(e2, q);
    if (t > tmin && t < tmax && t < best) {
        tout = t;
        uout = u;
        vout = v;
        return true;
    }
    return false;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ unsigned long long wave_max(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t lane_prefix(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Reserve `want ? 1 : 0` queue entries per thread of a whole workgroup, for two queues at once:
// wave ballots + mbcnt prefixes, per-wave counts through LDS, one returning atomic per queue per
// workgroup (issued by two different waves, so the two round trips overlap).  A single counter
// word sustains only ~88 returning atomics/us chip-wide (MI355X_MICROARCH.md, dequeue), so one
// atomic per WAVE made the shade kernel atomic-bound; per workgroup it is 4x fewer.
// Must be reached by every thread of the block; a second call in the same kernel needs a barrier
// before it (the LDS words are the same).
template <int BS = kBlock>
__device__ __forceinline__ void block_append2(bool want_a, uint32_t *ctr_a, uint32_t &pos_a, bool want_b,
                                              uint32_t *ctr_b, uint32_t &pos_b) {
    constexpr int kWaves = BS / 64;
    __shared__ uint32_t s_cnt[2][kWaves];
    __shared__ uint32_t s_base[2];
    const unsigned long long ma = __ballot(want_a), mb = __ballot(want_b);
    const uint32_t w = threadIdx.x / 64;
    if (__lane_id() == 0) {
        s_cnt[0][w] = (uint32_t)__popcll(ma);
        s_cnt[1][w] = (uint32_t)__popcll(mb);
    }
    __syncthreads();
    if (threadIdx.x == 0 || threadIdx.x == 64 % BS) {
        const int q = threadIdx.x == 0 ? 0 : 1;
        uint32_t tot = 0;
        for (int k = 0; k < kWaves; k++) tot += s_cnt[q][k];
        s_base[q] = tot ? atomicAdd(q == 0 ? ctr_a : ctr_b, tot) : 0;
    }
    __syncthreads();
    uint32_t ba = s_base[0], bb = s_base[1];
    for (uint32_t k = 0; k < w; k++) {
        ba += s_cnt[0][k];
        bb += s_cnt[1][k];
    }
    pos_a = ba + lane_prefix(ma);
    pos_b = bb + lane_prefix(mb);
}

// ------------------------------------------------------------------------------------- trace
// The leaf phase's triangle records are loaded with the leaf's header in one batch (EXPERIMENTS.md
// §9, r18).  They are used only once the leaf's box test has passed, so without this the compiler
// sinks their loads behind that test: a second dependent round trip before the first triangle test
// (MT's first operation needs e2).  An empty asm that reads them keeps the loads in the batch.
__device__ __forceinline__ void issue_together(const float4 &a, const float4 &b, const float4 &c, const float4 &d,
                                               const float4 &e, const float4 &f) {
    asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(c.x), "v"(c.y),
                 "v"(c.z), "v"(d.x), "v"(d.y), "v"(d.z), "v"(d.w), "v"(e.x), "v"(e.y), "v"(e.z), "v"(f.x), "v"(f.y),
                 "v"(f.z));
}

__device__ __forceinline__ bool is_internal(uint32_t c) { return !(c & AKR_CHILD_LEAF); }
__device__ __forceinline__ bool is_leaf(uint32_t c) { return (c & AKR_CHILD_LEAF) && c != AKR_CHILD_EMPTY; }

// Traversal stack pointers carry their address space in the type (LDS = 3, global = 1), so the
// compiler cannot merge the LDS push/pop with the overflow one of the other branch into a single
// flat (generic-address) access — which it does with plain pointers, turning every push/pop flat.
// An entry is one u64: node ref in the low word, entry-distance bits in the high word.
typedef __attribute__((address_space(3))) unsigned long long lds_u64;
typedef __attribute__((address_space(1))) unsigned long long glb_u64;

// An LDS stack entry: 8 B, [entry][thread]
constexpr int kStackLdsU64 = kStackLds * kTraceBlock;
__device__ __forceinline__ unsigned long long lds_get(const lds_u64 *s, int e, uint32_t tid) {
    return s[e * kTraceBlock + tid];
}
__device__ __forceinline__ void lds_put(lds_u64 *s, int e, uint32_t tid, unsigned long long v) {
    s[e * kTraceBlock + tid] = v;
}

// Pop the next stacked node whose stored entry distance is not beyond `lim` (the reference
// re-tests a popped node's box against the current best, bvh-accelerator.h:500-503).
__device__ __forceinline__ uint32_t stack_pop(const lds_u64 *s_stack, const glb_u64 *ovf, uint32_t ovf_threads,
                                              uint32_t tid, uint32_t gtid, int &sp, float lim) {
    // while no lane of the wave is past the LDS part, an LDS-only loop: the overflow branch's
    // exec-mask split stays out of the common pop (with the uniform push below: whole frame -1.8 %,
    // profiles/r21_uniform_ovf_ab.log)
    if (__ballot(sp > kStackLds) == 0) {
        while (sp > 0) {
            --sp;
            const unsigned long long e = lds_get(s_stack, sp, tid);
            if (!(__uint_as_float((uint32_t)(e >> 32)) > lim)) return (uint32_t)e;
        }
        return AKR_CHILD_EMPTY;
    }
    while (sp > 0) {
        --sp;
        unsigned long long e;
        if (sp < kStackLds) e = lds_get(s_stack, sp, tid);
        else e = ovf[(size_t)(sp - kStackLds) * ovf_threads + gtid];
        if (!(__uint_as_float((uint32_t)(e >> 32)) > lim)) return (uint32_t)e;
    }
    return AKR_CHILD_EMPTY;
}

// Visit internal node `cur`: test both child boxes, continue with the near one (near = left iff
// d[axis] > 0), push the far one with its entry distance, or pop when neither is entered.
template <bool TIGHT, bool FAST, bool ANY>
__device__ __forceinline__ void visit_node(const float4 *nodesf, const uint4 *nodesu, uint32_t &cur, V3 o, V3 d,
                                           V3 invd, float tmin, float tmax, float best, lds_u64 *s_stack, glb_u64 *ovf,
                                           uint32_t ovf_threads, uint32_t tid, uint32_t gtid, int &sp) {
    const float4 q0 = nodesf[4 * (size_t)cur + 0];
    const float4 q1 = nodesf[4 * (size_t)cur + 1];
    const float4 q2 = nodesf[4 * (size_t)cur + 2];
    const uint4 q3 = nodesu[4 * (size_t)cur + 3];
    const float t0 = box_test<TIGHT, FAST>(q0.x, q0.y, q0.z, q0.w, q2.x, q2.y, o, invd, tmin, tmax);
    const float t1 = box_test<TIGHT, FAST>(q1.x, q1.y, q1.z, q1.w, q2.z, q2.w, o, invd, tmin, tmax);
    const float lim = ANY ? tmax : best;
    const bool p0 = !(t0 < 0.0f || t0 > lim);
    const bool p1 = !(t1 < 0.0f || t1 > lim);
    const float dax = q3.z == 0 ? d.x : (q3.z == 1 ? d.y : d.z);
    const bool left_first = dax > 0;
    const uint32_t near_ref = left_first ? q3.x : q3.y;
    const uint32_t far_ref = left_first ? q3.y : q3.x;
    const bool pn = left_first ? p0 : p1;
    const bool pf = left_first ? p1 : p0;
    const float tf = left_first ? t1 : t0;
    if (pn && pf) {
        const unsigned long long e = (unsigned long long)far_ref | ((unsigned long long)__float_as_uint(tf) << 32);
        if (sp < kStackLds) lds_put(s_stack, sp, tid, e);
        else ovf[(size_t)(sp - kStackLds) * ovf_threads + gtid] = e;
        sp++;
    }
    cur = pn ? near_ref : (pf ? far_ref : stack_pop(s_stack, ovf, ovf_threads, tid, gtid, sp, lim));
}

// Visit wide node `cur` (akr_bvh4_node): test the four outward-quantized slot boxes, continue with
// the first entered slot in the BVH2 depth-first order and push the other entered slots behind
// it, each with its (conservative, <= exact) entry distance.  Returns the number of slot boxes
// tested.  Only for rays with fast_box_ok(): the conservative boxes then pass whenever the exact
// ones do (slab arithmetic is monotone in the bounds), so no leaf the BVH2 traversal reaches is
// skipped; leaves are re-tested with their exact boxes before their triangles.
__device__ __forceinline__ float ubyte(uint32_t w, int k) {  // v_cvt_f32_ubyte{k}
    return (float)((w >> (8 * k)) & 0xFFu);
}

// Continue with the first entered slot of a wide node in the BVH2 depth-first order and push the
// other entered slots behind it, each with its entry distance; pop when no slot is entered.
// `dpos` holds the ray's direction signs: bit a = (d[a] > 0), the octant.  The node's order words
// (akr_bvh4_node::order) give each slot's position in the depth-first order of that octant: byte
// dpos, two bits per slot.  Entered slots are ranked by position without moving any data: the first
// becomes `cur`, each other one is written straight to its stack entry sp + (number of entered
// slots at later positions), so the earliest is popped first.
// NOPOP: when no slot is entered, return true instead of popping, so the caller pops at one site
// for this case and for a postponed leaf
template <bool ANY, bool NOPOP = false>
__device__ __forceinline__ bool wide_order_push(uint32_t order_lo, uint32_t order_hi, uint32_t dpos, const float (&t)[4],
                                                const bool (&hit)[4], const uint32_t (&ref)[4], uint32_t &cur, float lim,
                                                lds_u64 *s_stack, glb_u64 *ovf, uint32_t ovf_threads, uint32_t tid,
                                                uint32_t gtid, int &sp) {
    const uint32_t perm = ((dpos & 4u) ? order_hi : order_lo) >> ((dpos & 3u) << 3);
    const uint32_t pos[4] = {perm & 3u, (perm >> 2) & 3u, (perm >> 4) & 3u, (perm >> 6) & 3u};
    uint32_t pm = 0;  // entered slots, by position
#pragma unroll
    for (int k = 0; k < 4; k++) pm |= hit[k] ? (1u << pos[k]) : 0u;
    if (pm == 0) {
        if constexpr (NOPOP) return true;
        cur = stack_pop(s_stack, ovf, ovf_threads, tid, gtid, sp, lim);
        return false;
    }
    const uint32_t rest = pm & (pm - 1u);  // entered slots after the first: pushed
    if (__ballot(sp + 4 > kStackLds) == 0) {  // wave-uniform: no exec-mask split in the common case
        // all in LDS: four unconditional writes, no exec-mask branches; a slot that is not pushed
        // writes entry sp + 3, which lies above the new top (sp grows by at most 3) and is dead
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool push = (rest >> pos[k]) & 1u;
            const int e = sp + (push ? (int)__popc(rest >> (pos[k] + 1u)) : 3);
            lds_put(s_stack, e, tid, (unsigned long long)ref[k] | ((unsigned long long)__float_as_uint(t[k]) << 32));
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if ((rest >> pos[k]) & 1u) {
                const int e = sp + (int)__popc(rest >> (pos[k] + 1u));
                const unsigned long long v = (unsigned long long)ref[k] | ((unsigned long long)__float_as_uint(t[k]) << 32);
                if (e < kStackLds) lds_put(s_stack, e, tid, v);
                else ovf[(size_t)(e - kStackLds) * ovf_threads + gtid] = v;
            }
        }
    }
    sp += (int)__popc(rest);
    // the slot at the first entered position (selects on static indices: no private array)
    const uint32_t first = pm ^ rest;
    uint32_t c = AKR_CHILD_EMPTY;
#pragma unroll
    for (int k = 0; k < 4; k++) c = ((first >> pos[k]) & 1u) ? ref[k] : c;
    cur = c;
    return false;
}

template <bool TIGHT, bool ANY>
__device__ __forceinline__ int visit_wide(const float4 *wn, uint32_t &cur, V3 o, uint32_t dpos, V3 invd, float tmin, float tmax,
                                          float best, lds_u64 *s_stack, glb_u64 *ovf, uint32_t ovf_threads,
                                          uint32_t tid, uint32_t gtid, int &sp) {
    const char *wb = reinterpret_cast<const char *>(wn);  // 32-bit byte offset, as visit_wide_lean
    const uint32_t off = cur << 6;
    const float4 h = *reinterpret_cast<const float4 *>(wb + off);       // origin.xyz, meta
    const uint4 c = *reinterpret_cast<const uint4 *>(wb + off + 16);    // slot refs
    const uint4 qa = *reinterpret_cast<const uint4 *>(wb + off + 32);   // qlo_x, qhi_x, qlo_y, qhi_y
    const uint4 qb = *reinterpret_cast<const uint4 *>(wb + off + 48);   // qlo_z, qhi_z, order[2]
    const uint32_t meta = __float_as_uint(h.w);
    const float sx = __uint_as_float((meta & 0xFFu) << 23);
    const float sy = __uint_as_float(((meta >> 8) & 0xFFu) << 23);
    const float sz = __uint_as_float(((meta >> 16) & 0xFFu) << 23);
    const float lim = ANY ? tmax : best;
    float t[4];
    bool hit[4];
    uint32_t ref[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        // bound = fmaf(q, 2^e, origin): the product is exact, the one rounding is the builder's
        const float lox = __builtin_fmaf(ubyte(qa.x, k), sx, h.x), hix = __builtin_fmaf(ubyte(qa.y, k), sx, h.x);
        const float loy = __builtin_fmaf(ubyte(qa.z, k), sy, h.y), hiy = __builtin_fmaf(ubyte(qa.w, k), sy, h.y);
        const float loz = __builtin_fmaf(ubyte(qb.x, k), sz, h.z), hiz = __builtin_fmaf(ubyte(qb.y, k), sz, h.z);
        t[k] = box_test<TIGHT, true>(lox, hix, loy, hiy, loz, hiz, o, invd, tmin, tmax);
        hit[k] = ref[k] != AKR_CHILD_EMPTY && !(t[k] < 0.0f || t[k] > lim);
    }
    const int tested = (c.x != AKR_CHILD_EMPTY) + (c.y != AKR_CHILD_EMPTY) + (c.z != AKR_CHILD_EMPTY) +
                       (c.w != AKR_CHILD_EMPTY);
    wide_order_push<ANY>(qb.z, qb.w, dpos, t, hit, ref, cur, lim, s_stack, ovf, ovf_threads, tid, gtid, sp);
    return tested;
}

// Lean slot test ("lean slot test"): the same conservative test in fewer VALU
// operations.  Per node and axis it forms oq = (origin - o) * invd and sc = 2^e * invd (exact), and
// per slot bound one fma: q * sc + oq is (bound - o) * invd in real arithmetic.  An error slack
// E = 8u * (|oq| + 255 |sc|) + 2^-120 (u = 2^-24), folded into oq once per node (oq - E for the
// entry side, oq + E for the exit side), makes the per-axis entry value <= and the exit value >=
// the reference's RN(RN(b - o) * invd) for the exact BVH2 box (the builder quantizes outward in
// real arithmetic, bvh_wide.cpp).  Entry and exit bounds are chosen per node from the sign of invd
// instead of a min/max per slot.  So the test passes whenever the exact one does, with an entry
// distance no larger: leaves are still reached, in order, and re-tested exactly.  Only for rays
// with `lean_ok` (fast_box_ok, tmin >= 0, |o| <= 2^60, |invd| <= 2^64) on a wide view whose frame
// origins and steps are <= 2^40, which bounds every term below 2^126 (no overflow, no NaN); with
// tmin >= 0 the reference's "t < 0" reject cannot fire and TIGHT's t <= m1 implies m0 <= m1, and
// t < tmax is t <= tmaxp (the float below tmax).
// The wide node's four 16-B loads (a 32-bit byte offset from the array base: SGPR base + VGPR offset
// addressing, one 32-bit shift instead of two 64-bit address operations per visit, 0.7 % of the
// frame; the wide view holds fewer than 2^26 nodes, checked when it is uploaded, kMaxWideNodes)
struct WideNode {
    float4 h;
    uint4 c, qa, qb;
};
__device__ __forceinline__ WideNode wide_load(const float4 *wn, uint32_t cur) {
    const char *wb = reinterpret_cast<const char *>(wn);
    const uint32_t off = cur << 6;
    WideNode nd;
    nd.h = *reinterpret_cast<const float4 *>(wb + off);
    nd.c = *reinterpret_cast<const uint4 *>(wb + off + 16);
    nd.qa = *reinterpret_cast<const uint4 *>(wb + off + 32);
    nd.qb = *reinterpret_cast<const uint4 *>(wb + off + 48);
    return nd;
}

template <bool ANY, bool NOPOP = false>
__device__ __forceinline__ int visit_wide_lean_node(const WideNode &nd, uint32_t &cur, V3 o, uint32_t dpos, V3 invd,
                                                    float tmin, float tmaxp, float best, lds_u64 *s_stack, glb_u64 *ovf,
                                                    uint32_t ovf_threads, uint32_t tid, uint32_t gtid, int &sp,
                                                    bool *need_pop = nullptr) {
    const float4 h = nd.h;
    const uint4 c = nd.c, qa = nd.qa, qb = nd.qb;
    const uint32_t meta = __float_as_uint(h.w);
    constexpr float kRel = 0x1p-21f;   // 8u
    constexpr float kAbs = 0x1p-120f;  // covers an underflowing sc
    const float scx = __uint_as_float((meta & 0xFFu) << 23) * invd.x;
    const float scy = __uint_as_float(((meta >> 8) & 0xFFu) << 23) * invd.y;
    const float scz = __uint_as_float(((meta >> 16) & 0xFFu) << 23) * invd.z;
    const float oqx = (h.x - o.x) * invd.x, oqy = (h.y - o.y) * invd.y, oqz = (h.z - o.z) * invd.z;
    const float ex = __builtin_fmaf(__builtin_fmaf(255.0f, fabsf(scx), fabsf(oqx)), kRel, kAbs);
    const float ey = __builtin_fmaf(__builtin_fmaf(255.0f, fabsf(scy), fabsf(oqy)), kRel, kAbs);
    const float ez = __builtin_fmaf(__builtin_fmaf(255.0f, fabsf(scz), fabsf(oqz)), kRel, kAbs);
    const float nox = oqx - ex, noy = oqy - ey, noz = oqz - ez;  // entry side
    const float fox = oqx + ex, foy = oqy + ey, foz = oqz + ez;  // exit side
    const bool px = invd.x > 0.0f, py = invd.y > 0.0f, pz = invd.z > 0.0f;
    const uint32_t qnx = px ? qa.x : qa.y, qfx = px ? qa.y : qa.x;
    const uint32_t qny = py ? qa.z : qa.w, qfy = py ? qa.w : qa.z;
    const uint32_t qnz = pz ? qb.x : qb.y, qfz = pz ? qb.y : qb.x;
    const float lim = ANY ? tmaxp : fminf(best, tmaxp);
    float t[4];
    bool hit[4];
    uint32_t ref[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const float nx = __builtin_fmaf(ubyte(qnx, k), scx, nox), fx = __builtin_fmaf(ubyte(qfx, k), scx, fox);
        const float ny = __builtin_fmaf(ubyte(qny, k), scy, noy), fy = __builtin_fmaf(ubyte(qfy, k), scy, foy);
        const float nz = __builtin_fmaf(ubyte(qnz, k), scz, noz), fz = __builtin_fmaf(ubyte(qfz, k), scz, foz);
        const float tk = fmaxf(fmaxf(nx, ny), fmaxf(nz, tmin));
        const float m1 = fminf(fminf(fx, fy), fminf(fz, lim));
        t[k] = tk;
        hit[k] = ref[k] != AKR_CHILD_EMPTY && tk <= m1;
    }
    const int tested = (c.x != AKR_CHILD_EMPTY) + (c.y != AKR_CHILD_EMPTY) + (c.z != AKR_CHILD_EMPTY) +
                       (c.w != AKR_CHILD_EMPTY);
    const bool np = wide_order_push<ANY, NOPOP>(qb.z, qb.w, dpos, t, hit, ref, cur, ANY ? tmaxp : best, s_stack, ovf,
                                                ovf_threads, tid, gtid, sp);
    if (NOPOP) *need_pop = np;
    return tested;
}

template <bool ANY>
__device__ __forceinline__ int visit_wide_lean(const float4 *wn, uint32_t &cur, V3 o, uint32_t dpos, V3 invd, float tmin,
                                               float tmaxp, float best, lds_u64 *s_stack, glb_u64 *ovf,
                                               uint32_t ovf_threads, uint32_t tid, uint32_t gtid, int &sp) {
    const WideNode nd = wide_load(wn, cur);
    return visit_wide_lean_node<ANY>(nd, cur, o, dpos, invd, tmin, tmaxp, best, s_stack, ovf, ovf_threads, tid, gtid, sp);
}

// The float just below `x` (x not NaN): t < x  <=>  t <= below(x) for every float t.
__device__ __forceinline__ float float_below(float x) {
    const uint32_t b = __float_as_uint(x);
    if (x > 0.0f) return __uint_as_float(b - 1u);
    if (x == 0.0f) return -0x1p-149f;
    return __uint_as_float(b + 1u);  // negative (incl. -inf -> NaN never: -inf has no float below)
}

__device__ __forceinline__ bool lean_ok(V3 o, V3 invd, float tmin, float tmax) {
    const float mo = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float mi = fmaxf(fmaxf(fabsf(invd.x), fabsf(invd.y)), fabsf(invd.z));
    return fast_box_ok(o, invd, tmin, tmax) && tmin >= 0.0f && tmax > -INFINITY && mo <= 0x1p60f && mi <= 0x1p64f;
}

// Result of one finished ray: the closest hit (float4 queue record or akr_hit), or for a shadow
// ray the NEE contribution L[slot] += colour when unoccluded (a slot has at most one shadow ray
// per bounce, so there is no write race).
template <int MODE>
__device__ __forceinline__ void emit_result(const TraceArgs &a, uint32_t idx, float best, float bu, float bv,
                                            uint32_t bgid, bool occluded) {
    constexpr bool ANY = MODE != TRACE_CLOSEST;
    if (MODE == TRACE_SHADOW) {
        if (!occluded) {
            const float4 c = a.shadow_color[idx];
            const uint32_t slot = fbits(c.w);
            float4 l = a.L[slot];
            l.x += c.x;
            l.y += c.y;
            l.z += c.z;
            a.L[slot] = l;
        }
    } else if (a.abi_hits) {
        akr_hit h;
        const bool hit = ANY ? occluded : (bgid != kNoHit);
        h.t = hit ? best : kInf;
        h.u = hit ? bu : 0.0f;
        h.v = hit ? bv : 0.0f;
        h.geom_id = -1;
        h.prim_id = -1;
        if (hit) {
            int lo = 0, hi = a.n_meshes;  // largest m with mesh_base[m] <= gid
            while (hi - lo > 1) {
                const int mid = (lo + hi) / 2;
                if (a.mesh_base[mid] <= bgid) lo = mid; else hi = mid;
            }
            h.geom_id = lo;
            h.prim_id = (int32_t)(bgid - a.mesh_base[lo]);
        }
        h._pad[0] = h._pad[1] = h._pad[2] = 0;
        a.abi_hits[idx] = h;
    } else {
        a.hits[idx] = make_float4(best, bu, bv, bitsf(bgid));
    }
}

// Exact BVH2 traversal of one lane's ray to completion (reference order and NaN semantics), for
// the rare rays the wide kernel cannot take (fast_box_ok false: a zero or denormal direction
// component, a non-finite origin or a NaN interval).  Runs inline while the rest of the wave
// waits, so no extra launch is ever needed; the lane's LDS stack is free (it holds no ray).
template <bool ANY, bool TIGHT>
__device__ __forceinline__ void trace_exact_core(const TraceArgs &a, V3 o, V3 d, V3 invd, float tmin, float tmax,
                                                 lds_u64 *s_stack, glb_u64 *ovf, uint32_t tid, uint32_t gtid, float &best,
                                                 float &bu, float &bv, uint32_t &bgid, bool &occluded) {
    const float4 *nodesf = reinterpret_cast<const float4 *>(a.nodes);
    const uint4 *nodesu = reinterpret_cast<const uint4 *>(a.nodes);
    const float4 r0 = nodesf[0], r2 = nodesf[2];
    const uint32_t root = nodesu[3].x;
    best = kInf;
    bu = bv = 0.0f;
    bgid = kNoHit;
    occluded = false;
    int sp = 0;
    const float tr = box_test<TIGHT, false>(r0.x, r0.y, r0.z, r0.w, r2.x, r2.y, o, invd, tmin, tmax);
    uint32_t cur = (root == AKR_CHILD_EMPTY || tr < 0.0f || tr > (ANY ? tmax : best)) ? AKR_CHILD_EMPTY : root;
    while (cur != AKR_CHILD_EMPTY) {
        if (is_internal(cur)) {
            visit_node<TIGHT, false, ANY>(nodesf, nodesu, cur, o, d, invd, tmin, tmax, best, s_stack, ovf, a.ovf_threads,
                                          tid, gtid, sp);
            continue;
        }
        const uint32_t first = akr_leaf_first(cur), cnt = akr_leaf_count(cur);
        for (uint32_t k = 0; k < cnt; k++) {
            const float4 ta = a.tris[3 * (size_t)(first + k) + 0];
            const float4 tb = a.tris[3 * (size_t)(first + k) + 1];
            const float4 tc = a.tris[3 * (size_t)(first + k) + 2];
            float t, u, v;
            if (mt(o, d, tmin, tmax, ta, tb, tc, ANY ? kInf : best, t, u, v)) {
                best = t;
                bu = u;
                bv = v;
                bgid = fbits(ta.w);
                if (ANY) {
                    occluded = true;
                    break;
                }
            }
        }
        if (ANY && occluded) break;
        cur = stack_pop(s_stack, ovf, a.ovf_threads, tid, gtid, sp, ANY ? tmax : best);
    }
}

template <int MODE, bool TIGHT>
__device__ __forceinline__ void trace_exact_lane(const TraceArgs &a, uint32_t idx, V3 o, V3 d, V3 invd, float tmin,
                                              float tmax, lds_u64 *s_stack, glb_u64 *ovf, uint32_t tid, uint32_t gtid) {
    float best, bu, bv;
    uint32_t bgid;
    bool occluded;
    trace_exact_core<MODE != TRACE_CLOSEST, TIGHT>(a, o, d, invd, tmin, tmax, s_stack, ovf, tid, gtid, best, bu, bv, bgid,
                                                   occluded);
    emit_result<MODE>(a, idx, best, bu, bv, bgid, occluded);
}

// One ray per lane; persistent waves.  Per outer iteration a wave
//   1. refills idle lanes from the queue (one atomic; the new rays' loads overlap step 2),
//   2. runs the traversal phase: visit internal nodes until every busy lane holds a pending leaf
//      or has run out of nodes.  A lane that finds a leaf postpones it and keeps descending
//      (speculative traversal, Aila & Laine 2009) so it does not idle while others search,
//   3. runs the leaf phase: Moller-Trumbore on the pending leaf of every lane.
// Leaves are still tested in the reference's depth-first order (near = left iff d[axis] > 0);
// speculation only visits extra internal nodes, against a stale (larger) best t, which can add
// box tests but never a different hit.  A node's two child boxes are tested when the node is
// visited and the far child is pushed with its entry distance, re-compared against the current
// best when popped — the reference's pop-time test of the node's own box.
// Registers are capped for 5 waves per SIMD (<= 96 VGPRs; the LDS stack allows 6 workgroups of
// 4 waves per CU): at the 6-wave cap (80 VGPRs) the kernel spills and the closest-hit launch is
// 4 % slower, the small (8-way split) launches 5 % slower.
#ifndef AKR_TRACE_WAVES
#define AKR_TRACE_WAVES 5
#endif
#define AKR_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(AKR_TRACE_WAVES)))
template <int MODE, bool COUNT, bool TIGHT, bool WIDE>
__global__ __launch_bounds__(kTraceBlock) AKR_TRACE_ATTR void k_trace(TraceArgs a) {
    constexpr bool ANY = MODE == TRACE_ANY || MODE == TRACE_SHADOW;  // occlusion query: any hit in (tmin, tmax)
    // the pilot's steps-only build (TRACE_PILOT) counts steps without the counting build's tallies
    constexpr bool STEPS = COUNT || MODE == TRACE_PILOT;
    __shared__ unsigned long long s_stack_mem[kStackLdsU64];
    lds_u64 *s_stack = (lds_u64 *)s_stack_mem;
    glb_u64 *stack_ovf = (glb_u64 *)a.stack_ovf;
    const uint32_t tid = threadIdx.x;
    const uint32_t gtid = blockIdx.x * kTraceBlock + tid;
    const uint32_t n = a.count ? *a.count : a.n;
    const float4 *nodesf = reinterpret_cast<const float4 *>(a.nodes);
    const uint4 *nodesu = reinterpret_cast<const uint4 *>(a.nodes);
    // virtual root (node 0): child 0 = real root with its box
    const float4 r0 = nodesf[0], r2 = nodesf[2];
    const uint32_t root = WIDE ? a.wide_root : nodesu[3].x;
    const float4 *wn = a.wide_nodes;
    unsigned long long c_rays = 0, c_box = 0, c_tri = 0, c_strav = 0, c_sleaf = 0, c_stri = 0, c_visit = 0, c_deep = 0,
                       c_leaf = 0;
    bool deep = false;  // COUNT only: this lane's ray has pushed past the LDS stack

    V3 o{0, 0, 0}, d{0, 0, 0}, invd{0, 0, 0};
    float tmin = 0.0f, tmax = 0.0f, tmaxp = 0.0f, best = kInf, bu = 0.0f, bv = 0.0f;
    bool lean = false;  // this ray may take the lean slot test (visit_wide_lean)
    uint32_t dpos = 0;  // direction signs: bit a = (d[a] > 0)
    uint32_t bgid = kNoHit, idx = 0, cur = AKR_CHILD_EMPTY, leaf = AKR_CHILD_EMPTY;
    int sp = 0;
    uint32_t steps = 0;  // COUNT only (ray_steps diagnostic)
    bool busy = false, occluded = false, drained = n == 0;
    bool need_exact = false;  // trace this lane's ray with the exact BVH2 walk (end of iteration)
    // The queue [0, n) is cut into kWorkShards contiguous ranges, each with its own counter on its
    // own 128-B line: one counter word saturates at ~88 returning atomics/us chip-wide, so a
    // single shared counter capped the refill rate.  A wave starts on shard blockIdx % 8 (the
    // blocks of one XCD share it: speed only, correctness never depends on placement) and moves
    // to the next shard when its shard is exhausted; every index is handed out exactly once.
    uint32_t shard = blockIdx.x % kWorkShards;
    int shards_left = kWorkShards;
    uint32_t s_lo = shard_begin(n, shard), s_hi = shard_begin(n, shard + 1);
    while (true) {
        // ---- 1. refill idle lanes (wave-uniform control flow): one atomic per refill; the new
        // rays' loads are consumed after this iteration's traversal phase, which hides them.
        bool fresh = false;
        float4 ra = {}, rb = {};
        if (!drained) {
            const unsigned long long idle = __ballot(!busy);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (nidle >= (uint32_t)(ANY ? kRefillMinAny : kRefillMin) || nidle == (uint32_t)__popcll(__ballot(1))) {
                const int leader = __ffsll((long long)idle) - 1;
                uint32_t base = 0;
                if ((int)__lane_id() == leader) base = atomicAdd(a.work + shard * kWorkStride, nidle);
                base = __shfl(base, leader);
                const uint32_t first = s_lo + base;  // may exceed s_hi once the shard is exhausted
                if (!busy) {
                    const uint32_t my = first + lane_prefix(idle);
                    if (my < s_hi && base < s_hi - s_lo) {
                        idx = my;
                        ra = a.rays[2 * (size_t)my];
                        rb = a.rays[2 * (size_t)my + 1];
                        fresh = true;
                    }
                }
                if (base + nidle >= s_hi - s_lo) {  // this shard is exhausted: move to the next open one
                    while (true) {
                        if (--shards_left == 0) {
                            drained = true;
                            break;
                        }
                        shard = (shard + 1) % kWorkShards;
                        s_lo = shard_begin(n, shard);
                        s_hi = shard_begin(n, shard + 1);
                        const uint32_t taken = __builtin_amdgcn_readfirstlane(__hip_atomic_load(
                            a.work + shard * kWorkStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        if (taken < s_hi - s_lo) break;
                    }
                }
            }
        }
        if (!__any(busy || fresh || need_exact)) {
            if (drained) break;
            continue;
        }
        if (__any(busy)) {
            // ---- 2. traversal phase (fast min/max box tests unless a lane's ray could make NaNs;
            // the wide kernel only ever holds rays with fast_box_ok)
            const bool wave_fast = WIDE || !__any(busy && !fast_box_ok(o, invd, tmin, tmax));
            while (true) {
                if (COUNT) {
                    c_strav++;  // every lane of the (converged) wave
                    c_sleaf += busy ? 1 : 0;
                }
                if (STEPS) steps += busy ? 1 : 0;
                // lean visits pop at one site with the leaf postponement below (as path_traverse);
                // the pilot (STEPS) keeps its step metric's old loop, on which the form rule is calibrated
                constexpr bool kOnePop = TIGHT && !STEPS;
                bool need_pop = false;
                if (WIDE && busy && is_internal(cur)) {
                    int nt;
                    if (kOnePop)
                        nt = visit_wide_lean_node<ANY, true>(wide_load(wn, cur), cur, o, dpos, invd, tmin, tmaxp, best,
                                                             s_stack, stack_ovf, a.ovf_threads, tid, gtid, sp, &need_pop);
                    else if (TIGHT)  // every wide-loop ray of the tight kernel is lean (others: exact lane)
                        nt = visit_wide_lean<ANY>(wn, cur, o, dpos, invd, tmin, tmaxp, best, s_stack, stack_ovf,
                                                  a.ovf_threads, tid, gtid, sp);
                    else
                        nt = visit_wide<TIGHT, ANY>(wn, cur, o, dpos, invd, tmin, tmax, best, s_stack, stack_ovf,
                                                    a.ovf_threads, tid, gtid, sp);
                    if (COUNT) {
                        c_box += nt;
                        c_visit++;
                        deep = deep || sp > kStackLds;
                    }
                    if (STEPS && a.step_cap && steps >= a.step_cap) cur = AKR_CHILD_EMPTY;  // pilot: cost capped
                } else if (!WIDE && busy && is_internal(cur)) {
                    if (COUNT) {
                        c_box += 2;
                        c_visit++;
                    }
                    if (wave_fast)
                        visit_node<TIGHT, true, ANY>(nodesf, nodesu, cur, o, d, invd, tmin, tmax, best, s_stack,
                                                     stack_ovf, a.ovf_threads, tid, gtid, sp);
                    else
                        visit_node<TIGHT, false, ANY>(nodesf, nodesu, cur, o, d, invd, tmin, tmax, best, s_stack,
                                                      stack_ovf, a.ovf_threads, tid, gtid, sp);
                    if (COUNT) deep = deep || sp > kStackLds;
                }
                if (busy && !need_pop && leaf == AKR_CHILD_EMPTY && is_leaf(cur)) {
                    leaf = cur;  // postpone the leaf and keep descending
                    need_pop = true;
                }
                // (an any-hit ray culls at the float below tmax, as the visit's own pop did: an entry at
                // tmax holds no hit below it)
                if (need_pop)
                    cur = stack_pop(s_stack, stack_ovf, a.ovf_threads, tid, gtid, sp, ANY ? (kOnePop ? tmaxp : tmax) : best);
                // leave for the leaf phase once at most kWhileExit lanes are still searching for
                // their first leaf (0: every lane holds a leaf or is done — classic while-while),
                // but not while nobody holds a leaf yet and someone still searches: the leaf phase
                // would have nothing to do (a wave's last rays would pay a full outer iteration per
                // node visit)
                const unsigned long long searching = __ballot(busy && leaf == AKR_CHILD_EMPTY && cur != AKR_CHILD_EMPTY);
                if ((uint32_t)__popcll(searching) <= (uint32_t)(ANY ? kWhileExitAny : kWhileExit) &&
                    (searching == 0 || __ballot(busy && leaf != AKR_CHILD_EMPTY) != 0))
                    break;
            }
            // ---- 3. leaf phase
            if (busy && leaf != AKR_CHILD_EMPTY) {
                uint32_t cnt;
                const float4 *tp;  // this leaf's triangle records (3 x float4 each)
                float4 pa, pb, pc;     // the first one, fetched together with the leaf header
                float4 pa1, pb1, pc1;  // and the second one (wide view only: its blob is padded)
                if (WIDE) {  // the leaf's exact box, with the current best: the BVH2 pop-time test
                    const float4 *lr = a.wide_leaves + (leaf & 0x7FFFFFFFu);
                    const float4 l0 = lr[0], l1 = lr[1];  // lo.xyz hi.x | hi.yz first count
                    pa = lr[2];
                    pb = lr[3];
                    pc = lr[4];
                    pa1 = lr[5];
                    pb1 = lr[6];
                    pc1 = lr[7];
                    issue_together(pa, pb, pc, pa1, pb1, pc1);
                    const float tl = box_test<TIGHT, true>(l0.x, l0.w, l0.y, l1.x, l0.z, l1.y, o, invd, tmin, tmax);
                    const bool in = !(tl < 0.0f || tl > (ANY ? tmax : best));
                    if (COUNT) {
                        c_box++;
                        c_leaf++;
                    }
                    cnt = in ? fbits(l1.w) : 0u;
                    tp = lr + 2;
                } else {
                    tp = a.tris + 3 * (size_t)akr_leaf_first(leaf);
                    cnt = akr_leaf_count(leaf);
                    pa = tp[0];
                    pb = tp[1];
                    pc = tp[2];
                }
                for (uint32_t k = 0; k < cnt; k++) {
                    if (COUNT && lane_prefix(__ballot(1)) == 0) c_stri += 64;
                    const float4 ta = k == 0 ? pa : (WIDE && k == 1 ? pa1 : tp[3 * k + 0]);
                    const float4 tb = k == 0 ? pb : (WIDE && k == 1 ? pb1 : tp[3 * k + 1]);
                    const float4 tc = k == 0 ? pc : (WIDE && k == 1 ? pc1 : tp[3 * k + 2]);
                    if (COUNT) c_tri++;
                    if (STEPS) steps++;
                    float t, u, v;
                    if (mt(o, d, tmin, tmax, ta, tb, tc, ANY ? kInf : best, t, u, v)) {
                        best = t;
                        bu = u;
                        bv = v;
                        bgid = fbits(ta.w);
                        if (ANY) {
                            occluded = true;
                            break;
                        }
                    }
                }
                leaf = AKR_CHILD_EMPTY;
            }
            if (busy && ((ANY && occluded) || cur == AKR_CHILD_EMPTY)) {
                busy = false;
                if constexpr (MODE != TRACE_PILOT) emit_result<MODE>(a, idx, best, bu, bv, bgid, occluded);
                if (STEPS && a.ray_steps) a.ray_steps[idx] = steps;
                if (COUNT) c_deep += deep ? 1 : 0;
            }
        }
        if (fresh) {
            o = V3{ra.x, ra.y, ra.z};
            d = V3{rb.x, rb.y, rb.z};
            tmin = ra.w;
            tmax = rb.w;
            invd = V3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
            dpos = (d.x > 0.0f ? 1u : 0u) | (d.y > 0.0f ? 2u : 0u) | (d.z > 0.0f ? 4u : 0u);
            // boolean occlusion (shadow mode): far slots first — the answer is order-free;
            // the ABI's any-hit query reports the t of the hit it finds, so it keeps the BVH2 order
            if (MODE == TRACE_SHADOW && a.any_far_first) dpos ^= 7u;
            if (WIDE && TIGHT) {
                lean = a.lean && lean_ok(o, invd, tmin, tmax);
                tmaxp = float_below(tmax);
            }
            // rare: exact BVH2 traversal, inline — rays with possible NaN slabs, and in the tight
            // kernel rays outside the lean test's bounds (tmin < 0, |o| > 2^60, |d| < 2^-64)
            if (WIDE && (TIGHT ? !lean : !fast_box_ok(o, invd, tmin, tmax))) {
                if (COUNT) c_rays++;
                need_exact = true;
                fresh = false;
            }
        }
        if (need_exact) {
            if constexpr (MODE != TRACE_PILOT)  // the pilot only ranks such a ray costliest
                trace_exact_lane<MODE, TIGHT>(a, idx, o, d, invd, tmin, tmax, s_stack, stack_ovf, tid, gtid);
            if (STEPS && a.ray_steps) a.ray_steps[idx] = 0xFFFFFFFFu;  // traced outside the wide loop
            need_exact = false;
        }
        if (fresh) {
            best = kInf;
            bu = bv = 0.0f;
            bgid = kNoHit;
            occluded = false;
            sp = 0;
            leaf = AKR_CHILD_EMPTY;
            if (COUNT) { c_rays++; c_box++; deep = false; }
            if (STEPS) steps = 0;
            const float tr = box_test<TIGHT, WIDE>(r0.x, r0.y, r0.z, r0.w, r2.x, r2.y, o, invd, tmin, tmax);
            cur = (root == AKR_CHILD_EMPTY || tr < 0.0f || tr > (ANY ? tmax : best)) ? AKR_CHILD_EMPTY : root;
            busy = true;
        }
    }
    if (COUNT) {
        c_rays = wave_sum(c_rays);
        c_box = wave_sum(c_box);
        c_tri = wave_sum(c_tri);
        c_strav = wave_sum(c_strav);
        c_sleaf = wave_sum(c_sleaf);
        c_stri = wave_sum(c_stri);
        c_visit = wave_sum(c_visit);
        c_deep = wave_sum(c_deep);
        c_leaf = wave_sum(c_leaf);
        if (__lane_id() == 0) {
            atomicAdd(&a.counters[MODE].rays, c_rays);
            atomicAdd(&a.counters[MODE].box, c_box);
            atomicAdd(&a.counters[MODE].tri, c_tri);
            atomicAdd(&a.counters[MODE].slots_trav, c_strav);
            atomicAdd(&a.counters[MODE].slots_leaf, c_sleaf);
            atomicAdd(&a.counters[MODE].slots_tri, c_stri);
            atomicAdd(&a.counters[MODE].visits, c_visit);
            atomicAdd(&a.counters[MODE].deep, c_deep);
            atomicAdd(&a.counters[MODE].leaves, c_leaf);
        }
    }
}

// ------------------------------------------------------------------------------------ raygen
__device__ __forceinline__ void apply_rows(const float *m, float x, float y, float z, float w, float *r, int rows) {
    for (int i = 0; i < rows; i++) {
        float s = m[4 * i + 0] * x;
        s += m[4 * i + 1] * y;
        s += m[4 * i + 2] * z;
        s += m[4 * i + 3] * w;
        r[i] = s;
    }
}

// camera_ray: generate_ray(next2d() /*lens*/, next2d() /*film*/, p) — pathtracer.h:61-64
__device__ __forceinline__ void camera_ray(const CameraDev &cam, int x, int y, uint32_t &seed, float4 &r0, float4 &r1) {
    lcg_next2(seed);
    const V2 u2 = lcg_next2(seed);
    const float pfx = (float)x + u2.x, pfy = (float)y + u2.y;
    float r[4];
    apply_rows(cam.r2c, pfx, pfy, 0.0f, 1.0f, r, 4);  // Transform::apply_point, math.h:243-251
    float px_ = r[0], py_ = r[1];
    if (r[3] != 1.0f) {
        px_ = px_ / r[3];
        py_ = py_ / r[3];
    }
    V3 d = normalize(v3(px_ - 0.0f, py_ - 0.0f, 0.0f - 1.0f));
    float ro[4];
    apply_rows(cam.c2w, 0.0f, 0.0f, 0.0f, 1.0f, ro, 4);
    V3 o = v3(ro[0], ro[1], ro[2]);
    if (ro[3] != 1.0f) o = divs(o, ro[3]);
    float rd[3];
    for (int k = 0; k < 3; k++) {  // apply_vector: m3 * v, math.h:253
        float s = cam.c2w[4 * k + 0] * d.x;
        s += cam.c2w[4 * k + 1] * d.y;
        s += cam.c2w[4 * k + 2] * d.z;
        rd[k] = s;
    }
    r0 = make_float4(o.x, o.y, o.z, kEps);
    r1 = make_float4(rd[0], rd[1], rd[2], kInf);
}

__global__ __launch_bounds__(kBlock) void k_raygen(RaygenArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    // queue entry i holds slot sl: with the cost order the costliest camera rays are fetched first
    // in each XCD shard of the closest-hit launch (the order's shards are the launch's shards)
    const uint32_t sl = a.order ? a.order[i] : a.slot_base + i;
    const uint32_t px = a.pixel[sl];
    const int x = (int)(px & 0xFFFFu), y = (int)(px >> 16);
    uint32_t seed = a.first_pass ? (uint32_t)(x + y * a.cam.width) : a.seed[sl];
    float4 r0, r1;
    camera_ray(a.cam, x, y, seed, r0, r1);
    a.L[sl] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    a.ray_out[2 * (size_t)i] = r0;
    a.ray_out[2 * (size_t)i + 1] = r1;
    a.state_out[i] = make_float4(1.0f, 1.0f, 1.0f, bitsf(seed));
    a.slot_out[i] = sl;
    if (a.probe) a.probe[sl].y += 1u;  // the camera ray (always traced)
    if (i == 0) *a.count_out = a.n;
}

// LCG state after n draws: the affine step s -> A s + C raised to the n-th power by squaring
__device__ __forceinline__ uint32_t lcg_advance(uint32_t s, uint32_t n) {
    uint32_t A = 1103515245u, C = 12345u, ra = 1u, rc = 0u;
    while (n) {
        if (n & 1u) {
            ra = A * ra;
            rc = A * rc + C;
        }
        C = A * C + C;
        A = A * A;
        n >>= 1;
    }
    return ra * s + rc;
}

// ------------------------------------------------------------------------------------- shade
// Texture::evaluate (texture.h:30-66; image lookup core/image.hpp:83-99)
__device__ __forceinline__ V3 tex_eval(const SceneDev &s, int32_t ti, V2 tc) {
    const TexDev t = s.texs[ti];
    if (t.type == AKR_TEX_CONSTANT) return v3(t.value[0], t.value[1], t.value[2]);
    float x = fmodf(tc.x, 1.0f);
    float y = 1.0f - fmodf(tc.y, 1.0f);
    const int w = t.w, h = t.h;
    int ix = (int)(x * (float)w), iy = (int)(y * (float)h);
    ix = ix < 0 ? 0 : (ix > w - 1 ? w - 1 : ix);
    iy = iy < 0 ? 0 : (iy > h - 1 ? h - 1 : iy);
    const AKR_GLOBAL float *p = s.images + t.off + 4 * ((int64_t)ix + (int64_t)iy * w);
    return v3(p[0], p[1], p[2]);
}

template <class P>  // a float pointer in any address space (global scene arrays, LDS tables)
__device__ __forceinline__ V3 ld3(P p) { return v3(p[0], p[1], p[2]); }

// One bounce of GenericPathTracer::run_megakernel at a closest hit (pathtracer.h:137-162):
// on_surface_scatter (:96-132) then compute_direct_lighting(select_light) (:65-91).  Shared by the
// wavefront shade kernel and the persistent path kernel, so both run the same arithmetic.
struct Bounce {
    bool emit;        // L += e (depth 0, front-facing or double-sided emitter)
    V3 e;
    bool ext;         // next ray (e0 = p | tmin, e1 = wi | tmax) with throughput nb
    float4 e0, e1;
    V3 nb;
    bool sh;          // shadow ray (s0 = light point | tmin, s1 = direction | tmax), contribution col
    float4 s0, s1;
    V3 col;
};

// Material channel: the resolved constant, or the image texture's texel
template <class C>  // float[3] in any address space
__device__ __forceinline__ V3 mat_rgb(const SceneDev &s, const C &c, int32_t img, V2 tc) {
    return img < 0 ? v3(c[0], c[1], c[2]) : tex_eval(s, img, tc);
}
__device__ __forceinline__ float mat_x(const SceneDev &s, float c, int32_t img, V2 tc) {
    return img < 0 ? c : tex_eval(s, img, tc).x;
}

// The shading's small per-scene tables (materials, lights, light CDF) behind one accessor: read
// from HBM (GlobalTab), or from an LDS copy that the persistent path kernels make at launch when the
// tables fit kTabBytes (LdsTab).  A processing phase's material -> CDF -> light chain of dependent
// loads then waits on LDS instead of L2/HBM.  Same values, same arithmetic.
#define AKR_LDS __attribute__((address_space(3)))
constexpr uint32_t kTabBytes = 1024;
struct GlobalTab {
    const AKR_GLOBAL MatDev *mats;
    const AKR_GLOBAL LightDev *lights;
    const AKR_GLOBAL float *cdf;
    __device__ const AKR_GLOBAL MatDev *mat(int i) const { return mats + i; }
    __device__ const AKR_GLOBAL LightDev *light(int i) const { return lights + i; }
    __device__ float cdf_at(int i) const { return cdf[i]; }
};
struct LdsTab {
    const AKR_LDS MatDev *mats;
    const AKR_LDS LightDev *lights;
    const AKR_LDS float *cdf;
    __device__ const AKR_LDS MatDev *mat(int i) const { return mats + i; }
    __device__ const AKR_LDS LightDev *light(int i) const { return lights + i; }
    __device__ float cdf_at(int i) const { return cdf[i]; }
};
__host__ __device__ constexpr uint32_t tab_bytes(uint32_t n_mats, uint32_t n_lights) {
    return n_lights * (uint32_t)sizeof(LightDev) + n_mats * (uint32_t)sizeof(MatDev) + (n_lights + 1) * 4u;
}
static_assert(sizeof(LightDev) % 16 == 0 && sizeof(MatDev) % 16 == 0, "LDS table records stay 16-B aligned");
bool path_tab_fits(int32_t n_mats, int32_t n_lights) {
    return n_mats >= 0 && n_lights >= 0 && n_mats <= 64 && n_lights <= 64 &&
           tab_bytes((uint32_t)n_mats, (uint32_t)n_lights) <= kTabBytes;
}
__device__ __forceinline__ GlobalTab global_tab(const SceneDev &s) { return GlobalTab{s.mats, s.lights, s.light_cdf}; }

// TAB: the workgroup copies the tables into `buf` (lights, materials, CDF; one barrier at launch)
template <bool TAB> struct PathTab;
template <> struct PathTab<false> {
    static __device__ __forceinline__ GlobalTab make(const SceneDev &s, uint4 *) { return global_tab(s); }
};
template <> struct PathTab<true> {
    static __device__ __forceinline__ LdsTab make(const SceneDev &s, uint4 *buf) {
        AKR_LDS uint32_t *d = (AKR_LDS uint32_t *)buf;
        const uint32_t wl = (uint32_t)s.n_lights * (uint32_t)(sizeof(LightDev) / 4);
        const uint32_t wm = (uint32_t)s.n_mats * (uint32_t)(sizeof(MatDev) / 4);
        const uint32_t wc = s.n_lights > 0 ? (uint32_t)s.n_lights + 1 : 0u;
        const AKR_GLOBAL uint32_t *gl = (const AKR_GLOBAL uint32_t *)s.lights;
        const AKR_GLOBAL uint32_t *gm = (const AKR_GLOBAL uint32_t *)s.mats;
        const AKR_GLOBAL uint32_t *gc = (const AKR_GLOBAL uint32_t *)s.light_cdf;
        for (uint32_t i = threadIdx.x; i < wl; i += blockDim.x) d[i] = gl[i];
        for (uint32_t i = threadIdx.x; i < wm; i += blockDim.x) d[wl + i] = gm[i];
        for (uint32_t i = threadIdx.x; i < wc; i += blockDim.x) d[wl + wm + i] = gc[i];
        __syncthreads();
        return LdsTab{(const AKR_LDS MatDev *)(d + wl), (const AKR_LDS LightDev *)d, (const AKR_LDS float *)(d + wl + wm)};
    }
};

// Scene::select_light's index: upper_bound over the light CDF (distribution.h:32-44), clamped
template <class Tab>
__device__ __forceinline__ int select_light_index(const SceneDev &s, const Tab &tab, float x) {
    int lo = 0, hi = s.n_lights + 1;
    while (lo < hi) {
        const int m = (lo + hi) / 2;
        if (tab.cdf_at(m) <= x) lo = m + 1; else hi = m;
    }
    const int li = hi - 1;
    return li < 0 ? 0 : (li > s.n_lights - 1 ? s.n_lights - 1 : li);
}

template <class Tab>
__device__ __forceinline__ void shade_hit_tab(const SceneDev &s, const Tab &tab, uint32_t gid, float u, float v, V3 wo,
                                              V3 beta, uint32_t &seed, int depth, int max_depth, bool last, Bounce &o,
                                              unsigned long long *t_load = nullptr) {
    o.emit = o.ext = o.sh = false;
    unsigned long long t0 = 0;  // counting builds (t_load): ticks until the shading record is in
    if (t_load) t0 = wall_clock64();
    const ShadeTri tr = s.tri[gid];
    // the whole record in one round trip: without this the compiler loads the material id alone, tests
    // it, then loads the rest (two dependent trips; whole frame -0.6 %, profiles/r21_shade_trip_ab.log)
    asm volatile("" ::"v"(tr.a.x), "v"(tr.a.y), "v"(tr.a.z), "v"(tr.a.w), "v"(tr.b.x), "v"(tr.b.y), "v"(tr.b.z),
                 "v"(tr.b.w), "v"(tr.c.x), "v"(tr.c.y), "v"(tr.c.z), "v"(tr.c.w), "v"(tr.d.x), "v"(tr.d.y), "v"(tr.d.z),
                 "v"(tr.d.w), "v"(tr.e.x), "v"(tr.e.y), "v"(tr.e.z));
    if (t_load) *t_load += wall_clock64() - t0;
    const int32_t mid = (int32_t)fbits(tr.a.w);
    if (mid < 0) return;  // a null material ends the path (undefined in the reference)
    const V3 v0{tr.a.x, tr.a.y, tr.a.z}, v1{tr.b.x, tr.b.y, tr.b.z}, v2{tr.c.x, tr.c.y, tr.c.z};
    // SurfaceInteraction(uv, triangle) (interaction.h:40-41, shape.h:31-40)
    const V3 p = lerp3(v0, v1, v2, u, v);
    const V3 ng = normalize(cross(sub(v1, v0), sub(v2, v0)));
    const V3 ns = lerp3(v3(tr.b.w, tr.c.w, tr.d.x), v3(tr.d.y, tr.d.z, tr.d.w), v3(tr.e.x, tr.e.y, tr.e.z), u, v);
    V2 tc{0.0f, 0.0f};  // only image textures read it
    if (s.has_image_tex) {
        const AKR_GLOBAL float *tt = s.texcoords + 6 * (size_t)gid;
        tc = lerp3(V2{tt[0], tt[1]}, V2{tt[2], tt[3]}, V2{tt[4], tt[5]}, u, v);
    }
    auto mat = tab.mat(mid);
    if (mat->type == AKR_MAT_EMISSIVE) {
        if (depth == 0) {
            const bool face_front = dot(neg(wo), ng) < 0.0f;
            if (mat->double_sided || face_front) {
                o.emit = true;
                o.e = mul(beta, mat_rgb(s, mat->color, mat->color_img, tc));
            }
        }
        return;
    }
    if (depth >= max_depth) return;
    // MaterialEvalContext holds a COPY of the sampler: u1.x is the next draw
    uint32_t copy = seed;
    float sel_u = lcg_next(copy);
    float choice_pdf = 1.0f;
    while (mat->type == AKR_MAT_MIX) {  // Material::select_material, material.h:251-268
        const float frac = mat_x(s, mat->frac, mat->frac_img, tc);
        if (sel_u < frac) {
            sel_u = sel_u / frac;
            mat = tab.mat(mat->second);
            choice_pdf *= 1.0f / frac;
        } else {
            sel_u = (sel_u - frac) / (1.0f - frac);
            mat = tab.mat(mat->first);
            choice_pdf *= 1.0f / (1.0f - frac);
        }
    }
    Closure cl{CL_NONE, v3(0, 0, 0), 0.0f};
    if (mat->type == AKR_MAT_DIFFUSE) {
        cl.kind = CL_DIFFUSE;
        cl.R = mat_rgb(s, mat->color, mat->color_img, tc);
    } else if (mat->type == AKR_MAT_GLOSSY) {
        cl.kind = CL_GLOSSY;
        cl.R = mat_rgb(s, mat->color, mat->color_img, tc);
        float r = mat_x(s, mat->rough, mat->rough_img, tc);
        r *= r;
        cl.alpha = r;
    }
    const Frame frame = make_frame(ns);
    const V2 bu = lcg_next2(seed);  // BSDFSampleContext(sampler.next2d(), wo)
    if (cl.kind == CL_NONE) return;
    V3 wi_l;
    float pdf = 0.0f;
    const V3 f = closure_sample(cl, bu, to_local(frame, wo), wi_l, pdf);
    const V3 wi = to_world(frame, wi_l);
    pdf *= choice_pdf;
    if (pdf == 0.0f) return;
    const float cng = fabsf(dot(ng, wi));
    const V3 ev_beta = divs(muls(f, cng), pdf);
    // select_light(sampler.next2d()) — scene.h:79-90
    const V2 su = lcg_next2(seed);
    if (s.n_lights > 0) {
        const auto &lt = *tab.light(select_light_index(s, tab, su.x));
        const V2 lu = lcg_next2(seed);
        // AreaLight::sample (light.h:58-71); lng, the area and the selection pdf are precomputed
        const float su0 = sqrtf(lu.x);
        const float b0 = 1 - su0, b1 = lu.y * su0;
        const V3 lp = lerp3(ld3(lt.v), ld3(lt.v + 3), ld3(lt.v + 6), b0, b1);
        const V3 lng = ld3(lt.lng);
        V3 lwi = sub(lp, p);
        const float dist_sqr = dot(lwi, lwi);
        lwi = divs(lwi, sqrtf(dist_sqr));
        V3 Le;
        if (lt.color_img < 0) {
            Le = ld3(lt.Le);
        } else {
            const V2 ltc = lerp3(V2{lt.tc[0], lt.tc[1]}, V2{lt.tc[2], lt.tc[3]}, V2{lt.tc[4], lt.tc[5]}, b0, b1);
            Le = tex_eval(s, lt.color_img, ltc);
        }
        const float lpdf = dist_sqr / rmax(0.0f, -dot(lwi, lng)) / lt.area_half;
        if (!(lpdf <= 0.0f)) {
            const float light_pdf = lt.sel_pdf * lpdf;
            const V3 fe = closure_eval(cl, to_local(frame, wo), to_local(frame, lwi));
            const V3 fl = muls(mul(Le, fe), fabsf(dot(ns, lwi)));
            const V3 col = divs(mul(beta, fl), light_pdf);
            if (!is_black(col)) {
                o.sh = true;
                const V3 sdir = neg(lwi);
                o.s0 = make_float4(lp.x, lp.y, lp.z, kEps / fabsf(dot(lwi, lng)));
                o.s1 = make_float4(sdir.x, sdir.y, sdir.z, sqrtf(dist_sqr) * (1.0f - kShadowEps));
                o.col = col;
            }
        }
    }
    if (!last) {
        o.ext = true;
        o.nb = mul(beta, ev_beta);
        o.e0 = make_float4(p.x, p.y, p.z, kEps / cng);
        o.e1 = make_float4(wi.x, wi.y, wi.z, kInf);
    }
}

__device__ __forceinline__ void shade_hit(const SceneDev &s, uint32_t gid, float u, float v, V3 wo, V3 beta,
                                          uint32_t &seed, int depth, int max_depth, bool last, Bounce &o) {
    shade_hit_tab(s, global_tab(s), gid, u, v, wo, beta, seed, depth, max_depth, last, o);
}

// One bounce for every queued hit (wavefront form)
#ifndef AKR_SHADE_BLOCK
#define AKR_SHADE_BLOCK 256
#endif
constexpr int kShadeBlock = AKR_SHADE_BLOCK;  // threads per shade workgroup (one queue atomic each)
__global__ __launch_bounds__(kShadeBlock) void k_shade(ShadeArgs a) {
    const uint32_t i = blockIdx.x * kShadeBlock + threadIdx.x;
    const uint32_t n = *a.count_in;
    if (blockIdx.x * kShadeBlock >= n) return;  // whole workgroup past the queue (uniform: before any barrier)
    Bounce bo;
    bo.ext = bo.sh = false;
    uint32_t slot = 0, seed = 0;
    if (i < n) {
        slot = a.slot_in[i];
        const float4 stv = a.state_in[i];
        seed = fbits(stv.w);
        const float4 hv = a.hit_in[i];
        const uint32_t gid = fbits(hv.w);
        if (gid != kNoHit) {  // miss -> on_miss (no-op), the path ends
            const float4 rdv = a.ray_in[2 * (size_t)i + 1];
            shade_hit(a.sc, gid, hv.y, hv.z, neg(v3(rdv.x, rdv.y, rdv.z)), V3{stv.x, stv.y, stv.z}, seed, a.depth,
                      a.max_depth, a.last != 0, bo);
            if (bo.emit) {
                float4 l = a.L[slot];
                l.x += bo.e.x;
                l.y += bo.e.y;
                l.z += bo.e.z;
                a.L[slot] = l;
            }
        }
        // the path does not reach another traced bounce: persist its sampler stream for the next
        // sample (the stream continues across spp, cpu/integrator.cpp:124-134)
        if (!bo.ext) a.seed[slot] = seed;
        if (a.probe && (bo.ext || bo.sh)) {  // one queue entry per slot per launch: no race
            uint4 q = a.probe[slot];
            q.y += bo.ext ? 1u : 0u;
            q.z += bo.sh ? 1u : 0u;
            a.probe[slot] = q;
        }
    }
    uint32_t pos, spos;
    block_append2<kShadeBlock>(bo.ext, a.count_out, pos, bo.sh, a.shadow_count, spos);
    if (bo.ext) {  // the seed travels with the path state
        a.ray_out[2 * (size_t)pos] = bo.e0;
        a.ray_out[2 * (size_t)pos + 1] = bo.e1;
        a.state_out[pos] = make_float4(bo.nb.x, bo.nb.y, bo.nb.z, bitsf(seed));
        a.slot_out[pos] = slot;
    }
    if (bo.sh) {  // the shadow trace adds the colour to L[colour.w] when unoccluded
        a.shadow_ray[2 * (size_t)spos] = bo.s0;
        a.shadow_ray[2 * (size_t)spos + 1] = bo.s1;
        a.shadow_color[spos] = make_float4(bo.col.x, bo.col.y, bo.col.z, bitsf(slot));
    }
}

// --------------------------------------------------------------------------- ambient occlusion
// cpu::AmbientOcclusion's Li after the camera ray (kernel/integrators/cpu/integrator.cpp:46-56):
// on a hit, one cosine-hemisphere direction in the frame of the geometric normal, from trig.p(uv)
// with the default tmin Eps; the sampler state is persisted for the next sample pass either way.
__global__ __launch_bounds__(kBlock) void k_ao_shade(AoShadeArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t n = *a.count_in;
    if (blockIdx.x * kBlock >= n) return;  // uniform per workgroup: before the barrier
    bool want = false;
    float4 r0 = {}, r1 = {};
    uint32_t slot = 0;
    if (i < n) {
        slot = a.slot_in[i];
        uint32_t seed = fbits(a.state_in[i].w);
        const float4 hv = a.hit_in[i];
        const uint32_t gid = fbits(hv.w);
        if (gid != kNoHit) {
            const ShadeTri tr = a.tri[gid];
            const V3 v0{tr.a.x, tr.a.y, tr.a.z}, v1{tr.b.x, tr.b.y, tr.b.z}, v2{tr.c.x, tr.c.y, tr.c.z};
            const Frame frame = make_frame(normalize(cross(sub(v1, v0), sub(v2, v0))));
            const V3 w = to_world(frame, cosine_hemisphere(lcg_next2(seed)));
            const V3 p = lerp3(v0, v1, v2, hv.y, hv.z);
            want = true;
            r0 = make_float4(p.x, p.y, p.z, kEps);
            r1 = make_float4(w.x, w.y, w.z, kInf);
        }
        a.seed[slot] = seed;
    }
    uint32_t pos, unused;
    block_append2(want, a.count_out, pos, false, a.count_out, unused);
    if (want) {
        a.ray_out[2 * (size_t)pos] = r0;
        a.ray_out[2 * (size_t)pos + 1] = r1;
        if (a.color_out) a.color_out[pos] = make_float4(1.0f, 1.0f, 1.0f, bitsf(slot));
        if (a.slot_out) a.slot_out[pos] = slot;
    }
}

// `scene.intersect(ray, &its) && its.t < occlude` -> 0, else 1 (integrator.cpp:53-55)
__global__ __launch_bounds__(kBlock) void k_ao_resolve(AoResolveArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= *a.count) return;
    const float4 h = a.hits[i];
    if (fbits(h.w) != kNoHit && h.x < a.occlude) return;
    const uint32_t slot = a.slot[i];
    float4 l = a.L[slot];
    l.x += 1.0f;
    l.y += 1.0f;
    l.z += 1.0f;
    a.L[slot] = l;
}

// ------------------------------------------------------------------------------------- splat
__device__ __forceinline__ void splat_one(float4 &f, float4 l, float ray_clamp) {
    float r = l.x, g = l.y, b = l.z;
    if (ray_clamp > 0.0f) {  // clamp_zero + min (gpu/cuda/integrator.cpp:397-398)
        r = isnan(r) ? 0.0f : rmax(0.0f, r);
        g = isnan(g) ? 0.0f : rmax(0.0f, g);
        b = isnan(b) ? 0.0f : rmax(0.0f, b);
        r = rmin(r, ray_clamp);
        g = rmin(g, ray_clamp);
        b = rmin(b, ray_clamp);
    }
    f.x += r;
    f.y += g;
    f.z += b;
    f.w += 1.0f;
}

// Tile::add_sample per pixel, in sample order
__global__ __launch_bounds__(kBlock) void k_splat(SplatArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t sl = a.order ? a.order[i] : a.slot_base + i;
    float4 f = a.film[sl];
    splat_one(f, a.L[sl], a.ray_clamp);
    a.film[sl] = f;
}

// ------------------------------------------------------------------------------ persistent path
// k_path: the whole per-pixel sample loop of cpu::PathTracer::render (cpu/integrator.cpp:89-142,
// run_megakernel pathtracer.h:133-164) in one persistent launch.  A lane owns one pixel at a time
// and runs its spp samples in order, so the sampler stream, the order of the L additions and the
// film sums are exactly the sequential loop's; it takes the next pixel from the XCD-sharded pixel
// counters when it finishes one.  Per outer iteration a wave
//   A. processes the lanes whose ray has finished, once enough of them wait: a shadow ray adds its
//      contribution and hands over to the pending extension ray; a closest hit is shaded inline
//      (shade_hit), which yields a shadow ray (traced first) and/or the next extension ray; a
//      finished sample is splatted into the pixel's film sums and the next camera ray is made;
//   B. runs the traversal phase of k_trace's while-while loop (lean wide slot tests, speculative
//      leaves, early exit) over every lane's current ray, closest-hit or shadow alike;
//   C. runs the leaf phase.
// No launch boundary separates the bounces of a pixel from those of its neighbours, so a slow ray
// delays only its own pixel's chain: the per-bounce tails and gaps of the wavefront form (DESIGN.md
// §7) are gone.  A shadow ray is any-hit with best initialised to tmax, which makes every bound of
// the closest-hit loop the occlusion test's bound.
#ifndef AKR_PATH_WAVES
#define AKR_PATH_WAVES 4
#endif

// One lane's ray in the persistent path kernels' traversal loop (k_trace's registers) and the
// counting build's tallies ([0] closest-hit rays, [1] shadow rays).
struct PathRay {
    V3 o, d, invd;
    float tmin, tmax, tmaxp, best, bu, bv;
    uint32_t dpos, bgid, cur, leaf;
    int sp;
};
struct PathCount {
    unsigned long long rays[2] = {0, 0}, box[2] = {0, 0}, tri[2] = {0, 0}, visit[2] = {0, 0}, deep[2] = {0, 0},
                       leaf[2] = {0, 0};
    unsigned long long strav = 0, sleaf = 0, stri = 0, iters = 0;
    // time split of the traversal (v) and leaf (l) phases, wave ticks: issuing the node / leaf
    // loads, waiting for them (an explicit vmcnt(0) wait between two clock reads), the dependent
    // work after they return (slot tests, stack, ballots; leaf box and triangle loop)
    unsigned long long tv_issue = 0, tv_wait = 0, tv_comp = 0, tl_issue = 0, tl_wait = 0, tl_comp = 0;
    // leaf phases entered with at least one lane holding a leaf, and those lanes summed
    unsigned long long lphases = 0, lholders = 0;
    bool deep_now = false;
    // option count_lines (k_path): the bitmap of 128-B lines read, wide nodes in bits [0, span[1]), the
    // leaf blob in [span[1], span[2]) (distinct lines per sample pass against the
    // fabric reads)
    uint32_t *lines = nullptr;
    uint32_t span[3] = {0, 0, 0};
    const float4 *leaf_base = nullptr;
};

// Counting build, option count_lines: marks the 128-B lines of [p, p + bytes) (bytes <= 128) in the
// bitmap, line l of the region that starts at `region` as bit lo + l; a bit outside [lo, hi) is never
// written
__device__ __forceinline__ void mark_lines(uint32_t *map, uint32_t lo, uint32_t hi, const void *region, const void *p,
                                           uint32_t bytes) {
    const uint64_t r0 = (uint64_t)region >> 7, a = (uint64_t)p;
    if (a < (uint64_t)region) return;
    for (uint64_t l = (a >> 7) - r0; l <= ((a + bytes - 1) >> 7) - r0; l++) {
        const uint64_t b = lo + l;
        if (b < hi) atomicOr(map + (b >> 5), 1u << (b & 31u));
    }
}

// B. k_trace's traversal phase over every busy lane's ray (all rays here are lean)
template <bool COUNT, int EXIT = kWhileExit>  // EXIT: the phase ends when <= EXIT lanes still search
__device__ __forceinline__ void path_traverse(bool busy, int kind, PathRay &r, const float4 *wn, lds_u64 *s_stack,
                                              glb_u64 *ovf, uint32_t ovf_threads, uint32_t tid, uint32_t gtid,
                                              PathCount &c) {
    while (true) {
        [[maybe_unused]] unsigned long long tc = 0;
        bool need_pop = false;  // the visit entered no slot: pop below
        if constexpr (COUNT) {
            c.strav++;
            c.sleaf += busy ? 1 : 0;
            c.iters++;
            // the counting build splits the iteration's time: issue, wait, work
            const bool vis = busy && is_internal(r.cur);
            const unsigned long long ta = wall_clock64();
            // every lane loads (an idle lane node 0, a cache hit): a load under a branch makes the
            // compiler wait for it inside the branch, before the clock below
            const WideNode nd = wide_load(wn, vis ? r.cur : 0u);
            const unsigned long long tb = wall_clock64();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            tc = wall_clock64();
            c.tv_issue += tb - ta;
            c.tv_wait += tc - tb;
            if (vis) {
                const uint32_t node = r.cur;  // the visit moves r.cur on
                const int nt = visit_wide_lean_node<false, true>(nd, r.cur, r.o, r.dpos, r.invd, r.tmin, r.tmaxp, r.best,
                                                                 s_stack, ovf, ovf_threads, tid, gtid, r.sp, &need_pop);
                c.box[kind] += nt;
                c.visit[kind]++;
                c.deep_now = c.deep_now || r.sp > kStackLds;
                if (c.lines)
                    mark_lines(c.lines, 0u, c.span[1], wn, reinterpret_cast<const char *>(wn) + ((size_t)node << 6), 64u);
            }
        } else if (busy && is_internal(r.cur)) {
            const WideNode nd = wide_load(wn, r.cur);
            visit_wide_lean_node<false, true>(nd, r.cur, r.o, r.dpos, r.invd, r.tmin, r.tmaxp, r.best, s_stack, ovf,
                                              ovf_threads, tid, gtid, r.sp, &need_pop);
        }
        // One pop site per iteration, for a visit that entered no slot and for a leaf to postpone (a
        // popped leaf is postponed in the next iteration: every ray visits the same nodes and leaves
        // in the same order).  Popping at two sites chained two LDS round trips into one iteration
        // whenever the first pop returned a leaf: one site runs the whole frame 4.3 % and the 8-way
        // share 6.5 % faster (profiles/r21_one_pop_ab.log).
        if (busy && !need_pop && r.leaf == AKR_CHILD_EMPTY && is_leaf(r.cur)) {
            r.leaf = r.cur;  // postpone the leaf and keep descending
            need_pop = true;
        }
        if (need_pop) r.cur = stack_pop(s_stack, ovf, ovf_threads, tid, gtid, r.sp, r.best);
        const unsigned long long searching = __ballot(busy && r.leaf == AKR_CHILD_EMPTY && r.cur != AKR_CHILD_EMPTY);
        if constexpr (COUNT) {
            const bool stop = (uint32_t)__popcll(searching) <= (uint32_t)EXIT &&
                              (searching == 0 || __ballot(busy && r.leaf != AKR_CHILD_EMPTY) != 0);
            c.tv_comp += wall_clock64() - tc;
            if (stop) break;
        } else if ((uint32_t)__popcll(searching) <= (uint32_t)EXIT &&
                   (searching == 0 || __ballot(busy && r.leaf != AKR_CHILD_EMPTY) != 0)) {
            break;
        }
    }
}

// The counting build's leaf tests: the leaf's exact box with the current best, then its triangles
// (the header, the first and the second triangle's records already loaded)
template <bool COUNT>
__device__ __forceinline__ bool leaf_tests(int kind, PathRay &r, const float4 *lr, float4 l0, float4 l1, float4 pa0,
                                           float4 pb0, float4 pc0, float4 pa1, float4 pb1, float4 pc1, PathCount &c) {
    bool hit_any = false;
    const float tl = box_test<true, true>(l0.x, l0.w, l0.y, l1.x, l0.z, l1.y, r.o, r.invd, r.tmin, r.tmax);
    const bool in = !(tl < 0.0f || tl > r.best);
    if (COUNT) {
        c.box[kind]++;
        c.leaf[kind]++;
    }
    const uint32_t cnt = in ? fbits(l1.w) : 0u;
    const float4 *tp = lr + 2;
    for (uint32_t k = 0; k < cnt; k++) {
        if (COUNT && lane_prefix(__ballot(1)) == 0) c.stri += 64;
        const float4 ta = k == 0 ? pa0 : (k == 1 ? pa1 : tp[3 * k + 0]);
        const float4 tb = k == 0 ? pb0 : (k == 1 ? pb1 : tp[3 * k + 1]);
        const float4 tc = k == 0 ? pc0 : (k == 1 ? pc1 : tp[3 * k + 2]);
        if (COUNT) {
            c.tri[kind]++;
            if (c.lines && k >= 2) mark_lines(c.lines, c.span[1], c.span[2], c.leaf_base, tp + 3 * k, 48u);
        }
        float t, u, v;
        if (mt(r.o, r.d, r.tmin, r.tmax, ta, tb, tc, r.best, t, u, v)) {
            r.best = t;
            r.bu = u;
            r.bv = v;
            r.bgid = fbits(ta.w);
            if (kind) {
                hit_any = true;
                break;
            }
        }
    }
    r.leaf = AKR_CHILD_EMPTY;
    return hit_any;
}

// C. the leaf phase: the pending leaf's exact box with the current best, then its triangles;
// returns true when an occlusion ray (kind 1) found its first hit.  The leaf's header and its first
// two triangle records are one batch of eight 16-B loads: one dependent round trip less for leaves of
// two or more triangles (whole frame 5.00 -> 4.86 ms per spp, profiles/r18_leaf_pf2_ab.log); the blob
// is padded, so this never reads past its end.
template <bool COUNT>
__device__ __forceinline__ bool path_leaf(bool busy, int kind, PathRay &r, const float4 *wide_leaves, PathCount &c) {
    if constexpr (!COUNT) {  // (the loads and tests written out here: through leaf_tests the compiler
                             // allocates the persistent kernels' registers differently)
        bool hit_any = false;
        if (busy && r.leaf != AKR_CHILD_EMPTY) {
            const float4 *lr = wide_leaves + (r.leaf & 0x7FFFFFFFu);
            const float4 l0 = lr[0], l1 = lr[1];
            const float4 pa0 = lr[2], pb0 = lr[3], pc0 = lr[4];
            const float4 pa1 = lr[5], pb1 = lr[6], pc1 = lr[7];
            issue_together(pa0, pb0, pc0, pa1, pb1, pc1);
            const float tl = box_test<true, true>(l0.x, l0.w, l0.y, l1.x, l0.z, l1.y, r.o, r.invd, r.tmin, r.tmax);
            const bool in = !(tl < 0.0f || tl > r.best);
            const uint32_t cnt = in ? fbits(l1.w) : 0u;
            const float4 *tp = lr + 2;
            for (uint32_t k = 0; k < cnt; k++) {
                const float4 ta = k == 0 ? pa0 : (k == 1 ? pa1 : tp[3 * k + 0]);
                const float4 tb = k == 0 ? pb0 : (k == 1 ? pb1 : tp[3 * k + 1]);
                const float4 tc = k == 0 ? pc0 : (k == 1 ? pc1 : tp[3 * k + 2]);
                float t, u, v;
                if (mt(r.o, r.d, r.tmin, r.tmax, ta, tb, tc, r.best, t, u, v)) {
                    r.best = t;
                    r.bu = u;
                    r.bv = v;
                    r.bgid = fbits(ta.w);
                    if (kind) {
                        hit_any = true;
                        break;
                    }
                }
            }
            r.leaf = AKR_CHILD_EMPTY;
        }
        return hit_any;
    } else {  // the counting build splits the phase's time: issue, wait, tests
        bool hit_any = false;
        const unsigned long long ta = wall_clock64();
        const bool in_leaf = busy && r.leaf != AKR_CHILD_EMPTY;
        const uint32_t holders = (uint32_t)__popcll(__ballot(in_leaf));
        c.lphases += holders ? 1u : 0u;
        c.lholders += holders;
        // every lane loads (a lane without a leaf the blob's first record: see path_traverse)
        const float4 *lr = wide_leaves + (in_leaf ? (r.leaf & 0x7FFFFFFFu) : 0u);
        const float4 l0 = lr[0], l1 = lr[1], pa0 = lr[2], pb0 = lr[3], pc0 = lr[4], pa1 = lr[5], pb1 = lr[6],
                     pc1 = lr[7];
        const unsigned long long tb = wall_clock64();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long tc = wall_clock64();
        if (in_leaf && c.lines) mark_lines(c.lines, c.span[1], c.span[2], wide_leaves, lr, 128u);
        if (in_leaf) hit_any = leaf_tests<true>(kind, r, lr, l0, l1, pa0, pb0, pc0, pa1, pb1, pc1, c);
        c.tl_issue += tb - ta;
        c.tl_wait += tc - tb;
        c.tl_comp += wall_clock64() - tc;
        return hit_any;
    }
}

// A fresh ray into the traversal state: lean rays enter the loop (returns true: the lane is busy),
// others are traced inline with the exact BVH2 walk and come back finished (false).  An occlusion
// ray's best starts at tmax (§3.8).  A return value, not bool references: a reference to one of two
// flags picked per lane puts both in scratch.
template <bool COUNT>
__device__ __forceinline__ bool path_begin(const TraceArgs &a, bool occl, float4 ra, float4 rb, PathRay &r,
                                           lds_u64 *s_stack, glb_u64 *ovf, uint32_t tid, uint32_t gtid, PathCount &c) {
    r.o = V3{ra.x, ra.y, ra.z};
    r.d = V3{rb.x, rb.y, rb.z};
    r.tmin = ra.w;
    r.tmax = rb.w;
    r.invd = V3{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
    r.dpos = (r.d.x > 0.0f ? 1u : 0u) | (r.d.y > 0.0f ? 2u : 0u) | (r.d.z > 0.0f ? 4u : 0u);
    if (occl && a.any_far_first) r.dpos ^= 7u;
    r.tmaxp = float_below(r.tmax);
    if (COUNT) c.rays[occl]++;
    if (!lean_ok(r.o, r.invd, r.tmin, r.tmax)) {  // rare: exact BVH2 walk inline (k_trace's exact lane)
        bool hit;
        if (occl)
            trace_exact_core<true, true>(a, r.o, r.d, r.invd, r.tmin, r.tmax, s_stack, ovf, tid, gtid, r.best, r.bu,
                                         r.bv, r.bgid, hit);
        else
            trace_exact_core<false, true>(a, r.o, r.d, r.invd, r.tmin, r.tmax, s_stack, ovf, tid, gtid, r.best, r.bu,
                                          r.bv, r.bgid, hit);
        return false;
    }
    r.best = occl ? r.tmax : kInf;
    r.bu = r.bv = 0.0f;
    r.bgid = kNoHit;
    r.sp = 0;
    r.leaf = AKR_CHILD_EMPTY;
    if (COUNT) {
        c.box[occl]++;
        c.deep_now = false;
    }
    const float4 *nodesf = reinterpret_cast<const float4 *>(a.nodes);
    const float4 r0 = nodesf[0], r2 = nodesf[2];
    const float tr = box_test<true, true>(r0.x, r0.y, r0.z, r0.w, r2.x, r2.y, r.o, r.invd, r.tmin, r.tmax);
    r.cur = (a.wide_root == AKR_CHILD_EMPTY || tr < 0.0f || tr > r.best) ? AKR_CHILD_EMPTY : a.wide_root;
    return true;
}

__device__ __forceinline__ void path_park(uint32_t (*s_park)[kTraceBlock], uint32_t tid, const PathRay &r);
__device__ __forceinline__ void path_unpark(uint32_t (*s_park)[kTraceBlock], uint32_t tid, PathRay &r, bool far_first,
                                            bool occl);

// Wave-level pixel fetch from the XCD shards (k_trace's refill): every lane with `need` set gets
// the next pixel of its wave's shard, or `done` once every shard is exhausted.  Fetch index i of a
// shard maps to its slot by `mode`: FETCH_LINEAR (i), FETCH_SCRAMBLE ((i * (2^31 - 1)) mod len, a
// bijection: the lanes of a wave hold pixels from all over their shard instead of one tile's rows),
// or FETCH_PAIR (i/2 from the front for even i, from the back for odd i: over a cost-ordered shard
// each wave holds the costliest and the cheapest pixels left, so lanes whose pixel ends early can
// take the long pixels' shadow rays).  `order` (optional) maps the position to the
// slot.  With `prio`, a wave whose fetch lies in the first `prio` / 256 of its shard (the costliest
// pixels of a cost order) raises its issue priority, else lowers it.
enum : uint32_t { FETCH_LINEAR = 0, FETCH_SCRAMBLE = 1, FETCH_PAIR = 2, FETCH_STRIDE = 3 };
struct PixelFetch {
    uint32_t shard, s_lo, s_hi;
    int shards_left;
    bool drained;
    uint32_t stride = 0;  // FETCH_STRIDE: the shard's step (coprime with its length), 0 = not computed
};
__device__ __forceinline__ uint32_t gcd_u32(uint32_t x, uint32_t y) {
    while (y) {
        const uint32_t t = x % y;
        x = y;
        y = t;
    }
    return x;
}
__device__ __forceinline__ void fetch_pixels(PixelFetch &f, uint32_t n, uint32_t *work, uint32_t mode,
                                             const uint32_t *order, uint32_t prio, bool &need, bool &done,
                                             uint32_t &pix) {
    while (true) {
        const unsigned long long want = __ballot(need && !done);
        if (want == 0) break;
        if (f.drained) {
            if (need) done = true;
            break;
        }
        const uint32_t nw = (uint32_t)__popcll(want);
        const int leader = __ffsll((long long)want) - 1;
        uint32_t base = 0;
        if ((int)__lane_id() == leader) base = atomicAdd(work + f.shard * kWorkStride, nw);
        base = __builtin_amdgcn_readfirstlane(__shfl(base, leader));
        const uint32_t len = f.s_hi - f.s_lo;
        if (prio && base < len) {  // wave-uniform
            if ((uint64_t)base * 256u < (uint64_t)len * prio) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(0);
        }
        if (need && !done) {
            const uint32_t my = base + lane_prefix(want);
            if (base < len && my < len) {
                uint32_t pos = my;
                if (mode == FETCH_SCRAMBLE) pos = (uint32_t)(((uint64_t)my * 2147483647ull) % len);
                else if (mode == FETCH_PAIR) pos = (my & 1u) ? len - 1u - (my >> 1) : (my >> 1);
                else if (mode == FETCH_STRIDE) {  // consecutive fetches len/64 apart: every wave spans the cost order
                    if (f.stride == 0) {
                        uint32_t st = max(1u, len / 64u) | 1u;
                        while (gcd_u32(st, len) != 1u) st += 2u;
                        f.stride = st;
                    }
                    pos = (uint32_t)(((uint64_t)my * f.stride) % len);
                }
                const uint32_t at = f.s_lo + pos;
                pix = order ? order[at] : at;
                need = false;
            }
        }
        if (base + nw >= len) {  // this shard is exhausted: move to the next open one
            while (true) {
                if (--f.shards_left == 0) {
                    f.drained = true;
                    break;
                }
                f.shard = (f.shard + 1) % kWorkShards;
                f.s_lo = shard_begin(n, f.shard);
                f.s_hi = shard_begin(n, f.shard + 1);
                f.stride = 0;
                const uint32_t taken = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(work + f.shard * kWorkStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (taken < f.s_hi - f.s_lo) break;
            }
        }
    }
}

// Counting build: a wave's phase profile and ray tallies into PathProfile / TraceCounters
__device__ __forceinline__ void path_count_flush(const PathArgs &pa, PathCount &c, unsigned long long p_outer,
                                                 unsigned long long p_procs, unsigned long long p_tp,
                                                 unsigned long long p_tt, unsigned long long p_tl, unsigned long long p_t0,
                                                 unsigned long long p_lanes, unsigned long long p_tsh) {
    const TraceArgs &a = pa.t;
    if (__lane_id() == 0 && pa.prof) {
        const unsigned long long tot = wall_clock64() - p_t0;
        PathProfile &q = *pa.prof;
        atomicAdd(&q.waves, 1ull);
        atomicAdd(&q.outer, p_outer);
        atomicAdd(&q.procs, p_procs);
        atomicAdd(&q.trav_iters, c.iters);
        atomicAdd(&q.t_proc, p_tp);
        atomicAdd(&q.t_trav, p_tt);
        atomicAdd(&q.t_leaf, p_tl);
        atomicAdd(&q.t_total, tot);
        atomicMax(&q.t_max, tot);
        atomicAdd(&q.lanes_proc, p_lanes);
        atomicAdd(&q.t_shade, p_tsh);
        atomicAdd(&q.tv_issue, c.tv_issue);
        atomicAdd(&q.tv_wait, c.tv_wait);
        atomicAdd(&q.tv_comp, c.tv_comp);
        atomicAdd(&q.tl_issue, c.tl_issue);
        atomicAdd(&q.tl_wait, c.tl_wait);
        atomicAdd(&q.tl_comp, c.tl_comp);
        atomicAdd(&q.leaf_phases, c.lphases);
        atomicAdd(&q.leaf_holders, c.lholders);
    }
    const int slot_of[2] = {TRACE_CLOSEST, TRACE_SHADOW};
    for (int m = 0; m < 2; m++) {
        const unsigned long long rr = wave_sum(c.rays[m]), b = wave_sum(c.box[m]), t = wave_sum(c.tri[m]),
                                 v = wave_sum(c.visit[m]), dp = wave_sum(c.deep[m]), lf = wave_sum(c.leaf[m]);
        if (__lane_id() == 0) {
            TraceCounters &tc = a.counters[slot_of[m]];
            atomicAdd(&tc.rays, rr);
            atomicAdd(&tc.box, b);
            atomicAdd(&tc.tri, t);
            atomicAdd(&tc.visits, v);
            atomicAdd(&tc.deep, dp);
            atomicAdd(&tc.leaves, lf);
        }
    }
    // lane-slot utilisation of the shared loop: under the closest-hit set
    const unsigned long long st = wave_sum(c.strav), sl = wave_sum(c.sleaf), sr = wave_sum(c.stri);
    if (__lane_id() == 0) {
        atomicAdd(&a.counters[TRACE_CLOSEST].slots_trav, st);
        atomicAdd(&a.counters[TRACE_CLOSEST].slots_leaf, sl);
        atomicAdd(&a.counters[TRACE_CLOSEST].slots_tri, sr);
    }
}

// The traversal state of every lane is parked in LDS ([field][thread]) while the wave processes its
// waiting lanes, so the shading code's registers are not stacked on top of it (128 VGPRs and ~80
// spilled without this).  Only the ray (o.xyz d.xyz tmin tmax) goes to LDS; best, u, v, gid, node
// and stack pointer stay in registers across the processing phase, where the waiting lanes read
// their finished ray's hit.  Parking all 14 words measured 4.5 % slower: the 6 KB
// per workgroup it takes holds three more stack entries per lane.
// The probe record's flags (akr_pixel_probe): the seed always, the ray counts in the counting
// build, and with option "pixel_probe" 2 the pixel's completion time (wall clock / 16 above bit 8)
template <bool COUNT>
__device__ __forceinline__ uint32_t probe_flags(const PathArgs &pa) {
    if (!COUNT) return AKR_PROBE_SEED;
    uint32_t f = AKR_PROBE_SEED | AKR_PROBE_RAYS;
    if (pa.probe_clock) f |= 4u | (uint32_t)((wall_clock64() >> 4) << 8);
    return f;
}

constexpr int kParkSlots = 8;

template <bool COUNT, bool TAB>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(AKR_PATH_WAVES))) void k_path(PathArgs pa) {
    if (pa.gate && *pa.gate != pa.gate_want) return;  // the other candidate form runs (uniform: before any barrier)
    const TraceArgs &a = pa.t;
    __shared__ unsigned long long s_stack_mem[kStackLdsU64];
    __shared__ uint32_t s_park[kParkSlots][kTraceBlock];
    __shared__ uint4 s_tab[TAB ? kTabBytes / 16 : 1];
    lds_u64 *s_stack = (lds_u64 *)s_stack_mem;
    glb_u64 *stack_ovf = (glb_u64 *)a.stack_ovf;
    const uint32_t tid = threadIdx.x;
    const uint32_t gtid = blockIdx.x * kTraceBlock + tid;
    const uint32_t n = pa.n_pix;
    const int nb = pa.max_depth == 0 ? 1 : pa.max_depth;  // the trace at depth == max_depth is skipped (§3.3)
    const bool ff = a.any_far_first != 0;
    const auto tab = PathTab<TAB>::make(pa.sc, s_tab);  // one workgroup barrier when TAB
    PathCount c;
    if (COUNT) {
        c.lines = pa.lines;
        c.span[1] = pa.lines_span[1];
        c.span[2] = pa.lines_span[2];
        c.leaf_base = a.wide_leaves;
    }
    PixelFetch f{blockIdx.x % kWorkShards, 0, 0, (int)kWorkShards, n == 0};
    f.s_lo = shard_begin(n, f.shard);
    f.s_hi = shard_begin(n, f.shard + 1);

    // per-lane path state
    uint32_t pix = 0, left = 0, seed = 0, pxr = 0;
    int depth = 0;
    V3 beta{1.0f, 1.0f, 1.0f}, Lr{0.0f, 0.0f, 0.0f}, scol{0.0f, 0.0f, 0.0f};
    float4 film = {0.0f, 0.0f, 0.0f, 0.0f};
    float4 pe0 = {}, pe1 = {};  // extension ray waiting behind the shadow ray
    bool pend = false;
    bool any = false;           // the lane's ray is a shadow ray (a hit is bgid != kNoHit)
    bool need_pixel = true, done = false, fin = false, busy = false;
    uint32_t pc_closest = 0, pc_shadow = 0;  // counting build: the pixel's rays (akr_pixel_probe)
    PathRay r{};
    r.best = kInf;
    r.bgid = kNoHit;
    r.cur = r.leaf = AKR_CHILD_EMPTY;
    unsigned long long p_outer = 0, p_procs = 0, p_tp = 0, p_tt = 0, p_tl = 0, p_lanes = 0, p_t0 = 0, p_t = 0, p_tsh = 0;
    unsigned long long p_tpark = 0, p_tnext = 0, p_tbegin = 0, p_tload = 0;  // counting build: the split of A
    if (COUNT) p_t0 = wall_clock64();

    while (true) {
        // ---- A. lanes without a ray in flight
        const unsigned long long waiting = __ballot(!busy && !done);
        const uint32_t nwait = (uint32_t)__popcll(waiting);
        const uint32_t nbusy = (uint32_t)__popcll(__ballot(busy));
        if (nwait == 0 && nbusy == 0) break;
        if (COUNT) {
            p_outer++;
            p_t = wall_clock64();
        }
        // process once min_wait of a full wave's lanes wait, or that fraction of a sparser wave's
        if (nwait > 0 && 64u * nwait >= pa.min_wait * (nwait + nbusy)) {
            if (COUNT) {
                p_procs++;
                p_lanes += nwait;
            }
            path_park(s_park, tid, r);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            asm volatile("" ::: "memory");
            bool fresh = false, next_any = false, sample_end = false, start = false;
            float4 ra = {}, rb = {};
            unsigned long long p_ts = 0;
            unsigned long long tl_phase = 0;  // counting build: this phase's wait for the shading records
            if (COUNT) {
                p_ts = wall_clock64();
                p_tpark += p_ts - p_t;
            }
            if (!busy && !done && fin) {
                fin = false;
                const uint32_t hgid = r.bgid;
                if (any) {  // shadow ray: NEE contribution when unoccluded (pathtracer.h:84-88)
                    if (hgid == kNoHit) {
                        Lr.x += scol.x;
                        Lr.y += scol.y;
                        Lr.z += scol.z;
                    }
                    if (pend) {
                        ra = pe0;
                        rb = pe1;
                        fresh = true;
                        pend = false;
                    } else {
                        sample_end = true;
                    }
                } else if (hgid == kNoHit) {  // on_miss: the sample ends
                    sample_end = true;
                } else {
                    const V3 wo{-bitsf(s_park[3][tid]), -bitsf(s_park[4][tid]), -bitsf(s_park[5][tid])};
                    Bounce bo;
                    if (COUNT && pa.lines)
                        mark_lines(pa.lines, pa.lines_span[2], pa.lines_span[3], pa.sc.tri, pa.sc.tri + hgid,
                                   (uint32_t)sizeof(ShadeTri));
                    // inlined: 3 % faster than an out-of-line call once every load is global
                    shade_hit_tab(pa.sc, tab, hgid, r.bu, r.bv, wo, beta, seed, depth,
                              pa.max_depth, depth == nb - 1, bo, COUNT ? &tl_phase : nullptr);
                    if (bo.emit) {
                        Lr.x += bo.e.x;
                        Lr.y += bo.e.y;
                        Lr.z += bo.e.z;
                    }
                    if (bo.ext) {
                        beta = bo.nb;
                        depth++;
                    }
                    if (bo.sh) {  // the shadow ray first, the extension ray waits behind it
                        ra = bo.s0;
                        rb = bo.s1;
                        scol = bo.col;
                        next_any = true;
                        fresh = true;
                        pend = bo.ext;
                        pe0 = bo.e0;
                        pe1 = bo.e1;
                    } else if (bo.ext) {
                        ra = bo.e0;
                        rb = bo.e1;
                        fresh = true;
                    } else {
                        sample_end = true;
                    }
                }
            }
            if (COUNT) {
                const unsigned long long t = wall_clock64();
                p_tsh += t - p_ts;
                p_ts = t;
                p_tload += wave_max(tl_phase);  // wave-uniform: the shading lanes share the wait
            }
            if (sample_end) {  // Tile::add_sample (core/film.h:66-70), in sample order
                splat_one(film, make_float4(Lr.x, Lr.y, Lr.z, 0.0f), pa.ray_clamp);
                if (--left == 0) {
                    pa.film[pix] = film;
                    if (pa.probe)
                        pa.probe[pix] = make_uint4(seed, COUNT ? pc_closest : 0u, COUNT ? pc_shadow : 0u,
                                                   probe_flags<COUNT>(pa));
                    need_pixel = true;
                } else {
                    start = true;
                }
            }
            // next pixel for the lanes that finished theirs: one atomic per wave per attempt
            const bool asked = need_pixel && !done;
            fetch_pixels(f, n, pa.work, pa.order ? pa.order_mode : FETCH_LINEAR, pa.order, pa.prio, need_pixel, done, pix);
            if (asked && !need_pixel) {
                const uint32_t px = pa.pixel[pix];
                pxr = px;
                left = pa.spp;
                seed = (uint32_t)((int)(px & 0xFFFFu) + (int)(px >> 16) * pa.cam.width);
                film = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                start = true;
                if (COUNT) pc_closest = pc_shadow = 0;
            }
            if (start) {  // a new sample: camera ray (pathtracer.h:61-64), L = 0, beta = 1
                Lr = V3{0.0f, 0.0f, 0.0f};
                beta = V3{1.0f, 1.0f, 1.0f};
                depth = 0;
                // the pixel's coordinates from a register set at its fetch: no dependent load per sample
                // (measured: whole frame -0.6 %, profiles/r21_px_reg_ab.log; the reload
                // was cheaper before the r21 traversal changes freed registers)
                const uint32_t px = pxr;
                camera_ray(pa.cam, (int)(px & 0xFFFFu), (int)(px >> 16), seed, ra, rb);
                fresh = true;
            }
            asm volatile("" ::: "memory");
            if (COUNT) {
                const unsigned long long t = wall_clock64();
                p_tnext += t - p_ts;
                p_ts = t;
            }
            path_unpark(s_park, tid, r, ff, any);  // the busy lanes' traversal continues unchanged
            if (fresh) {
                any = next_any;
                if (COUNT) {
                    pc_closest += any ? 0u : 1u;
                    pc_shadow += any ? 1u : 0u;
                }
                busy = path_begin<COUNT>(a, any, ra, rb, r, s_stack, stack_ovf, tid, gtid, c);
                fin = !busy;
            }
            if (COUNT) p_tbegin += wall_clock64() - p_ts;
        }
        if (COUNT) {
            const unsigned long long t = wall_clock64();
            p_tp += t - p_t;
            p_t = t;
        }
        if (!__any(busy)) continue;
        // ---- B. traversal phase, C. leaf phase (k_trace's, shared with k_path_defer)
        const int kd = any ? 1 : 0;
        path_traverse<COUNT, kWhileExitPath>(busy, kd, r, a.wide_nodes, s_stack, stack_ovf, a.ovf_threads, tid, gtid, c);
        if (COUNT) {
            const unsigned long long t = wall_clock64();
            p_tt += t - p_t;
            p_t = t;
        }
        const bool hit_any = path_leaf<COUNT>(busy, kd, r, a.wide_leaves, c);
        if (busy && (hit_any || r.cur == AKR_CHILD_EMPTY)) {
            busy = false;
            fin = true;
            if (COUNT) c.deep[kd] += c.deep_now ? 1 : 0;
        }
        if (COUNT) p_tl += wall_clock64() - p_t;
    }
    if (COUNT) {
        path_count_flush(pa, c, p_outer, p_procs, p_tp, p_tt, p_tl, p_t0, p_lanes, p_tsh);
        if (__lane_id() == 0 && pa.prof) {
            atomicAdd(&pa.prof->tp_park, p_tpark);
            atomicAdd(&pa.prof->tp_next, p_tnext);
            atomicAdd(&pa.prof->tp_begin, p_tbegin);
            atomicAdd(&pa.prof->tp_load, p_tload);
        }
    }
}

__device__ __forceinline__ void path_park(uint32_t (*s_park)[kTraceBlock], uint32_t tid, const PathRay &r) {
    const float pv[8] = {r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, r.tmin, r.tmax};
#pragma unroll
    for (int k = 0; k < 8; k++) s_park[k][tid] = fbits(pv[k]);
}
__device__ __forceinline__ void path_unpark(uint32_t (*s_park)[kTraceBlock], uint32_t tid, PathRay &r, bool far_first,
                                            bool occl) {
    r.o = V3{bitsf(s_park[0][tid]), bitsf(s_park[1][tid]), bitsf(s_park[2][tid])};
    r.d = V3{bitsf(s_park[3][tid]), bitsf(s_park[4][tid]), bitsf(s_park[5][tid])};
    r.tmin = bitsf(s_park[6][tid]);
    r.tmax = bitsf(s_park[7][tid]);
    r.invd = V3{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
    r.dpos = (r.d.x > 0.0f ? 1u : 0u) | (r.d.y > 0.0f ? 2u : 0u) | (r.d.z > 0.0f ? 4u : 0u);
    if (occl && far_first) r.dpos ^= 7u;
    r.tmaxp = float_below(r.tmax);
    r.leaf = AKR_CHILD_EMPTY;
}

// Position of the r-th set bit of m (r < popcount(m)): binary search on popcounts
__device__ __forceinline__ int nth_set_bit(unsigned long long m, uint32_t r) {
    int base = 0;
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
        const unsigned long long low = m & ((1ull << s) - 1ull);
        const uint32_t c = (uint32_t)__popcll(low);
        if (r >= c) {
            r -= c;
            m >>= s;
            base += s;
        } else {
            m = low;
        }
    }
    return base;
}

// ------------------------------------------------------------------- persistent path, deferred NEE
// k_path_defer: k_path with the shadow rays taken off a pixel's chain.  When a bounce
// yields a shadow ray, its contribution goes to the lane's scratch (slot parity * 8 + bounce) and the
// ray is handed, by lane shuffles inside the wave, to a lane with no work of its own (pixel done, or
// waiting on its own shadow results); that lane traces it and posts (resolved, occluded) into the
// owner's LDS word.  The owner goes on with its extension ray at once.  A sample whose path has ended
// closes once all its shadow results are in: L = (emission) + the unoccluded contributions in bounce
// order, exactly the sequential order of pathtracer.h:84-88, then Tile::add_sample.  At most two
// samples of a pixel are in flight (the older one waiting to close), so the film sums stay in
// sample order.  A shadow ray with no free lane in the wave is traced by its owner, as in k_path.
// Every hand-off and result stays inside one wave: no cross-wave synchronisation.
constexpr uint32_t kDeferSlots = 8;  // shadow rays per sample (one per bounce below max_depth <= 8)
enum : uint32_t { RAY_NONE = 0, RAY_OWN = 1, RAY_OWN_SHADOW = 2, RAY_FOREIGN = 3 };

// The per-lane sample bookkeeping of k_path_defer in one word (registers are the limit there)
struct DeferState {
    uint32_t w = 0;
    static constexpr uint32_t KIND = 0, RP = 2, LAST = 3, OPEN = 4, NSH = 6, DEPTH = 14, FTAG = 18, PEND = 30, RUN = 31;
    __device__ __forceinline__ uint32_t get(uint32_t off, uint32_t bits) const { return (w >> off) & ((1u << bits) - 1u); }
    __device__ __forceinline__ void set(uint32_t off, uint32_t bits, uint32_t v) {
        const uint32_t m = ((1u << bits) - 1u) << off;
        w = (w & ~m) | ((v << off) & m);
    }
    __device__ __forceinline__ uint32_t kind() const { return get(KIND, 2); }
    __device__ __forceinline__ uint32_t rp() const { return get(RP, 1); }
    __device__ __forceinline__ uint32_t last() const { return get(LAST, 1); }
    __device__ __forceinline__ uint32_t open() const { return get(OPEN, 2); }
    __device__ __forceinline__ uint32_t nsh(uint32_t q) const { return get(NSH + 4 * q, 4); }
    __device__ __forceinline__ int depth() const { return (int)get(DEPTH, 4); }
    __device__ __forceinline__ uint32_t ftag() const { return get(FTAG, 12); }  // owner lane | slot << 8
    __device__ __forceinline__ bool pend() const { return get(PEND, 1) != 0; }
    __device__ __forceinline__ bool running() const { return get(RUN, 1) != 0; }
};

template <bool COUNT, bool TAB>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(AKR_PATH_WAVES))) void k_path_defer(PathArgs pa) {
    if (pa.gate && *pa.gate != pa.gate_want) return;  // the other candidate form runs (uniform: before any barrier)
    const TraceArgs &a = pa.t;
    __shared__ unsigned long long s_stack_mem[kStackLdsU64];
    __shared__ uint32_t s_park[kParkSlots][kTraceBlock];
    __shared__ uint4 s_tab[TAB ? kTabBytes / 16 : 1];
    __shared__ uint32_t s_res[kTraceBlock];  // per owner lane: resolved bit (slot), occluded bit (16 + slot)
    lds_u64 *s_stack = (lds_u64 *)s_stack_mem;
    glb_u64 *stack_ovf = (glb_u64 *)a.stack_ovf;
    const uint32_t tid = threadIdx.x;
    const uint32_t gtid = blockIdx.x * kTraceBlock + tid;
    const size_t lanes = (size_t)gridDim.x * kTraceBlock;
    float4 *const contrib = pa.contrib + gtid;  // slot s at contrib[s * lanes]; 16, 17: the waiting extension ray
    const uint32_t n = pa.n_pix;
    const int nb = pa.max_depth == 0 ? 1 : pa.max_depth;
    const bool ff = a.any_far_first != 0;
    const auto tab = PathTab<TAB>::make(pa.sc, s_tab);  // one workgroup barrier when TAB
    PathCount c;
    PixelFetch f{blockIdx.x % kWorkShards, 0, 0, (int)kWorkShards, n == 0};
    f.s_lo = shard_begin(n, f.shard);
    f.s_hi = shard_begin(n, f.shard + 1);
    s_res[tid] = 0;

    uint32_t pix = 0, left = 0, seed = 0, pxy = 0;
    V3 beta{1.0f, 1.0f, 1.0f}, Lr{0.0f, 0.0f, 0.0f};
    // a pixel's film sums live in its (zeroed) film slot, not in registers: 23 -> 15 VGPRs spilled, time
    // unchanged (the same change made k_path 0.7 % slower, §3.8); samples close in
    // sample order, so the sums are the sequential ones
#define DEFER_SPLAT(l)                                 \
    do {                                               \
        float4 fm_ = pa.film[pix];                     \
        splat_one(fm_, (l), pa.ray_clamp);             \
        pa.film[pix] = fm_;                            \
    } while (0)
    DeferState s;
    bool need_pixel = true, done = false, fin = false, busy = false;
    uint32_t idle_rounds = 0;    // hang guard: consecutive rounds with no ray in flight in the wave
    uint32_t pc_closest = 0, pc_shadow = 0;  // counting build: the owned pixel's rays (akr_pixel_probe)
    PathRay r{};
    r.best = kInf;
    r.bgid = kNoHit;
    r.cur = r.leaf = AKR_CHILD_EMPTY;
    unsigned long long p_outer = 0, p_procs = 0, p_tp = 0, p_tt = 0, p_tl = 0, p_lanes = 0, p_t0 = 0, p_t = 0, p_tsh = 0;
    if (COUNT) p_t0 = wall_clock64();

    // a new sample of the lane's pixel, when nothing else is in hand and at most one older sample
    // is still waiting to close (sample k has parity k & 1)
    auto try_start = [&](bool free_lane, bool &fresh, float4 &ra, float4 &rb) {
        if (free_lane && !done && !need_pixel && !s.running() && left > 0 && __popc(s.open()) <= 1) {
            s.set(DeferState::RP, 1, (pa.spp - left) & 1u);
            left--;
            s.set(DeferState::RUN, 1, 1);
            s.set(DeferState::DEPTH, 4, 0);
            Lr = V3{0.0f, 0.0f, 0.0f};
            beta = V3{1.0f, 1.0f, 1.0f};
            camera_ray(pa.cam, (int)(pxy & 0xFFFFu), (int)(pxy >> 16), seed, ra, rb);
            fresh = true;
            s.set(DeferState::KIND, 2, RAY_OWN);
        }
    };

    while (true) {
        if (!__any(!done || busy || fin)) break;
        const uint32_t nfin = (uint32_t)__popcll(__ballot(fin));
        const uint32_t nbusy = (uint32_t)__popcll(__ballot(busy));
        if (COUNT) {
            p_outer++;
            p_t = wall_clock64();
        }
        if (nfin > 0 ? 64u * nfin >= pa.min_wait * (nfin + nbusy) : nbusy == 0) {
            if (COUNT) {
                p_procs++;
                p_lanes += nfin;
            }
            path_park(s_park, tid, r);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            asm volatile("" ::: "memory");
            bool fresh = false, occl = false, want_sh = false, sample_end = false;
            float4 ra = {}, rb = {}, sh0 = {}, sh1 = {};
            uint32_t shtag = 0;
            unsigned long long p_ts = 0;
            if (COUNT) p_ts = wall_clock64();
            // 1. the finished ray's result
            if (fin) {
                fin = false;
                const uint32_t hgid = r.bgid;
                const uint32_t kind = s.kind();
                if (kind == RAY_FOREIGN || kind == RAY_OWN_SHADOW) {
                    const uint32_t tag = s.ftag();
                    const uint32_t owner = kind == RAY_FOREIGN ? (tag & 0xFFu) : tid, slot = tag >> 8;
                    atomicOr(&s_res[owner], (1u << slot) | (hgid != kNoHit ? (1u << (16 + slot)) : 0u));
                    s.set(DeferState::KIND, 2, RAY_NONE);
                    if (kind == RAY_OWN_SHADOW && s.pend()) {  // the extension ray waited behind it
                        ra = contrib[16 * lanes];
                        rb = contrib[17 * lanes];
                        s.set(DeferState::PEND, 1, 0);
                        fresh = true;
                        s.set(DeferState::KIND, 2, RAY_OWN);
                    }
                } else {  // the running sample's closest hit
                    s.set(DeferState::KIND, 2, RAY_NONE);
                    if (hgid == kNoHit) {
                        sample_end = true;
                    } else {
                        const V3 wo{-bitsf(s_park[3][tid]), -bitsf(s_park[4][tid]), -bitsf(s_park[5][tid])};
                        const int depth = s.depth();
                        Bounce bo;
                        shade_hit_tab(pa.sc, tab, hgid, r.bu, r.bv, wo, beta, seed, depth,
                                  pa.max_depth, depth == nb - 1, bo);
                        if (bo.emit) {
                            Lr.x += bo.e.x;
                            Lr.y += bo.e.y;
                            Lr.z += bo.e.z;
                        }
                        if (bo.ext) {
                            beta = bo.nb;
                            s.set(DeferState::DEPTH, 4, (uint32_t)depth + 1u);
                        }
                        if (bo.sh) {
                            if (COUNT) pc_shadow++;  // the owner's pixel, whichever lane traces it
                            const uint32_t rp = s.rp(), b = s.nsh(rp), slot = rp * kDeferSlots + b;
                            s.set(DeferState::NSH + 4 * rp, 4, b + 1u);
                            contrib[slot * lanes] = make_float4(bo.col.x, bo.col.y, bo.col.z, 0.0f);
                            want_sh = true;
                            sh0 = bo.s0;
                            sh1 = bo.s1;
                            shtag = tid | (slot << 8);
                            if (bo.ext) {  // may have to wait behind the shadow ray (step 5)
                                ra = bo.e0;
                                rb = bo.e1;
                            } else {
                                sample_end = true;
                            }
                        } else if (bo.ext) {
                            ra = bo.e0;
                            rb = bo.e1;
                            fresh = true;
                            s.set(DeferState::KIND, 2, RAY_OWN);
                        } else {
                            sample_end = true;
                        }
                    }
                }
            }
            if (COUNT) p_tsh += wall_clock64() - p_ts;
            // 2. a path that ended: close at once when nothing waits, else leave it open
            if (sample_end) {
                const uint32_t rp = s.rp();
                s.set(DeferState::RUN, 1, 0);
                s.set(DeferState::LAST, 1, rp);
                if (s.nsh(rp) == 0 && s.open() == 0)
                    DEFER_SPLAT(make_float4(Lr.x, Lr.y, Lr.z, 0.0f));
                else
                    s.set(DeferState::OPEN, 2, s.open() | (1u << rp));
            }
            // 3. close the oldest open samples whose shadow results are all in, in sample order
            for (int it = 0; it < 2 && s.open(); it++) {
                const uint32_t om = s.open();
                const uint32_t q = __popc(om) == 2 ? (s.last() ^ 1u) : (om == 1u ? 0u : 1u);
                const uint32_t k = s.nsh(q);
                const uint32_t need = ((1u << k) - 1u) << (kDeferSlots * q);
                const uint32_t res = s_res[tid];
                if ((res & need) != need) break;
                V3 L = (q == s.last() && !s.running()) ? Lr : V3{0.0f, 0.0f, 0.0f};
                for (uint32_t b = 0; b < k; b++)  // pathtracer.h:84-88, in bounce order
                    if (!((res >> (16 + kDeferSlots * q + b)) & 1u)) {
                        const float4 cc = contrib[(q * kDeferSlots + b) * lanes];
                        L.x += cc.x;
                        L.y += cc.y;
                        L.z += cc.z;
                    }
                DEFER_SPLAT(make_float4(L.x, L.y, L.z, 0.0f));
                s.set(DeferState::OPEN, 2, om & ~(1u << q));
                s.set(DeferState::NSH + 4 * q, 4, 0);
                atomicAnd(&s_res[tid], ~((0xFFu << (kDeferSlots * q)) | (0xFFu << (16 + kDeferSlots * q))));
            }
            // 4. a finished pixel stores its film and fetches the next; free lanes start samples
            const bool free_lane = !busy && !fresh && !want_sh && s.kind() == RAY_NONE;
            if (free_lane && !done && !need_pixel && !s.running() && left == 0 && s.open() == 0) {
                if (pa.probe)
                    pa.probe[pix] = make_uint4(seed, COUNT ? pc_closest : 0u, COUNT ? pc_shadow : 0u,
                                               probe_flags<COUNT>(pa));
                need_pixel = true;
            }
            const bool asked = need_pixel && !done;
            fetch_pixels(f, n, pa.work, pa.order ? pa.order_mode : (pa.mix ? FETCH_SCRAMBLE : FETCH_LINEAR), pa.order, pa.prio,
                         need_pixel, done, pix);  // the cost order replaces the scramble
            if (asked && !need_pixel) {
                pxy = pa.pixel[pix];
                left = pa.spp;
                seed = (uint32_t)((int)(pxy & 0xFFFFu) + (int)(pxy >> 16) * pa.cam.width);
                if (COUNT) pc_closest = pc_shadow = 0;
            }
            try_start(free_lane, fresh, ra, rb);
            // 5. hand the new shadow rays to the wave's lanes that have nothing in hand, in lane order
            const unsigned long long pm = __ballot(want_sh);
            if (pm) {
                const bool helper = !busy && !fresh && !want_sh && s.kind() == RAY_NONE;
                const unsigned long long hm = __ballot(helper);
                const uint32_t np = (uint32_t)__popcll(pm), nh = (uint32_t)__popcll(hm);
                const uint32_t k = np < nh ? np : nh;
                const uint32_t hr = lane_prefix(hm), pr = lane_prefix(pm);
                const bool take = helper && hr < k;
                const int src = take ? nth_set_bit(pm, hr) : (int)__lane_id();
                float4 x0, x1;
                x0.x = __shfl(sh0.x, src);
                x0.y = __shfl(sh0.y, src);
                x0.z = __shfl(sh0.z, src);
                x0.w = __shfl(sh0.w, src);
                x1.x = __shfl(sh1.x, src);
                x1.y = __shfl(sh1.y, src);
                x1.z = __shfl(sh1.z, src);
                x1.w = __shfl(sh1.w, src);
                const uint32_t tg = (uint32_t)__shfl((int)shtag, src);
                if (take) {
                    ra = x0;
                    rb = x1;
                    s.set(DeferState::FTAG, 12, tg);
                    s.set(DeferState::KIND, 2, RAY_FOREIGN);
                    occl = true;
                    fresh = true;
                }
                if (want_sh) {
                    const bool has_ext = s.running();  // the path goes on (its ray is in ra / rb)
                    if (pr < k) {  // handed over: go on with the extension ray, or start the next sample
                        if (has_ext) {
                            fresh = true;
                            s.set(DeferState::KIND, 2, RAY_OWN);
                        } else {
                            try_start(true, fresh, ra, rb);
                        }
                    } else {  // no free lane: trace it here, the extension ray waits behind it
                        if (has_ext) {
                            contrib[16 * lanes] = ra;
                            contrib[17 * lanes] = rb;
                            s.set(DeferState::PEND, 1, 1);
                        }
                        ra = sh0;
                        rb = sh1;
                        s.set(DeferState::FTAG, 12, shtag);
                        s.set(DeferState::KIND, 2, RAY_OWN_SHADOW);
                        occl = true;
                        fresh = true;
                    }
                }
            }
            asm volatile("" ::: "memory");
            // 6. unpark; fresh rays begin
            const uint32_t kind_now = s.kind();
            path_unpark(s_park, tid, r, ff, kind_now == RAY_OWN_SHADOW || kind_now == RAY_FOREIGN);
            if (fresh) {
                if (COUNT) pc_closest += occl ? 0u : 1u;  // own extension / camera rays
                busy = path_begin<COUNT>(a, occl, ra, rb, r, s_stack, stack_ovf, tid, gtid, c);
                fin = !busy;
            }
        }
        if (COUNT) {
            const unsigned long long t = wall_clock64();
            p_tp += t - p_t;
            p_t = t;
        }
        if (!__any(busy)) {
            // nothing in flight: every result is posted, so the next round makes progress; a wave
            // that idles for many rounds has lost its state (a bug): stop instead of spinning, and
            // raise the fault word the host checks after every render (akr_hip_ctx::check_fault)
            if (++idle_rounds > 1024) {
                if (pa.fault && __lane_id() == 0) __hip_atomic_fetch_or(pa.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            continue;
        }
        idle_rounds = 0;
        const uint32_t kind_now = s.kind();
        const int kd = (kind_now == RAY_OWN_SHADOW || kind_now == RAY_FOREIGN) ? 1 : 0;
        path_traverse<COUNT>(busy, kd, r, a.wide_nodes, s_stack, stack_ovf, a.ovf_threads, tid, gtid, c);
        if (COUNT) {
            const unsigned long long t = wall_clock64();
            p_tt += t - p_t;
            p_t = t;
        }
        const bool hit_any = path_leaf<COUNT>(busy, kd, r, a.wide_leaves, c);
        if (busy && (hit_any || r.cur == AKR_CHILD_EMPTY)) {
            busy = false;
            fin = true;
            if (COUNT) c.deep[kd] += c.deep_now ? 1 : 0;
        }
        if (COUNT) p_tl += wall_clock64() - p_t;
    }
    if (COUNT) path_count_flush(pa, c, p_outer, p_procs, p_tp, p_tt, p_tl, p_t0, p_lanes, p_tsh);
    // test-only (option "fault_test"): raise the hang guard's fault word once, so the host-side
    // reporting path can be exercised without a hang
    if (pa.fault_test && pa.fault && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_fetch_or(pa.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

#undef DEFER_SPLAT

// ------------------------------------------------------------- persistent path, speculative samples
// k_path_spec: k_path whose lanes, once the pixel queue is drained, help the busy
// pixels of their wave by running their later samples speculatively.  A pixel's samples are
// sequential only through its sampler state (cpu/integrator.cpp:124-134): sample s + 1 starts where
// sample s stopped drawing, 4 + 6 k draws later for k scattering events (pathtracer.h:96-164).
// A pixel is run by a group of lanes: its owner (the pixel, its film slot, the committed state C and
// count) and up to kSpecHelpers helpers.  Each lane of a group runs one node of a speculation tree:
// node 0 is the head, the next sample to commit, started from C; a node on level l (1..3) is the
// sample l places after the head, started from lcg_advance(C, the draws of the l samples before it),
// each of which it assumes to be full length (4 + 6 max_depth) or one bounce long (4 + 6) — the two
// common lengths of the C3 soup's samples (46 % and 34 %, tools/sample_lengths.py); its code holds
// those l choices.  Idle lanes take the free nodes in order of expected use.  When the head ends the
// owner commits it (Tile::add_sample, core/film.h:66-70), C becomes its end state, and its length
// picks the branch: the nodes whose first choice it is move up a level (the level-1 one becomes the
// head: it did start from the new C), the others are dropped; a length that is neither drops every
// node.  So a committed sample is always the one that starts from the committed state, and the film
// sums and the final sampler state are the sequential loop's, bit for bit.  The lanes of a group find
// each other with wave ballots against the owner's group mask; every hand-off is a lane shuffle.
constexpr uint32_t kSpecNodes = 15;     // the head and 2 + 4 + 8 nodes on levels 1-3 (a group spans at most 15 lanes)
// nodes in order of expected use (a sample full length with p = 0.6, one bounce with q = 0.35):
// 0, 1, 3, 2, 7, 4, 5, 8, 9, 11, 6, 12, 13, 10, 14, one per nibble
constexpr unsigned long long kSpecNodeOrder = 0xEADC6B985472310ull;
enum : uint32_t { ROLE_FREE = 0, ROLE_OWNER = 1, ROLE_HELPER = 2 };
enum : uint32_t { BR_FULL = 0, BR_ONE = 1, BR_NONE = 2, BR_NOCOMMIT = 3 };  // the head's branch, broadcast

__device__ __forceinline__ uint32_t node_lvl(uint32_t nd) { return 31u - __clz(nd + 1u); }
__device__ __forceinline__ uint32_t node_code(uint32_t nd) { return nd + 1u - (1u << node_lvl(nd)); }

struct SpecState {
    uint32_t w = 0;
    // ROLE: free / owner / helper; OL: a helper's owner lane; SRUN: the lane's sample runs; SEND: it
    // ended, (Lr, seed) wait for the commit; NODE: the lane's node in its group's tree; NH (owner):
    // helpers
    static constexpr uint32_t ROLE = 0, OL = 2, SRUN = 8, SEND = 9, ANY = 10, PEND = 11, NODE = 12, NH = 17;
    __device__ __forceinline__ uint32_t get(uint32_t off, uint32_t bits) const { return (w >> off) & ((1u << bits) - 1u); }
    __device__ __forceinline__ void set(uint32_t off, uint32_t bits, uint32_t v) {
        const uint32_t m = ((1u << bits) - 1u) << off;
        w = (w & ~m) | ((v << off) & m);
    }
    __device__ __forceinline__ uint32_t role() const { return get(ROLE, 2); }
    __device__ __forceinline__ uint32_t ol() const { return get(OL, 6); }
    __device__ __forceinline__ bool srun() const { return get(SRUN, 1) != 0; }
    __device__ __forceinline__ bool send() const { return get(SEND, 1) != 0; }
    __device__ __forceinline__ bool any() const { return get(ANY, 1) != 0; }
    __device__ __forceinline__ bool pend() const { return get(PEND, 1) != 0; }
    __device__ __forceinline__ uint32_t node() const { return get(NODE, 4); }
    __device__ __forceinline__ uint32_t nh() const { return get(NH, 5); }
};

template <bool COUNT, bool TAB>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(AKR_PATH_WAVES))) void k_path_spec(PathArgs pa) {
    if (pa.gate && *pa.gate != pa.gate_want) return;  // the other candidate form runs (uniform: before any barrier)
    const TraceArgs &a = pa.t;
    __shared__ unsigned long long s_stack_mem[kStackLdsU64];
    __shared__ uint32_t s_park[kParkSlots][kTraceBlock];
    __shared__ uint4 s_tab[TAB ? kTabBytes / 16 : 1];
    lds_u64 *s_stack = (lds_u64 *)s_stack_mem;
    glb_u64 *stack_ovf = (glb_u64 *)a.stack_ovf;
    const uint32_t tid = threadIdx.x;
    const uint32_t gtid = blockIdx.x * kTraceBlock + tid;
    const uint32_t lane = __lane_id();
    const unsigned long long below = (1ull << lane) - 1ull;  // lanes under this one
    const uint32_t n = pa.n_pix;
    const int nb = pa.max_depth == 0 ? 1 : pa.max_depth;  // the trace at depth == max_depth is skipped (§3.3)
    const uint32_t g_full = 4u + 6u * (uint32_t)pa.max_depth;  // draws of a full-length sample
    const uint32_t g_one = 4u + 6u;                             // draws of a one-bounce sample
    const uint32_t lvl_cap = min(pa.spec_depth, 3u);            // tree levels used (option path_spec_depth)
    // the chain of full-length guesses only: the tree's one-bounce branches measured slower
    const uint32_t spp = pa.spp;
    const bool ff = a.any_far_first != 0;
    const auto tab = PathTab<TAB>::make(pa.sc, s_tab);  // one workgroup barrier when TAB
    PathCount c;
    PixelFetch f{blockIdx.x % kWorkShards, 0, 0, (int)kWorkShards, n == 0};
    f.s_lo = shard_begin(n, f.shard);
    f.s_hi = shard_begin(n, f.shard + 1);

    // owner: the committed state and count, the tree nodes in flight (bit per node), its group's
    // lanes; every group lane: the pixel, and the sample it runs
    uint32_t pix = 0, C = 0, cseq = 0, occ = 0;
    unsigned long long grp = 0;
    uint32_t seed = 0;
    int depth = 0;
    V3 beta{1.0f, 1.0f, 1.0f}, Lr{0.0f, 0.0f, 0.0f}, scol{0.0f, 0.0f, 0.0f};
    float4 pe0 = {}, pe1 = {};  // extension ray waiting behind the shadow ray
    SpecState s;
    bool done = false, fin = false, busy = false;
    uint32_t idle_rounds = 0;
    uint32_t pc_closest = 0, pc_shadow = 0, sc_closest = 0, sc_shadow = 0;  // counting build: pixel / sample rays
    unsigned long long n_spec = 0, n_abort = 0;                              // counting build: speculation
    PathRay r{};
    r.best = kInf;
    r.bgid = kNoHit;
    r.cur = r.leaf = AKR_CHILD_EMPTY;
    unsigned long long p_outer = 0, p_procs = 0, p_tp = 0, p_tt = 0, p_tl = 0, p_lanes = 0, p_t0 = 0, p_t = 0, p_tsh = 0;
    if (COUNT) p_t0 = wall_clock64();

    while (true) {
        if (!__any(s.role() != ROLE_FREE || !done || busy || fin)) break;
        const uint32_t nfin = (uint32_t)__popcll(__ballot(fin));
        const uint32_t nbusy = (uint32_t)__popcll(__ballot(busy));
        if (COUNT) {
            p_outer++;
            p_t = wall_clock64();
        }
        if (nfin > 0 ? 64u * nfin >= pa.min_wait * (nfin + nbusy) : nbusy == 0) {
            if (COUNT) {
                p_procs++;
                p_lanes += nfin;
            }
            path_park(s_park, tid, r);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            asm volatile("" ::: "memory");
            bool fresh = false, next_any = false, start = false;
            float4 ra = {}, rb = {};
            unsigned long long p_ts = 0;
            if (COUNT) p_ts = wall_clock64();
            // 1. the finished ray (k_path's processing); a sample that ended waits for its commit
            if (fin) {
                fin = false;
                bool sample_end = false;
                const uint32_t hgid = r.bgid;
                if (s.any()) {  // shadow ray: NEE contribution when unoccluded (pathtracer.h:84-88)
                    if (hgid == kNoHit) {
                        Lr.x += scol.x;
                        Lr.y += scol.y;
                        Lr.z += scol.z;
                    }
                    if (s.pend()) {
                        ra = pe0;
                        rb = pe1;
                        fresh = true;
                        s.set(SpecState::PEND, 1, 0);
                    } else {
                        sample_end = true;
                    }
                } else if (hgid == kNoHit) {  // on_miss: the sample ends
                    sample_end = true;
                } else {
                    const V3 wo{-bitsf(s_park[3][tid]), -bitsf(s_park[4][tid]), -bitsf(s_park[5][tid])};
                    Bounce bo;
                    shade_hit_tab(pa.sc, tab, hgid, r.bu, r.bv, wo, beta, seed, depth, pa.max_depth, depth == nb - 1, bo);
                    if (bo.emit) {
                        Lr.x += bo.e.x;
                        Lr.y += bo.e.y;
                        Lr.z += bo.e.z;
                    }
                    if (bo.ext) {
                        beta = bo.nb;
                        depth++;
                    }
                    if (bo.sh) {  // the shadow ray first, the extension ray waits behind it
                        ra = bo.s0;
                        rb = bo.s1;
                        scol = bo.col;
                        next_any = true;
                        fresh = true;
                        s.set(SpecState::PEND, 1, bo.ext ? 1u : 0u);
                        pe0 = bo.e0;
                        pe1 = bo.e1;
                    } else if (bo.ext) {
                        ra = bo.e0;
                        rb = bo.e1;
                        fresh = true;
                    } else {
                        sample_end = true;
                    }
                }
                if (sample_end) {
                    s.set(SpecState::SRUN, 1, 0);
                    s.set(SpecState::SEND, 1, 1);
                }
            }
            if (COUNT) p_tsh += wall_clock64() - p_ts;
            // Until a lane of the wave finds the pixel queue drained no lane can be a helper: every group
            // is its owner alone, running its head.  Steps 2-5 then reduce to k_path's processing: commit
            // a finished head, fetch a pixel, start the next head from C, without the group bookkeeping.
            const bool fast = !__any(done);
            if (fast) {
                bool head = false;  // start the head sample from C
                if (s.role() == ROLE_OWNER && s.send()) {  // Tile::add_sample, C = the head's end state
                    float4 fm = pa.film[pix];
                    splat_one(fm, make_float4(Lr.x, Lr.y, Lr.z, 0.0f), pa.ray_clamp);
                    pa.film[pix] = fm;
                    if (COUNT) {
                        pc_closest += sc_closest;
                        pc_shadow += sc_shadow;
                    }
                    C = seed;
                    cseq++;
                    occ = 0;
                    s.set(SpecState::SEND, 1, 0);
                    if (cseq == spp) {
                        if (pa.probe)
                            pa.probe[pix] = make_uint4(C, COUNT ? pc_closest : 0u, COUNT ? pc_shadow : 0u, probe_flags<COUNT>(pa));
                        s.set(SpecState::ROLE, 2, ROLE_FREE);
                        s.set(SpecState::NH, 5, 0);
                        grp = 0;
                    } else {
                        head = true;
                    }
                }
                bool need = s.role() == ROLE_FREE && !done;
                const bool asked = need;
                fetch_pixels(f, n, pa.work, pa.order ? pa.order_mode : FETCH_LINEAR, pa.order, pa.prio, need, done, pix);
                if (asked && !need) {
                    const uint32_t px = pa.pixel[pix];
                    C = (uint32_t)((int)(px & 0xFFFFu) + (int)(px >> 16) * pa.cam.width);
                    cseq = 0;
                    occ = 0;
                    grp = 1ull << lane;
                    s.set(SpecState::ROLE, 2, ROLE_OWNER);
                    s.set(SpecState::NH, 5, 0);
                    if (COUNT) pc_closest = pc_shadow = 0;
                    head = true;
                }
                if (head) {
                    seed = C;
                    occ |= 1u;
                    s.set(SpecState::NODE, 4, 0);
                    start = true;
                }
            } else {
            // 2. commits, in sample order: a finished head is committed and its length picks the
            // branch of the tree that moves up; rounds until no group has a finished head
            const int ol = s.role() == ROLE_HELPER ? (int)s.ol() : (int)lane;
            for (int it = 0; it <= (int)kSpecNodes; it++) {
                const bool hd = s.role() != ROLE_FREE && s.send() && s.node() == 0u;  // a finished head
                const unsigned long long hm = __ballot(hd);
                if (hm == 0) break;
                const bool act = s.role() == ROLE_OWNER && (grp & hm) != 0;
                const int hl = act ? __ffsll((long long)(grp & hm)) - 1 : (int)lane;
                V3 L;
                L.x = __shfl(Lr.x, hl);
                L.y = __shfl(Lr.y, hl);
                L.z = __shfl(Lr.z, hl);
                const uint32_t E = (uint32_t)__shfl((int)seed, hl);
                uint32_t hcc = 0, hcs = 0;
                if (COUNT) {
                    hcc = (uint32_t)__shfl((int)sc_closest, hl);
                    hcs = (uint32_t)__shfl((int)sc_shadow, hl);
                }
                uint32_t br = BR_NOCOMMIT;
                if (act) {  // Tile::add_sample, C = the head's end state
                    float4 fm = pa.film[pix];  // the film sums live in the (zeroed) film slot
                    splat_one(fm, make_float4(L.x, L.y, L.z, 0.0f), pa.ray_clamp);
                    pa.film[pix] = fm;
                    if (COUNT) {
                        pc_closest += hcc;
                        pc_shadow += hcs;
                    }
                    br = E == lcg_advance(C, g_full) ? BR_FULL : (E == lcg_advance(C, g_one) ? BR_ONE : BR_NONE);
                    C = E;
                    cseq++;
                    // the nodes on branch br move up a level, the others go
                    uint32_t nocc = 0;
                    for (uint32_t nd = 1; nd < kSpecNodes; nd++) {
                        const uint32_t lv = node_lvl(nd), cd = node_code(nd);
                        if (((occ >> nd) & 1u) && br != BR_NONE && (cd & 1u) == br)
                            nocc |= 1u << ((1u << (lv - 1u)) - 1u + (cd >> 1));
                    }
                    occ = nocc;
                }
                const uint32_t obr = (uint32_t)__shfl((int)br, ol);
                if (s.role() != ROLE_FREE && obr != BR_NOCOMMIT && (s.srun() || s.send())) {
                    const uint32_t nd = s.node();
                    bool drop = false;
                    if (nd == 0u) {  // the committed head: its lane is free
                        s.set(SpecState::SEND, 1, 0);
                    } else if (obr == BR_NONE || (node_code(nd) & 1u) != obr) {
                        drop = true;
                    } else {
                        s.set(SpecState::NODE, 4, (1u << (node_lvl(nd) - 1u)) - 1u + (node_code(nd) >> 1));
                    }
                    if (drop) {  // a dropped sample: its ray goes with it
                        if (COUNT) n_abort++;
                        s.set(SpecState::SRUN, 1, 0);
                        s.set(SpecState::SEND, 1, 0);
                        s.set(SpecState::PEND, 1, 0);
                        fresh = false;
                        busy = false;
                    }
                }
            }
            // a pixel that is done frees its group
            {
                if (s.role() == ROLE_OWNER && cseq == spp) {
                    if (pa.probe)
                        pa.probe[pix] = make_uint4(C, COUNT ? pc_closest : 0u, COUNT ? pc_shadow : 0u, probe_flags<COUNT>(pa));
                    s.set(SpecState::ROLE, 2, ROLE_FREE);
                    s.set(SpecState::NH, 5, 0);
                    grp = 0;
                    occ = 0;
                }
                SpecState os;
                os.w = (uint32_t)__shfl((int)s.w, ol);
                const uint32_t o_pix = (uint32_t)__shfl((int)pix, ol);
                if (s.role() == ROLE_HELPER && (os.role() != ROLE_OWNER || o_pix != pix))
                    s.set(SpecState::ROLE, 2, ROLE_FREE);  // its pixel is done (its lane may own another)
                if (s.role() == ROLE_FREE && (s.srun() || s.send())) {  // none is left past the last sample
                    if (COUNT) n_abort++;
                    s.set(SpecState::SRUN, 1, 0);
                    s.set(SpecState::SEND, 1, 0);
                    s.set(SpecState::PEND, 1, 0);
                    fresh = false;
                    busy = false;
                }
            }
            // 3. free lanes fetch the next pixel while the queue lasts
            {
                bool need = s.role() == ROLE_FREE && !done;
                const bool asked = need;
                fetch_pixels(f, n, pa.work, pa.order ? pa.order_mode : FETCH_LINEAR, pa.order, pa.prio, need, done, pix);
                if (asked && !need) {
                    const uint32_t px = pa.pixel[pix];
                    C = (uint32_t)((int)(px & 0xFFFFu) + (int)(px >> 16) * pa.cam.width);
                    cseq = 0;
                    occ = 0;
                    grp = 1ull << lane;
                    s.set(SpecState::ROLE, 2, ROLE_OWNER);
                    s.set(SpecState::NH, 5, 0);
                    if (COUNT) pc_closest = pc_shadow = 0;
                }
            }
            // 4. lanes with nothing left to fetch join the groups of owners with samples to speculate
            // on, one per owner per phase; the owners with at least half the wave's most samples left
            // first
            {
                const uint32_t left = spp - cseq;  // samples not committed
                const bool avail = s.role() == ROLE_FREE && done;
                const bool want = s.role() == ROLE_OWNER && s.nh() < lvl_cap && left > 1u;
                const unsigned long long fm = __ballot(avail), owm = __ballot(want);
                int nol = -1;  // a free lane's new owner
                if (fm && owm) {
                    uint32_t ml = want ? left : 0u;
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) ml = max(ml, (uint32_t)__shfl_xor((int)ml, o));
                    const bool t1 = want && 2u * left >= ml;
                    const unsigned long long om1 = __ballot(t1), om2 = owm & ~om1;
                    const uint32_t nf = (uint32_t)__popcll(fm);
                    const uint32_t k1 = min(nf, (uint32_t)__popcll(om1));
                    const uint32_t k2 = min(nf - k1, (uint32_t)__popcll(om2));
                    if (avail) {
                        const uint32_t fr = lane_prefix(fm);
                        if (fr < k1 + k2) nol = fr < k1 ? nth_set_bit(om1, fr) : nth_set_bit(om2, fr - k1);
                    }
                    if (want) {
                        const uint32_t orank = t1 ? lane_prefix(om1) : lane_prefix(om2);
                        if (orank < (t1 ? k1 : k2)) {
                            grp |= 1ull << nth_set_bit(fm, t1 ? orank : k1 + orank);
                            s.set(SpecState::NH, 5, s.nh() + 1u);
                        }
                    }
                }
                const uint32_t np = (uint32_t)__shfl((int)pix, nol >= 0 ? nol : (int)lane);
                if (nol >= 0) {
                    s.set(SpecState::ROLE, 2, ROLE_HELPER);
                    s.set(SpecState::OL, 6, (uint32_t)nol);
                    pix = np;
                }
            }
            // 5. starts: the idle lanes of a group take the free nodes in order of expected use, the
            // head first (from C); a node l levels down starts after its l assumed sample lengths
            {
                const int ol2 = s.role() == ROLE_HELPER ? (int)s.ol() : (int)lane;
                const bool idle = s.role() != ROLE_FREE && !s.srun() && !s.send();
                const unsigned long long im = __ballot(idle);
                unsigned long long pick = 0;  // the nodes handed out, one per nibble, in idle-lane order
                uint32_t npick = 0;
                if (s.role() == ROLE_OWNER) {
                    const uint32_t nfree = (uint32_t)__popcll(grp & im);
                    const uint32_t lv_max = min(lvl_cap, spp - cseq - 1u);  // nodes past the last sample are useless
                    for (uint32_t k = 0; k < kSpecNodes && npick < nfree; k++) {
                        const uint32_t nd = (uint32_t)(kSpecNodeOrder >> (4u * k)) & 15u;
                        if (((occ >> nd) & 1u) || node_lvl(nd) > lv_max || node_code(nd)) continue;
                        pick |= (unsigned long long)nd << (4u * npick);
                        npick++;
                        occ |= 1u << nd;
                    }
                }
                const uint32_t o_np = (uint32_t)__shfl((int)npick, ol2);
                const uint32_t plo = (uint32_t)__shfl((int)(uint32_t)pick, ol2);
                const uint32_t phi = (uint32_t)__shfl((int)(uint32_t)(pick >> 32), ol2);
                const uint32_t o_C = (uint32_t)__shfl((int)C, ol2);
                const uint32_t glo = (uint32_t)__shfl((int)(uint32_t)grp, ol2);
                const uint32_t ghi = (uint32_t)__shfl((int)(uint32_t)(grp >> 32), ol2);
                if (idle && o_np) {
                    const unsigned long long og = ((unsigned long long)ghi << 32) | glo;
                    const uint32_t k = (uint32_t)__popcll(og & im & below);  // this lane's rank among the idle
                    if (k < o_np) {
                        const unsigned long long pk = ((unsigned long long)phi << 32) | plo;
                        const uint32_t nd = (uint32_t)(pk >> (4u * k)) & 15u;
                        const uint32_t lv = node_lvl(nd), cd = node_code(nd), ones = (uint32_t)__popc(cd);
                        const uint32_t ahead = (lv - ones) * g_full + ones * g_one;
                        seed = ahead ? lcg_advance(o_C, ahead) : o_C;
                        if (COUNT && lv) n_spec++;
                        s.set(SpecState::NODE, 4, nd);
                        start = true;
                    }
                }
            }
            }  // general path
            {
                if (start) {  // a new sample: camera ray (pathtracer.h:61-64), L = 0, beta = 1
                    const uint32_t px = pa.pixel[pix];  // reloaded: a register shuffled to the helpers measured slower (profiles/r21_px_reg_spec_ab.log)
                    Lr = V3{0.0f, 0.0f, 0.0f};
                    beta = V3{1.0f, 1.0f, 1.0f};
                    depth = 0;
                    camera_ray(pa.cam, (int)(px & 0xFFFFu), (int)(px >> 16), seed, ra, rb);
                    s.set(SpecState::SRUN, 1, 1);
                    s.set(SpecState::PEND, 1, 0);
                    next_any = false;
                    fresh = true;
                    if (COUNT) sc_closest = sc_shadow = 0;
                }
            }
            asm volatile("" ::: "memory");
            path_unpark(s_park, tid, r, ff, s.any());  // the busy lanes' traversal continues unchanged
            if (fresh) {
                s.set(SpecState::ANY, 1, next_any ? 1u : 0u);
                if (COUNT) {
                    sc_closest += next_any ? 0u : 1u;
                    sc_shadow += next_any ? 1u : 0u;
                }
                busy = path_begin<COUNT>(a, next_any, ra, rb, r, s_stack, stack_ovf, tid, gtid, c);
                fin = !busy;
            }
        }
        if (COUNT) {
            const unsigned long long t = wall_clock64();
            p_tp += t - p_t;
            p_t = t;
        }
        if (!__any(busy)) {
            // nothing in flight: the next processing phase commits or starts something; a wave that
            // idles for many rounds has lost its state (a bug): stop and raise the fault word
            if (++idle_rounds > 1024) {
                if (pa.fault && __lane_id() == 0) __hip_atomic_fetch_or(pa.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            continue;
        }
        idle_rounds = 0;
        // ---- B. traversal phase, C. leaf phase (k_trace's, shared with the other persistent kernels)
        const int kd = s.any() ? 1 : 0;
        path_traverse<COUNT, kWhileExitSpec>(busy, kd, r, a.wide_nodes, s_stack, stack_ovf, a.ovf_threads, tid, gtid, c);
        if (COUNT) {
            const unsigned long long t = wall_clock64();
            p_tt += t - p_t;
            p_t = t;
        }
        const bool hit_any = path_leaf<COUNT>(busy, kd, r, a.wide_leaves, c);
        if (busy && (hit_any || r.cur == AKR_CHILD_EMPTY)) {
            busy = false;
            fin = true;
            if (COUNT) c.deep[kd] += c.deep_now ? 1 : 0;
        }
        if (COUNT) p_tl += wall_clock64() - p_t;
    }
    if (COUNT) {
        path_count_flush(pa, c, p_outer, p_procs, p_tp, p_tt, p_tl, p_t0, p_lanes, p_tsh);
        const unsigned long long ns = wave_sum(n_spec), na = wave_sum(n_abort);
        if (__lane_id() == 0 && pa.prof) {
            atomicAdd(&pa.prof->spec_started, ns);
            atomicAdd(&pa.prof->spec_aborted, na);
        }
    }
    if (pa.fault_test && pa.fault && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_fetch_or(pa.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Film::merge_tile (core/film.h:85-95) on the device: a context's packed film (one float4 per
// slot: radiance sums, weight) added into full-frame buffers at its pixels.  `order` (optional)
// lists the slots of one launch; a launch never holds the same pixel twice, so the adds of a pixel
// happen in launch order — the host loop's order.
__global__ __launch_bounds__(kBlock) void k_merge_film(const float4 *film, const uint32_t *pixel, const uint32_t *order,
                                                      uint32_t n, int32_t width, float *rad, float *w) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = order ? order[i] : i;
    const uint32_t px = pixel[j];
    const size_t p = (size_t)(px & 0xFFFFu) + (size_t)(px >> 16) * (size_t)width;
    const float4 f = film[j];
    rad[3 * p + 0] += f.x;
    rad[3 * p + 1] += f.y;
    rad[3 * p + 2] += f.z;
    w[p] += f.w;
}

// The render's pixel list from its tile list, on the device: `tiles` holds each non-empty clipped
// tile as (x0, y0, width, first slot), in list order; slot i lies in the last tile whose first slot
// is <= i, row-major inside it (the order the host list had, capi.hip setup_pixels).  One thread
// per slot, a binary search over the (few thousand) tiles, which stay in L2.
__global__ __launch_bounds__(kBlock) void k_expand_pixels(const uint4 *tiles, uint32_t n_tiles, uint32_t n,
                                                          uint32_t *pixel) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint32_t lo = 0, hi = n_tiles;  // largest k with tiles[k].w <= i (tiles[0].w == 0)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (tiles[mid].w <= i) lo = mid; else hi = mid;
    }
    const uint4 t = tiles[lo];
    const uint32_t local = i - t.w;
    pixel[i] = (t.x + local % t.z) | ((t.y + local / t.z) << 16);
}

__global__ __launch_bounds__(kBlock) void k_unpack_film(const float4 *film, uint32_t n, float *rad, float *w) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float4 f = film[i];
    rad[3 * (size_t)i + 0] = f.x;
    rad[3 * (size_t)i + 1] = f.y;
    rad[3 * (size_t)i + 2] = f.z;
    w[i] = f.w;
}

// In-band read-back check: counts the film slots whose sample weight is not `expect` (one atomic
// per wave); a render that lost samples, or a film read before its last splat, cannot pass.
__global__ __launch_bounds__(kBlock) void k_check_weights(const float4 *film, uint32_t n, float expect, uint32_t *bad) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const unsigned long long m = __ballot(i < n && film[i].w != expect);
    if (__lane_id() == 0 && m) atomicAdd(bad, (uint32_t)__popcll(m));
}

// Cost-ordered pixel fetch of the persistent path kernels.  Pilot: the camera ray
// of each slot's first sample, made from a copy of its seed (nothing is committed), traced by the
// counting kernel, whose per-ray steps (traversal iterations + triangle tests) rank the pixels.
// With `sub` > 0 only every 2^sub-th slot gets a pilot ray (ray k: slot k << sub; neighbours in a
// tile row share a cost estimate), which shortens the pilot launch.
__global__ __launch_bounds__(kBlock) void k_pilot_rays(CameraDev cam, const uint32_t *pixel, uint32_t n, uint32_t sub,
                                                      float4 *rays) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t px = pixel[i << sub];
    const int x = (int)(px & 0xFFFFu), y = (int)(px >> 16);
    uint32_t seed = (uint32_t)(x + y * cam.width);
    float4 r0, r1;
    camera_ray(cam, x, y, seed, r0, r1);
    rays[2 * (size_t)i] = r0;
    rays[2 * (size_t)i + 1] = r1;
}

// Sort key of slot i: its XCD shard above its cost class (steps >> shift, capped at cmax <=
// kOrderClassMask, descending), so a stable sort orders each shard by decreasing cost and keeps tile
// order within a class (few classes keep more of the tile order: a smaller cache footprint).
// With `sum` set, the pilot rays' steps are summed (one atomic per wave; a ray the exact walk traced
// adds nothing): the form rule's mean steps per camera ray (capi.hip).
__global__ __launch_bounds__(kBlock) void k_order_keys(const uint32_t *steps, uint32_t n, uint32_t shift, uint32_t cmax,
                                                       uint32_t sub, uint32_t *key, uint32_t *idx,
                                                       unsigned long long *sum) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    uint32_t add = 0;
    if (i < n) {
        uint32_t sh = 0;
        for (uint32_t k = 1; k < kWorkShards; k++) sh += i >= shard_begin(n, k) ? 1u : 0u;
        const uint32_t s = steps[i >> sub];  // 0xFFFFFFFF: traced by the exact BVH2 walk (rare): costliest class
        const uint32_t cls = s == 0xFFFFFFFFu ? cmax : min(s >> shift, cmax);
        key[i] = (sh << kOrderClassBits) | (kOrderClassMask - cls);
        idx[i] = i;
        // one pilot ray per 2^sub slots: counted at its first slot
        add = (s != 0xFFFFFFFFu && (i & ((1u << sub) - 1u)) == 0u) ? s : 0u;
    }
    if (sum) {
        const unsigned long long w = wave_sum(add);
        if (__lane_id() == 0 && w) atomicAdd(sum, w);
    }
}

// Path pilot (option path_order_pilot_spp): a slot's cost is the rays (closest-hit + shadow) its first
// samples took in a counting render, from the pixel probe of that render
__global__ __launch_bounds__(kBlock) void k_probe_cost(const uint4 *probe, uint32_t n, uint32_t *cost) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) cost[i] = probe[i].y + probe[i].z;
}

// one word from device memory into mapped host memory (the host polls it after an event)
// Wavefront form: the final sampler state of every slot into its pixel probe (the ray counts were
// added by k_raygen / k_shade)
__global__ __launch_bounds__(kBlock) void k_probe_seed(const uint32_t *seed, uint32_t n, uint4 *probe) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint4 q = probe[i];
    q.x = seed[i];
    q.w = AKR_PROBE_SEED | AKR_PROBE_RAYS;
    probe[i] = q;
}

// The form rule's tail test on the device: gate = 1 when the pilot's camera rays
// took at least `thresh` traversal steps in all
__global__ void k_pick_form(const unsigned long long *sum, unsigned long long thresh, uint32_t *gate) {
    if (threadIdx.x == 0) *gate = *sum >= thresh ? 1u : 0u;
}

__global__ void k_store_word(const uint32_t *src, uint32_t *dst) {
    if (threadIdx.x == 0) {
        __atomic_store_n(dst, *src, __ATOMIC_RELAXED);
        __threadfence_system();
    }
}

// ------------------------------------------------------------------------------------ launch
static inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock); }

template <int MODE, bool WIDE>
static void launch_trace_mode(bool count, bool tight, const TraceArgs &a, uint32_t grid, hipStream_t st) {
    if (count) {
        if (tight) hipLaunchKernelGGL((k_trace<MODE, true, true, WIDE>), dim3(grid), dim3(kTraceBlock), 0, st, a);
        else hipLaunchKernelGGL((k_trace<MODE, true, false, WIDE>), dim3(grid), dim3(kTraceBlock), 0, st, a);
    } else {
        if (tight) hipLaunchKernelGGL((k_trace<MODE, false, true, WIDE>), dim3(grid), dim3(kTraceBlock), 0, st, a);
        else hipLaunchKernelGGL((k_trace<MODE, false, false, WIDE>), dim3(grid), dim3(kTraceBlock), 0, st, a);
    }
}

void launch_trace(int mode, bool count, bool tight, bool wide, const TraceArgs &a, uint32_t grid, hipStream_t st) {
    if (grid == 0) return;
    if (wide) {
        if (mode == TRACE_CLOSEST) launch_trace_mode<TRACE_CLOSEST, true>(count, tight, a, grid, st);
        else if (mode == TRACE_ANY) launch_trace_mode<TRACE_ANY, true>(count, tight, a, grid, st);
        else if (mode == TRACE_PILOT) {  // steps only: the tight, uncounted wide kernel
            if (count || !tight) throw std::runtime_error("launch_trace: the pilot mode is tight and uncounted");
            hipLaunchKernelGGL((k_trace<TRACE_PILOT, false, true, true>), dim3(grid), dim3(kTraceBlock), 0, st, a);
        } else launch_trace_mode<TRACE_SHADOW, true>(count, tight, a, grid, st);
    } else {
        if (mode == TRACE_PILOT) throw std::runtime_error("launch_trace: the pilot mode needs the wide view");
        if (mode == TRACE_CLOSEST) launch_trace_mode<TRACE_CLOSEST, false>(count, tight, a, grid, st);
        else if (mode == TRACE_ANY) launch_trace_mode<TRACE_ANY, false>(count, tight, a, grid, st);
        else launch_trace_mode<TRACE_SHADOW, false>(count, tight, a, grid, st);
    }
}

int trace_blocks_per_cu(int mode) {
    int nb = 0;
    hipError_t e;
    if (mode == TRACE_CLOSEST)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_trace<TRACE_CLOSEST, false, true, true>, kTraceBlock, 0);
    else if (mode == TRACE_ANY)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_trace<TRACE_ANY, false, true, true>, kTraceBlock, 0);
    else
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_trace<TRACE_SHADOW, false, true, true>, kTraceBlock, 0);
    if (e != hipSuccess || nb <= 0) nb = 1;
    return nb;
}

void launch_raygen(const RaygenArgs &a, hipStream_t st) {
    if (a.n == 0) return;
    hipLaunchKernelGGL(k_raygen, dim3(blocks_for(a.n)), dim3(kBlock), 0, st, a);
}
void launch_shade(const ShadeArgs &a, uint32_t max_items, hipStream_t st) {
    if (max_items == 0) return;
    const dim3 grid((uint32_t)((max_items + kShadeBlock - 1) / kShadeBlock));
    hipLaunchKernelGGL(k_shade, grid, dim3(kShadeBlock), 0, st, a);
}
void launch_pick_form(const unsigned long long *sum, unsigned long long thresh, uint32_t *gate, hipStream_t st) {
    hipLaunchKernelGGL(k_pick_form, dim3(1), dim3(64), 0, st, sum, thresh, gate);
}
void launch_store_word(const uint32_t *src, uint32_t *dst, hipStream_t st) {
    hipLaunchKernelGGL(k_store_word, dim3(1), dim3(64), 0, st, src, dst);
}
void launch_ao_shade(const AoShadeArgs &a, uint32_t max_items, hipStream_t st) {
    if (max_items == 0) return;
    hipLaunchKernelGGL(k_ao_shade, dim3(blocks_for(max_items)), dim3(kBlock), 0, st, a);
}
void launch_ao_resolve(const AoResolveArgs &a, uint32_t max_items, hipStream_t st) {
    if (max_items == 0) return;
    hipLaunchKernelGGL(k_ao_resolve, dim3(blocks_for(max_items)), dim3(kBlock), 0, st, a);
}
void launch_splat(const SplatArgs &a, uint32_t max_items, hipStream_t st) {
    if (max_items == 0) return;
    hipLaunchKernelGGL(k_splat, dim3(blocks_for(max_items)), dim3(kBlock), 0, st, a);
}
template <bool COUNT, bool TAB>
static void launch_path_t(int kind, const PathArgs &a, uint32_t grid, hipStream_t st) {
    if (kind == PATH_DEFER) hipLaunchKernelGGL((k_path_defer<COUNT, TAB>), dim3(grid), dim3(kTraceBlock), 0, st, a);
    else if (kind == PATH_SPEC) hipLaunchKernelGGL((k_path_spec<COUNT, TAB>), dim3(grid), dim3(kTraceBlock), 0, st, a);
    else hipLaunchKernelGGL((k_path<COUNT, TAB>), dim3(grid), dim3(kTraceBlock), 0, st, a);
}
void launch_path(bool count, int kind, bool tab, const PathArgs &a, uint32_t grid, hipStream_t st) {
    if (grid == 0) return;
    if (tab && !path_tab_fits(a.sc.n_mats, a.sc.n_lights)) tab = false;  // the LDS copy must hold every record
    if (count) {
        if (tab) launch_path_t<true, true>(kind, a, grid, st);
        else launch_path_t<true, false>(kind, a, grid, st);
    } else {
        if (tab) launch_path_t<false, true>(kind, a, grid, st);
        else launch_path_t<false, false>(kind, a, grid, st);
    }
}
int path_blocks_per_cu(int kind, bool tab) {
    int nb = 0;
    hipError_t e;
    if (kind == PATH_SPEC)
        e = tab ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_path_spec<false, true>, kTraceBlock, 0)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_path_spec<false, false>, kTraceBlock, 0);
    else if (kind == PATH_DEFER)
        e = tab ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_path_defer<false, true>, kTraceBlock, 0)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_path_defer<false, false>, kTraceBlock, 0);
    else
        e = tab ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_path<false, true>, kTraceBlock, 0)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_path<false, false>, kTraceBlock, 0);
    if (e != hipSuccess || nb <= 0) nb = 1;
    return nb;
}
void launch_check_weights(const float4 *film, uint32_t n, float expect, uint32_t *bad, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_check_weights, dim3(blocks_for(n)), dim3(kBlock), 0, st, film, n, expect, bad);
}
void launch_merge_film(const float4 *film, const uint32_t *pixel, const uint32_t *order, uint32_t n, int32_t width,
                       float *rad, float *w, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_merge_film, dim3(blocks_for(n)), dim3(kBlock), 0, st, film, pixel, order, n, width, rad, w);
}
void launch_pilot_rays(const CameraDev &cam, const uint32_t *pixel, uint32_t n, uint32_t sub, float4 *rays,
                       hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_pilot_rays, dim3(blocks_for(n)), dim3(kBlock), 0, st, cam, pixel, n, sub, rays);
}
void launch_order_keys(const uint32_t *steps, uint32_t n, uint32_t shift, uint32_t cmax, uint32_t sub, uint32_t *key,
                       uint32_t *idx, hipStream_t st, unsigned long long *sum) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_order_keys, dim3(blocks_for(n)), dim3(kBlock), 0, st, steps, n, shift,
                       cmax < kOrderClassMask ? cmax : kOrderClassMask, sub, key, idx, sum);
}
void launch_probe_cost(const uint4 *probe, uint32_t n, uint32_t *cost, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_probe_cost, dim3(blocks_for(n)), dim3(kBlock), 0, st, probe, n, cost);
}
void launch_probe_seed(const uint32_t *seed, uint32_t n, uint4 *probe, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_probe_seed, dim3(blocks_for(n)), dim3(kBlock), 0, st, seed, n, probe);
}
void launch_expand_pixels(const uint4 *tiles, uint32_t n_tiles, uint32_t n, uint32_t *pixel, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_expand_pixels, dim3(blocks_for(n)), dim3(kBlock), 0, st, tiles, n_tiles, n, pixel);
}
void launch_unpack(const float4 *film, uint32_t n, float *rad, float *w, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_unpack_film, dim3(blocks_for(n)), dim3(kBlock), 0, st, film, n, rad, w);
}

}  // namespace akr
