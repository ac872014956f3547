// akr_math.h — f32 math of the AkariRender hot path for gfx950 device code.
//
// Every routine keeps the reference's operation order (sequential dot products, std::min/max
// ternary semantics, no FMA contraction: the library is built with -ffp-contract=off and IEEE
// division/sqrt), so that the device results are bit-identical to the CPU restatement.
// Citations are to the reference tree (src/akari/...).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "akr_trig.h"

namespace akr {

constexpr float kInf = __builtin_huge_valf();
constexpr float kPi = 3.1415926535897932384f;  // Constants::Pi, common/math.h:37
constexpr float kPi2 = kPi / 2.0f;
constexpr float kPi4 = kPi / 4.0f;
constexpr float kInvPi = 1.0f / kPi;
constexpr float kEps = 0.001f;                 // Constants::Eps, math.h:41
constexpr float kShadowEps = 0.0001f;          // Constants::ShadowEps, math.h:42

struct V3 { float x, y, z; };
struct V2 { float x, y; };

__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ V3 muls(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ V3 divs(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ float get(V3 a, uint32_t i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
// common/array.h:210-216
__device__ __forceinline__ float dot(V3 a, V3 b) { float s = a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s; }
// common/math.h:176-181
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return {(a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)};
}
__device__ __forceinline__ V3 normalize(V3 a) { return divs(a, sqrtf(dot(a, a))); }
__device__ __forceinline__ float length(V3 a) { return sqrtf(dot(a, a)); }
// std::min / std::max (common/array.h:41-46): NaN handling of the ternaries is kept.
__device__ __forceinline__ float rmin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float rmax(float a, float b) { return (a < b) ? b : a; }
// lerp3 (common/math.h:47-50)
__device__ __forceinline__ V3 lerp3(V3 a, V3 b, V3 c, float u, float v) {
    float w = 1.0f - u - v;
    return add(add(muls(a, w), muls(b, u)), muls(c, v));
}
__device__ __forceinline__ V2 lerp3(V2 a, V2 b, V2 c, float u, float v) {
    float w = 1.0f - u - v;
    return {(a.x * w + b.x * u) + c.x * v, (a.y * w + b.y * u) + c.y * v};
}
// Scalar sin/cos in f64 rounded to f32 (the correctly rounded f32 value), see DESIGN.md §4;
// akr_trig.h's bounded-range f64 kernels (identical to glibc's f64 results after rounding on every
// f32 in [-2 pi, 2 pi], tests/test_host.py).
__device__ __forceinline__ void fsincos(float x, float &s, float &c) { trig_sincosf(x, s, c); }

// LCGSampler::next1d (kernel/sampler.h:60-63)
__device__ __forceinline__ float lcg_next(uint32_t &s) {
    s = 1103515245u * s + 12345u;
    return (float)s / (float)0xFFFFFFFFu;
}
__device__ __forceinline__ V2 lcg_next2(uint32_t &s) { float a = lcg_next(s); float b = lcg_next(s); return {a, b}; }

// Color::is_black (common/color.h:48-50): bool-accumulator reduce seeded with c[0]
__device__ __forceinline__ bool is_black(V3 c) {
    bool acc = (c.x != 0.0f);
    acc = acc || (c.y > 0.0f);
    acc = acc || (c.z > 0.0f);
    return !acc;
}

// Frame (common/math.h:201-225), normal = y axis of the local frame
struct Frame { V3 n, t, b; };
__device__ __forceinline__ Frame make_frame(V3 v1) {
    Frame f;
    f.n = v1;
    if (fabsf(v1.x) > fabsf(v1.y))
        f.t = divs(v3(-v1.z, 0, v1.x), sqrtf(v1.x * v1.x + v1.z * v1.z));
    else
        f.t = divs(v3(0, v1.z, -v1.y), sqrtf(v1.y * v1.y + v1.z * v1.z));
    f.b = normalize(cross(v1, f.t));
    return f;
}
__device__ __forceinline__ V3 to_local(const Frame &f, V3 v) { return v3(dot(f.t, v), dot(f.n, v), dot(f.b, v)); }
__device__ __forceinline__ V3 to_world(const Frame &f, V3 v) {
    return add(add(muls(f.t, v.x), muls(f.n, v.y)), muls(f.b, v.z));
}

// sampling.h:32-53
__device__ __forceinline__ V2 concentric_disk(V2 u) {
    V2 o{2.f * u.x - 1.0f, 2.f * u.y - 1.0f};
    if (o.x == 0 && o.y == 0) return {0, 0};
    float theta, r;
    if (fabsf(o.x) > fabsf(o.y)) {
        r = o.x;
        theta = kPi4 * (o.y / o.x);
    } else {
        r = o.y;
        theta = kPi2 - kPi4 * (o.x / o.y);
    }
    float s, c;
    fsincos(theta, s, c);
    return {r * c, r * s};
}
__device__ __forceinline__ V3 cosine_hemisphere(V2 u) {
    V2 d = concentric_disk(u);
    float r = d.x * d.x + d.y * d.y;
    float h = sqrtf(rmax(0.0f, 1.0f - r));
    return v3(d.x, h, d.y);
}

__device__ __forceinline__ bool same_hemisphere(V3 a, V3 b) { return a.y * b.y >= 0; }
__device__ __forceinline__ float cos2_theta(V3 w) { return w.y * w.y; }
__device__ __forceinline__ float tan2_theta(V3 w) { return (1 - cos2_theta(w)) / cos2_theta(w); }

// microfacet.h:74-89 (GGX D and G1; G1 is evaluated in f64 as written there)
__device__ __forceinline__ float ggx_d(float alpha, V3 m) {
    if (m.y <= 0.0f) return 0.0f;
    float a2 = alpha * alpha;
    float c2 = cos2_theta(m);
    float t2 = tan2_theta(m);
    float at = a2 + t2;
    return a2 / (kPi * c2 * c2 * at * at);
}
__device__ __forceinline__ float ggx_g1(float alpha, V3 v, V3 m) {
    if (dot(v, m) * v.y <= 0) return 0.0f;
    return (float)(2.0 / (1.0 + sqrt(1.0 + (double)(alpha * alpha * tan2_theta(m)))));
}

// BSDF closure kinds (material.h:139-155)
enum : int { CL_NONE = 0, CL_DIFFUSE = 1, CL_GLOSSY = 2 };
struct Closure { int kind; V3 R; float alpha; };

// DiffuseBSDF::evaluate (material.h:72-77) / MicrofacetReflection::evaluate (:99-121)
__device__ __forceinline__ V3 closure_eval(const Closure &c, V3 wo, V3 wi) {
    if (c.kind == CL_DIFFUSE) {
        if (same_hemisphere(wo, wi)) return muls(c.R, kInvPi);
        return v3(0, 0, 0);
    }
    if (c.kind == CL_GLOSSY) {
        if (same_hemisphere(wo, wi)) {
            float co = fabsf(wo.y), ci = fabsf(wi.y);
            V3 wh = add(wo, wi);
            if (ci == 0 || co == 0) return v3(0, 0, 0);
            if (wh.x == 0 && wh.y == 0 && wh.z == 0) return v3(0, 0, 0);
            wh = normalize(wh);
            if (wh.y < 0) wh = neg(wh);
            float F = 1.0f;
            float g = ggx_g1(c.alpha, wo, wh) * ggx_g1(c.alpha, wi, wh);
            return muls(c.R, ggx_d(c.alpha, wh) * g * F / (4.0f * ci * co));
        }
        return v3(0, 0, 0);
    }
    return v3(0, 0, 0);
}

// DiffuseBSDF::sample (material.h:79-85) / MicrofacetReflection::sample (:123-137) with
// MicrofacetModel::sample_wh (microfacet.h:125-149) and reflect (bsdf-funcs.h:52-54)
__device__ __forceinline__ V3 closure_sample(const Closure &c, V2 u, V3 wo, V3 &wi, float &pdf) {
    if (c.kind == CL_DIFFUSE) {
        wi = cosine_hemisphere(u);
        if (!same_hemisphere(wo, wi)) wi.y = -wi.y;
        pdf = fabsf(wi.y) * kInvPi;
        return muls(c.R, kInvPi);
    }
    float phi = 2 * kPi * u.y;
    float t2 = c.alpha * c.alpha * u.x / (1 - u.x);
    float cos_t = 1.0f / sqrtf(1 + t2);
    float sin_t = sqrtf(rmax(0.0f, 1 - cos_t * cos_t));
    float sp, cp;
    fsincos(phi, sp, cp);
    V3 wh = v3(cp * sin_t, cos_t, sp * sin_t);
    if (!same_hemisphere(wo, wh)) wh = neg(wh);
    wi = add(muls(wo, -1.0f), muls(wh, 2.0f * dot(wo, wh)));
    if (!same_hemisphere(wo, wi)) {
        pdf = 0;
        return v3(0, 0, 0);
    }
    if (wh.y < 0) wh = neg(wh);
    pdf = ggx_d(c.alpha, wh) * fabsf(wh.y) / (4.0f * fabsf(dot(wo, wh)));
    return closure_eval(c, wo, wi);
}

}  // namespace akr
