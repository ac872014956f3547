// akr_oracle.cpp — CPU restatement of the AkariRender hot path.
//
// TEST INFRASTRUCTURE ONLY (see akr_oracle.h): the checker for the HIP backend and the
// cpu_baseline leg of bench.py.  Every function cites the reference file:line it restates
// (paths relative to the reference root, src/akari/...).  Build: oracle/Makefile
// (g++ -O3 -mavx2 -ffp-contract=off: no FMA contraction, IEEE div/sqrt, like the reference's
// x86 build flags CMakeLists.txt:28).
//
// Conventions fixed where the reference is unspecified:
//  * function arguments that each draw from the sampler are evaluated left to right
//    (pathtracer.h:62 camera u1 then u2; sampler.h:64 next2d = (first, second));
//  * the CPU path's RNG consumption (no extra next1d for material selection; Mix selection
//    uses the first draw of the sampler COPY held by MaterialEvalContext, material.h:198-202);
//  * scalar sin/cos/atan are evaluated in double and rounded to float (the correctly rounded
//    float result in all but ~2^-29 of inputs, which is what the reference's float calls give).

#include "akr_oracle.h"

#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>
#include <algorithm>
#include <limits>

namespace {

constexpr float kInf = std::numeric_limits<float>::infinity();
constexpr float kPi = 3.1415926535897932384f;          // Constants::Pi, common/math.h:37
constexpr float kPi2 = kPi / 2.0f;                     // :38
constexpr float kPi4 = kPi / 4.0f;                     // :39
constexpr float kInvPi = 1.0f / kPi;                   // :40
constexpr float kEps = 0.001f;                         // :41
constexpr float kShadowEps = 0.0001f;                  // :42

struct V3 { float x, y, z; };
struct V2 { float x, y; };

inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 mul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 muls(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 divs(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
inline float get(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
// dot: sequential, common/array.h:210-216
inline float dot(V3 a, V3 b) { float s = a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s; }
// cross: common/math.h:176-181
inline V3 cross(V3 a, V3 b) {
    return {(a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)};
}
// normalize: a / sqrt(dot(a, a)), common/array.h:284-286
inline V3 normalize(V3 a) { return divs(a, std::sqrt(dot(a, a))); }
inline float length(V3 a) { return std::sqrt(dot(a, a)); }
// std::min / std::max as used through akari::min/max (common/array.h:41-46)
inline float rmin(float a, float b) { return (b < a) ? b : a; }
inline float rmax(float a, float b) { return (a < b) ? b : a; }
// lerp3: (1 - u - v) * v0 + u * v1 + v * v2, common/math.h:47-50
inline V3 lerp3(V3 a, V3 b, V3 c, float u, float v) {
    float w = 1.0f - u - v;
    return add(add(muls(a, w), muls(b, u)), muls(c, v));
}
inline V2 lerp3(V2 a, V2 b, V2 c, float u, float v) {
    float w = 1.0f - u - v;
    return {(a.x * w + b.x * u) + c.x * v, (a.y * w + b.y * u) + c.y * v};
}
inline float fsin(float x) { return (float)std::sin((double)x); }
inline float fcos(float x) { return (float)std::cos((double)x); }

// ---------------------------------------------------------------- sampler (kernel/sampler.h)
struct Lcg {
    uint32_t seed;
    // LCGSampler::next1d, sampler.h:60-63
    float next1d() {
        seed = 1103515245u * seed + 12345u;
        return (float)seed / (float)0xFFFFFFFFu;
    }
    V2 next2d() { float a = next1d(); float b = next1d(); return {a, b}; }
};

struct Pcg {
    uint64_t state;
    static constexpr uint64_t mult = 6364136223846793005ull;
    static constexpr uint64_t inc = 1442695040888963407ull;
    static uint32_t rotr32(uint32_t x, unsigned r) { return x >> r | x << (-r & 31); }
    uint32_t pcg32() {  // sampler.h:33-40
        uint64_t x = state;
        unsigned count = (unsigned)(x >> 59);
        state = x * mult + inc;
        x ^= x >> 18;
        return rotr32((uint32_t)(x >> 27), count);
    }
    void init(uint64_t seed) { state = seed + inc; (void)pcg32(); }  // :41-44
    float next1d() { return (float)pcg32() / (float)0xffffffffu; }   // :49
};

// ---------------------------------------------------------------- matrices (common/math.h)
struct M4 { float m[4][4]; };
M4 ident() { M4 r{}; for (int i = 0; i < 4; i++) r.m[i][i] = 1.0f; return r; }
M4 from16(const float *a) { M4 r; for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) r.m[i][j] = a[i * 4 + j]; return r; }
// Matrix::operator* (math.h:93-101): m(i,j) = dot(row(i), rhs.col(j)), sequential dot
M4 mmul(const M4 &a, const M4 &b) {
    M4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float s = a.m[i][0] * b.m[0][j];
            s += a.m[i][1] * b.m[1][j];
            s += a.m[i][2] * b.m[2][j];
            s += a.m[i][3] * b.m[3][j];
            r.m[i][j] = s;
        }
    return r;
}
M4 scale(float x, float y, float z) { float m[16] = {x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0, 0, 0, 0, 1}; return from16(m); }
M4 translate(float x, float y, float z) { float m[16] = {1, 0, 0, x, 0, 1, 0, y, 0, 0, 1, z, 0, 0, 0, 1}; return from16(m); }
M4 rotate_x(float t) { float s = fsin(t), c = fcos(t); float m[16] = {1, 0, 0, 0, 0, c, -s, 0, 0, s, c, 0, 0, 0, 0, 1}; return from16(m); }
M4 rotate_y(float t) { float s = fsin(t), c = fcos(t); float m[16] = {c, 0, s, 0, 0, 1, 0, 0, -s, 0, c, 0, 0, 0, 0, 1}; return from16(m); }
M4 rotate_z(float t) { float s = fsin(t), c = fcos(t); float m[16] = {c, -s, 0, 0, s, c, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}; return from16(m); }
// Transform::apply_point (math.h:243-251)
V3 apply_point(const M4 &m, V3 p) {
    float v[4] = {p.x, p.y, p.z, 1.0f}, r[4];
    for (int i = 0; i < 4; i++) {
        float s = m.m[i][0] * v[0];
        s += m.m[i][1] * v[1];
        s += m.m[i][2] * v[2];
        s += m.m[i][3] * v[3];
        r[i] = s;
    }
    V3 q{r[0], r[1], r[2]};
    if (r[3] != 1.0f) q = divs(q, r[3]);
    return q;
}
// Transform::apply_vector = m3 * v (math.h:253)
V3 apply_vector(const M4 &m, V3 v) {
    float r[3];
    for (int i = 0; i < 3; i++) {
        float s = m.m[i][0] * v.x;
        s += m.m[i][1] * v.y;
        s += m.m[i][2] * v.z;
        r[i] = s;
    }
    return {r[0], r[1], r[2]};
}

struct Camera {
    M4 r2c, c2w;
    int w, h;
};
Camera make_camera(const akr_camera &c) {
    Camera cam;
    cam.w = c.resolution[0];
    cam.h = c.resolution[1];
    // radians(float3): x * Pi / 180.0f (math.h:352-354) applied to rotation (camera.cpp:45)
    float rx = c.rotation_deg[0] * kPi / 180.0f;
    float ry = c.rotation_deg[1] * kPi / 180.0f;
    float rz = c.rotation_deg[2] * kPi / 180.0f;
    // camera.cpp:32-36
    M4 c2w = rotate_z(rz);
    c2w = mmul(rotate_x(ry), c2w);
    c2w = mmul(rotate_y(rx), c2w);
    c2w = mmul(translate(c.position[0], c.position[1], c.position[2]), c2w);
    cam.c2w = c2w;
    // fov = radians(double): x * double(Pi_f) / 180 (camera.cpp:43), narrowed to Float (:37)
    float fov = (float)(c.fov_deg * (double)kPi / 180.0);
    // PerspectiveCamera::preprocess, camera.h:45-59
    M4 m = ident();
    m = mmul(scale(1.0f / cam.w, 1.0f / cam.h, 1), m);
    m = mmul(scale(2, 2, 1), m);
    m = mmul(translate(-1, -1, 0), m);
    m = mmul(scale(1, -1, 1), m);
    float s = (float)std::atan((double)(fov / 2));
    if (cam.w > cam.h)
        m = mmul(scale(s, s * float(cam.h) / cam.w, 1), m);
    else
        m = mmul(scale(s * float(cam.w) / cam.h, s, 1), m);
    cam.r2c = m;
    return cam;
}
// generate_ray(u1 = lens, u2 = film jitter, raster), camera.h:67-86 (lens_radius = 0)
akr_ray generate_ray(const Camera &cam, V2 u2, int x, int y) {
    V2 pf{(float)x + u2.x, (float)y + u2.y};
    V3 p = apply_point(cam.r2c, v3(pf.x, pf.y, 0.0f));
    V3 d = normalize(sub(v3(p.x, p.y, 0), v3(0, 0, 1)));
    V3 o = apply_point(cam.c2w, v3(0, 0, 0));
    d = apply_vector(cam.c2w, d);
    akr_ray r;
    r.o[0] = o.x; r.o[1] = o.y; r.o[2] = o.z;
    r.d[0] = d.x; r.d[1] = d.y; r.d[2] = d.z;
    r.tmin = kEps;  // Ray default tmin (math.h:190-193)
    r.tmax = kInf;
    return r;
}

// ---------------------------------------------------------------- geometry
struct Ray { V3 o, d; float tmin, tmax; };
inline Ray to_ray(const akr_ray &r) { return {v3(r.o[0], r.o[1], r.o[2]), v3(r.d[0], r.d[1], r.d[2]), r.tmin, r.tmax}; }

// intersectAABB, bvh-accelerator.h:89-103
// tight = additionally reject boxes wholly behind the origin (t > m1), the device default
inline float intersect_aabb(V3 lo, V3 hi, const Ray &ray, V3 invd, bool tight) {
    V3 t0 = mul(sub(lo, ray.o), invd);
    V3 t1 = mul(sub(hi, ray.o), invd);
    V3 tmn{rmin(t0.x, t1.x), rmin(t0.y, t1.y), rmin(t0.z, t1.z)};
    V3 tmx{rmax(t0.x, t1.x), rmax(t0.y, t1.y), rmax(t0.z, t1.z)};
    float m0 = rmax(rmax(tmn.x, tmn.y), tmn.z);  // hmax via reduce, array.h:238-240
    float m1 = rmin(rmin(tmx.x, tmx.y), tmx.z);
    if (m0 <= m1) {
        float t = rmax(ray.tmin, m0);
        if (t >= ray.tmax) return -1;
        if (tight && !(t <= m1)) return -1;
        return t;
    }
    return -1;
}

struct Best { float t, u, v; uint32_t gid; };

// MeshInstance::intersect (Moller-Trumbore), instance.h:42-80; e1/e2 pre-subtracted in f32
inline bool mt(const Ray &ray, V3 v0, V3 e1, V3 e2, uint32_t gid, Best &best) {
    V3 h = cross(ray.d, e2);
    float a = dot(e1, h);
    if (a > -1e-6f && a < 1e-6f) return false;
    float f = 1.0f / a;
    V3 s = sub(ray.o, v0);
    float u = f * dot(s, h);
    if (u < 0.0f || u > 1.0f) return false;
    V3 q = cross(s, e1);
    float v = f * dot(ray.d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    float t = f * dot(e2, q);
    if (t > ray.tmin && t < ray.tmax) {
        if (t < best.t) {
            best.u = u; best.v = v; best.gid = gid; best.t = t;
            return true;
        }
        return false;
    }
    return false;
}

struct ChildRef { uint32_t ref; V3 lo, hi; };
inline ChildRef child_of(const akr_bvh_node &n, int k) {
    ChildRef c;
    c.ref = n.child[k];
    const float *b = k == 0 ? n.bxy0 : n.bxy1;
    c.lo = v3(b[0], b[2], n.bz[2 * k + 0]);
    c.hi = v3(b[1], b[3], n.bz[2 * k + 1]);
    return c;
}

// TBVHAccelerator::intersect / occlude (bvh-accelerator.h:488-547) restated on the
// child-boxes-in-parent layout: a stack entry carries the child's box, which is tested when the
// entry is popped, exactly like the reference tests a popped node's own box.
bool traverse(const orc_scene &s, const Ray &ray, bool any_hit, bool tight, Best &best, uint64_t &nbox,
              uint64_t &ntri) {
    best.t = kInf; best.u = best.v = 0; best.gid = 0xFFFFFFFFu;
    if (s.n_nodes == 0) return false;
    V3 invd{1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z};
    ChildRef stack[AKR_BVH_MAX_DEPTH + 8];
    int sp = 0;
    ChildRef cur = child_of(s.nodes[0], 0);
    bool have = cur.ref != AKR_CHILD_EMPTY;
    bool hit = false;
    while (have) {
        nbox++;
        float t = intersect_aabb(cur.lo, cur.hi, ray, invd, tight);
        float lim = any_hit ? ray.tmax : best.t;
        if (t < 0 || t > lim) {
            if (sp > 0) cur = stack[--sp]; else have = false;
            continue;
        }
        if (cur.ref & AKR_CHILD_LEAF) {
            uint32_t first = akr_leaf_first(cur.ref), cnt = akr_leaf_count(cur.ref);
            for (uint32_t i = first; i < first + cnt; i++) {
                const akr_bvh_tri &tr = s.tris[i];
                ntri++;
                if (any_hit) {
                    Best tmp; tmp.t = kInf;
                    if (mt(ray, v3(tr.v0[0], tr.v0[1], tr.v0[2]), v3(tr.e1[0], tr.e1[1], tr.e1[2]),
                           v3(tr.e2[0], tr.e2[1], tr.e2[2]), tr.gid, tmp)) {
                        best = tmp;
                        return true;
                    }
                } else if (mt(ray, v3(tr.v0[0], tr.v0[1], tr.v0[2]), v3(tr.e1[0], tr.e1[1], tr.e1[2]),
                              v3(tr.e2[0], tr.e2[1], tr.e2[2]), tr.gid, best)) {
                    hit = true;
                }
            }
            if (sp > 0) cur = stack[--sp]; else have = false;
        } else {
            const akr_bvh_node &n = s.nodes[cur.ref];
            ChildRef l = child_of(n, 0), r = child_of(n, 1);
            if (get(ray.d, (int)n.axis) > 0) {
                stack[sp++] = r;
                cur = l;
            } else {
                stack[sp++] = l;
                cur = r;
            }
        }
    }
    return hit;
}

inline V3 vert(const orc_scene &s, int32_t vi) {
    return v3(s.vertices[3 * (int64_t)vi + 0], s.vertices[3 * (int64_t)vi + 1], s.vertices[3 * (int64_t)vi + 2]);
}

bool brute(const orc_scene &s, const Ray &ray, bool any_hit, Best &best) {
    best.t = kInf; best.u = best.v = 0; best.gid = 0xFFFFFFFFu;
    bool hit = false;
    for (uint64_t g = 0; g < s.n_tris; g++) {
        V3 v0 = vert(s, s.indices[3 * g + 0]);
        V3 v1 = vert(s, s.indices[3 * g + 1]);
        V3 v2 = vert(s, s.indices[3 * g + 2]);
        Best tmp = best;
        if (any_hit) tmp.t = kInf;
        if (mt(ray, v0, sub(v1, v0), sub(v2, v0), (uint32_t)g, any_hit ? tmp : best)) {
            hit = true;
            if (any_hit) { best = tmp; return true; }
        }
    }
    return hit;
}

// ---------------------------------------------------------------- scene data
struct Tri {  // Triangle<C> (kernel/shape.h:26-42) via get_triangle (instance.h:83-97)
    V3 v[3], n[3];
    V2 tc[3];
    int32_t mat;
};
Tri get_triangle(const orc_scene &s, uint32_t g) {
    Tri t;
    for (int i = 0; i < 3; i++) {
        t.v[i] = vert(s, s.indices[3 * (int64_t)g + i]);
        int64_t vi = 3 * (int64_t)g + i;
        t.n[i] = v3(s.normals[3 * vi + 0], s.normals[3 * vi + 1], s.normals[3 * vi + 2]);
        t.tc[i] = V2{s.texcoords[2 * vi + 0], s.texcoords[2 * vi + 1]};
    }
    t.mat = s.matid[g];
    return t;
}
inline V3 tri_ng(const Tri &t) { return normalize(cross(sub(t.v[1], t.v[0]), sub(t.v[2], t.v[0]))); }
inline float tri_area(const Tri &t) { return length(cross(sub(t.v[1], t.v[0]), sub(t.v[2], t.v[0]))) * 0.5f; }

// Texture::evaluate (texture.h:30-66; image lookup core/image.hpp:83-99)
V3 tex_eval(const orc_scene &s, int32_t ti, V2 tc) {
    const akr_texture &t = s.textures[ti];
    if (t.type == AKR_TEX_CONSTANT) return v3(t.value[0], t.value[1], t.value[2]);
    float x = std::fmod(tc.x, 1.0f);
    float y = 1.0f - std::fmod(tc.y, 1.0f);
    int w = s.image_w[t.image], h = s.image_h[t.image];
    int ix = (int)(x * (float)w), iy = (int)(y * (float)h);
    ix = std::clamp(ix, 0, w - 1);
    iy = std::clamp(iy, 0, h - 1);
    const float *px = s.images + s.image_offset[t.image] + 4 * ((int64_t)ix + (int64_t)iy * w);
    return v3(px[0], px[1], px[2]);
}

// bsdf-funcs.h helpers (local frame, y up)
inline bool same_hemisphere(V3 a, V3 b) { return a.y * b.y >= 0; }
inline float cos2_theta(V3 w) { return w.y * w.y; }
inline float tan2_theta(V3 w) { return (1 - cos2_theta(w)) / cos2_theta(w); }

// Frame (math.h:201-225)
struct Frame { V3 n, t, b; };
Frame make_frame(V3 v1) {
    Frame f;
    f.n = v1;
    if (std::abs(v1.x) > std::abs(v1.y))
        f.t = divs(v3(-v1.z, 0, v1.x), std::sqrt(v1.x * v1.x + v1.z * v1.z));
    else
        f.t = divs(v3(0, v1.z, -v1.y), std::sqrt(v1.y * v1.y + v1.z * v1.z));
    f.b = normalize(cross(v1, f.t));
    return f;
}
inline V3 to_local(const Frame &f, V3 v) { return v3(dot(f.t, v), dot(f.n, v), dot(f.b, v)); }
inline V3 to_world(const Frame &f, V3 v) { return add(add(muls(f.t, v.x), muls(f.n, v.y)), muls(f.b, v.z)); }

// sampling.h:32-53
V2 concentric_disk(V2 u) {
    V2 o{2.f * u.x - 1.0f, 2.f * u.y - 1.0f};
    if (o.x == 0 && o.y == 0) return {0, 0};
    float theta, r;
    if (std::abs(o.x) > std::abs(o.y)) {
        r = o.x;
        theta = kPi4 * (o.y / o.x);
    } else {
        r = o.y;
        theta = kPi2 - kPi4 * (o.x / o.y);
    }
    return {r * fcos(theta), r * fsin(theta)};
}
V3 cosine_hemisphere(V2 u) {
    V2 d = concentric_disk(u);
    float r = d.x * d.x + d.y * d.y;
    float h = std::sqrt(rmax(0.0f, 1.0f - r));
    return v3(d.x, h, d.y);
}

// microfacet.h:74-89 (GGX)
float ggx_d(float alpha, V3 m) {
    if (m.y <= 0.0f) return 0.0f;
    float a2 = alpha * alpha;
    float c2 = cos2_theta(m);
    float t2 = tan2_theta(m);
    float at = a2 + t2;
    return a2 / (kPi * c2 * c2 * at * at);
}
float ggx_g1(float alpha, V3 v, V3 m) {
    if (dot(v, m) * v.y <= 0) return 0.0f;
    return (float)(2.0 / (1.0 + std::sqrt(1.0 + (double)(alpha * alpha * tan2_theta(m)))));
}

struct Closure {
    int kind;  // 0 none, 1 diffuse, 2 microfacet
    V3 R;
    float alpha;
};
// DiffuseBSDF / MicrofacetReflection evaluate (material.h:72-77, 99-121)
V3 closure_eval(const Closure &c, V3 wo, V3 wi) {
    if (c.kind == 1) {
        if (same_hemisphere(wo, wi)) return muls(c.R, kInvPi);
        return v3(0, 0, 0);
    }
    if (c.kind == 2) {
        if (same_hemisphere(wo, wi)) {
            float co = std::abs(wo.y), ci = std::abs(wi.y);
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
// closure sample (material.h:79-85, 123-137; microfacet sample_wh :125-149)
V3 closure_sample(const Closure &c, V2 u, V3 wo, V3 &wi, float &pdf) {
    if (c.kind == 1) {
        wi = cosine_hemisphere(u);
        if (!same_hemisphere(wo, wi)) wi.y = -wi.y;
        pdf = std::abs(wi.y) * kInvPi;
        return muls(c.R, kInvPi);
    }
    // GGX sample_wh
    float phi = 2 * kPi * u.y;
    float t2 = c.alpha * c.alpha * u.x / (1 - u.x);
    float cos_t = 1.0f / std::sqrt(1 + t2);
    float sin_t = std::sqrt(rmax(0.0f, 1 - cos_t * cos_t));
    V3 wh = v3(fcos(phi) * sin_t, cos_t, fsin(phi) * sin_t);
    if (!same_hemisphere(wo, wh)) wh = neg(wh);
    // reflect: -1 * w + 2 * dot(w, n) * n (bsdf-funcs.h:52-54)
    wi = add(muls(wo, -1.0f), muls(wh, 2.0f * dot(wo, wh)));
    if (!same_hemisphere(wo, wi)) {
        pdf = 0;
        return v3(0, 0, 0);
    }
    if (wh.y < 0) wh = neg(wh);
    pdf = ggx_d(c.alpha, wh) * std::abs(wh.y) / (4.0f * std::abs(dot(wo, wh)));
    return closure_eval(c, wo, wi);
}

struct Distribution {  // Distribution1D (common/distribution.h:46-102)
    std::vector<float> func, cdf;
    float func_int = 0;
    void build(const float *f, size_t n) {
        func.assign(f, f + n);
        cdf.assign(n + 1, 0.0f);
        cdf[0] = 0;
        for (size_t i = 0; i < n; i++) cdf[i + 1] = cdf[i] + func[i] / n;
        func_int = cdf[n];
        if (func_int == 0) {
            for (uint32_t i = 1; i < n + 1; ++i) cdf[i] = float(i) / float(n);
        } else {
            for (uint32_t i = 1; i < n + 1; ++i) cdf[i] /= func_int;
        }
    }
    int sample_discrete(float u, float *pdf) const {
        int first = 0, last = (int)cdf.size();
        int lo = first, hi = last;
        while (lo < hi) {  // upper_bound, distribution.h:32-44
            int mid = (lo + hi) / 2;
            if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
        }
        int i = std::clamp<int>(hi - 1, 0, (last - first) - 2);
        if (pdf) *pdf = func[i] / (func_int * func.size());
        return i;
    }
};

struct Scene {
    const orc_scene *s;
    Camera cam;
    Distribution dist;
    std::vector<Tri> lights;
};

inline bool is_black(V3 c) {
    // Color::is_black reduces with a bool accumulator seeded by c[0] (color.h:48-50)
    bool acc = (c.x != 0.0f);
    acc = acc || (c.y > 0.0f);
    acc = acc || (c.z > 0.0f);
    return !acc;
}

struct PathStats { uint64_t cam = 0, ext = 0, shd = 0, box = 0, tri = 0; };

// Per-pixel fingerprint of the sample loop (akr_pixel_probe): closest-hit traces the device makes
// (every trace below max(1, max_depth): the one at depth == max_depth can add nothing and the
// device skips it) and shadow traces; the final sampler state is taken by the caller.
struct PixelTally { uint32_t closest = 0, shadow = 0; };

// GenericPathTracer::run_megakernel (pathtracer.h:133-164) with on_surface_scatter (:96-132)
// and compute_direct_lighting (:69-91); returns L.
V3 trace_path(const Scene &sc, Lcg &sampler, int x, int y, int max_depth, bool tight, PathStats &st,
               PixelTally &pt) {
    const orc_scene &s = *sc.s;
    V3 L = v3(0, 0, 0), beta = v3(1, 1, 1);
    int depth = 0;
    const int traced_below = max_depth == 0 ? 1 : max_depth;
    V2 u1 = sampler.next2d();  // lens sample (unused: lens_radius = 0)
    (void)u1;
    V2 u2 = sampler.next2d();
    akr_ray cr = generate_ray(sc.cam, u2, x, y);
    Ray ray = to_ray(cr);
    st.cam++;
    while (true) {
        Best hit;
        if (depth < traced_below) pt.closest++;
        if (!traverse(s, ray, false, tight, hit, st.box, st.tri)) break;
        V3 wo = neg(ray.d);
        Tri tri = get_triangle(s, hit.gid);
        float u = hit.u, v = hit.v;
        // SurfaceInteraction(uv, triangle), interaction.h:40-41
        V3 p = lerp3(tri.v[0], tri.v[1], tri.v[2], u, v);
        V3 ng = tri_ng(tri);
        V3 ns = lerp3(tri.n[0], tri.n[1], tri.n[2], u, v);
        V2 tc = lerp3(tri.tc[0], tri.tc[1], tri.tc[2], u, v);
        if (tri.mat < 0) break;  // reference dereferences a null material here (undefined)
        const akr_material *mat = &s.materials[tri.mat];
        // MaterialEvalContext copies the sampler: u1 = copy.next2d() (material.h:198-202)
        Lcg copy = sampler;
        V2 cu1 = copy.next2d();
        if (mat->type == AKR_MAT_EMISSIVE) {
            if (depth == 0) {
                bool face_front = dot(neg(wo), ng) < 0.0f;
                if (mat->double_sided || face_front) {
                    L = add(L, mul(beta, tex_eval(s, mat->color, tc)));
                }
            }
            break;
        }
        if (depth >= max_depth) break;
        // Material::get_bsdf -> select_material (material.h:251-268) -> get_bsdf0
        float sel_u = cu1.x, choice_pdf = 1.0f;
        while (mat->type == AKR_MAT_MIX) {
            float frac = tex_eval(s, mat->fraction, tc).x;
            if (sel_u < frac) {
                sel_u = sel_u / frac;
                mat = &s.materials[mat->second];
                choice_pdf *= 1.0f / frac;
            } else {
                sel_u = (sel_u - frac) / (1.0f - frac);
                mat = &s.materials[mat->first];
                choice_pdf *= 1.0f / (1.0f - frac);
            }
        }
        Closure cl{0, v3(0, 0, 0), 0};
        if (mat->type == AKR_MAT_DIFFUSE) {
            cl.kind = 1;
            cl.R = tex_eval(s, mat->color, tc);
        } else if (mat->type == AKR_MAT_GLOSSY) {
            cl.kind = 2;
            cl.R = tex_eval(s, mat->color, tc);
            float r = tex_eval(s, mat->roughness, tc).x;
            r *= r;
            cl.alpha = r;
        }
        Frame frame = make_frame(ns);
        // BSDF::sample (material.h:180-188)
        V2 bu = sampler.next2d();
        if (cl.kind == 0) break;  // null closure (Mix resolving to Emissive): undefined in reference
        V3 wo_l = to_local(frame, wo);
        V3 wi_l;
        float pdf = 0;
        V3 f = closure_sample(cl, bu, wo_l, wi_l, pdf);
        V3 wi = to_world(frame, wi_l);
        pdf *= choice_pdf;
        if (pdf == 0.0f) break;
        float cng = std::abs(dot(ng, wi));
        Ray next{p, wi, kEps / cng, kInf};
        V3 ev_beta = divs(muls(f, cng), pdf);
        // compute_direct_lighting(select_light(next2d)) (pathtracer.h:65-91, scene.h:79-90)
        V2 su = sampler.next2d();
        if (!sc.lights.empty()) {
            float sel_pdf;
            size_t idx = (size_t)sc.dist.sample_discrete(su.x, &sel_pdf);
            if (idx == sc.lights.size()) idx -= 1;
            const Tri &lt = sc.lights[idx];
            V2 lu = sampler.next2d();
            // AreaLight::sample (light.h:58-71)
            float su0 = std::sqrt(lu.x);
            float b0 = 1 - su0, b1 = lu.y * su0;
            V3 lp = lerp3(lt.v[0], lt.v[1], lt.v[2], b0, b1);
            V3 lng = tri_ng(lt);
            V3 lwi = sub(lp, p);
            float dist_sqr = dot(lwi, lwi);
            lwi = divs(lwi, std::sqrt(dist_sqr));
            V2 ltc = lerp3(lt.tc[0], lt.tc[1], lt.tc[2], b0, b1);
            V3 Le = tex_eval(s, s.materials[lt.mat].color, ltc);
            float lpdf = dist_sqr / rmax(0.0f, -dot(lwi, lng)) / tri_area(lt);
            Ray shadow{lp, neg(lwi), kEps / std::abs(dot(lwi, lng)), std::sqrt(dist_sqr) * (1.0f - kShadowEps)};
            if (!(lpdf <= 0.0f)) {
                float light_pdf = sel_pdf * lpdf;
                V3 fe = closure_eval(cl, to_local(frame, wo), to_local(frame, lwi));
                V3 fl = muls(mul(Le, fe), std::abs(dot(ns, lwi)));
                V3 color = divs(mul(beta, fl), light_pdf);
                if (!is_black(color)) {
                    st.shd++;
                    pt.shadow++;
                    Best sh;
                    if (!traverse(s, shadow, true, tight, sh, st.box, st.tri)) L = add(L, color);
                }
            }
        }
        beta = mul(beta, ev_beta);
        depth++;
        ray = next;
        st.ext++;
    }
    return L;
}

int hw_threads(int n) {
    if (n > 0) return n;
    int h = (int)std::thread::hardware_concurrency();
    return h > 0 ? h : 1;
}

template <class F>
void parallel_for(uint64_t n, int threads, uint64_t chunk, F &&f) {
    std::atomic<uint64_t> next{0};
    auto worker = [&](int tid) {
        while (true) {
            uint64_t b = next.fetch_add(chunk);
            if (b >= n) break;
            uint64_t e = std::min(n, b + chunk);
            for (uint64_t i = b; i < e; i++) f(i, tid);
        }
    };
    if (threads <= 1) { worker(0); return; }
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) ts.emplace_back(worker, t);
    for (auto &t : ts) t.join();
}

// split every rect into 16x16 work tiles (cpu/integrator.h:47, TileSize film.h:37)
struct Work { int x0, y0, x1, y1; };
std::vector<Work> split_work(const akr_rect *tiles, int n_tiles, int W, int H) {
    std::vector<Work> work;
    for (int k = 0; k < n_tiles; k++) {
        int x0 = std::max(0, tiles[k].x0), y0 = std::max(0, tiles[k].y0);
        int x1 = std::min(W, tiles[k].x1), y1 = std::min(H, tiles[k].y1);
        for (int ty = y0; ty < y1; ty += 16)
            for (int tx = x0; tx < x1; tx += 16) work.push_back({tx, ty, std::min(x1, tx + 16), std::min(y1, ty + 16)});
    }
    return work;
}

// Per-work-tile results (rgb sum, weight per pixel) merged into the frame after the parallel loop,
// serially in work order.  The reference merges each finished tile under a mutex
// (cpu/integrator.cpp:138-140, Film::merge_tile film.h:85-95); merging in a fixed order also keeps
// overlapping tiles deterministic.  (An unlocked += from the worker threads lost updates where tiles
// overlap: the flaky short weights of earlier parity runs.)
struct TileFilm {
    std::vector<size_t> off;   // first pixel of each work tile
    std::vector<float> px;     // 4 floats per pixel: rgb sum, weight
    explicit TileFilm(const std::vector<Work> &work) {
        off.resize(work.size() + 1, 0);
        for (size_t i = 0; i < work.size(); i++)
            off[i + 1] = off[i] + (size_t)(work[i].x1 - work[i].x0) * (size_t)(work[i].y1 - work[i].y0);
        px.assign(4 * off.back(), 0.0f);
    }
    float *at(size_t wi, const Work &w, int x, int y) {
        return &px[4 * (off[wi] + (size_t)(y - w.y0) * (size_t)(w.x1 - w.x0) + (size_t)(x - w.x0))];
    }
    void merge(const std::vector<Work> &work, int W, float *radiance, float *weight) {
        for (size_t wi = 0; wi < work.size(); wi++) {
            const Work &w = work[wi];
            for (int y = w.y0; y < w.y1; y++)
                for (int x = w.x0; x < w.x1; x++) {
                    const float *v = at(wi, w, x, y);
                    const int64_t pix = (int64_t)x + (int64_t)y * W;
                    radiance[3 * pix + 0] += v[0];
                    radiance[3 * pix + 1] += v[1];
                    radiance[3 * pix + 2] += v[2];
                    weight[pix] += v[3];
                }
        }
    }
};

// cpu::AmbientOcclusion::render's Li (kernel/integrators/cpu/integrator.cpp:43-60).  The camera
// sample is generate_ray(sampler.next2d(), sampler.next2d(), p) (:76-77): C++ leaves the order of
// the two argument evaluations unspecified; we take them left to right (lens draw first, film draw
// second), the order the path tracer's camera_ray spells out (pathtracer.h:61-64), so the AO and
// path-traced camera rays of a sample coincide.
float trace_ao(const Scene &sc, Lcg &sampler, int x, int y, float occlude, bool tight, PathStats &st) {
    const orc_scene &s = *sc.s;
    V2 u1 = sampler.next2d();  // lens sample (unused: lens_radius = 0)
    (void)u1;
    V2 u2 = sampler.next2d();
    Ray ray = to_ray(generate_ray(sc.cam, u2, x, y));
    st.cam++;
    Best hit;
    if (!traverse(s, ray, false, tight, hit, st.box, st.tri)) return 0.0f;
    Tri tri = get_triangle(s, hit.gid);
    Frame frame = make_frame(tri_ng(tri));  // Frame3f frame(trig.ng())
    V3 w = to_world(frame, cosine_hemisphere(sampler.next2d()));
    Ray ao{lerp3(tri.v[0], tri.v[1], tri.v[2], hit.u, hit.v), w, kEps, kInf};  // Ray3f(trig.p(uv), w)
    st.shd++;
    Best h2;
    if (traverse(s, ao, false, tight, h2, st.box, st.tri) && h2.t < occlude) return 0.0f;
    return 1.0f;
}

}  // namespace

extern "C" {

int orc_version(void) { return 1; }

uint32_t orc_lcg(uint32_t seed, int32_t n, float *out) {
    Lcg l{seed};
    for (int i = 0; i < n; i++) out[i] = l.next1d();
    return l.seed;
}

void orc_pcg(uint64_t seed, int64_t n, float *out) {
    Pcg p;
    p.init(seed);
    for (int64_t i = 0; i < n; i++) out[i] = p.next1d();
}

void orc_camera_matrices(const akr_camera *c, float *r2c16, float *c2w16) {
    Camera cam = make_camera(*c);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            r2c16[i * 4 + j] = cam.r2c.m[i][j];
            c2w16[i * 4 + j] = cam.c2w.m[i][j];
        }
}

int orc_camera_ray(const akr_camera *c, int32_t x, int32_t y, uint32_t *seed, akr_ray *out) {
    Camera cam = make_camera(*c);
    Lcg l{*seed};
    V2 u1 = l.next2d();
    (void)u1;
    V2 u2 = l.next2d();
    *out = generate_ray(cam, u2, x, y);
    *seed = l.seed;
    return 0;
}

void orc_distribution_sample(const float *func, int32_t n, const float *u, int32_t m, int32_t *idx, float *pdf) {
    Distribution d;
    d.build(func, (size_t)n);
    for (int i = 0; i < m; i++) idx[i] = d.sample_discrete(u[i], &pdf[i]);
}

void orc_frame_roundtrip(const float *n3, const float *w3, float *ltw3, float *back3) {
    Frame f = make_frame(v3(n3[0], n3[1], n3[2]));
    V3 u = to_world(f, v3(w3[0], w3[1], w3[2]));
    V3 v = to_local(f, u);
    ltw3[0] = u.x; ltw3[1] = u.y; ltw3[2] = u.z;
    back3[0] = v.x; back3[1] = v.y; back3[2] = v.z;
}

void orc_cosine_hemisphere(const float *u2, int32_t n, float *out3) {
    for (int i = 0; i < n; i++) {
        V3 w = cosine_hemisphere(V2{u2[2 * i], u2[2 * i + 1]});
        out3[3 * i] = w.x; out3[3 * i + 1] = w.y; out3[3 * i + 2] = w.z;
    }
}

int orc_trace(const orc_scene *s, const akr_ray *rays, uint64_t n, orc_hit *hits, int any_hit, int32_t tight,
              int32_t n_threads, uint64_t *box_tests, uint64_t *tri_tests) {
    int T = hw_threads(n_threads);
    std::vector<uint64_t> nb(T, 0), nt(T, 0);
    parallel_for(n, T, 1024, [&](uint64_t i, int tid) {
        Best b;
        bool h = traverse(*s, to_ray(rays[i]), any_hit != 0, tight != 0, b, nb[tid], nt[tid]);
        if (any_hit) {
            hits[i].t = h ? b.t : kInf;
            hits[i].u = h ? b.u : 0;
            hits[i].v = h ? b.v : 0;
            hits[i].gid = h ? b.gid : 0xFFFFFFFFu;
        } else {
            hits[i].t = b.t; hits[i].u = b.u; hits[i].v = b.v; hits[i].gid = b.gid;
        }
    });
    uint64_t sb = 0, st = 0;
    for (int t = 0; t < T; t++) { sb += nb[t]; st += nt[t]; }
    if (box_tests) *box_tests = sb;
    if (tri_tests) *tri_tests = st;
    return 0;
}

int orc_trace_brute(const orc_scene *s, const akr_ray *rays, uint64_t n, orc_hit *hits, int any_hit, int32_t n_threads) {
    int T = hw_threads(n_threads);
    parallel_for(n, T, 64, [&](uint64_t i, int) {
        Best b;
        brute(*s, to_ray(rays[i]), any_hit != 0, b);
        hits[i].t = b.t; hits[i].u = b.u; hits[i].v = b.v; hits[i].gid = b.gid;
    });
    return 0;
}

int orc_render_probe(const orc_scene *s, const akr_pt_params *p, const akr_rect *tiles, int32_t n_tiles,
                     float *radiance, float *weight, int32_t n_threads, orc_render_stats *stats,
                     akr_pixel_probe *probe) {
    Scene sc;
    sc.s = s;
    sc.cam = make_camera(s->camera);
    if (s->n_lights > 0) {
        sc.dist.build(s->light_power, (size_t)s->n_lights);
        for (int i = 0; i < s->n_lights; i++) sc.lights.push_back(get_triangle(*s, s->light_gid[i]));
    }
    const int W = sc.cam.w, H = sc.cam.h;
    const std::vector<Work> work = split_work(tiles, n_tiles, W, H);
    int T = hw_threads(n_threads);
    std::vector<PathStats> pst(T);
    const float clampv = p->ray_clamp;
    const bool tight = !(p->flags & AKR_PT_EXACT_CULL);
    TileFilm tf(work);
    parallel_for(work.size(), T, 1, [&](uint64_t wi, int tid) {
        const Work &w = work[wi];
        for (int y = w.y0; y < w.y1; y++)
            for (int x = w.x0; x < w.x1; x++) {
                Lcg sampler{(uint32_t)(x + y * W)};  // set_sample_index(x + y * W), integrator.cpp:124
                V3 acc = v3(0, 0, 0);
                float wsum = 0;
                PixelTally pt;
                for (int sidx = 0; sidx < p->spp; sidx++) {
                    V3 L = trace_path(sc, sampler, x, y, p->max_depth, tight, pst[tid], pt);
                    if (clampv > 0) {  // gpu/cuda/integrator.cpp:397-398 (GPU-only clamp)
                        V3 c;
                        c.x = std::isnan(L.x) ? 0.0f : rmax(0.0f, L.x);
                        c.y = std::isnan(L.y) ? 0.0f : rmax(0.0f, L.y);
                        c.z = std::isnan(L.z) ? 0.0f : rmax(0.0f, L.z);
                        L = v3(rmin(c.x, clampv), rmin(c.y, clampv), rmin(c.z, clampv));
                    }
                    acc = add(acc, L);  // Tile::add_sample, film.h:66-70
                    wsum += 1.0f;
                }
                float *o = tf.at(wi, w, x, y);
                o[0] = acc.x;
                o[1] = acc.y;
                o[2] = acc.z;
                o[3] = wsum;
                if (probe) {  // frame-indexed; a pixel listed twice computes the same values
                    akr_pixel_probe &q = probe[(size_t)x + (size_t)y * (size_t)W];
                    q.seed = sampler.seed;
                    q.closest_rays = pt.closest;
                    q.shadow_rays = pt.shadow;
                    q.flags = AKR_PROBE_SEED | AKR_PROBE_RAYS;
                }
            }
    });
    tf.merge(work, W, radiance, weight);
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        for (auto &q : pst) {
            stats->camera_rays += q.cam;
            stats->extension_rays += q.ext;
            stats->shadow_rays += q.shd;
            stats->box_tests += q.box;
            stats->tri_tests += q.tri;
        }
    }
    return 0;
}

int orc_render(const orc_scene *s, const akr_pt_params *p, const akr_rect *tiles, int32_t n_tiles, float *radiance,
               float *weight, int32_t n_threads, orc_render_stats *stats) {
    return orc_render_probe(s, p, tiles, n_tiles, radiance, weight, n_threads, stats, nullptr);
}

int orc_render_ao(const orc_scene *s, const akr_ao_params *p, const akr_rect *tiles, int32_t n_tiles, float *radiance,
                  float *weight, int32_t n_threads, orc_render_stats *stats) {
    Scene sc;
    sc.s = s;
    sc.cam = make_camera(s->camera);
    const int W = sc.cam.w, H = sc.cam.h;
    const std::vector<Work> work = split_work(tiles, n_tiles, W, H);
    int T = hw_threads(n_threads);
    std::vector<PathStats> pst(T);
    const bool tight = !(p->flags & AKR_PT_EXACT_CULL);
    TileFilm tf(work);
    parallel_for(work.size(), T, 1, [&](uint64_t wi, int tid) {
        const Work &w = work[wi];
        for (int y = w.y0; y < w.y1; y++)
            for (int x = w.x0; x < w.x1; x++) {
                Lcg sampler{(uint32_t)(x + y * W)};  // set_sample_index(x + y * W), integrator.cpp:73
                float acc = 0, wsum = 0;
                for (int sidx = 0; sidx < p->spp; sidx++) {
                    acc += trace_ao(sc, sampler, x, y, p->occlude, tight, pst[tid]);  // Spectrum(L) per channel
                    wsum += 1.0f;
                }
                float *o = tf.at(wi, w, x, y);
                o[0] = o[1] = o[2] = acc;  // Spectrum(L) per channel
                o[3] = wsum;
            }
    });
    tf.merge(work, W, radiance, weight);
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        for (auto &q : pst) {
            stats->camera_rays += q.cam;
            stats->shadow_rays += q.shd;
            stats->box_tests += q.box;
            stats->tri_tests += q.tri;
        }
    }
    return 0;
}

}  // extern "C"
