// lbvh.hip — GPU BVH2 builder: linear BVH (Karras 2012) over 63-bit Morton
// codes of the triangle centroids, built entirely on the device, in the same akr_bvh_node /
// akr_bvh_tri format as the host SAH builder (bvh_build.cpp), so every traversal kernel, the
// wide collapse and the oracle work on it unchanged.
//
// The reference's SBVH build (bvh-accelerator.h:125-475) runs on the host and is the slow step
// before the path at 10M triangles; this one trades tree quality for build time:
//   1. k_tri_bounds   per-triangle box + centroid, scene bounds (block reduction + ordered atomics)
//   2. k_morton       21 bits per axis, interleaved x, y, z from the most significant bit
//   3. rocprim radix sort of (code, triangle) pairs
//   4. k_karras       one thread per internal node: range and split from common prefixes
//                     (equal codes are separated by their sorted index)
//   5. k_refit        one thread per leaf walks up; the second child to arrive at a node (agent-
//                     scope acq_rel counter) writes the node's box into its parent's child slot
//   6. k_leaf_tris    leaf-ordered akr_bvh_tri records (v0, gid, e1, e2 as f32 host subtraction)
// The split axis stored for the traversal order is the axis of the node's splitting Morton bit,
// so the left child is the lower one along it.  Leaves hold one triangle.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include "kernels.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "bvh_build.h"

namespace akr {

namespace {

#define LB_CHECK(x)                                                                              \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) throw std::runtime_error(std::string("lbvh: ") + #x + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int kB = 256;

// order-preserving float <-> uint for atomicMin/Max on floats
__device__ __forceinline__ uint32_t f2o(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float o2f(uint32_t u) {
    const uint32_t b = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}

__global__ void k_tri_bounds(const float *v, const int32_t *idx, uint32_t n, float4 *cen, uint32_t *bounds) {
    __shared__ uint32_t s[6][kB];
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    uint32_t lo[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, hi[3] = {0, 0, 0};
    if (i < n) {
        float c[3];
        for (int k = 0; k < 3; k++) {
            const float a = v[3 * (size_t)idx[3 * (size_t)i + 0] + k], b = v[3 * (size_t)idx[3 * (size_t)i + 1] + k],
                        d = v[3 * (size_t)idx[3 * (size_t)i + 2] + k];
            const float mn = fminf(a, fminf(b, d)), mx = fmaxf(a, fmaxf(b, d));
            c[k] = 0.5f * mn + 0.5f * mx;  // box centre, like the host builder's centroid
            lo[k] = f2o(c[k]);
            hi[k] = f2o(c[k]);
        }
        cen[i] = make_float4(c[0], c[1], c[2], 0.0f);
    }
    for (int k = 0; k < 3; k++) {
        s[k][threadIdx.x] = lo[k];
        s[3 + k][threadIdx.x] = hi[k];
    }
    __syncthreads();
    for (int off = kB / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off)
            for (int k = 0; k < 3; k++) {
                s[k][threadIdx.x] = min(s[k][threadIdx.x], s[k][threadIdx.x + off]);
                s[3 + k][threadIdx.x] = max(s[3 + k][threadIdx.x], s[3 + k][threadIdx.x + off]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int k = 0; k < 3; k++) {
            atomicMin(&bounds[k], s[k][0]);
            atomicMax(&bounds[3 + k], s[3 + k][0]);
        }
}

__device__ __forceinline__ uint64_t spread21(uint64_t x) {  // 21 bits -> every third bit
    x &= 0x1FFFFFull;
    x = (x | x << 32) & 0x1F00000000FFFFull;
    x = (x | x << 16) & 0x1F0000FF0000FFull;
    x = (x | x << 8) & 0x100F00F00F00F00Full;
    x = (x | x << 4) & 0x10C30C30C30C30C3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

__global__ void k_morton(const float4 *cen, uint32_t n, const uint32_t *bounds, uint64_t *code, uint32_t *id) {
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const float4 c = cen[i];
    const float cc[3] = {c.x, c.y, c.z};
    uint64_t q[3];
    for (int k = 0; k < 3; k++) {
        const float lo = o2f(bounds[k]), hi = o2f(bounds[3 + k]);
        const float ext = hi - lo;
        float t = ext > 0.0f ? (cc[k] - lo) / ext : 0.0f;
        t = fminf(fmaxf(t, 0.0f), 1.0f);
        q[k] = (uint64_t)(t * 2097151.0f);
    }
    code[i] = spread21(q[0]) << 2 | spread21(q[1]) << 1 | spread21(q[2]);  // bit 62 = x's MSB
    id[i] = i;
}

struct Tree {
    int32_t *left, *right, *parent;  // internal nodes [0, n-1), leaves n-1 + i; child < 0 encodes leaf ~i
    uint32_t *axis;
};

__device__ __forceinline__ int delta(const uint64_t *c, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint64_t a = c[i], b = c[j];
    return a == b ? 64 + __clz((uint32_t)(i ^ j)) : __clzll((long long)(a ^ b));
}

__global__ void k_karras(const uint64_t *c, int n, Tree t) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n - 1) return;
    const int d = delta(c, n, i, i + 1) - delta(c, n, i, i - 1) >= 0 ? 1 : -1;
    const int dmin = delta(c, n, i, i - d);
    int lmax = 2;
    while (delta(c, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int s = lmax / 2; s >= 1; s /= 2)
        if (delta(c, n, i, i + (l + s) * d) > dmin) l += s;
    const int j = i + l * d;
    const int dnode = delta(c, n, i, j);
    int s = 0;
    for (int div = 2;; div *= 2) {
        const int st = (l + div - 1) / div;
        if (delta(c, n, i, i + (s + st) * d) > dnode) s += st;
        if (st <= 1) break;
    }
    const int gamma = i + s * d + min(d, 0);
    const int lo = min(i, j), hi = max(i, j);
    const int L = lo == gamma ? ~gamma : gamma;          // leaf gamma or internal gamma
    const int R = hi == gamma + 1 ? ~(gamma + 1) : gamma + 1;
    t.left[i] = L;
    t.right[i] = R;
    t.parent[L < 0 ? (n - 1) + ~L : L] = i;
    t.parent[R < 0 ? (n - 1) + ~R : R] = i;
    // split bit: the highest bit where the range's first and last codes differ (Morton bit
    // 62 - 3k is x, 61 - 3k is y, 60 - 3k is z); equal codes (index split) get axis 0
    const uint64_t x = c[lo] ^ c[hi];
    t.axis[i] = x ? (uint32_t)((__clzll((long long)x) - 1) % 3) : 0u;
}

// Child boxes are handed between threads of any CU / XCD: written with agent-scope (sc1) stores
// and read with agent-scope loads, ordered by the acq_rel counter (MI355X_MICROARCH.md,
// inter-workgroup visibility).
__device__ __forceinline__ void st_agent(float *p, float x) {
    __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float *p) {
    return __hip_atomic_load(const_cast<float *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// node record slot of child `side` of internal node i (our node index = i + 1; node 0 = virtual root)
__device__ __forceinline__ void write_child_box(akr_bvh_node *nodes, int node, int side, const float lo[3],
                                                const float hi[3]) {
    akr_bvh_node &nd = nodes[node];
    float *xy = side == 0 ? nd.bxy0 : nd.bxy1;
    st_agent(&xy[0], lo[0]);
    st_agent(&xy[1], hi[0]);
    st_agent(&xy[2], lo[1]);
    st_agent(&xy[3], hi[1]);
    st_agent(&nd.bz[2 * side], lo[2]);
    st_agent(&nd.bz[2 * side + 1], hi[2]);
}

__global__ void k_refit(const float *v, const int32_t *idx, const uint32_t *sorted_id, int n, Tree t,
                        uint32_t *flags, akr_bvh_node *nodes) {
    const int leaf = blockIdx.x * kB + threadIdx.x;
    if (leaf >= n) return;
    const uint32_t tri = sorted_id[leaf];
    float lo[3], hi[3];
    for (int k = 0; k < 3; k++) {
        const float a = v[3 * (size_t)idx[3 * (size_t)tri + 0] + k], b = v[3 * (size_t)idx[3 * (size_t)tri + 1] + k],
                    d = v[3 * (size_t)idx[3 * (size_t)tri + 2] + k];
        lo[k] = fminf(a, fminf(b, d));
        hi[k] = fmaxf(a, fmaxf(b, d));
    }
    if (n == 1) {  // the virtual root's child is the leaf itself
        write_child_box(nodes, 0, 0, lo, hi);
        return;
    }
    int child = ~leaf;
    int node = t.parent[(n - 1) + leaf];
    while (true) {
        const int side = t.left[node] == child ? 0 : 1;
        write_child_box(nodes, node + 1, side, lo, hi);
        // agent-scope acq_rel: the first arrival's box is visible to the second (other CU / XCD)
        const uint32_t old = __hip_atomic_fetch_add(&flags[node], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old == 0) return;
        const akr_bvh_node &nd = nodes[node + 1];
        const float *oxy = side == 0 ? nd.bxy1 : nd.bxy0;
        const float olo[3] = {ld_agent(&oxy[0]), ld_agent(&oxy[2]), ld_agent(&nd.bz[2 * (1 - side)])};
        const float ohi[3] = {ld_agent(&oxy[1]), ld_agent(&oxy[3]), ld_agent(&nd.bz[2 * (1 - side) + 1])};
        for (int k = 0; k < 3; k++) {
            lo[k] = fminf(lo[k], olo[k]);
            hi[k] = fmaxf(hi[k], ohi[k]);
        }
        if (node == 0) {  // the root: its box goes to the virtual root's child 0
            write_child_box(nodes, 0, 0, lo, hi);
            return;
        }
        child = node;
        node = t.parent[node];
    }
}

__global__ void k_links(int n, Tree t, akr_bvh_node *nodes) {
    const int i = blockIdx.x * kB + threadIdx.x;
    auto ref = [&](int c) -> uint32_t {  // leaf ~p -> LEAF | p << 3 | (1 - 1); internal c -> node c + 1
        return c < 0 ? (AKR_CHILD_LEAF | ((uint32_t)~c << 3)) : (uint32_t)(c + 1);
    };
    if (i == 0) {  // virtual root
        akr_bvh_node &r = nodes[0];
        r.child[0] = n == 1 ? ref(~0) : 1u;
        r.child[1] = AKR_CHILD_EMPTY;
        r.bxy1[0] = r.bxy1[2] = r.bz[2] = INFINITY;
        r.bxy1[1] = r.bxy1[3] = r.bz[3] = -INFINITY;
        r.axis = 0;
        r._pad = 0;
    }
    if (i >= n - 1) return;
    akr_bvh_node &nd = nodes[i + 1];
    nd.child[0] = ref(t.left[i]);
    nd.child[1] = ref(t.right[i]);
    nd.axis = t.axis[i];
    nd._pad = 0;
}

__global__ void k_leaf_tris(const float *v, const int32_t *idx, const uint32_t *sorted_id, uint32_t n, akr_bvh_tri *out) {
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const uint32_t tri = sorted_id[i];
    float p[3][3];
    for (int c = 0; c < 3; c++)
        for (int k = 0; k < 3; k++) p[c][k] = v[3 * (size_t)idx[3 * (size_t)tri + c] + k];
    akr_bvh_tri r;
    for (int k = 0; k < 3; k++) {
        r.v0[k] = p[0][k];
        r.e1[k] = p[1][k] - p[0][k];
        r.e2[k] = p[2][k] - p[0][k];
    }
    r.gid = tri;
    r._pad0 = r._pad1 = 0;
    out[i] = r;
}

template <class T>
struct Dev {
    T *p = nullptr;
    explicit Dev(size_t n) { LB_CHECK(hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T))); }
    ~Dev() { (void)hipFree(p); }
    Dev(const Dev &) = delete;
    Dev &operator=(const Dev &) = delete;
};

inline unsigned blocks(size_t n) { return (unsigned)((n + kB - 1) / kB); }

int tree_depth(const std::vector<akr_bvh_node> &nodes) {
    int best = 0;
    std::vector<std::pair<uint32_t, int>> st{{nodes[0].child[0], 1}};
    while (!st.empty()) {
        auto [r, dep] = st.back();
        st.pop_back();
        if (r == AKR_CHILD_EMPTY) continue;
        best = std::max(best, dep);
        if (r & AKR_CHILD_LEAF) continue;
        st.push_back({nodes[r].child[0], dep + 1});
        st.push_back({nodes[r].child[1], dep + 1});
    }
    return best;
}

}  // namespace

void build_lbvh_gpu(const BvhInput &in, BvhOutput &out, hipStream_t st) {
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t n64 = in.n_tris;
    if (n64 >= (1ull << 28)) throw std::runtime_error("lbvh: too many triangles");
    const int n = (int)n64;
    out.nodes.assign(1, akr_bvh_node{});
    out.tris.clear();
    out.max_leaf = n ? 1 : 0;
    out.sah_cost = 0;
    akr_bvh_node &vr = out.nodes[0];
    vr.child[0] = vr.child[1] = AKR_CHILD_EMPTY;
    for (int k = 0; k < 2; k++) {
        float *xy = k == 0 ? vr.bxy0 : vr.bxy1;
        xy[0] = xy[2] = vr.bz[2 * k] = INFINITY;
        xy[1] = xy[3] = vr.bz[2 * k + 1] = -INFINITY;
    }
    if (n == 0) {
        out.max_depth = 0;
        out.build_ms = 0;
        return;
    }
    uint64_t nv = 0;
    for (uint64_t i = 0; i < 3 * n64; i++) nv = std::max<uint64_t>(nv, (uint64_t)in.indices[i] + 1);
    Dev<float> v(3 * nv);
    Dev<int32_t> idx(3 * n64);
    LB_CHECK(hipMemcpyAsync(v.p, in.vertices, 3 * nv * sizeof(float), hipMemcpyHostToDevice, st));
    LB_CHECK(hipMemcpyAsync(idx.p, in.indices, 3 * n64 * sizeof(int32_t), hipMemcpyHostToDevice, st));
    Dev<float4> cen(n64);
    Dev<uint32_t> bounds(6);
    const uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
    LB_CHECK(hipMemcpyAsync(bounds.p, init, sizeof(init), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_tri_bounds, dim3(blocks(n64)), dim3(kB), 0, st, v.p, idx.p, (uint32_t)n, cen.p, bounds.p);
    Dev<uint64_t> code(n64), code_s(n64);
    Dev<uint32_t> id(n64), id_s(n64);
    hipLaunchKernelGGL(k_morton, dim3(blocks(n64)), dim3(kB), 0, st, cen.p, (uint32_t)n, bounds.p, code.p, id.p);
    size_t tmp_bytes = 0;
    LB_CHECK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, code.p, code_s.p, id.p, id_s.p, n64, 0, 63, st));
    Dev<uint8_t> tmp(tmp_bytes);
    LB_CHECK(rocprim::radix_sort_pairs(tmp.p, tmp_bytes, code.p, code_s.p, id.p, id_s.p, n64, 0, 63, st));
    const size_t n_int = (size_t)std::max(0, n - 1);
    Dev<int32_t> left(n_int), right(n_int), parent(2 * n64);
    Dev<uint32_t> axis(n_int), flags(n_int);
    Tree t{left.p, right.p, parent.p, axis.p};
    Dev<akr_bvh_node> nodes(1 + n_int);
    LB_CHECK(hipMemcpyAsync(nodes.p, out.nodes.data(), sizeof(akr_bvh_node), hipMemcpyHostToDevice, st));
    if (n > 1) {
        LB_CHECK(hipMemsetAsync(flags.p, 0, n_int * sizeof(uint32_t), st));
        hipLaunchKernelGGL(k_karras, dim3(blocks(n_int)), dim3(kB), 0, st, code_s.p, n, t);
    }
    hipLaunchKernelGGL(k_refit, dim3(blocks(n64)), dim3(kB), 0, st, v.p, idx.p, id_s.p, n, t, flags.p, nodes.p);
    hipLaunchKernelGGL(k_links, dim3(blocks(std::max<size_t>(1, n_int))), dim3(kB), 0, st, n, t, nodes.p);
    Dev<akr_bvh_tri> tris(n64);
    hipLaunchKernelGGL(k_leaf_tris, dim3(blocks(n64)), dim3(kB), 0, st, v.p, idx.p, id_s.p, (uint32_t)n, tris.p);
    LB_CHECK(hipGetLastError());
    out.nodes.resize(1 + n_int);
    out.tris.resize(n64);
    LB_CHECK(hipMemcpyAsync(out.nodes.data(), nodes.p, (1 + n_int) * sizeof(akr_bvh_node), hipMemcpyDeviceToHost, st));
    LB_CHECK(hipMemcpyAsync(out.tris.data(), tris.p, n64 * sizeof(akr_bvh_tri), hipMemcpyDeviceToHost, st));
    LB_CHECK(hipStreamSynchronize(st));
    out.max_depth = tree_depth(out.nodes);
    if (out.max_depth > AKR_BVH_MAX_DEPTH)
        throw std::runtime_error("lbvh: tree deeper than " + std::to_string(AKR_BVH_MAX_DEPTH) +
                                 " levels (use the SAH builder for this scene)");
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Stable sort of the cost-ordered fetch's (shard, class) keys with their slot indices.
size_t pixel_order_tmp_bytes(uint32_t n) {
    size_t bytes = 0;
    LB_CHECK(rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                       (const uint32_t *)nullptr, (uint32_t *)nullptr, n, 0,
                                       (int)(kOrderClassBits + 3), (hipStream_t)0));
    return bytes;
}
void sort_pixel_order(void *tmp, size_t tmp_bytes, const uint32_t *key_in, uint32_t *key_out, const uint32_t *idx_in,
                      uint32_t *idx_out, uint32_t n, hipStream_t st) {
    static_assert(kWorkShards <= 8, "the sort key holds the shard in 3 bits");
    LB_CHECK(rocprim::radix_sort_pairs(tmp, tmp_bytes, key_in, key_out, idx_in, idx_out, n, 0,
                                       (int)(kOrderClassBits + 3), st));
}

}  // namespace akr
