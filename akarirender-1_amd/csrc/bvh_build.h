// bvh_build.h — host binned-SAH builder for the BVH2 of akr_bvh_format.h.
//
// Replaces the reference's SBVH build (src/akari/kernel/bvh-accelerator.h:125-475, called from
// BVHAccelerator::build :673-678).  Closest-hit and occlusion results do not depend on the
// builder (up to exact ties in t), so the builder is free to target GPU traversal cost:
// 32-bin SAH per axis (like the reference's nBuckets, :104), leaves of at most `max_leaf_size`
// triangles, task-parallel over std::thread.  AKR_BUILDER_SAH: object splits only (no duplicated
// references).  AKR_BUILDER_SBVH: the reference's spatial splits as well (clipped, duplicated
// references, up to spatial_budget * n extra).
#pragma once
#include <stdint.h>
#include <exception>
#include <thread>
#include <vector>
#include "../../include/akr_hip.h"
#include "../../include/akr_bvh_format.h"

namespace akr {

// Runs f(k) for k in [0, n): k >= 1 on threads of their own, k = 0 on the calling thread.  Every
// thread that was started is joined before this returns or rethrows (a joinable std::thread that is
// destroyed during unwinding calls std::terminate); a share whose thread cannot be created
// (std::system_error under thread or resource limits) runs on the calling thread instead.  The first
// exception thrown by any f(k) is rethrown after the join.
template <class F>
void run_on_threads(int n, F &&f) {
    std::vector<std::exception_ptr> err((size_t)(n > 0 ? n : 0));
    auto call = [&](int k) {
        try {
            f(k);
        } catch (...) {
            err[(size_t)k] = std::current_exception();
        }
    };
    std::vector<std::thread> ts;
    std::vector<int> inline_k;
    for (int k = 1; k < n; k++) {
        try {
            ts.emplace_back(call, k);
        } catch (...) {
            inline_k.push_back(k);
        }
    }
    if (n > 0) call(0);
    for (int k : inline_k) call(k);
    for (auto &t : ts) t.join();
    for (auto &e : err)
        if (e) std::rethrow_exception(e);
}

struct BvhInput {
    const float *vertices;   // 3 * n_vertices
    const int32_t *indices;  // 3 * n_tris
    uint64_t n_tris;
};

struct BvhOutput {
    std::vector<akr_bvh_node> nodes;
    std::vector<akr_bvh_tri> tris;
    int max_depth = 0;
    int max_leaf = 0;
    double sah_cost = 0;
    double build_ms = 0;
};

void build_bvh(const BvhInput &in, const akr_build_params &params, BvhOutput &out);

#ifdef __HIPCC__
// GPU linear BVH (lbvh.hip): Morton sort + Karras hierarchy + parallel refit on the device of the
// current HIP context, on stream `st`; one triangle per leaf.  Same output format.
void build_lbvh_gpu(const BvhInput &in, BvhOutput &out, hipStream_t st);
#endif

// Wide view of a BVH2 (akr_bvh4_node / akr_bvh_leaf, akr_bvh_format.h).  root_ref is the wide
// reference of the BVH2's real root (wide node 0, a leaf, or EMPTY for an empty scene).
struct Bvh4Output {
    std::vector<akr_bvh4_node> nodes;
    std::vector<akr_bvh_leaf> leaves;
    uint32_t root_ref = AKR_CHILD_EMPTY;
    int max_depth = 0;
    float max_abs = 0.0f;  // largest |frame origin| and frame step 2^e over all wide nodes (lean test bound)
};

// n_threads <= 0: one per hardware thread (at most 64).  collapse: AKR_COLLAPSE_SAH (default) or
// AKR_COLLAPSE_BALANCED (akr_hip.h; bvh_wide.cpp gather_slots).
void build_bvh4(const std::vector<akr_bvh_node> &bvh2, Bvh4Output &out, int n_threads = 0, int collapse = 0);

// Checks a BVH2 handed in from outside (akr_hip_import_accel) before the library adopts it: node 0 is
// the virtual root (child[1] EMPTY), every internal reference is < n_nodes and reached once from
// the root (a tree), every leaf's triangle range lies inside `tris` with 1..AKR_LEAF_MAX triangles,
// split axes are 0..2, boxes are not NaN, the depth is <= AKR_BVH_MAX_DEPTH and every triangle id
// is < n_scene_tris.  Returns the depth (and the largest leaf in max_leaf); throws on violation.
int validate_bvh2(const akr_bvh_node *nodes, uint64_t n_nodes, const akr_bvh_tri *tris, uint64_t n_tris,
                  uint64_t n_scene_tris, int &max_leaf);

// Outward 8-bit quantization of one bound (exposed for tests): the q with fmaf(q, s, origin) on
// the correct side of `bound`, s = 2^(e - 127).
uint32_t quantize_lo(float bound, float origin, float s);
uint32_t quantize_hi(float bound, float origin, float s);

}  // namespace akr
