/*
 * akr_bvh_format.h — in-memory layout of the acceleration structure produced by
 * akr_hip_build_accel (data format only; no algorithms live here).
 *
 * BVH2 with both child boxes stored in the parent ("child boxes in parent"): one 64-byte node
 * fetch (one half of a 128-byte HBM line) serves the two AABB tests of a traversal step, and a
 * culled child is never fetched.  This replaces the reference's per-node 64-byte BVHNode
 * (src/akari/kernel/bvh-accelerator.h:34-57) whose box is tested when the node is popped; the
 * traversal order (near child = left iff ray.d[axis] > 0, bvh-accelerator.h:43-56, 508-514) and
 * the cull rule (entry t < 0 or entry t > best t, :500) are kept, see DESIGN.md §3.
 *
 * Node 0 is a virtual root: child[0] is the real root (or a leaf), child[1] is EMPTY, so the
 * root box is tested exactly once like the reference's first intersectAABB.
 */
#ifndef AKR_BVH_FORMAT_H
#define AKR_BVH_FORMAT_H
#include <stdint.h>

#define AKR_CHILD_EMPTY 0xFFFFFFFFu
#define AKR_CHILD_LEAF 0x80000000u   /* leaf reference: LEAF | (first << 3) | (count - 1) */
#define AKR_LEAF_MAX 8
#define AKR_BVH_MAX_DEPTH 64

#if defined(__HIPCC__)
#define AKR_HD __host__ __device__
#else
#define AKR_HD
#endif

typedef struct akr_bvh_node {
    float bxy0[4]; /* child 0: lo.x, hi.x, lo.y, hi.y */
    float bxy1[4]; /* child 1: lo.x, hi.x, lo.y, hi.y */
    float bz[4];   /* child 0: lo.z, hi.z; child 1: lo.z, hi.z */
    uint32_t child[2];
    uint32_t axis; /* split axis of this node (0, 1, 2) */
    uint32_t _pad;
} akr_bvh_node;

/* Leaf-ordered triangle: v0, e1 = v1 - v0, e2 = v2 - v0 (computed in f32 on the host, the same
 * rounding as the reference's in-loop subtraction, instance.h:49-50), global triangle id. */
typedef struct akr_bvh_tri {
    float v0[3];
    uint32_t gid;
    float e1[3];
    uint32_t _pad0;
    float e2[3];
    uint32_t _pad1;
} akr_bvh_tri;

/* Wide (4-child) view of the same tree, which the traversal kernels walk.
 * A wide node is a treelet of at most three BVH2 internal nodes (a node and up to two nodes below
 * it, chosen by surface area) whose frontier children are its slots, stored in the treelet's
 * depth-first order.  order[] gives, for each ray direction octant o (bit a = d[a] > 0), the slots'
 * positions in the BVH2 depth-first order for that octant (near = left iff d[axis] > 0 at every
 * node of the treelet): byte o of the pair, two bits per slot.  Slot boxes are quantized OUTWARD to
 * 8 bits per bound: bound = fmaf(q, 2^(e - 127), origin) is <= (lo) / >= (hi) the exact bound, so
 * a slot test can only pass more often than the exact one.  Every leaf keeps its exact f32 box in
 * an akr_bvh_leaf record and is tested with it (with the current best t) before its triangles:
 * the leaves whose triangles are tested, and their order, are exactly the BVH2 traversal's. */
typedef struct akr_bvh4_node {
    float origin[3];
    uint32_t meta;     /* ex | ey << 8 | ez << 16 (frame step exponents, biased by 127) */
    uint32_t child[4]; /* wide node index, AKR_CHILD_LEAF | leaf index, or AKR_CHILD_EMPTY */
    uint32_t q[6];     /* qlo_x, qhi_x, qlo_y, qhi_y, qlo_z, qhi_z; byte k of each = slot k */
    uint32_t order[2]; /* per octant slot positions: octants 0-3 in order[0], 4-7 in order[1] */
} akr_bvh4_node;

typedef struct akr_bvh_leaf {
    float lo[3];
    float hi[3];
    uint32_t first; /* into the leaf-ordered akr_bvh_tri array */
    uint32_t count;
} akr_bvh_leaf;

static inline AKR_HD int akr_child_is_leaf(uint32_t c) { return c != AKR_CHILD_EMPTY && (c & AKR_CHILD_LEAF); }
static inline AKR_HD uint32_t akr_leaf_first(uint32_t c) { return (c & 0x7FFFFFFFu) >> 3; }
static inline AKR_HD uint32_t akr_leaf_count(uint32_t c) { return (c & 7u) + 1u; }

#endif
