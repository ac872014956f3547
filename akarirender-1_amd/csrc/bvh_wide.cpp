// bvh_wide.cpp — collapse the BVH2 into the 4- and 8-wide, outward-quantized views the traversal
// kernels walk (akr_bvh4_node / akr_bvh8_node / akr_bvh_leaf, akr_bvh_format.h).
//
// Each wide node is a BVH2 node with its two children folded in, so a traversal step replaces
// two BVH2 levels and fetches 64 B for four child boxes instead of 2 x 64 B.  Correctness does
// not rest on the quantized boxes: they only have to CONTAIN the exact ones (checked here in real
// arithmetic, which implies the device's fmaf decode), and every leaf is re-tested with its exact box.
#include <cmath>
#include <cstring>
#include <stdexcept>
#include "bvh_build.h"

namespace akr {

// The quantized bound must lie outside the exact one in REAL arithmetic (origin + q * s, no
// rounding), not only after the device's fmaf rounding: the lean slot test (kernels.hip
// visit_wide_lean) folds origin and q * s into one fma per bound with an error slack derived for
// the real value.  Real containment implies the fmaf one (rounding is monotone and `bound` is a
// float).  The real value is evaluated in long double with a margin that covers its own rounding.
static bool real_le(uint32_t q, float s, float origin, float bound) {
    const long double v = (long double)origin + (long double)q * (long double)s;
    const long double m = std::ldexp(1.0L, -60) * (std::fabs((long double)origin) + 255.0L * s + std::fabs((long double)bound));
    return v + m <= (long double)bound;
}

static bool real_ge(uint32_t q, float s, float origin, float bound) {
    const long double v = (long double)origin + (long double)q * (long double)s;
    const long double m = std::ldexp(1.0L, -60) * (std::fabs((long double)origin) + 255.0L * s + std::fabs((long double)bound));
    return v - m >= (long double)bound;
}

namespace {

inline float pow2f(int k) { return std::ldexp(1.0f, k); }

struct Box {
    float lo[3], hi[3];
};

Box child_box(const akr_bvh_node &n, int c) {
    Box b;
    const float *xy = c == 0 ? n.bxy0 : n.bxy1;
    b.lo[0] = xy[0];
    b.hi[0] = xy[1];
    b.lo[1] = xy[2];
    b.hi[1] = xy[3];
    b.lo[2] = n.bz[2 * c];
    b.hi[2] = n.bz[2 * c + 1];
    return b;
}

// A wide node before packing: W slots (BVH2 references + exact boxes) and the split axes of the
// W - 1 folded BVH2 nodes, in heap order (node, its children, its grandchildren ...).
template <int W>
struct WideSlots {
    uint32_t ref2[W];
    Box box[W];
    uint32_t axis[W - 1];
};

// Collapses a BVH2 into W-wide nodes (W = 4 or 8), depth-first preorder, leaves in BVH2
// depth-first order.  Out is Bvh4Output or Bvh8Output; pack() writes the format's node.
template <int W, class Out, class Node>
struct Collapser {
    static constexpr int L = W == 4 ? 2 : 3;  // folded BVH2 levels
    const std::vector<akr_bvh_node> &in;
    Out &out;

    uint32_t leaf_ref(uint32_t ref2, const Box &b) {
        akr_bvh_leaf l;
        for (int k = 0; k < 3; k++) {
            l.lo[k] = b.lo[k];
            l.hi[k] = b.hi[k];
        }
        l.first = akr_leaf_first(ref2);
        l.count = akr_leaf_count(ref2);
        out.leaves.push_back(l);
        const uint64_t idx = out.leaves.size() - 1;
        if (idx >= AKR_CHILD_LEAF) throw std::runtime_error("too many BVH leaves for the wide format");
        return AKR_CHILD_LEAF | (uint32_t)idx;
    }

    // slot group [base, base + span) at `level` below the wide node's BVH2 node: a leaf (or the
    // bottom level) takes slot `base`; an internal node records its axis and splits the group
    void gather(WideSlots<W> &ws, uint32_t ref, const Box &b, int level, int base, int span) {
        if (ref == AKR_CHILD_EMPTY) return;
        if (level == L || (ref & AKR_CHILD_LEAF)) {
            ws.ref2[base] = ref;
            ws.box[base] = b;
            return;
        }
        const akr_bvh_node &m = in[ref];
        ws.axis[(1 << level) - 1 + base / span] = m.axis;
        for (int g = 0; g < 2; g++) gather(ws, m.child[g], child_box(m, g), level + 1, base + g * span / 2, span / 2);
    }

    // Wide node for BVH2 internal node `n2`, laid out in depth-first preorder.
    uint32_t build(uint32_t n2, int depth) {
        if (depth > out.max_depth) out.max_depth = depth;
        const uint32_t me = (uint32_t)out.nodes.size();
        out.nodes.emplace_back();
        WideSlots<W> ws;
        for (int s = 0; s < W; s++) ws.ref2[s] = AKR_CHILD_EMPTY;
        for (int a = 0; a < W - 1; a++) ws.axis[a] = 0;
        const akr_bvh_node &n = in[n2];
        ws.axis[0] = n.axis;
        for (int c = 0; c < 2; c++) gather(ws, n.child[c], child_box(n, c), 1, c * W / 2, W / 2);
        // quantization frame: the union of the slot boxes
        float plo[3], phi[3];
        for (int k = 0; k < 3; k++) {
            plo[k] = INFINITY;
            phi[k] = -INFINITY;
        }
        bool any = false;
        for (int s = 0; s < W; s++) {
            if (ws.ref2[s] == AKR_CHILD_EMPTY) continue;
            any = true;
            for (int k = 0; k < 3; k++) {
                plo[k] = std::min(plo[k], ws.box[s].lo[k]);
                phi[k] = std::max(phi[k], ws.box[s].hi[k]);
            }
        }
        float origin[3];
        uint32_t ex[3] = {1, 1, 1};
        for (int k = 0; k < 3; k++) {
            if (!any) {
                origin[k] = 0.0f;
                continue;
            }
            if (!std::isfinite(plo[k]) || !std::isfinite(phi[k]))
                throw std::runtime_error("non-finite BVH bounds");
            origin[k] = plo[k];
            const double ext = (double)phi[k] - (double)plo[k];
            int e = -126;
            if (ext > 0) {
                int k2 = 0;
                std::frexp(ext / 255.0, &k2);  // ext / 255 < 2^k2
                e = std::max(-126, k2 - 1);
            }
            while (e < 127 && 255.0 * std::ldexp(1.0, e) < ext) e++;
            while (e < 127 && (std::fmaf(255.0f, pow2f(e), plo[k]) < phi[k] || !real_ge(255, pow2f(e), plo[k], phi[k]))) e++;
            if (std::fmaf(255.0f, pow2f(e), plo[k]) < phi[k] || !real_ge(255, pow2f(e), plo[k], phi[k]))
                throw std::runtime_error("BVH bounds too large to quantize");
            out.max_abs = std::max(out.max_abs, std::max(std::fabs(plo[k]), pow2f(e)));
            ex[k] = (uint32_t)(e + 127);
        }
        uint8_t qlo[W][3], qhi[W][3];
        for (int s = 0; s < W; s++)
            for (int k = 0; k < 3; k++) {
                qlo[s][k] = qhi[s][k] = 0;
                if (ws.ref2[s] == AKR_CHILD_EMPTY) continue;
                const float sc = pow2f((int)ex[k] - 127);
                qlo[s][k] = (uint8_t)quantize_lo(ws.box[s].lo[k], origin[k], sc);
                qhi[s][k] = (uint8_t)quantize_hi(ws.box[s].hi[k], origin[k], sc);
            }
        // children (preorder: this node first, then its slots' subtrees in slot order)
        uint32_t child[W];
        for (int s = 0; s < W; s++) {
            const uint32_t r = ws.ref2[s];
            child[s] = r == AKR_CHILD_EMPTY ? AKR_CHILD_EMPTY
                                            : ((r & AKR_CHILD_LEAF) ? leaf_ref(r, ws.box[s]) : build(r, depth + 1));
        }
        Node w;
        std::memset(&w, 0, sizeof(w));
        pack(w, origin, ex, ws.axis, child, qlo, qhi);
        out.nodes[me] = w;
        return me;
    }

    static void pack(akr_bvh4_node &w, const float *origin, const uint32_t *ex, const uint32_t *axis,
                     const uint32_t *child, const uint8_t (*qlo)[3], const uint8_t (*qhi)[3]) {
        for (int k = 0; k < 3; k++) w.origin[k] = origin[k];
        w.meta = ex[0] | ex[1] << 8 | ex[2] << 16 | (axis[0] | axis[1] << 2 | axis[2] << 4) << 24;
        for (int s = 0; s < 4; s++) {
            w.child[s] = child[s];
            for (int k = 0; k < 3; k++) {
                w.q[2 * k] |= (uint32_t)qlo[s][k] << (8 * s);
                w.q[2 * k + 1] |= (uint32_t)qhi[s][k] << (8 * s);
            }
        }
    }

    static void pack(akr_bvh8_node &w, const float *origin, const uint32_t *ex, const uint32_t *axis,
                     const uint32_t *child, const uint8_t (*qlo)[3], const uint8_t (*qhi)[3]) {
        for (int k = 0; k < 3; k++) w.origin[k] = origin[k];
        w.meta = ex[0] | ex[1] << 8 | ex[2] << 16;
        w.axes = 0;
        for (int a = 0; a < 7; a++) w.axes |= axis[a] << (2 * a);
        for (int s = 0; s < 8; s++) {
            w.child[s] = child[s];
            for (int k = 0; k < 3; k++) {
                w.q[2 * (2 * k) + (s >> 2)] |= (uint32_t)qlo[s][k] << (8 * (s & 3));
                w.q[2 * (2 * k + 1) + (s >> 2)] |= (uint32_t)qhi[s][k] << (8 * (s & 3));
            }
        }
    }
};

template <int W, class Out, class Node>
void build_wide(const std::vector<akr_bvh_node> &bvh2, Out &out) {
    out.nodes.clear();
    out.leaves.clear();
    out.max_depth = 0;
    out.max_abs = 0.0f;
    out.root_ref = AKR_CHILD_EMPTY;
    if (bvh2.empty()) return;
    const akr_bvh_node &vroot = bvh2[0];  // virtual root: child 0 = the real root
    const uint32_t r = vroot.child[0];
    if (r == AKR_CHILD_EMPTY) return;
    Collapser<W, Out, Node> c{bvh2, out};
    out.nodes.reserve(bvh2.size() / (W - 1) + 1);
    if (r & AKR_CHILD_LEAF) out.root_ref = c.leaf_ref(r, child_box(vroot, 0));
    else out.root_ref = c.build(r, 1);
}

}  // namespace

uint32_t quantize_lo(float bound, float origin, float s) {
    double q = std::floor(((double)bound - (double)origin) / (double)s);
    q = std::min(255.0, std::max(0.0, q));
    uint32_t qi = (uint32_t)q;
    while (qi > 0 && (std::fmaf((float)qi, s, origin) > bound || !real_le(qi, s, origin, bound))) qi--;
    if (std::fmaf((float)qi, s, origin) > bound || (qi > 0 && !real_le(qi, s, origin, bound)))
        throw std::runtime_error("quantize_lo: bound below origin");
    return qi;  // q = 0 is the origin itself, which is <= every bound of the frame
}

uint32_t quantize_hi(float bound, float origin, float s) {
    double q = std::ceil(((double)bound - (double)origin) / (double)s);
    q = std::min(255.0, std::max(0.0, q));
    uint32_t qi = (uint32_t)q;
    while (qi < 255 && (std::fmaf((float)qi, s, origin) < bound || !real_ge(qi, s, origin, bound))) qi++;
    if (std::fmaf((float)qi, s, origin) < bound || !real_ge(qi, s, origin, bound))
        throw std::runtime_error("quantize_hi: bound beyond the frame");
    return qi;
}

void build_bvh4(const std::vector<akr_bvh_node> &bvh2, Bvh4Output &out) {
    build_wide<4, Bvh4Output, akr_bvh4_node>(bvh2, out);
}

void build_bvh8(const std::vector<akr_bvh_node> &bvh2, Bvh8Output &out) {
    build_wide<8, Bvh8Output, akr_bvh8_node>(bvh2, out);
}

}  // namespace akr
