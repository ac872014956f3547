// bvh_wide.cpp — collapse the BVH2 into the 4-wide, outward-quantized view the traversal kernels
// walk (akr_bvh4_node / akr_bvh_leaf, akr_bvh_format.h).
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

struct Collapser {
    const std::vector<akr_bvh_node> &in;
    Bvh4Output &out;

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

    // Wide node for BVH2 internal node `n2`, laid out in depth-first preorder.
    uint32_t build(uint32_t n2, int depth) {
        if (depth > out.max_depth) out.max_depth = depth;
        const uint32_t me = (uint32_t)out.nodes.size();
        out.nodes.emplace_back();
        const akr_bvh_node &n = in[n2];
        uint32_t slot_ref2[4] = {AKR_CHILD_EMPTY, AKR_CHILD_EMPTY, AKR_CHILD_EMPTY, AKR_CHILD_EMPTY};
        Box slot_box[4];
        uint32_t axis[3] = {n.axis, 0, 0};
        for (int c = 0; c < 2; c++) {
            const uint32_t r = n.child[c];
            if (r == AKR_CHILD_EMPTY) continue;
            if (r & AKR_CHILD_LEAF) {
                slot_ref2[2 * c] = r;
                slot_box[2 * c] = child_box(n, c);
            } else {
                const akr_bvh_node &m = in[r];
                axis[1 + c] = m.axis;
                for (int g = 0; g < 2; g++) {
                    slot_ref2[2 * c + g] = m.child[g];
                    slot_box[2 * c + g] = child_box(m, g);
                }
            }
        }
        // quantization frame: the union of the slot boxes
        float plo[3], phi[3];
        for (int k = 0; k < 3; k++) {
            plo[k] = INFINITY;
            phi[k] = -INFINITY;
        }
        bool any = false;
        for (int s = 0; s < 4; s++) {
            if (slot_ref2[s] == AKR_CHILD_EMPTY) continue;
            any = true;
            for (int k = 0; k < 3; k++) {
                plo[k] = std::min(plo[k], slot_box[s].lo[k]);
                phi[k] = std::max(phi[k], slot_box[s].hi[k]);
            }
        }
        akr_bvh4_node w;
        std::memset(&w, 0, sizeof(w));
        uint32_t ex[3] = {1, 1, 1};
        for (int k = 0; k < 3; k++) {
            if (!any) {
                w.origin[k] = 0.0f;
                continue;
            }
            if (!std::isfinite(plo[k]) || !std::isfinite(phi[k]))
                throw std::runtime_error("non-finite BVH bounds");
            w.origin[k] = plo[k];
            const double ext = (double)phi[k] - (double)plo[k];
            int e = -126;
            if (ext > 0) {
                int k = 0;
                std::frexp(ext / 255.0, &k);  // ext / 255 < 2^k
                e = std::max(-126, k - 1);
            }
            while (e < 127 && 255.0 * std::ldexp(1.0, e) < ext) e++;
            while (e < 127 && (std::fmaf(255.0f, pow2f(e), plo[k]) < phi[k] || !real_ge(255, pow2f(e), plo[k], phi[k]))) e++;
            if (std::fmaf(255.0f, pow2f(e), plo[k]) < phi[k] || !real_ge(255, pow2f(e), plo[k], phi[k]))
                throw std::runtime_error("BVH bounds too large to quantize");
            out.max_abs = std::max(out.max_abs, std::max(std::fabs(plo[k]), pow2f(e)));
            ex[k] = (uint32_t)(e + 127);
        }
        w.meta = ex[0] | ex[1] << 8 | ex[2] << 16 | (axis[0] | axis[1] << 2 | axis[2] << 4) << 24;
        for (int s = 0; s < 4; s++) {
            const uint32_t r = slot_ref2[s];
            if (r == AKR_CHILD_EMPTY) {
                w.child[s] = AKR_CHILD_EMPTY;
                continue;
            }
            for (int k = 0; k < 3; k++) {
                const float sc = pow2f((int)ex[k] - 127);
                w.q[2 * k] |= quantize_lo(slot_box[s].lo[k], w.origin[k], sc) << (8 * s);
                w.q[2 * k + 1] |= quantize_hi(slot_box[s].hi[k], w.origin[k], sc) << (8 * s);
            }
        }
        // children (preorder: this node first, then its slots' subtrees in slot order)
        for (int s = 0; s < 4; s++) {
            const uint32_t r = slot_ref2[s];
            if (r == AKR_CHILD_EMPTY) continue;
            w.child[s] = (r & AKR_CHILD_LEAF) ? leaf_ref(r, slot_box[s]) : build(r, depth + 1);
        }
        out.nodes[me] = w;
        return me;
    }
};

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
    out.nodes.clear();
    out.leaves.clear();
    out.max_depth = 0;
    out.max_abs = 0.0f;
    out.root_ref = AKR_CHILD_EMPTY;
    if (bvh2.empty()) return;
    const akr_bvh_node &vroot = bvh2[0];  // virtual root: child 0 = the real root
    const uint32_t r = vroot.child[0];
    if (r == AKR_CHILD_EMPTY) return;
    Collapser c{bvh2, out};
    out.nodes.reserve(bvh2.size() / 2 + 1);
    if (r & AKR_CHILD_LEAF) out.root_ref = c.leaf_ref(r, child_box(vroot, 0));
    else out.root_ref = c.build(r, 1);
}

}  // namespace akr
