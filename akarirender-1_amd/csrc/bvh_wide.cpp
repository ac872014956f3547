// bvh_wide.cpp — collapse the BVH2 into the 4-wide, outward-quantized view the traversal kernels
// walk (akr_bvh4_node / akr_bvh_leaf, akr_bvh_format.h).
//
// Each wide node is a BVH2 node with its two children folded in, so a traversal step replaces
// two BVH2 levels and fetches 64 B for four child boxes instead of 2 x 64 B.  Correctness does
// not rest on the quantized boxes: they only have to CONTAIN the exact ones (checked here in real
// arithmetic, which implies the device's fmaf decode), and every leaf is re-tested with its exact box.
#include <atomic>
#include <cmath>
#include <exception>
#include <thread>
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

// Slots of the wide node for BVH2 internal node `n`: a treelet of at most three BVH2 internal nodes
// (n and up to two nodes below it) whose at most four frontier children are the slots.  `code`
// names the treelet (n with children a, b; a0, a1 the children of a):
//   0 {n}, 1 {n, a}, 2 {n, b}, 3 {n, a, b}, 4 {n, a, a0}, 5 {n, a, a1}, 6 {n, b, b0}, 7 {n, b, b1}
// (Collapser::choose picks it).  Slots are stored in the treelet's depth-first order with no flips;
// order[0..1] hold, per ray direction octant o (bit a = d[a] > 0), the slot permutation of the BVH2
// depth-first order: byte o of the pair, two bits per slot = that slot's position (near = left iff
// d[axis] > 0 at each node).
int gather_slots(const std::vector<akr_bvh_node> &in, uint32_t n2, int code, uint32_t slot_ref2[4], Box slot_box[4],
                 uint32_t order[2]) {
    struct TN {
        uint32_t ref;  // BVH2 reference of a frontier entry (leaf, EMPTY or an unopened node)
        Box box;
        int kid[2];    // opened: treelet indices of its children; -1 while a frontier entry
        uint32_t axis;
    };
    TN tn[7];
    int n_tn = 1;
    tn[0].ref = n2;
    auto open = [&](int i) {
        const akr_bvh_node &m = in[tn[i].ref];
        tn[i].axis = m.axis;
        for (int c = 0; c < 2; c++) {
            tn[n_tn].ref = m.child[c];
            tn[n_tn].box = child_box(m, c);
            tn[n_tn].kid[0] = tn[n_tn].kid[1] = -1;
            tn[i].kid[c] = n_tn++;
        }
    };
    open(0);  // tn[1] = a, tn[2] = b
    if (code == 1 || code == 3 || code == 4 || code == 5) open(1);  // tn[3], tn[4] = a0, a1
    if (code == 2 || code == 6 || code == 7) open(2);                // tn[3], tn[4] = b0, b1
    if (code == 3) open(2);
    if (code == 4 || code == 6) open(3);
    if (code == 5 || code == 7) open(4);
    // depth-first frontier of the treelet, each opened node's children swapped when `flip` says so
    auto frontier = [&](auto &&flip, int out[4]) {
        int st[8], sp = 0, n = 0;
        st[sp++] = 0;
        while (sp) {
            const int i = st[--sp];
            if (tn[i].kid[0] < 0) {
                out[n++] = i;
                continue;
            }
            const bool f = flip(tn[i].axis);
            st[sp++] = tn[i].kid[f ? 0 : 1];
            st[sp++] = tn[i].kid[f ? 1 : 0];
        }
        return n;
    };
    int slot_tn[4];
    const int n_slots = frontier([](uint32_t) { return false; }, slot_tn);
    for (int s = 0; s < 4; s++) slot_ref2[s] = AKR_CHILD_EMPTY;
    for (int s = 0; s < n_slots; s++) {
        slot_ref2[s] = tn[slot_tn[s]].ref;
        slot_box[s] = tn[slot_tn[s]].box;
    }
    order[0] = order[1] = 0;
    for (uint32_t o = 0; o < 8; o++) {
        int seq[4];
        frontier([o](uint32_t axis) { return !((o >> axis) & 1u); }, seq);
        uint32_t byte = 0, used = 0;
        for (int s = 0; s < n_slots; s++)
            for (int p = 0; p < n_slots; p++)
                if (seq[p] == slot_tn[s]) {
                    byte |= (uint32_t)p << (2 * s);
                    used |= 1u << p;
                }
        for (int s = n_slots, p = 0; s < 4; s++) {  // empty slots: the positions left (never entered)
            while (used & (1u << p)) p++;
            byte |= (uint32_t)p << (2 * s);
            used |= 1u << p;
        }
        order[o >> 2] |= byte << (8 * (o & 3));
    }
    return n_slots;
}

// Layout: wide nodes in depth-first preorder (a node, then its slots' subtrees in slot order) and
// leaves in the order that walk meets them.  Both are fixed by per-subtree counts, so every subtree
// is written at a precomputed offset and independent subtrees are collapsed on several threads;
// the output is the same as a serial recursive walk.
struct Collapser {
    const std::vector<akr_bvh_node> &in;
    Bvh4Output &out;
    int collapse;
    std::vector<uint32_t> n_nodes, n_leaves;  // per BVH2 node: wide nodes / leaves of its wide subtree
    std::vector<uint8_t> choice;              // AKR_COLLAPSE_SAH: per BVH2 node, its treelet code

    bool internal(uint32_t r) const { return r != AKR_CHILD_EMPTY && !(r & AKR_CHILD_LEAF); }

    int code_of(uint32_t n2) const {
        if (collapse == AKR_COLLAPSE_SAH) return choice[n2];
        const bool ia = internal(in[n2].child[0]), ib = internal(in[n2].child[1]);  // balanced
        return ia && ib ? 3 : (ia ? 1 : (ib ? 2 : 0));
    }

    // AKR_COLLAPSE_SAH: the treelet of every node that minimises the expected number of wide-node
    // visits of its subtree, sum over wide nodes of the area of their box (a ray's chance to enter
    // it), by dynamic programming from the leaves up.  Leaves do not enter the sum: every leaf is a
    // slot of exactly one wide node whatever the treelets, and is tested when that slot is entered.
    // cost[x] = the sum for the wide subtree below a wide node rooted at x (x's own area excluded).
    void choose(uint32_t root) {
        choice.assign(in.size(), 0);
        std::vector<double> cost(in.size(), 0.0);
        auto area = [](const Box &b) {
            const double dx = (double)b.hi[0] - b.lo[0], dy = (double)b.hi[1] - b.lo[1], dz = (double)b.hi[2] - b.lo[2];
            return dx * dy + dy * dz + dz * dx;
        };
        // a frontier entry: child c of node p, reached as a wide node of its own when internal
        auto G = [&](uint32_t p, int c) {
            const uint32_t r = in[p].child[c];
            return internal(r) ? area(child_box(in[p], c)) + cost[r] : 0.0;
        };
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        while (!st.empty()) {
            auto [n, done] = st.back();
            st.pop_back();
            const uint32_t a = in[n].child[0], b = in[n].child[1];
            if (!done) {
                st.push_back({n, true});
                if (internal(a)) st.push_back({a, false});
                if (internal(b)) st.push_back({b, false});
                continue;
            }
            const bool ia = internal(a), ib = internal(b);
            double c[8];
            for (double &x : c) x = INFINITY;
            c[0] = G(n, 0) + G(n, 1);
            if (ia) {
                c[1] = G(a, 0) + G(a, 1) + G(n, 1);
                if (internal(in[a].child[0])) c[4] = G(in[a].child[0], 0) + G(in[a].child[0], 1) + G(a, 1) + G(n, 1);
                if (internal(in[a].child[1])) c[5] = G(a, 0) + G(in[a].child[1], 0) + G(in[a].child[1], 1) + G(n, 1);
            }
            if (ib) {
                c[2] = G(n, 0) + G(b, 0) + G(b, 1);
                if (internal(in[b].child[0])) c[6] = G(n, 0) + G(in[b].child[0], 0) + G(in[b].child[0], 1) + G(b, 1);
                if (internal(in[b].child[1])) c[7] = G(n, 0) + G(b, 0) + G(in[b].child[1], 0) + G(in[b].child[1], 1);
            }
            if (ia && ib) c[3] = G(a, 0) + G(a, 1) + G(b, 0) + G(b, 1);
            int best = 0;
            for (int k = 1; k < 8; k++)
                if (c[k] < c[best]) best = k;
            choice[n] = (uint8_t)best;
            cost[n] = c[best];
        }
    }

    struct Task {
        uint32_t n2, node_at, leaf_at;
        int depth;
    };

    // Post-order count pass over the wide tree (iterative: SBVH trees can be deep).
    void count(uint32_t root) {
        n_nodes.assign(in.size(), 0);
        n_leaves.assign(in.size(), 0);
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        uint32_t ref[4], order[2];
        Box box[4];
        while (!st.empty()) {
            auto [n2, done] = st.back();
            st.pop_back();
            gather_slots(in, n2, code_of(n2), ref, box, order);
            if (!done) {
                st.push_back({n2, true});
                for (int s = 0; s < 4; s++)
                    if (ref[s] != AKR_CHILD_EMPTY && !(ref[s] & AKR_CHILD_LEAF)) st.push_back({ref[s], false});
                continue;
            }
            uint64_t nn = 1, nl = 0;
            for (int s = 0; s < 4; s++) {
                if (ref[s] == AKR_CHILD_EMPTY) continue;
                if (ref[s] & AKR_CHILD_LEAF) nl++;
                else {
                    nn += n_nodes[ref[s]];
                    nl += n_leaves[ref[s]];
                }
            }
            if (nn >= 0xffffffffull || nl >= AKR_CHILD_LEAF) throw std::runtime_error("too many BVH leaves for the wide format");
            n_nodes[n2] = (uint32_t)nn;
            n_leaves[n2] = (uint32_t)nl;
        }
    }

    void put_leaf(uint32_t at, uint32_t ref2, const Box &b) {
        akr_bvh_leaf &l = out.leaves[at];
        for (int k = 0; k < 3; k++) {
            l.lo[k] = b.lo[k];
            l.hi[k] = b.hi[k];
        }
        l.first = akr_leaf_first(ref2);
        l.count = akr_leaf_count(ref2);
    }

    // Collapse the wide subtree of `t.n2` into its slots.  Subtrees with fewer than `spawn_below`
    // wide nodes are collapsed in place; larger ones are handed to `spawn` (when given).
    template <class Spawn>
    void build(const Task &t, int &max_depth, float &max_abs, uint32_t spawn_below, Spawn &&spawn) {
        if (t.depth > max_depth) max_depth = t.depth;
        uint32_t slot_ref2[4], order[2];
        Box slot_box[4];
        gather_slots(in, t.n2, code_of(t.n2), slot_ref2, slot_box, order);
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
            max_abs = std::max(max_abs, std::max(std::fabs(plo[k]), pow2f(e)));
            ex[k] = (uint32_t)(e + 127);
        }
        w.meta = ex[0] | ex[1] << 8 | ex[2] << 16;
        w.order[0] = order[0];
        w.order[1] = order[1];
        uint32_t node_at = t.node_at + 1, leaf_at = t.leaf_at;
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
            if (r & AKR_CHILD_LEAF) {
                put_leaf(leaf_at, r, slot_box[s]);
                w.child[s] = AKR_CHILD_LEAF | leaf_at++;
            } else {
                const Task c{r, node_at, leaf_at, t.depth + 1};
                w.child[s] = node_at;
                if (n_nodes[r] >= spawn_below) spawn(c);
                else build(c, max_depth, max_abs, spawn_below, spawn);
                node_at += n_nodes[r];
                leaf_at += n_leaves[r];
            }
        }
        out.nodes[t.node_at] = w;
    }

    void run(uint32_t root, int threads) {
        if (collapse == AKR_COLLAPSE_SAH) choose(root);
        count(root);
        out.nodes.resize(n_nodes[root]);
        out.leaves.resize(n_leaves[root]);
        const int n_threads = threads > 0 ? std::min(threads, 64) : (int)std::min(64u, std::max(1u, std::thread::hardware_concurrency()));
        // Top of the tree on this thread: subtrees of at least `cut` wide nodes are split further,
        // the rest become tasks (about 32 per thread) collapsed on the pool.
        const uint32_t cut = std::max<uint32_t>(4096, n_nodes[root] / (32u * (uint32_t)n_threads));
        std::vector<Task> tasks, top{{root, 0, 0, 1}};
        int max_depth = 0;
        float max_abs = 0.0f;
        auto defer = [&](const Task &c) { top.push_back(c); };
        auto leave = [&](const Task &c) { tasks.push_back(c); };
        while (!top.empty()) {
            const Task t = top.back();
            top.pop_back();
            if (n_nodes[t.n2] < cut && t.node_at != 0) {
                tasks.push_back(t);
                continue;
            }
            // one level here; large children go back on `top`, small ones straight to `tasks`
            build(t, max_depth, max_abs, 1, [&](const Task &c) {
                if (n_nodes[c.n2] >= cut) defer(c);
                else leave(c);
            });
        }
        std::atomic<size_t> next{0};
        std::vector<int> depth_of(n_threads, 0);
        std::vector<float> abs_of(n_threads, 0.0f);
        run_on_threads(n_threads, [&](int w) {
            auto no_spawn = [](const Task &) {};
            for (size_t i; (i = next.fetch_add(1)) < tasks.size();)
                build(tasks[i], depth_of[w], abs_of[w], 0xffffffffu, no_spawn);
        });
        for (int w = 0; w < n_threads; w++) {
            max_depth = std::max(max_depth, depth_of[w]);
            max_abs = std::max(max_abs, abs_of[w]);
        }
        out.max_depth = max_depth;
        out.max_abs = max_abs;
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

int validate_bvh2(const akr_bvh_node *nodes, uint64_t n_nodes, const akr_bvh_tri *tris, uint64_t n_tris,
                  uint64_t n_scene_tris, int &max_leaf) {
    max_leaf = 0;
    if (n_nodes == 0) throw std::runtime_error("BVH: no nodes");
    if (n_nodes >= AKR_CHILD_LEAF) throw std::runtime_error("BVH: too many nodes");
    if (nodes[0].child[1] != AKR_CHILD_EMPTY) throw std::runtime_error("BVH: node 0 is not the virtual root");
    for (uint64_t t = 0; t < n_tris; t++)
        if (tris[t].gid >= n_scene_tris) throw std::runtime_error("BVH: triangle id beyond the scene");
    std::vector<uint8_t> seen(n_nodes, 0);
    std::vector<std::pair<uint32_t, int>> st;  // (node, depth)
    int depth = 0;
    auto child = [&](uint32_t r, int d) {
        if (r == AKR_CHILD_EMPTY) return;
        if (r & AKR_CHILD_LEAF) {
            const uint64_t first = akr_leaf_first(r), cnt = akr_leaf_count(r);
            if (cnt > AKR_LEAF_MAX || first + cnt > n_tris) throw std::runtime_error("BVH: leaf outside the triangles");
            max_leaf = std::max(max_leaf, (int)cnt);
            depth = std::max(depth, d);
            return;
        }
        if (r == 0 || r >= n_nodes) throw std::runtime_error("BVH: node reference out of range");
        if (seen[r]) throw std::runtime_error("BVH: a node is reached twice (not a tree)");
        seen[r] = 1;
        st.push_back({r, d});
    };
    seen[0] = 1;
    child(nodes[0].child[0], 1);
    while (!st.empty()) {
        const auto [n, d] = st.back();
        st.pop_back();
        if (d > AKR_BVH_MAX_DEPTH) throw std::runtime_error("BVH: deeper than AKR_BVH_MAX_DEPTH");
        depth = std::max(depth, d);
        const akr_bvh_node &x = nodes[n];
        if (x.axis > 2) throw std::runtime_error("BVH: split axis out of range");
        const float *v[3] = {x.bxy0, x.bxy1, x.bz};
        for (int a = 0; a < 3; a++)
            for (int k = 0; k < 4; k++)
                if (std::isnan(v[a][k])) throw std::runtime_error("BVH: NaN in a node box");
        child(x.child[0], d + 1);
        child(x.child[1], d + 1);
    }
    return depth;
}

void build_bvh4(const std::vector<akr_bvh_node> &bvh2, Bvh4Output &out, int n_threads, int collapse) {
    out.nodes.clear();
    out.leaves.clear();
    out.max_depth = 0;
    out.max_abs = 0.0f;
    out.root_ref = AKR_CHILD_EMPTY;
    if (bvh2.empty()) return;
    const akr_bvh_node &vroot = bvh2[0];  // virtual root: child 0 = the real root
    const uint32_t r = vroot.child[0];
    if (r == AKR_CHILD_EMPTY) return;
    if (r & AKR_CHILD_LEAF) {
        out.leaves.resize(1);
        Collapser c{bvh2, out, collapse, {}, {}, {}};
        c.put_leaf(0, r, child_box(vroot, 0));
        out.root_ref = AKR_CHILD_LEAF;
    } else {
        Collapser c{bvh2, out, collapse, {}, {}, {}};
        c.run(r, n_threads);
        out.root_ref = 0;
    }
}

}  // namespace akr
