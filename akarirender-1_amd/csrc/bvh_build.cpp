// bvh_build.cpp — task-parallel binned-SAH BVH2 builder (see bvh_build.h).
#include "bvh_build.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <functional>
#include <limits>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace akr {
namespace {

constexpr int kMaxBins = 64;
constexpr int kMedianDepth = 40;        // below this depth fall back to object-median splits
constexpr uint32_t kTaskMin = 8192;     // subtrees at least this big become pool tasks
constexpr uint32_t kParBinMin = 262144; // ranges at least this big are binned by all threads

struct Box {
    float lo[3], hi[3];
    void reset() {
        for (int i = 0; i < 3; i++) {
            lo[i] = std::numeric_limits<float>::infinity();
            hi[i] = -std::numeric_limits<float>::infinity();
        }
    }
    void grow(const Box &b) {
        for (int i = 0; i < 3; i++) {
            lo[i] = std::min(lo[i], b.lo[i]);
            hi[i] = std::max(hi[i], b.hi[i]);
        }
    }
    void grow(const float *p) {
        for (int i = 0; i < 3; i++) {
            lo[i] = std::min(lo[i], p[i]);
            hi[i] = std::max(hi[i], p[i]);
        }
    }
    double area() const {
        double e[3];
        for (int i = 0; i < 3; i++) {
            e[i] = (double)hi[i] - (double)lo[i];
            if (!(e[i] >= 0)) return 0.0;
        }
        return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
    }
};

struct BNode {
    Box box;
    uint32_t left = 0, right = 0;  // build-node indices
    uint32_t first = 0, count = 0; // leaf range in the reference array
    uint8_t axis = 0;
    bool leaf = false;
};

struct Bin {
    Box box, cbox;
    uint32_t n;
    void reset() { box.reset(); cbox.reset(); n = 0; }
};

struct Task {
    uint32_t node, begin, end;
    int depth;
    Box box, cbox;
};

// SBVH reference: a triangle and the part of its bounds this reference covers (spatial splits
// clip it; bvh-accelerator.h:568-607)
struct SRef {
    uint32_t prim;
    Box box;
};

struct STask {
    uint32_t node;
    int depth;
    Box box;
    std::vector<SRef> refs;
};

struct Job {
    Task t;
    std::shared_ptr<STask> s;  // non-null: an SBVH task
};

inline bool box_empty(const Box &b) { return !(b.lo[0] <= b.hi[0] && b.lo[1] <= b.hi[1] && b.lo[2] <= b.hi[2]); }
inline Box box_and(const Box &a, const Box &b) {
    Box r;
    for (int i = 0; i < 3; i++) {
        r.lo[i] = std::max(a.lo[i], b.lo[i]);
        r.hi[i] = std::min(a.hi[i], b.hi[i]);
    }
    return r;
}
inline float round_down(double x) {
    float f = (float)x;
    return (double)f > x ? std::nextafter(f, -std::numeric_limits<float>::infinity()) : f;
}
inline float round_up(double x) {
    float f = (float)x;
    return (double)f < x ? std::nextafter(f, std::numeric_limits<float>::infinity()) : f;
}

class Builder {
  public:
    Builder(const BvhInput &in, const akr_build_params &p) : in_(in) {
        n_ = (uint32_t)in.n_tris;
        threads_ = p.n_threads > 0 ? p.n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
        bins_ = std::clamp(p.n_bins > 0 ? p.n_bins : 32, 2, kMaxBins);
        max_leaf_ = std::clamp(p.max_leaf_size > 0 ? p.max_leaf_size : 4, 1, AKR_LEAF_MAX);
        ct_ = p.traversal_cost > 0 ? p.traversal_cost : 1.0f;
        ci_ = p.intersect_cost > 0 ? p.intersect_cost : 4.0f;
        sbvh_ = p.builder == AKR_BUILDER_SBVH;
        budget_ = p.spatial_budget > 0 ? std::min(p.spatial_budget, 4.0f) : 0.5f;
    }

    void run(BvhOutput &out) {
        if (n_ == 0) {
            out.nodes.assign(1, empty_vroot());
            out.tris.clear();
            return;
        }
        if (sbvh_) {
            run_sbvh(out);
            return;
        }
        pbox_.resize(n_);
        cen_.resize(3 * (size_t)n_);
        ref_.resize(n_);
        nodes_.resize(2 * (size_t)n_ + 1);
        next_node_ = 0;
        std::vector<Box> tb(threads_), tc(threads_);
        parallel_chunks(0, n_, [&](uint32_t b, uint32_t e, int t) {
            tb[t].reset();
            tc[t].reset();
            for (uint32_t i = b; i < e; i++) {
                Box bx;
                bx.reset();
                for (int k = 0; k < 3; k++) {
                    int32_t vi = in_.indices[3 * (size_t)i + k];
                    bx.grow(&in_.vertices[3 * (size_t)vi]);
                }
                pbox_[i] = bx;
                for (int k = 0; k < 3; k++) cen_[3 * (size_t)i + k] = 0.5f * bx.lo[k] + 0.5f * bx.hi[k];
                ref_[i] = i;
                tb[t].grow(bx);
                tc[t].grow(&cen_[3 * (size_t)i]);
            }
        });
        Box root, croot;
        root.reset();
        croot.reset();
        for (int t = 0; t < threads_; t++) {
            root.grow(tb[t]);
            croot.grow(tc[t]);
        }
        uint32_t r = alloc_node();
        submit(Task{r, 0, n_, 0, root, croot});
        drain();
        flatten(r, out);
    }

  private:
    static akr_bvh_node empty_vroot() {
        akr_bvh_node v;
        std::memset(&v, 0, sizeof(v));
        for (int k = 0; k < 2; k++) {
            float *b = k == 0 ? v.bxy0 : v.bxy1;
            b[0] = b[2] = std::numeric_limits<float>::infinity();
            b[1] = b[3] = -std::numeric_limits<float>::infinity();
            v.bz[2 * k] = std::numeric_limits<float>::infinity();
            v.bz[2 * k + 1] = -std::numeric_limits<float>::infinity();
        }
        v.child[0] = v.child[1] = AKR_CHILD_EMPTY;
        return v;
    }

    template <class F>
    void parallel_chunks(uint32_t b, uint32_t e, F &&f) {
        uint32_t n = e - b;
        int T = (n < 65536) ? 1 : threads_;
        if (T == 1) {
            f(b, e, 0);
            return;
        }
        uint32_t chunk = (n + T - 1) / T;
        run_on_threads(T, [&](int t) {
            uint32_t cb = b + t * chunk, ce = std::min(e, cb + chunk);
            if (cb < ce) f(cb, ce, t);
        });
    }

    uint32_t alloc_node() {
        uint32_t i = next_node_.fetch_add(1);
        if (i >= nodes_.size()) throw std::runtime_error("bvh: node pool exhausted");
        return i;
    }

    // ---------------------------------------------------------------- task pool
    void submit(const Task &t) {
        std::lock_guard<std::mutex> g(mu_);
        queue_.push_back(Job{t, nullptr});
        pending_++;
        cv_.notify_one();
    }
    void submit(std::shared_ptr<STask> t) {
        std::lock_guard<std::mutex> g(mu_);
        queue_.push_back(Job{Task{}, std::move(t)});
        pending_++;
        cv_.notify_one();
    }
    void drain() {
        run_on_threads(threads_, [this](int) { worker(); });
        if (!error_.empty()) throw std::runtime_error(error_);
    }
    void worker() {
        while (true) {
            Job j;
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return !queue_.empty() || pending_ == 0; });
                if (queue_.empty()) return;
                j = std::move(queue_.back());
                queue_.pop_back();
            }
            try {
                if (j.s) build_sbvh(std::move(*j.s));
                else build(j.t);
            } catch (const std::exception &e) {
                std::lock_guard<std::mutex> g(mu_);
                error_ = e.what();
            }
            {
                std::lock_guard<std::mutex> g(mu_);
                pending_--;
                if (pending_ == 0) cv_.notify_all();
            }
        }
    }

    // ---------------------------------------------------------------- recursion
    void make_leaf(BNode &nd, const Task &t) {
        nd.leaf = true;
        nd.first = t.begin;
        nd.count = t.end - t.begin;
        nd.box = t.box;
    }

    int bin_of(uint32_t prim, int axis, float cmin, float k) const {
        int b = (int)((cen_[3 * (size_t)prim + axis] - cmin) * k);
        return std::clamp(b, 0, bins_ - 1);
    }

    void build(Task t) {
        // iterative on the larger side to bound native stack use; small subtrees stay local
        while (true) {
            BNode &nd = nodes_[t.node];
            nd.box = t.box;
            uint32_t n = t.end - t.begin;
            if (n <= 1 || (t.depth >= AKR_BVH_MAX_DEPTH - 2 && n <= (uint32_t)max_leaf_)) {
                make_leaf(nd, t);
                return;
            }
            if (t.depth >= AKR_BVH_MAX_DEPTH - 2) throw std::runtime_error("bvh: depth limit exceeded");
            int axis = -1, split = -1;
            double best = std::numeric_limits<double>::infinity();
            Bin bins[3][kMaxBins];
            float kscale[3] = {0, 0, 0};
            bool median = t.depth >= kMedianDepth;
            if (!median) {
                for (int a = 0; a < 3; a++) {
                    float ext = t.cbox.hi[a] - t.cbox.lo[a];
                    kscale[a] = ext > 0 ? (float)bins_ * (1.0f - 1e-6f) / ext : 0.0f;
                }
                bin_range(t, kscale, bins);
                double parea = t.box.area();
                for (int a = 0; a < 3; a++) {
                    if (!(kscale[a] > 0)) continue;
                    double rarea[kMaxBins];
                    uint32_t rcnt[kMaxBins];
                    Box acc;
                    acc.reset();
                    uint32_t c = 0;
                    for (int b = bins_ - 1; b > 0; b--) {
                        acc.grow(bins[a][b].box);
                        c += bins[a][b].n;
                        rarea[b] = acc.area();
                        rcnt[b] = c;
                    }
                    acc.reset();
                    c = 0;
                    for (int b = 0; b < bins_ - 1; b++) {
                        acc.grow(bins[a][b].box);
                        c += bins[a][b].n;
                        uint32_t nl = c, nr = rcnt[b + 1];
                        if (nl == 0 || nr == 0) continue;
                        double cost = acc.area() * nl + rarea[b + 1] * nr;
                        if (cost < best) {
                            best = cost;
                            axis = a;
                            split = b;
                        }
                    }
                }
                double parea_safe = parea > 0 ? parea : 1.0;
                double split_cost = ct_ + ci_ * best / parea_safe;
                double leaf_cost = ci_ * (double)n;
                if (n <= (uint32_t)max_leaf_ && (axis < 0 || leaf_cost <= split_cost)) {
                    make_leaf(nd, t);
                    return;
                }
            }
            uint32_t mid;
            Task lt, rt;
            if (axis >= 0) {
                float cmin = t.cbox.lo[axis], k = kscale[axis];
                uint32_t *r = ref_.data();
                uint32_t *m = std::partition(r + t.begin, r + t.end,
                                             [&](uint32_t p) { return bin_of(p, axis, cmin, k) <= split; });
                mid = (uint32_t)(m - r);
                lt.box.reset(); lt.cbox.reset(); rt.box.reset(); rt.cbox.reset();
                for (int b = 0; b < bins_; b++) {
                    Task &dst = b <= split ? lt : rt;
                    dst.box.grow(bins[axis][b].box);
                    dst.cbox.grow(bins[axis][b].cbox);
                }
            } else {
                if (n <= (uint32_t)max_leaf_) {
                    make_leaf(nd, t);
                    return;
                }
                // object median along the widest centroid axis
                int a = 0;
                for (int k = 1; k < 3; k++)
                    if (t.cbox.hi[k] - t.cbox.lo[k] > t.cbox.hi[a] - t.cbox.lo[a]) a = k;
                axis = a;
                mid = t.begin + n / 2;
                uint32_t *r = ref_.data();
                std::nth_element(r + t.begin, r + mid, r + t.end, [&](uint32_t x, uint32_t y) {
                    return cen_[3 * (size_t)x + a] < cen_[3 * (size_t)y + a];
                });
                bounds(t.begin, mid, lt.box, lt.cbox);
                bounds(mid, t.end, rt.box, rt.cbox);
            }
            if (mid == t.begin || mid == t.end) throw std::runtime_error("bvh: empty partition");
            nd.leaf = false;
            nd.axis = (uint8_t)axis;
            nd.left = alloc_node();
            nd.right = alloc_node();
            lt.node = nd.left; lt.begin = t.begin; lt.end = mid; lt.depth = t.depth + 1;
            rt.node = nd.right; rt.begin = mid; rt.end = t.end; rt.depth = t.depth + 1;
            // hand the bigger child to the pool when it is large, continue with the other
            Task &big = (lt.end - lt.begin) >= (rt.end - rt.begin) ? lt : rt;
            Task &small = (&big == &lt) ? rt : lt;
            if (big.end - big.begin >= kTaskMin) {
                submit(big);
                t = small;
            } else {
                build(small);
                t = big;
            }
        }
    }

    void bounds(uint32_t b, uint32_t e, Box &box, Box &cbox) {
        box.reset();
        cbox.reset();
        for (uint32_t i = b; i < e; i++) {
            uint32_t p = ref_[i];
            box.grow(pbox_[p]);
            cbox.grow(&cen_[3 * (size_t)p]);
        }
    }

    void bin_range(const Task &t, const float *k, Bin (&bins)[3][kMaxBins]) {
        auto work = [&](uint32_t b, uint32_t e, Bin (&lb)[3][kMaxBins]) {
            for (int a = 0; a < 3; a++)
                for (int i = 0; i < bins_; i++) lb[a][i].reset();
            for (uint32_t i = b; i < e; i++) {
                uint32_t p = ref_[i];
                for (int a = 0; a < 3; a++) {
                    if (!(k[a] > 0)) continue;
                    Bin &bn = lb[a][bin_of(p, a, t.cbox.lo[a], k[a])];
                    bn.n++;
                    bn.box.grow(pbox_[p]);
                    bn.cbox.grow(&cen_[3 * (size_t)p]);
                }
            }
        };
        uint32_t n = t.end - t.begin;
        if (n < kParBinMin || threads_ == 1) {
            work(t.begin, t.end, bins);
            return;
        }
        std::vector<Bin> local((size_t)threads_ * 3 * kMaxBins);
        auto at = [&](int th) -> Bin (&)[3][kMaxBins] {
            return *reinterpret_cast<Bin(*)[3][kMaxBins]>(&local[(size_t)th * 3 * kMaxBins]);
        };
        uint32_t chunk = (n + threads_ - 1) / threads_;
        int used = 0;
        for (int th = 0; th < threads_; th++)
            if (t.begin + th * chunk < t.end) used = th + 1;
        run_on_threads(used, [&](int th) {
            uint32_t cb = t.begin + th * chunk, ce = std::min(t.end, cb + chunk);
            work(cb, ce, at(th));
        });
        for (int a = 0; a < 3; a++)
            for (int i = 0; i < bins_; i++) {
                bins[a][i].reset();
                for (int th = 0; th < used; th++) {
                    const Bin &s = at(th)[a][i];
                    bins[a][i].n += s.n;
                    bins[a][i].box.grow(s.box);
                    bins[a][i].cbox.grow(s.cbox);
                }
            }
    }

    // ---------------------------------------------------------------- SBVH
    // The reference's SBVH (TBVHAccelerator::recursiveBuild, bvh-accelerator.h:125-475): per node
    // the best binned object split and, above depth 40 and when the object split's children overlap
    // by more than 1e-5 of the root area, the best spatial split (references straddling the plane
    // are clipped into both children, TriangleHandle::split :568-607), with the reference's
    // unsplitting test for each straddling reference.  Task-parallel; a reference budget bounds the
    // duplication.
    void run_sbvh(BvhOutput &out) {
        ref_cap_ = (uint64_t)n_ + (uint64_t)((double)budget_ * n_);
        if (ref_cap_ >= (1ull << 31)) ref_cap_ = (1ull << 31) - 1;
        ref_.resize(ref_cap_);
        nodes_.resize(2 * (size_t)ref_cap_ + 1);
        next_node_ = 0;
        refs_total_ = n_;
        leaf_cursor_ = 0;
        auto root = std::make_shared<STask>();
        root->refs.resize(n_);
        std::vector<Box> tb(threads_);
        parallel_chunks(0, n_, [&](uint32_t b, uint32_t e, int t) {
            tb[t].reset();
            for (uint32_t i = b; i < e; i++) {
                SRef &r = root->refs[i];
                r.prim = i;
                r.box.reset();
                for (int k = 0; k < 3; k++) r.box.grow(vtx(i, k));
                tb[t].grow(r.box);
            }
        });
        root->box.reset();
        for (int t = 0; t < threads_; t++) root->box.grow(tb[t]);
        root_area_ = root->box.area();
        root->depth = 0;
        root->node = alloc_node();
        const uint32_t r = root->node;
        submit(std::move(root));
        drain();
        flatten(r, out);
    }

    const float *vtx(uint32_t prim, int k) const {
        return &in_.vertices[3 * (size_t)in_.indices[3 * (size_t)prim + k]];
    }

    // Clip reference r at plane `s` of `axis` (TriangleHandle::split): the parts of the triangle on
    // either side, intersected with r's box; crossing points rounded outward.
    void split_ref(const SRef &r, int axis, float s, SRef &l, SRef &rr) const {
        Box lb, rb;
        lb.reset();
        rb.reset();
        for (int i = 0; i < 3; i++) {
            const float *v0 = vtx(r.prim, i), *v1 = vtx(r.prim, (i + 1) % 3);
            const double p0 = v0[axis], p1 = v1[axis];
            if (p0 <= s) lb.grow(v0);
            if (p0 >= s) rb.grow(v0);
            if ((p0 < s && p1 > s) || (p1 < s && p0 > s)) {
                const double t = std::max(0.0, std::min(1.0, (s - p0) / (p1 - p0)));
                float lo[3], hi[3];
                for (int k = 0; k < 3; k++) {
                    const double q = (double)v0[k] + t * ((double)v1[k] - (double)v0[k]);
                    lo[k] = round_down(q);
                    hi[k] = round_up(q);
                }
                lo[axis] = hi[axis] = s;
                lb.grow(lo); lb.grow(hi);
                rb.grow(lo); rb.grow(hi);
            }
        }
        lb.hi[axis] = std::min(lb.hi[axis], s);
        rb.lo[axis] = std::max(rb.lo[axis], s);
        l.prim = rr.prim = r.prim;
        l.box = box_and(lb, r.box);
        rr.box = box_and(rb, r.box);
    }

    void sbvh_leaf(BNode &nd, const STask &t) {
        const uint32_t c = (uint32_t)t.refs.size();
        const uint64_t first = leaf_cursor_.fetch_add(c);
        if (first + c > ref_cap_) throw std::runtime_error("bvh: reference budget exceeded");
        for (uint32_t i = 0; i < c; i++) ref_[first + i] = t.refs[i].prim;
        nd.leaf = true;
        nd.first = (uint32_t)first;
        nd.count = c;
        nd.box = t.box;
    }

    static void centroid(const Box &b, float *c) {
        for (int k = 0; k < 3; k++) c[k] = 0.5f * b.lo[k] + 0.5f * b.hi[k];
    }

    void build_sbvh(STask t) {
        while (true) {
            BNode &nd = nodes_[t.node];
            nd.box = t.box;
            const uint32_t n = (uint32_t)t.refs.size();
            if (n <= 1 || (t.depth >= AKR_BVH_MAX_DEPTH - 2 && n <= (uint32_t)max_leaf_)) {
                sbvh_leaf(nd, t);
                return;
            }
            if (t.depth >= AKR_BVH_MAX_DEPTH - 2) throw std::runtime_error("bvh: depth limit exceeded");
            const int B = bins_;
            const bool par = n >= kParBinMin && threads_ > 1;
            const int T = par ? threads_ : 1;
            // centroid bounds
            Box cb;
            {
                std::vector<Box> tc(T);
                auto f = [&](uint32_t b, uint32_t e, int th) {
                    tc[th].reset();
                    float c[3];
                    for (uint32_t i = b; i < e; i++) {
                        centroid(t.refs[i].box, c);
                        tc[th].grow(c);
                    }
                };
                if (par) parallel_chunks(0, n, f); else f(0, n, 0);
                cb.reset();
                for (auto &x : tc) cb.grow(x);
            }
            const double parea = t.box.area();
            // object split: binned centroids
            float ks[3];
            for (int a = 0; a < 3; a++) {
                const float ext = cb.hi[a] - cb.lo[a];
                ks[a] = ext > 0 ? (float)B * (1.0f - 1e-6f) / ext : 0.0f;
            }
            auto obin = [&](const SRef &r, int a) {
                float c[3];
                centroid(r.box, c);
                return std::clamp((int)((c[a] - cb.lo[a]) * ks[a]), 0, B - 1);
            };
            std::vector<Bin> ob((size_t)T * 3 * kMaxBins);
            {
                auto f = [&](uint32_t b, uint32_t e, int th) {
                    Bin *lb = &ob[(size_t)th * 3 * kMaxBins];
                    for (int i = 0; i < 3 * kMaxBins; i++) lb[i].reset();
                    for (uint32_t i = b; i < e; i++)
                        for (int a = 0; a < 3; a++) {
                            if (!(ks[a] > 0)) continue;
                            Bin &x = lb[a * kMaxBins + obin(t.refs[i], a)];
                            x.n++;
                            x.box.grow(t.refs[i].box);
                        }
                };
                if (par) parallel_chunks(0, n, f); else f(0, n, 0);
                for (int th = 1; th < T; th++)
                    for (int i = 0; i < 3 * kMaxBins; i++) {
                        ob[i].n += ob[(size_t)th * 3 * kMaxBins + i].n;
                        ob[i].box.grow(ob[(size_t)th * 3 * kMaxBins + i].box);
                    }
            }
            int oaxis = -1, osplit = -1;
            double obest = std::numeric_limits<double>::infinity();
            Box ooverlap;
            ooverlap.reset();
            for (int a = 0; a < 3; a++) {
                if (!(ks[a] > 0)) continue;
                const Bin *bn = &ob[a * kMaxBins];
                double rarea[kMaxBins];
                uint32_t rcnt[kMaxBins];
                Box rbox[kMaxBins];
                Box acc;
                acc.reset();
                uint32_t c = 0;
                for (int b = B - 1; b > 0; b--) {
                    acc.grow(bn[b].box);
                    c += bn[b].n;
                    rarea[b] = acc.area();
                    rcnt[b] = c;
                    rbox[b] = acc;
                }
                acc.reset();
                c = 0;
                for (int b = 0; b < B - 1; b++) {
                    acc.grow(bn[b].box);
                    c += bn[b].n;
                    if (c == 0 || rcnt[b + 1] == 0) continue;
                    const double cost = acc.area() * c + rarea[b + 1] * rcnt[b + 1];
                    if (cost < obest) {
                        obest = cost;
                        oaxis = a;
                        osplit = b;
                        ooverlap = box_and(acc, rbox[b + 1]);
                    }
                }
            }
            // spatial split, like the reference: depth <= 40, object children overlapping
            int saxis = -1;
            float splane = 0.0f;
            double sbest = std::numeric_limits<double>::infinity();
            bool try_spatial = t.depth <= 40 && refs_total_.load() < ref_cap_ && parea > 0;
            if (try_spatial && oaxis >= 0)
                try_spatial = !box_empty(ooverlap) && ooverlap.area() / root_area_ > alpha_;
            if (try_spatial) {
                struct SBin {
                    Box box;
                    uint32_t enter, exit;
                };
                std::vector<SBin> sb((size_t)T * 3 * kMaxBins);
                float planes[3][kMaxBins];
                bool ok[3];
                for (int a = 0; a < 3; a++) {
                    const double lo = t.box.lo[a], ext = (double)t.box.hi[a] - lo;
                    ok[a] = ext > 0;
                    for (int j = 0; j < B - 1; j++) planes[a][j] = (float)(lo + ext * (j + 1) / B);
                }
                auto f = [&](uint32_t b, uint32_t e, int th) {
                    SBin *lb = &sb[(size_t)th * 3 * kMaxBins];
                    for (int i = 0; i < 3 * kMaxBins; i++) {
                        lb[i].box.reset();
                        lb[i].enter = lb[i].exit = 0;
                    }
                    for (uint32_t i = b; i < e; i++) {
                        const SRef &r = t.refs[i];
                        for (int a = 0; a < 3; a++) {
                            if (!ok[a]) continue;
                            const float *pl = planes[a];
                            // first / last bin the reference's box touches (bins are [p_{j-1}, p_j])
                            int first = (int)(std::upper_bound(pl, pl + B - 1, r.box.lo[a]) - pl);
                            int last = (int)(std::lower_bound(pl, pl + B - 1, r.box.hi[a]) - pl);
                            if (last < first) last = first;
                            SRef cur = r, L, R;
                            for (int j = first; j < last; j++) {
                                split_ref(cur, a, pl[j], L, R);
                                if (!box_empty(L.box)) lb[a * kMaxBins + j].box.grow(L.box);
                                cur = R;
                            }
                            if (!box_empty(cur.box)) lb[a * kMaxBins + last].box.grow(cur.box);
                            lb[a * kMaxBins + first].enter++;
                            lb[a * kMaxBins + last].exit++;
                        }
                    }
                };
                if (par) parallel_chunks(0, n, f); else f(0, n, 0);
                for (int th = 1; th < T; th++)
                    for (int i = 0; i < 3 * kMaxBins; i++) {
                        const SBin &x = sb[(size_t)th * 3 * kMaxBins + i];
                        sb[i].box.grow(x.box);
                        sb[i].enter += x.enter;
                        sb[i].exit += x.exit;
                    }
                for (int a = 0; a < 3; a++) {
                    if (!ok[a]) continue;
                    const SBin *bn = &sb[a * kMaxBins];
                    double rarea[kMaxBins];
                    uint32_t rcnt[kMaxBins];
                    Box acc;
                    acc.reset();
                    uint32_t c = 0;
                    for (int b = B - 1; b > 0; b--) {
                        acc.grow(bn[b].box);
                        c += bn[b].exit;
                        rarea[b] = acc.area();
                        rcnt[b] = c;
                    }
                    acc.reset();
                    c = 0;
                    for (int b = 0; b < B - 1; b++) {
                        acc.grow(bn[b].box);
                        c += bn[b].enter;
                        if (c == 0 || rcnt[b + 1] == 0) continue;
                        const double cost = acc.area() * c + rarea[b + 1] * rcnt[b + 1];
                        if (cost < sbest) {
                            sbest = cost;
                            saxis = a;
                            splane = planes[a][b];
                        }
                    }
                }
            }
            const bool use_spatial = saxis >= 0 && sbest < obest;
            const double best = use_spatial ? sbest : obest;
            if (n <= (uint32_t)max_leaf_ &&
                ((oaxis < 0 && saxis < 0) || ci_ * (double)n <= ct_ + ci_ * best / (parea > 0 ? parea : 1.0))) {
                sbvh_leaf(nd, t);
                return;
            }
            auto lt = std::make_shared<STask>(), rt = std::make_shared<STask>();
            int axis = -1;
            if (use_spatial) {
                axis = saxis;
                std::vector<SRef> mid;
                Box B1, B2;
                B1.reset();
                B2.reset();
                for (const SRef &r : t.refs) {
                    if (r.box.hi[axis] <= splane) {
                        lt->refs.push_back(r);
                        B1.grow(r.box);
                    } else if (r.box.lo[axis] >= splane) {
                        rt->refs.push_back(r);
                        B2.grow(r.box);
                    } else {
                        mid.push_back(r);
                    }
                }
                // straddling references: split, or kept whole on one side when that is cheaper
                // (the reference's unsplitting test); splits draw on the reference budget
                uint64_t want = mid.size();
                uint64_t before = refs_total_.fetch_add(want);
                const bool may_split = before + want <= ref_cap_;
                uint64_t added = 0;
                for (const SRef &r : mid) {
                    SRef L, R;
                    split_ref(r, axis, splane, L, R);
                    const double N1 = (double)lt->refs.size() + 1, N2 = (double)rt->refs.size() + 1;
                    Box b1 = B1, b2 = B2;
                    b1.grow(r.box);
                    b2.grow(r.box);
                    const double csplit = B1.area() * N1 + B2.area() * N2;
                    const double c1 = b1.area() * N1 + B2.area() * (N2 - 1);
                    const double c2 = B1.area() * (N1 - 1) + b2.area() * N2;
                    const bool le = box_empty(L.box), re = box_empty(R.box);
                    if (may_split && !le && !re && csplit < std::min(c1, c2)) {
                        lt->refs.push_back(L);
                        rt->refs.push_back(R);
                        B1.grow(L.box);
                        B2.grow(R.box);
                        added++;
                    } else if (re || (!le && c1 <= c2)) {
                        lt->refs.push_back(r);
                        B1 = b1;
                    } else {
                        rt->refs.push_back(r);
                        B2 = b2;
                    }
                }
                refs_total_.fetch_sub(want - added);
                lt->box = B1;
                rt->box = B2;
            }
            if (!use_spatial || lt->refs.empty() || rt->refs.empty()) {
                lt->refs.clear();
                rt->refs.clear();
                lt->box.reset();
                rt->box.reset();
                if (oaxis >= 0) {
                    axis = oaxis;
                    for (const SRef &r : t.refs) {
                        STask &d = obin(r, oaxis) <= osplit ? *lt : *rt;
                        d.refs.push_back(r);
                        d.box.grow(r.box);
                    }
                } else {  // centroids coincide: halve the list
                    if (n <= (uint32_t)max_leaf_) {
                        sbvh_leaf(nd, t);
                        return;
                    }
                    int a = 0;
                    for (int k = 1; k < 3; k++)
                        if (t.box.hi[k] - t.box.lo[k] > t.box.hi[a] - t.box.lo[a]) a = k;
                    axis = a;
                    for (uint32_t i = 0; i < n; i++) {
                        STask &d = i < n / 2 ? *lt : *rt;
                        d.refs.push_back(t.refs[i]);
                        d.box.grow(t.refs[i].box);
                    }
                }
            }
            if (lt->refs.empty() || rt->refs.empty()) throw std::runtime_error("bvh: empty partition");
            std::vector<SRef>().swap(t.refs);
            nd.leaf = false;
            nd.axis = (uint8_t)axis;
            nd.left = alloc_node();
            nd.right = alloc_node();
            lt->node = nd.left;
            rt->node = nd.right;
            lt->depth = rt->depth = t.depth + 1;
            std::shared_ptr<STask> big = lt->refs.size() >= rt->refs.size() ? lt : rt;
            std::shared_ptr<STask> small = big == lt ? rt : lt;
            if (big->refs.size() >= kTaskMin) {
                submit(big);
                t = std::move(*small);
            } else {
                build_sbvh(std::move(*small));
                t = std::move(*big);
            }
        }
    }

    // ---------------------------------------------------------------- output
    uint32_t emit(uint32_t bi, BvhOutput &out, int depth, double root_area) {
        const BNode &b = nodes_[bi];
        out.max_depth = std::max(out.max_depth, depth);
        if (b.leaf) {
            uint32_t first = (uint32_t)out.tris.size();
            if (first >= (1u << 28)) throw std::runtime_error("bvh: too many triangle records");
            for (uint32_t i = b.first; i < b.first + b.count; i++) {
                uint32_t g = ref_[i];
                const float *v0 = &in_.vertices[3 * (size_t)in_.indices[3 * (size_t)g + 0]];
                const float *v1 = &in_.vertices[3 * (size_t)in_.indices[3 * (size_t)g + 1]];
                const float *v2 = &in_.vertices[3 * (size_t)in_.indices[3 * (size_t)g + 2]];
                akr_bvh_tri tr;
                std::memset(&tr, 0, sizeof(tr));
                for (int k = 0; k < 3; k++) {
                    tr.v0[k] = v0[k];
                    tr.e1[k] = v1[k] - v0[k];  // instance.h:49
                    tr.e2[k] = v2[k] - v0[k];  // instance.h:50
                }
                tr.gid = g;
                out.tris.push_back(tr);
            }
            out.max_leaf = std::max(out.max_leaf, (int)b.count);
            out.sah_cost += ci_ * (double)b.count * (root_area > 0 ? b.box.area() / root_area : 1.0);
            return AKR_CHILD_LEAF | (first << 3) | (b.count - 1);
        }
        out.sah_cost += ct_ * (root_area > 0 ? b.box.area() / root_area : 1.0);
        uint32_t idx = (uint32_t)out.nodes.size();
        out.nodes.emplace_back();
        uint32_t l = emit(b.left, out, depth + 1, root_area);
        uint32_t r = emit(b.right, out, depth + 1, root_area);
        akr_bvh_node &o = out.nodes[idx];
        std::memset(&o, 0, sizeof(o));
        const Box &lb = nodes_[b.left].box, &rb = nodes_[b.right].box;
        o.bxy0[0] = lb.lo[0]; o.bxy0[1] = lb.hi[0]; o.bxy0[2] = lb.lo[1]; o.bxy0[3] = lb.hi[1];
        o.bxy1[0] = rb.lo[0]; o.bxy1[1] = rb.hi[0]; o.bxy1[2] = rb.lo[1]; o.bxy1[3] = rb.hi[1];
        o.bz[0] = lb.lo[2]; o.bz[1] = lb.hi[2]; o.bz[2] = rb.lo[2]; o.bz[3] = rb.hi[2];
        o.child[0] = l;
        o.child[1] = r;
        o.axis = b.axis;
        return idx;
    }

    void flatten(uint32_t root, BvhOutput &out) {
        out.nodes.clear();
        out.tris.clear();
        out.nodes.reserve(next_node_.load() / 2 + 2);
        out.tris.reserve(sbvh_ ? leaf_cursor_.load() : n_);
        out.nodes.push_back(empty_vroot());
        const Box &rb = nodes_[root].box;
        double ra = rb.area();
        uint32_t c = emit(root, out, 1, ra);
        akr_bvh_node &v = out.nodes[0];
        v.bxy0[0] = rb.lo[0]; v.bxy0[1] = rb.hi[0]; v.bxy0[2] = rb.lo[1]; v.bxy0[3] = rb.hi[1];
        v.bz[0] = rb.lo[2]; v.bz[1] = rb.hi[2];
        v.child[0] = c;
        v.child[1] = AKR_CHILD_EMPTY;
        v.axis = 0;
    }

    const BvhInput &in_;
    uint32_t n_ = 0;
    int threads_ = 1, bins_ = 32, max_leaf_ = 4;
    float ct_ = 1, ci_ = 1;
    std::vector<Box> pbox_;
    std::vector<float> cen_;
    std::vector<uint32_t> ref_;
    std::vector<BNode> nodes_;
    std::atomic<uint32_t> next_node_{0};
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Job> queue_;
    // SBVH state
    bool sbvh_ = false;
    float budget_ = 0.5f;                    // spatial splits may add up to budget_ * n references
    double alpha_ = 1e-5;                    // spatial splits only where object children overlap more
                                             // (the reference's alpha; 1e-6 / 1e-7 measured the same)
    uint64_t ref_cap_ = 0;
    std::atomic<uint64_t> refs_total_{0}, leaf_cursor_{0};
    double root_area_ = 0;
    int64_t pending_ = 0;
    std::string error_;
};

}  // namespace

void build_bvh(const BvhInput &in, const akr_build_params &params, BvhOutput &out) {
    auto t0 = std::chrono::steady_clock::now();
    out = BvhOutput();
    if (in.n_tris >= (1ull << 31)) throw std::runtime_error("bvh: too many triangles");
    Builder b(in, params);
    b.run(out);
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace akr
