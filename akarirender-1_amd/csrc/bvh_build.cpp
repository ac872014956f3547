// bvh_build.cpp — task-parallel binned-SAH BVH2 builder (see bvh_build.h).
#include "bvh_build.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
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

class Builder {
  public:
    Builder(const BvhInput &in, const akr_build_params &p) : in_(in) {
        n_ = (uint32_t)in.n_tris;
        threads_ = p.n_threads > 0 ? p.n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
        bins_ = std::clamp(p.n_bins > 0 ? p.n_bins : 32, 2, kMaxBins);
        max_leaf_ = std::clamp(p.max_leaf_size > 0 ? p.max_leaf_size : 4, 1, AKR_LEAF_MAX);
        ct_ = p.traversal_cost > 0 ? p.traversal_cost : 1.0f;
        ci_ = p.intersect_cost > 0 ? p.intersect_cost : 4.0f;
    }

    void run(BvhOutput &out) {
        if (n_ == 0) {
            out.nodes.assign(1, empty_vroot());
            out.tris.clear();
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
        std::vector<std::thread> ts;
        uint32_t chunk = (n + T - 1) / T;
        for (int t = 0; t < T; t++) {
            uint32_t cb = b + t * chunk, ce = std::min(e, cb + chunk);
            if (cb >= ce) break;
            ts.emplace_back([&, cb, ce, t] { f(cb, ce, t); });
        }
        for (auto &t : ts) t.join();
    }

    uint32_t alloc_node() {
        uint32_t i = next_node_.fetch_add(1);
        if (i >= nodes_.size()) throw std::runtime_error("bvh: node pool exhausted");
        return i;
    }

    // ---------------------------------------------------------------- task pool
    void submit(const Task &t) {
        std::lock_guard<std::mutex> g(mu_);
        queue_.push_back(t);
        pending_++;
        cv_.notify_one();
    }
    void drain() {
        std::vector<std::thread> ws;
        for (int i = 0; i < threads_; i++) ws.emplace_back([this] { worker(); });
        for (auto &w : ws) w.join();
        if (!error_.empty()) throw std::runtime_error(error_);
    }
    void worker() {
        while (true) {
            Task t;
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return !queue_.empty() || pending_ == 0; });
                if (queue_.empty()) return;
                t = queue_.back();
                queue_.pop_back();
            }
            try {
                build(t);
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
        std::vector<std::thread> ts;
        uint32_t chunk = (n + threads_ - 1) / threads_;
        int used = 0;
        for (int th = 0; th < threads_; th++) {
            uint32_t cb = t.begin + th * chunk, ce = std::min(t.end, cb + chunk);
            if (cb >= ce) break;
            used++;
            ts.emplace_back([&, cb, ce, th] { work(cb, ce, at(th)); });
        }
        for (auto &x : ts) x.join();
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
        out.tris.reserve(n_);
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
    std::deque<Task> queue_;
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
