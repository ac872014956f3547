// capi.hip — implementation of the C-ABI boundary declared in include/akr_hip.h.
//
// One context = one device + one stream.  Scene arrays are staged on the host, flattened across
// meshes (global triangle id = mesh base + prim id) and uploaded once; the BVH is built on the
// host (bvh_build.cpp) and uploaded.  akr_hip_render runs the wavefront pipeline
// raygen -> {closest-hit -> shade -> shadow}^depth -> splat once per sample pass, entirely on
// the stream (no host synchronisation inside a render; queue counts live in device memory).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "akr_device.h"
#include "bvh_build.h"
#include "kernels.h"

using namespace akr;

#define HIPCHK(x)                                                                                        \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + " failed: " + hipGetErrorString(e_)); \
    } while (0)

namespace {

template <class T>
struct DBuf {
    T *p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf &) = delete;
    DBuf &operator=(const DBuf &) = delete;
    ~DBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void reserve(size_t count) {
        if (count <= n && p) return;
        release();
        size_t c = std::max<size_t>(count, 1);
        HIPCHK(hipMalloc(reinterpret_cast<void **>(&p), c * sizeof(T)));
        n = c;
    }
    void upload(const T *h, size_t count, hipStream_t st) {
        reserve(count);
        if (count) HIPCHK(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, st));
    }
};

struct Stat {
    uint64_t launches = 0;
    double total = 0, mn = 1e30, mx = 0;
};

// Camera (restated from core/nodes/camera.cpp:26-52 and kernel/camera.h:45-59)
struct M4 {
    float m[4][4];
};
M4 m_ident() {
    M4 r{};
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.0f;
    return r;
}
M4 m_from(const float (&a)[16]) {
    M4 r;
    for (int i = 0; i < 16; i++) r.m[i / 4][i % 4] = a[i];
    return r;
}
M4 m_mul(const M4 &a, const M4 &b) {  // Matrix::operator*, math.h:93-101 (sequential dot)
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
float hsinf(float x) { return (float)std::sin((double)x); }
float hcosf(float x) { return (float)std::cos((double)x); }
M4 m_scale(float x, float y, float z) { return m_from({x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0, 0, 0, 0, 1}); }
M4 m_translate(float x, float y, float z) { return m_from({1, 0, 0, x, 0, 1, 0, y, 0, 0, 1, z, 0, 0, 0, 1}); }
M4 m_rx(float t) { float s = hsinf(t), c = hcosf(t); return m_from({1, 0, 0, 0, 0, c, -s, 0, 0, s, c, 0, 0, 0, 0, 1}); }
M4 m_ry(float t) { float s = hsinf(t), c = hcosf(t); return m_from({c, 0, s, 0, 0, 1, 0, 0, -s, 0, c, 0, 0, 0, 0, 1}); }
M4 m_rz(float t) { float s = hsinf(t), c = hcosf(t); return m_from({c, -s, 0, 0, s, c, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}); }

CameraDev make_camera(const akr_camera &c) {
    const float pi = 3.1415926535897932384f;
    if (c.resolution[0] <= 0 || c.resolution[1] <= 0 || c.resolution[0] > 65535 || c.resolution[1] > 65535)
        throw std::runtime_error("camera resolution must be in [1, 65535]");
    CameraDev cam;
    cam.width = c.resolution[0];
    cam.height = c.resolution[1];
    float rx = c.rotation_deg[0] * pi / 180.0f, ry = c.rotation_deg[1] * pi / 180.0f, rz = c.rotation_deg[2] * pi / 180.0f;
    M4 c2w = m_rz(rz);
    c2w = m_mul(m_rx(ry), c2w);
    c2w = m_mul(m_ry(rx), c2w);
    c2w = m_mul(m_translate(c.position[0], c.position[1], c.position[2]), c2w);
    float fov = (float)(c.fov_deg * (double)pi / 180.0);
    M4 m = m_ident();
    m = m_mul(m_scale(1.0f / cam.width, 1.0f / cam.height, 1), m);
    m = m_mul(m_scale(2, 2, 1), m);
    m = m_mul(m_translate(-1, -1, 0), m);
    m = m_mul(m_scale(1, -1, 1), m);
    float s = (float)std::atan((double)(fov / 2));  // atan, not tan (camera.h:51)
    if (cam.width > cam.height)
        m = m_mul(m_scale(s, s * float(cam.height) / cam.width, 1), m);
    else
        m = m_mul(m_scale(s * float(cam.width) / cam.height, s, 1), m);
    for (int i = 0; i < 16; i++) {
        cam.r2c[i] = m.m[i / 4][i % 4];
        cam.c2w[i] = c2w.m[i / 4][i % 4];
    }
    return cam;
}

// Mapped host words written by kernels (k_store_word) are set to this by the host before the
// store is issued.  The host never acts on a value it has not seen change from the sentinel, so a
// stale read (a store not yet visible when the event it waited on completed, or a value left by an
// earlier render) can only delay a decision, never make a wrong one.
constexpr uint32_t kMappedSentinel = 0xFFFFFFFFu;

// Waits (up to ~2 s) until a mapped word no longer holds the sentinel; returns the sentinel if it
// never changes.
uint32_t read_mapped(const volatile uint32_t *p) {
    const auto t0 = std::chrono::steady_clock::now();
    while (true) {
        const uint32_t v = *p;
        if (v != kMappedSentinel) return v;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) return kMappedSentinel;
        std::this_thread::yield();
    }
}

}  // namespace

struct akr_hip_ctx {
    int device = 0;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    std::string err;
    // Every trace / render of a context is ordered after the previous one, whatever streams the
    // caller passes: they share the refill counters, the overflow stacks and the queues.
    hipEvent_t ev_done = nullptr;
    bool done_recorded = false;
    // In-band check that every slot of a render's film holds exactly spp samples (option "verify",
    // default on): device counter + mapped host word
    bool verify = true;
    DBuf<uint32_t> d_bad;
    uint32_t *h_check = nullptr, *d_check_host = nullptr;
    // Fault word (mapped, coherent host memory): a persistent kernel's hang guard sets it
    // (k_path_defer).  Checked after every render on the host, whatever "verify" says.
    uint32_t *h_fault = nullptr, *d_fault_host = nullptr;
    // Test-only per-slot fingerprint of the last render (option "pixel_probe", akr_pixel_probe)
    bool probe = false;
    bool fault_test = false;  // option "fault_test": k_path_defer raises the fault word once (tests)
    bool probe_clock = false; // option "pixel_probe" 2: completion times in the probe (counting build, diagnostic)
    DBuf<uint4> d_probe;
    uint64_t probe_n = 0;
    bool probe_ok = false;

    // host staging (flattened over meshes)
    std::vector<float> verts;
    std::vector<int32_t> idx;
    std::vector<float> normals, texcoords;
    std::vector<int32_t> matid;
    std::vector<uint32_t> mesh_base{0};
    std::vector<akr_texture> texs;
    std::vector<akr_material> mats;
    std::vector<float> images;
    std::vector<int64_t> img_off;
    std::vector<int32_t> img_w, img_h;
    std::vector<akr_area_light> lights;
    std::vector<float> power;
    bool scene_dirty = true;
    bool accel_built = false;
    akr_accel_info info{};
    BvhOutput bvh;
    Bvh4Output bvh4;

    // device scene
    DBuf<akr_bvh_node> d_nodes;
    DBuf<akr_bvh4_node> d_wnodes;
    DBuf<float4> d_wleaves;          // leaf blob (see TraceArgs::wide_leaves)
    uint32_t wide_root_dev = AKR_CHILD_EMPTY;
    uint64_t bvh_dev_bytes = 0;       // the uploaded wide nodes + leaf blob
    DBuf<float4> d_tris;
    DBuf<ShadeTri> d_shade_tri;
    DBuf<float> d_tc, d_images, d_cdf, d_func;
    DBuf<MatDev> d_mats;
    DBuf<TexDev> d_texs;
    DBuf<LightDev> d_lights;
    DBuf<uint32_t> d_mesh_base;
    float func_int = 0;
    int32_t n_lights = 0;
    int32_t n_mats = 0;
    bool has_image_tex = false;
    bool simple_shading = true;  // every material Diffuse / Emissive with constant textures

    CameraDev cam{};
    bool cam_set = false;

    // path / queue buffers
    size_t cap = 0;
    // The last render's tile list, clipped, non-empty tiles only: (x0, y0, width, first slot).  The
    // pixel list is expanded from it on the device (k_expand_pixels); the host copy h_pixel is built
    // only for the host-side merges that need it (host_pixels()).
    std::vector<uint4> h_tiles;
    uint64_t n_pix_last = 0;
    DBuf<uint4> d_tiles;
    std::vector<uint32_t> h_pixel;
    bool h_pixel_ok = false;
    DBuf<uint32_t> d_pixel, d_seed, d_slot0, d_slot1, d_counts;
    DBuf<float4> d_ray0, d_ray1, d_state0, d_state1, d_hit, d_film;
    DBuf<float4> d_L[2];  // per-sample radiance, alternating by sample pass (passes overlap)
    DBuf<float4> d_sray[2], d_scolor[2];  // shadow queues, alternating by bounce
    DBuf<uint32_t> d_ao_slot[2];          // AO queues traced closest-hit (finite occlude): slots
    int last_passes = 0;
    int32_t last_form = AKR_FORM_NONE, last_ordered = 0;  // akr_hip_render_form
    // Shadow traces run on a second stream, so the shadow trace of bounce b overlaps the closest-hit
    // trace of bounce b+1 (independent work): each persistent launch's tail is filled by the other.
    // Both internal: `main` (high priority) runs raygen / closest-hit / shade, `side` (low priority)
    // runs shadow traces and splat, so the last shadow trace and splat of sample pass s overlap
    // raygen and the first closest-hit trace of pass s + 1.
    hipStream_t main_st = nullptr, side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_join_main = nullptr, ev_shade[2] = {nullptr, nullptr},
               ev_shadow[2] = {nullptr, nullptr}, ev_splat[2] = {nullptr, nullptr};
    DBuf<uint2> d_ovf, d_ovf_side;  // traversal stack overflow: main-stream and side-stream traces
    DBuf<uint32_t> d_work;  // dynamic-fetch counters of a standalone trace launch (kTraceWords)
    uint32_t ovf_threads = 0;
    uint32_t trace_grid[3] = {0, 0, 0};
    uint32_t path_grid[3][2] = {{0, 0}, {0, 0}, {0, 0}};  // resident workgroups of the persistent path kernels [kind][tab]
    // The render form of a constant-shading scene.  A "tail form"
    // (k_path_spec, or k_path_defer when path_spec is 0) pays where k_path's launch would end on a few
    // long pixel chains while most lanes idle: few pixels per resident lane, and many pixels whose
    // paths end at once (the camera ray leaves the scene), whose lanes then free up early.  Both come
    // from the render itself: pixels per resident lane from the occupancy query, the share of camera
    // rays that miss from the cost-ordering pilot (which marks them).  A render without a pilot
    // (below the order's spp floor, or path_order 0) runs k_path.
    // option "path_defer": 1 = k_path_defer (max_depth <= 8), 0 = k_path, 2 (default) = the rule above
    int path_defer = 2;
    // option "path_spec": k_path_spec (lanes left idle by the drained pixel queue run
    // later samples of a busy pixel from guessed sampler states; committed in order, bit-exact):
    // 1 = always, 0 = never (the rule's tail form is then k_path_defer), 2 (default) = the tail form
    // when path_defer is 2.  Measured on C3 at 1040 spp: 8-way share 0.89 -> 0.83 ms per spp against
    // k_path_defer, 2-way 2.55 -> 2.48 against k_path, the whole frame 5 % slower (profiles/r19_spec_*.log)
    int path_spec = 2;
    // option "path_tail_ppl10": tail forms only at most path_tail_ppl10 / 10 pixels per resident lane
    // (default 6.0).  1080p C3 on one MI355X: the whole frame has 7.9 pixels per lane (k_path 4.61 ms
    // against 4.85 for k_path_spec), a 2-way share 4.0 (2.55 against 2.48)
    int64_t path_tail_ppl10 = 60;
    // option "path_tail_steps": ... and a cost-ordering pilot whose camera rays take at least this many
    // traversal steps (wide-node visits + triangle tests) on average: long dependent-fetch chains, where
    // a lane freed early can run work that overlaps them (DESIGN.md §3.12 gives the measured means of
    // the soup's and the Cornell box's shares; the box's rays are a few steps long, its shares run k_path)
    int path_tail_steps = 12;
    // option "path_cache_mb": a BVH of at most this many MiB on the device (wide nodes + leaf blob) is
    // taken as cache-resident (half the 256-MiB Infinity Cache: the kernel streams its film and rays
    // beside it, MI355X_MICROARCH.md §Infinity Cache): its rule form is k_path_defer at every size
    // (the SBVH of a 100K-triangle soup is 10.7 MiB and of a 1M soup 109.8 MiB: both cache-resident,
    // k_path_defer 4-20 % faster than k_path there; the 10M soup's 1.5 GB tree takes k_path_spec on
    // rank shares)
    int64_t path_cache_mb = 128;
    // explicit overrides of the rule's size test (0, default: pixels per lane): a tail form for renders
    // of at most this many pixels (options "path_spec_pixels", "path_defer_pixels"); option
    // "path_defer_min_tris" (0, default: no test) keeps scenes below it on k_path
    int64_t path_spec_pixels = 0;
    int64_t path_defer_pixels = 0;
    int64_t path_defer_min_tris = 0;
    int path_spec_fetch = 3;   // option "path_spec_fetch": k_path_spec's ordered fetch, FETCH_STRIDE (3); -1 = the path_order_pair rule
    // ... for renders of at most 1.5 pixels per resident lane (the 8-way share) or, when set, at most
    // path_spec_fetch_pixels pixels; larger ones (2- and 4-way) take the path_order_pair rule: 2.500 /
    // 1.399 ms against 2.526 / 1.403 strided (profiles/r20_spec_fetch_ab.log)
    int64_t path_spec_fetch_pixels = 0;
    int path_spec_depth = 3;   // option "path_spec_depth": samples in flight beyond a pixel's head (1-3, the
                               // speculation tree's levels; the r19 main line measured 2, 4, 8, 15 alike, 1 slower,
                               // profiles/r19_spec_depth.log)
    // the last render's form inputs (akr_hip_render_form_inputs): pixels per lane x 1000, the pilot's
    // rays and their summed steps
    int64_t last_ppl1000 = 0, last_pilot_rays = -1, last_pilot_steps = -1;
    DBuf<unsigned long long> d_steps_sum;   // the pilot's summed steps
    DBuf<uint32_t> d_gate;                  // k_pick_form's choice between the two launched forms
    // the last render launched two gated forms (gate_forms[gate]) / read the pilot's step sum on the
    // device: resolved on the host by resolve_form() when the form or its inputs are queried
    bool form_pending = false, pilot_sum_pending = false;
    int32_t gate_forms[2] = {AKR_FORM_NONE, AKR_FORM_NONE};
    bool path_mix = true;     // option "path_mix": k_path_defer fetches pixels in scrambled order
    bool path_tab = true;     // option "path_tab": persistent kernels read the scene tables from an LDS copy
    // option "path_order": cost-ordered pixel fetch: a pilot camera ray per pixel
    // ranks the pixels, and each XCD shard hands out its costliest pixels first, so a launch ends on
    // cheap ones (in k_path_defer it replaces the scrambled fetch).  2 (default) = both persistent
    // kernels, 1 = k_path only, 0 = off; renders of at least path_order_min_spp samples only (the
    // pilot costs about one third of a sample pass); classes
    // of 2^path_order_shift pilot steps.  Measured on C3 at 64 spp: 2- / 4- / 8-way shares 2-5 % faster
    int path_order = 2;
    // option "path_order_pair": the cost-ordered fetch of k_path_defer pairs each shard's costliest
    // pixels with its cheapest inside a wave (lanes done early take the long pixels' shadow rays)
    // instead of costliest-first: 1 = on, 0 = off, 3 = on for k_path too, 2 (default) = on for renders of at most
    // 1.5 pixels per resident lane (the 8-way share of a 1080p frame; measured on C3 at 32 spp, DESIGN.md §3.10: 8-way share 1.007 -> 0.946 ms, 4-way share
    // 1.499 -> 1.548 ms); option "path_prio": waves whose pixels lie in the first path_prio / 256 of
    // a cost-ordered shard run at raised issue priority (0 = off; measured without effect)
    int path_order_pair = 2;
    int path_prio = 0;
    // (16: at the driver's 20 spp the order makes the whole 1080p C3 frame 1.6 % faster, pilot included:
    // 4.905 -> 4.826 ms per spp, three alternating runs each, profiles/r18_order_min_spp_ab.log; it was 64
    // until the leaf phase fetched two triangles with the header)
    int path_order_min_spp = 16;
    // renders of at most path_order_share_pixels pixels (a rank's share of a 2-, 4- or 8-way split)
    // take the order from path_order_share_min_spp samples: the pilot's cost shrinks with the pixel
    // count and the launch tail it shortens does not (C3 at 20 spp, DESIGN.md §3.10: 2- / 4- / 8-way
    // shares 1.5 / 4.5 / 3 % faster with the order, the whole frame unchanged)
    int64_t path_order_share_pixels = 1200000;
    int path_order_share_min_spp = 16;
    int path_order_shift = 2;
    // option "path_order_classes": at most this many cost classes (1..32), the costliest holding every
    // pixel above; fewer classes keep more of the tile order inside a shard (16 since r20: whole frame
    // 4.612 against 4.627 ms per spp, 8-way share 0.803 against 0.808, profiles/r20_order_classes_ab.log)
    int path_order_classes = 16;
    // option "path_order_cap": a pilot ray stops after this many steps (0: none); its cost class is
    // then the cap's.  The pilot is a small latency-bound launch whose length is set by its slowest
    // ray, while the order only needs coarse classes (soup against background).
    int path_order_cap = 64;
    // option "path_order_sub": one pilot ray per 2^path_order_sub slots (neighbours in a tile row
    // share its cost); 0 = a pilot ray per slot
    int path_order_sub = 0;
    // option "path_order_pilot_spp": S > 0 ranks slots by the rays their first S samples take in a
    // counting k_path render (a path pilot; nothing of it reaches the film or the sampler states)
    // instead of one pilot camera ray's steps (0, default)
    int path_order_pilot_spp = 0;
    // option "wave_order": the wavefront's camera rays queued in the cost order (costliest first in
    // each shard of the closest-hit launch), by the same rule and floors as the persistent kernels
    bool wave_order = true;
    DBuf<uint4> d_pprobe;  // the path pilot's per-slot probe
    DBuf<uint32_t> d_okey[2], d_oidx[2], d_owork;
    DBuf<uint8_t> d_otmp;
    DBuf<TraceCounters> d_ocnt;
    bool order_warm = false;
    DBuf<float4> d_contrib;   // k_path_defer: per-lane NEE contributions awaiting their shadow result
    // option "path": 1 = render with k_path, 0 = the wavefront kernels, 2 (default) = k_path when the
    // render has at most path_auto_pixels pixels (default: any size; measured on C3, DESIGN.md §3.8,
    // k_path is 5 % faster than the wavefront on a whole 1080p frame and 19-31 % faster on 2-, 4- and
    // 8-way shares)
    int path_kernel = 2;
    int64_t path_auto_pixels = INT64_MAX;
    bool path_auto_complex = false;  // option "path_auto_complex": auto also takes k_path for complex shading
    bool serial_shadow = false;  // option "serial_shadow": wavefront shadow traces on the main stream (isolated timing)
    bool any_far_first = false;  // option "any_far_first": shadow traversal visits far slots first (measured: more visits on C3)
    // option "path_min_wait": a persistent kernel's wave processes its waiting lanes once this many of
    // 64 wait (scaled to the wave's live lanes); 0 (default) = 40 (measured on C3, DESIGN.md §3.8: with
    // the paired order the 8-way share runs 0.944-0.948 ms at 40, 0.972 at 32, 1.007 at 56)
    int path_min_wait = 0;
    int path_grid_pct = 100;  // option "path_grid_pct": persistent path grid as a percentage of the resident maximum
    DBuf<float4> d_trace_rays;
    DBuf<akr_hit> d_trace_hits;
    // akr_hip_render_node on the lead context: the frame and the staging of other contexts' films
    DBuf<float> d_frame;
    std::vector<std::unique_ptr<DBuf<float4>>> g_film;     // [k]: context k's packed film (staging)
    std::vector<std::unique_ptr<DBuf<uint32_t>>> g_pix;    // [k]: its pixel list
    DBuf<uint32_t> d_gorder;                               // merge orders of overlapping tiles
    hipEvent_t ev_gather = nullptr;  // this context's push to the lead device is done

    // instrumentation
    bool stats = false, count = false;
    bool stats_closest_only = false;  // time trace_closest only (HIP events on every launch cost ~7 % at small ranks)
    bool exact_cull = false;  // true: the reference intersectAABB (no behind-origin cull)
    int rays_per_lane = 1;    // trace grid sizing: at least this many queued rays per lane
    // persistent shadow-trace grid as a percentage of the resident maximum: the shadow trace runs beside
    // the next closest-hit trace, and 75 % leaves it room (wavefront 5.368 / 5.353 ms per spp against
    // 5.400 / 5.389 at 100 %, 5.395 / 5.380 at 50 %; profiles/r20_shadow_grid_ab.log)
    int shadow_grid_pct = 75;
    bool wide = true;         // 4-wide quantized traversal (false: BVH2 kernel only, for A/B)
    bool lean = true;         // fused per-node slot-test arithmetic (kernels.hip visit_wide_lean; false: A/B)
    int wide_collapse = AKR_COLLAPSE_SAH;  // akr_build_params::wide_collapse of the last build
    // option "leaf_align" (taken by the next build or import): each leaf record of the device blob
    // starts on a multiple of this many 16-B words (1 = packed; 8 = a 128-B line, so a leaf of at
    // most two triangles is one fabric request and the leaf phase's eight-load batch never straddles
    // two lines, tools/fetch_calib: a straddling 128-B gather costs 1.4 requests per line)
    int leaf_align = 1;
    bool ray_steps = false;   // diagnostic: standalone traces record per-ray iterations (counted kernel)
    DBuf<uint32_t> d_steps;
    uint64_t n_steps = 0;
    DBuf<TraceCounters> d_counters;
    DBuf<PathProfile> d_pprof;  // k_path counting build: per-wave phase profile
    // option count_lines (counting build, k_path): the bitmap of 128-B lines a render read, and the
    // bit ranges of its three regions (wide nodes, leaf blob, shading records)
    bool count_lines = false;
    DBuf<uint32_t> d_lines;
    uint32_t lines_span[4] = {0, 0, 0, 0};
    std::vector<hipEvent_t> pool;
    struct Pending {
        const char *name;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::map<std::string, Stat> stat;

    ~akr_hip_ctx() {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        for (auto &p : pending) {
            (void)hipEventDestroy(p.a);
            (void)hipEventDestroy(p.b);
        }
        for (auto e : pool) (void)hipEventDestroy(e);
        if (side) (void)hipStreamSynchronize(side);
        if (main_st) (void)hipStreamSynchronize(main_st);
        for (hipEvent_t e : {ev_fork, ev_join, ev_join_main, ev_shade[0], ev_shade[1], ev_shadow[0], ev_shadow[1], ev_splat[0], ev_splat[1]})
            if (e) (void)hipEventDestroy(e);
        if (h_check) (void)hipHostFree(h_check);
        if (h_fault) (void)hipHostFree(h_fault);
        if (ev_done) (void)hipEventDestroy(ev_done);
        if (ev_gather) (void)hipEventDestroy(ev_gather);
        if (main_st) (void)hipStreamDestroy(main_st);
        if (side) (void)hipStreamDestroy(side);
        if (stream) (void)hipStreamDestroy(stream);
    }

    hipEvent_t event() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        return e;
    }

    template <class F>
    void timed(const char *name, hipStream_t st, F &&launch) {
        if (!stats || (stats_closest_only && std::strcmp(name, "trace_closest") != 0 && std::strcmp(name, "path") != 0)) {
            launch();
            return;
        }
        hipEvent_t a = event(), b = event();
        HIPCHK(hipEventRecord(a, st));
        launch();
        HIPCHK(hipEventRecord(b, st));
        pending.push_back({name, a, b});
        if (pending.size() > 4096) flush_stats();
    }

    void flush_stats() {
        for (auto &p : pending) {
            HIPCHK(hipEventSynchronize(p.b));
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
            Stat &s = stat[p.name];
            s.launches++;
            s.total += ms;
            s.mn = std::min(s.mn, (double)ms);
            s.mx = std::max(s.mx, (double)ms);
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
    }

    SceneDev scene_dev() const {
        SceneDev s{};
        s.tri = (decltype(s.tri))d_shade_tri.p;  // device code sees them as global pointers
        s.texcoords = (decltype(s.texcoords))d_tc.p;
        s.has_image_tex = has_image_tex ? 1 : 0;
        s.mats = (decltype(s.mats))d_mats.p;
        s.texs = (decltype(s.texs))d_texs.p;
        s.images = (decltype(s.images))d_images.p;
        s.lights = (decltype(s.lights))d_lights.p;
        s.light_cdf = (decltype(s.light_cdf))d_cdf.p;
        s.n_lights = n_lights;
        s.n_mats = n_mats;
        return s;
    }

    uint64_t n_tris() const { return matid.size(); }

    void commit_scene() {
        if (!scene_dirty) return;
        const uint64_t nt = n_tris();
        // validate references
        for (uint64_t g = 0; g < nt; g++)
            if (matid[g] >= (int32_t)mats.size()) throw std::runtime_error("material index out of range");
        for (size_t m = 0; m < mats.size(); m++) {
            const akr_material &x = mats[m];
            auto tex_ok = [&](int32_t t) { return t >= 0 && t < (int32_t)texs.size(); };
            auto mat_ok = [&](int32_t t) { return t >= 0 && t < (int32_t)mats.size(); };
            bool ok = true;
            if (x.type == AKR_MAT_DIFFUSE || x.type == AKR_MAT_EMISSIVE) ok = tex_ok(x.color);
            else if (x.type == AKR_MAT_GLOSSY) ok = tex_ok(x.color) && tex_ok(x.roughness);
            else if (x.type == AKR_MAT_MIX) ok = tex_ok(x.fraction) && mat_ok(x.first) && mat_ok(x.second);
            else ok = false;
            if (!ok) throw std::runtime_error("material " + std::to_string(m) + " has an invalid type or reference");
        }
        // shading the persistent path kernels run well inline: constant Diffuse / Emissive only
        simple_shading = true;
        for (auto &m : mats) simple_shading = simple_shading && (m.type == AKR_MAT_DIFFUSE || m.type == AKR_MAT_EMISSIVE);
        has_image_tex = false;
        for (auto &t : texs) {
            if (t.type == AKR_TEX_IMAGE && (t.image < 0 || t.image >= (int32_t)img_w.size()))
                throw std::runtime_error("image texture references a missing image");
            has_image_tex = has_image_tex || t.type == AKR_TEX_IMAGE;
        }
        simple_shading = simple_shading && !has_image_tex;
        // one 80-byte shading record per triangle: corners, per-face-vertex normals, material
        std::vector<ShadeTri> st(nt);
        for (uint64_t g = 0; g < nt; g++) {
            const float *v0 = &verts[3 * (size_t)idx[3 * g + 0]];
            const float *v1 = &verts[3 * (size_t)idx[3 * g + 1]];
            const float *v2 = &verts[3 * (size_t)idx[3 * g + 2]];
            const float *nn = &normals[9 * g];
            float mbits;
            std::memcpy(&mbits, &matid[g], 4);
            st[g].a = make_float4(v0[0], v0[1], v0[2], mbits);
            st[g].b = make_float4(v1[0], v1[1], v1[2], nn[0]);
            st[g].c = make_float4(v2[0], v2[1], v2[2], nn[1]);
            st[g].d = make_float4(nn[2], nn[3], nn[4], nn[5]);
            st[g].e = make_float4(nn[6], nn[7], nn[8], 0.0f);
        }
        d_shade_tri.upload(st.data(), st.size(), stream);
        if (has_image_tex) d_tc.upload(texcoords.data(), texcoords.size(), stream);
        // materials with constant textures resolved (MatDev)
        std::vector<MatDev> md(mats.size());
        for (size_t m = 0; m < mats.size(); m++) {
            const akr_material &x = mats[m];
            MatDev &d = md[m];
            std::memset(&d, 0, sizeof(d));
            d.type = x.type;
            d.double_sided = x.double_sided;
            d.first = x.first;
            d.second = x.second;
            d.color_img = d.rough_img = d.frac_img = -1;
            auto resolve = [&](int32_t ti, float *val, int n, int32_t &img) {
                if (ti < 0 || ti >= (int32_t)texs.size()) return;  // unused by this material type
                if (texs[ti].type == AKR_TEX_IMAGE) img = ti;
                else
                    for (int c = 0; c < n; c++) val[c] = texs[ti].value[c];
            };
            if (x.type == AKR_MAT_DIFFUSE || x.type == AKR_MAT_EMISSIVE || x.type == AKR_MAT_GLOSSY)
                resolve(x.color, d.color, 3, d.color_img);
            if (x.type == AKR_MAT_GLOSSY) resolve(x.roughness, &d.rough, 1, d.rough_img);
            if (x.type == AKR_MAT_MIX) resolve(x.fraction, &d.frac, 1, d.frac_img);
        }
        d_mats.upload(md.data(), md.size(), stream);
        n_mats = (int32_t)md.size();
        std::vector<TexDev> td(texs.size());
        for (size_t k = 0; k < texs.size(); k++) {
            const akr_texture &t = texs[k];
            TexDev &d = td[k];
            std::memset(&d, 0, sizeof(d));
            d.type = t.type;
            for (int c = 0; c < 3; c++) d.value[c] = t.value[c];
            if (t.type == AKR_TEX_IMAGE) {
                d.w = img_w[t.image];
                d.h = img_h[t.image];
                d.off = img_off[t.image];
            }
        }
        d_texs.upload(td.data(), td.size(), stream);
        d_images.upload(images.data(), images.size(), stream);
        d_mesh_base.upload(mesh_base.data(), mesh_base.size(), stream);
        // lights: AreaLight records + Distribution1D over `power` (common/distribution.h:46-64)
        std::vector<LightDev> ld;
        for (auto &l : lights) {
            if (l.geom_id < 0 || l.geom_id + 1 >= (int32_t)mesh_base.size())
                throw std::runtime_error("light geom_id out of range");
            uint64_t g = (uint64_t)mesh_base[l.geom_id] + (uint64_t)l.prim_id;
            if (l.prim_id < 0 || g >= mesh_base[l.geom_id + 1]) throw std::runtime_error("light prim_id out of range");
            int32_t m = matid[g];
            if (m < 0 || mats[m].type != AKR_MAT_EMISSIVE) throw std::runtime_error("light triangle is not emissive");
            LightDev x{};
            for (int k = 0; k < 3; k++) {
                const float *v = &verts[3 * (size_t)idx[3 * g + k]];
                x.v[3 * k + 0] = v[0];
                x.v[3 * k + 1] = v[1];
                x.v[3 * k + 2] = v[2];
                x.tc[2 * k + 0] = texcoords[6 * g + 2 * k + 0];
                x.tc[2 * k + 1] = texcoords[6 * g + 2 * k + 1];
            }
            const akr_texture &lt = texs[mats[m].color];
            x.color_img = lt.type == AKR_TEX_IMAGE ? mats[m].color : -1;
            for (int c = 0; c < 3; c++) x.Le[c] = lt.type == AKR_TEX_IMAGE ? 0.0f : lt.value[c];
            // AreaLight::sample's triangle constants (light.h:58-71), in the device's f32 order:
            // lx = cross(v1 - v0, v2 - v0) (math.h:176-181), lng = lx / sqrt(dot(lx, lx)),
            // area_half = sqrt(dot(lx, lx)) * 0.5
            const float e1[3] = {x.v[3] - x.v[0], x.v[4] - x.v[1], x.v[5] - x.v[2]};
            const float e2[3] = {x.v[6] - x.v[0], x.v[7] - x.v[1], x.v[8] - x.v[2]};
            const float lx[3] = {(e1[1] * e2[2]) - (e1[2] * e2[1]), (e1[2] * e2[0]) - (e1[0] * e2[2]),
                                 (e1[0] * e2[1]) - (e1[1] * e2[0])};
            float dd = lx[0] * lx[0];
            dd += lx[1] * lx[1];
            dd += lx[2] * lx[2];
            const float len = std::sqrt(dd);
            for (int c = 0; c < 3; c++) x.lng[c] = lx[c] / len;
            x.area_half = len * 0.5f;
            ld.push_back(x);
        }
        n_lights = (int32_t)ld.size();
        std::vector<float> cdf(ld.size() + 1, 0.0f), func(power.begin(), power.end());
        const size_t n = ld.size();
        for (size_t i = 0; i < n; i++) cdf[i + 1] = cdf[i] + func[i] / n;
        func_int = n ? cdf[n] : 0.0f;
        if (func_int == 0) {
            for (uint32_t i = 1; i < n + 1; ++i) cdf[i] = float(i) / float(n);
        } else {
            for (uint32_t i = 1; i < n + 1; ++i) cdf[i] /= func_int;
        }
        for (size_t i = 0; i < n; i++) ld[i].sel_pdf = func[i] / (func_int * (float)n_lights);  // scene.h:85-89
        d_lights.upload(ld.data(), ld.size(), stream);
        d_cdf.upload(cdf.data(), cdf.size(), stream);
        HIPCHK(hipStreamSynchronize(stream));
        scene_dirty = false;
    }

    void ensure_trace_grid() {
        if (trace_grid[0]) return;
        uint32_t mx = 0;
        for (int m = 0; m < 3; m++) {
            trace_grid[m] = (uint32_t)(n_cu * trace_blocks_per_cu(m));
            mx = std::max(mx, trace_grid[m]);
        }
        for (int d = 0; d < 3; d++)
            for (int t = 0; t < 2; t++) {
                path_grid[d][t] = (uint32_t)(n_cu * path_blocks_per_cu(d, t != 0));
                mx = std::max(mx, path_grid[d][t]);
            }
        ovf_threads = mx * kTraceBlock;
        d_ovf.reserve((size_t)ovf_threads * (kStackMax - kStackLds));
        d_ovf_side.reserve((size_t)ovf_threads * (kStackMax - kStackLds));
        d_work.reserve(kTraceWords);
    }

    void ensure_side_stream() {
        if (side) return;
        int least = 0, greatest = 0;  // numerically lower = higher priority
        HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIPCHK(hipStreamCreateWithPriority(&main_st, hipStreamNonBlocking, greatest));
        HIPCHK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, least));
        for (hipEvent_t *e : {&ev_fork, &ev_join, &ev_join_main, &ev_shade[0], &ev_shade[1], &ev_shadow[0], &ev_shadow[1], &ev_splat[0], &ev_splat[1]})
            HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&h_fault), sizeof(uint32_t),
                             hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&d_fault_host), h_fault, 0));
        *reinterpret_cast<volatile uint32_t *>(h_fault) = 0;
    }

    // A raised fault word fails the call that sees it (and is cleared): the hang guard of a
    // persistent kernel stopped a wave, so that render's film is incomplete.  Called after the host
    // has waited for a render; a render_device without "verify" reports it at the next call.
    void check_fault(const char *which = "the render that raised it") {
        if (!h_fault) return;
        volatile uint32_t *f = reinterpret_cast<volatile uint32_t *>(h_fault);
        if (*f == 0) return;
        *f = 0;
        throw std::runtime_error(std::string("persistent path kernel: a wave stopped on its hang guard; the film of ") +
                                 which + " is incomplete");
    }
    // The last render_device ran without "verify" (no host wait): its fault, if any, is found by the
    // next call, which first waits for that render so the fault is not blamed on its own film.
    bool unchecked_render = false;

    uint32_t grid_for(int mode, uint64_t n) const {
        const uint64_t per_block = (uint64_t)kTraceBlock * (uint64_t)rays_per_lane;
        uint64_t need = (n + per_block - 1) / per_block;
        uint64_t cap = trace_grid[mode];
        if (mode == TRACE_SHADOW) cap = std::max<uint64_t>(1, cap * (uint64_t)shadow_grid_pct / 100);
        return (uint32_t)std::min<uint64_t>(need, cap);
    }

    void ensure_capacity(size_t n) {
        if (n <= cap) return;
        d_pixel.reserve(n);
        d_seed.reserve(n);
        d_slot0.reserve(n);
        d_slot1.reserve(n);
        d_ray0.reserve(2 * n);
        d_ray1.reserve(2 * n);
        d_state0.reserve(n);
        d_state1.reserve(n);
        d_hit.reserve(n);
        for (int k = 0; k < 2; k++) {
            d_sray[k].reserve(2 * n);
            d_scolor[k].reserve(n);
        }
        d_L[0].reserve(n);
        d_L[1].reserve(n);
        d_film.reserve(n);
        // the cost-ordered fetch's pilot buffers, with the rest: a first ordered
        // render then allocates nothing inside the caller's timed region
        for (int k = 0; k < 2; k++) {
            d_okey[k].reserve(n);
            d_oidx[k].reserve(n);
        }
        d_owork.reserve(kTraceWords);
        d_ocnt.reserve(3);
        d_steps_sum.reserve(1);
        d_gate.reserve(1);
        d_otmp.reserve(pixel_order_tmp_bytes((uint32_t)std::min<size_t>(n, UINT32_MAX)));
        d_pprobe.reserve(n);  // the tail pilot's and the path pilot's probe (no allocation in a render)
        cap = n;
    }

    // One trace launch: the 4-wide kernel (which traces its rare NaN-prone rays inline with the
    // exact BVH2 walk), or the BVH2 kernel when the "wide" option is off.
    void trace_launch(int mode, bool tight, const TraceArgs &t, uint64_t n_max, hipStream_t st) {
        launch_trace(mode, count, tight, wide, t, grid_for(mode, n_max), st);
    }

    TraceArgs trace_args(uint32_t *work) {
        TraceArgs t{};
        t.nodes = d_nodes.p;
        t.wide_nodes = reinterpret_cast<const float4 *>(d_wnodes.p);
        t.wide_leaves = reinterpret_cast<const float4 *>(d_wleaves.p);
        t.wide_root = wide_root_dev;
        // the lean slot test's slack is derived for frame origins and steps below 2^40
        t.lean = lean && bvh4.max_abs <= 0x1p40f ? 1u : 0u;
        t.any_far_first = any_far_first ? 1u : 0u;
        t.tris = d_tris.p;
        t.stack_ovf = d_ovf.p;
        t.ovf_threads = ovf_threads;
        t.counters = d_counters.p;
        t.work = work;
        t.mesh_base = d_mesh_base.p;
        t.n_meshes = (int32_t)mesh_base.size() - 1;
        return t;
    }

    void require_ready() {
        if (!accel_built) throw std::runtime_error("acceleration structure not built (call akr_hip_build_accel)");
        commit_scene();
        ensure_trace_grid();
        if (count || ray_steps) {
            if (!d_counters.p) {
                d_counters.reserve(3);
                HIPCHK(hipMemset(d_counters.p, 0, 3 * sizeof(TraceCounters)));
                d_pprof.reserve(1);
                HIPCHK(hipMemset(d_pprof.p, 0, sizeof(PathProfile)));
            }
        }
    }

    void trace(const float4 *rays, uint64_t n, akr_hit *hits, int any, hipStream_t st) {
        require_ready();
        if (n >= (1ull << 32)) throw std::runtime_error("too many rays in one batch");
        serialize(st);
        HIPCHK(hipMemsetAsync(d_work.p, 0, kTraceWords * sizeof(uint32_t), st));
        TraceArgs t = trace_args(d_work.p);
        t.rays = rays;
        t.n = (uint32_t)n;
        t.abi_hits = hits;
        int mode = any ? TRACE_ANY : TRACE_CLOSEST;
        if (ray_steps) {
            d_steps.reserve(n);
            n_steps = n;
            t.ray_steps = d_steps.p;
            timed(any ? "trace_any" : "trace_closest", st,
                  [&] { launch_trace(mode, true, !exact_cull, wide, t, grid_for(mode, n), st); });
        } else {
            timed(any ? "trace_any" : "trace_closest", st, [&] { trace_launch(mode, !exact_cull, t, n, st); });
        }
        HIPCHK(hipGetLastError());
        mark_done(st);
    }

    // Cost-ordered pixel fetch: d_oidx[1] = the slots of each XCD shard in order of
    // decreasing pilot cost (tile order within a cost class).  The pilot traces the camera ray of
    // every slot's first sample with the counting kernel into scratch counters; nothing it does
    // reaches the film, the sampler states or the context's statistics.
    void pixel_order(uint32_t N, hipStream_t ms, bool sum_steps = false) {
        // sized for the capacity by ensure_capacity (the sort's scratch grows with n), so no size
        // query runs per render
        if (d_okey[0].n < N || d_oidx[0].n < N) throw std::runtime_error("pixel order buffers not sized");
        const size_t tb = d_otmp.n;
        HIPCHK(hipMemsetAsync(d_owork.p, 0, kTraceWords * sizeof(uint32_t), ms));
        const uint32_t sub = (uint32_t)path_order_sub, n_rays = (uint32_t)(((uint64_t)N + (1u << sub) - 1) >> sub);
        launch_pilot_rays(cam, d_pixel.p, n_rays, sub, d_ray0.p, ms);
        TraceArgs t = trace_args(d_owork.p);
        t.rays = d_ray0.p;
        t.n = n_rays;
        t.hits = d_hit.p;
        t.counters = d_ocnt.p;
        t.ray_steps = d_okey[1].p;
        t.step_cap = (uint32_t)path_order_cap;
        // the steps-only build: no hits, no tallies (the counting build spilled and ran ~20 % longer)
        launch_trace(TRACE_PILOT, false, true, true, t, grid_for(TRACE_CLOSEST, n_rays), ms);
        if (sum_steps) HIPCHK(hipMemsetAsync(d_steps_sum.p, 0, sizeof(unsigned long long), ms));
        launch_order_keys(d_okey[1].p, N, (uint32_t)path_order_shift, (uint32_t)(path_order_classes - 1), sub,
                          d_okey[0].p, d_oidx[0].p, ms, sum_steps ? d_steps_sum.p : nullptr);
        sort_pixel_order(d_otmp.p, tb, d_okey[0].p, d_okey[1].p, d_oidx[0].p, d_oidx[1].p, N, ms);
        HIPCHK(hipGetLastError());
    }

    // A counting k_path render of S samples per slot (the render's own first samples: a slot's sampler
    // starts from its seed in every render) into the zeroed film, whose pixel probe d_pprobe then holds
    // each slot's closest-hit and shadow rays; the film is zeroed again for the render.  Nothing of it
    // reaches the context's statistics (scratch counters, no phase profile).
    void probe_render(const PathArgs &base, bool tab, uint32_t N, int S, hipStream_t ms) {
        if (d_pprobe.n < N) throw std::runtime_error("pilot probe buffer not sized");
        HIPCHK(hipMemsetAsync(d_owork.p, 0, kTraceWords * sizeof(uint32_t), ms));
        PathArgs pp = base;
        pp.spp = (uint32_t)S;
        pp.work = d_owork.p;
        pp.t.counters = d_ocnt.p;
        pp.prof = nullptr;
        pp.probe = d_pprobe.p;
        pp.probe_clock = 0;
        pp.order = nullptr;
        pp.fault_test = 0;
        const uint32_t grid = (uint32_t)std::max<uint64_t>(
            1, std::min<uint64_t>(path_grid[PATH_PLAIN][tab], ((uint64_t)N + kTraceBlock - 1) / kTraceBlock));
        launch_path(true, PATH_PLAIN, tab, pp, grid, ms);
        HIPCHK(hipMemsetAsync(d_film.p, 0, (size_t)N * sizeof(float4), ms));
    }

    // The last render's form and pilot step sum, when they were left on the device (a gated launch):
    // waits for that render, then reads the gate word and the sum
    void resolve_form() {
        if (!form_pending && !pilot_sum_pending) return;
        if (done_recorded) HIPCHK(hipStreamWaitEvent(stream, ev_done, 0));
        unsigned long long sum = 0;
        uint32_t gate = 0;
        HIPCHK(hipMemcpyAsync(&sum, d_steps_sum.p, sizeof(sum), hipMemcpyDeviceToHost, stream));
        if (form_pending) HIPCHK(hipMemcpyAsync(&gate, d_gate.p, sizeof(gate), hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        last_pilot_steps = (int64_t)sum;
        if (form_pending) {
            if (gate > 1) throw std::runtime_error("render form gate holds " + std::to_string(gate));
            last_form = gate_forms[gate];
        }
        form_pending = pilot_sum_pending = false;
    }

    // Path pilot (option path_order_pilot_spp): slots ranked by the rays their first S samples take
    // (probe_render), in classes of 2^shift rays.
    void pixel_order_path(const PathArgs &base, bool tab, uint32_t N, int S, hipStream_t ms) {
        if (d_okey[0].n < N || d_oidx[0].n < N) throw std::runtime_error("pixel order buffers not sized");
        // S samples trace at most S * (2 max_depth + 1) rays (max(1, max_depth) closest-hit, max_depth shadow)
        const uint32_t max_rays = (uint32_t)S * (2u * (uint32_t)std::max(base.max_depth, 0) + 1u);
        probe_render(base, tab, N, S, ms);
        launch_probe_cost(d_pprobe.p, N, d_okey[1].p, ms);
        uint32_t shift = 0;
        while (((max_rays + 1u) >> shift) > (uint32_t)path_order_classes) shift++;
        launch_order_keys(d_okey[1].p, N, shift, (uint32_t)(path_order_classes - 1), 0, d_okey[0].p, d_oidx[0].p, ms);
        sort_pixel_order(d_otmp.p, d_otmp.n, d_okey[0].p, d_okey[1].p, d_oidx[0].p, d_oidx[1].p, N, ms);
        HIPCHK(hipGetLastError());
    }

    // Pixels of the tile list (tiles in order, row-major inside a tile) into d_pixel, expanded on
    // the device from the clipped tiles (the host loop over every pixel and the pageable upload of
    // its list cost 1.7 ms per 1080p render); sizes the queues and the per-pass counter sets.
    // Returns the pixel count.
    uint64_t setup_pixels(const akr_rect *tiles, int32_t n_tiles, size_t n_count_words, hipStream_t st) {
        require_ready();
        if (!cam_set) throw std::runtime_error("camera not set (call akr_hip_set_camera)");
        if (n_tiles < 0 || (n_tiles > 0 && !tiles)) throw std::runtime_error("invalid tile list");
        h_tiles.clear();
        h_pixel_ok = false;
        uint64_t N = 0;
        for (int k = 0; k < n_tiles; k++) {
            const int x0 = std::max(0, tiles[k].x0), y0 = std::max(0, tiles[k].y0);
            const int x1 = std::min(cam.width, tiles[k].x1), y1 = std::min(cam.height, tiles[k].y1);
            if (x1 <= x0 || y1 <= y0) continue;
            if (N >= (1ull << 31)) break;  // rejected below
            h_tiles.push_back(make_uint4((uint32_t)x0, (uint32_t)y0, (uint32_t)(x1 - x0), (uint32_t)N));
            N += (uint64_t)(x1 - x0) * (uint64_t)(y1 - y0);
        }
        if (N >= (1ull << 31)) throw std::runtime_error("too many pixels in one render call");
        serialize(st);
        ensure_capacity(N);  // before any upload: a reallocation drops contents
        d_counts.reserve(2 * n_count_words);  // two pass parities
        n_pix_last = N;
        if (N == 0) return 0;
        ensure_side_stream();
        d_tiles.upload(h_tiles.data(), h_tiles.size(), st);
        launch_expand_pixels(d_tiles.p, (uint32_t)h_tiles.size(), (uint32_t)N, d_pixel.p, st);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemsetAsync(d_film.p, 0, N * sizeof(float4), st));
        HIPCHK(hipEventRecord(ev_fork, st));  // both internal streams start after the caller's work
        HIPCHK(hipStreamWaitEvent(main_st, ev_fork, 0));
        HIPCHK(hipStreamWaitEvent(side, ev_fork, 0));
        return N;
    }

    // The last render's pixel list on the host (slot order), for the host-side film merges
    const std::vector<uint32_t> &host_pixels() {
        if (!h_pixel_ok) {
            h_pixel.resize(n_pix_last);
            for (const uint4 &t : h_tiles) {
                const uint64_t end = &t == &h_tiles.back() ? n_pix_last : (&t)[1].w;
                for (uint64_t i = t.w; i < end; i++) {
                    const uint32_t local = (uint32_t)(i - t.w);
                    h_pixel[i] = (t.x + local % t.z) | ((t.y + local / t.z) << 16);
                }
            }
            h_pixel_ok = true;
        }
        return h_pixel;
    }

    // order `st` after the context's previous trace / render ("one context, one
    // order"), and record the end of this one
    void serialize(hipStream_t st) {
        if (done_recorded) HIPCHK(hipStreamWaitEvent(st, ev_done, 0));
    }
    void mark_done(hipStream_t st) {
        HIPCHK(hipEventRecord(ev_done, st));
        done_recorded = true;
    }

    // In-band check (option "verify"): every one of the N film slots holds exactly `spp` samples.
    // Runs on `st` after the render has been joined into it and waits for it on the host, so a
    // render_device with the check on returns only after the film is complete.
    void verify_weights(hipStream_t st, uint64_t N, int spp) {
        if (!verify || N == 0) return;
        if (!h_check) {
            HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&h_check), sizeof(uint32_t),
                                 hipHostMallocMapped | hipHostMallocCoherent));
            HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&d_check_host), h_check, 0));
        }
        d_bad.reserve(1);
        *reinterpret_cast<volatile uint32_t *>(h_check) = kMappedSentinel;
        HIPCHK(hipMemsetAsync(d_bad.p, 0, sizeof(uint32_t), st));
        launch_check_weights(d_film.p, (uint32_t)N, (float)spp, d_bad.p, st);
        launch_store_word(d_bad.p, d_check_host, st);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(st));
        check_fault();
        const uint32_t bad = read_mapped(h_check);
        if (bad == kMappedSentinel) throw std::runtime_error("film check: the device never reported its result");
        if (bad != 0)
            throw std::runtime_error("film check: " + std::to_string(bad) + " of " + std::to_string(N) +
                                     " pixels do not hold " + std::to_string(spp) + " samples");
    }

    // host waits for both internal streams (before a DMA read-back of the film)
    void host_join() {
        if (side) HIPCHK(hipStreamSynchronize(side));
        if (main_st) HIPCHK(hipStreamSynchronize(main_st));
    }

    // the caller's stream sees every pass of both internal streams complete
    void join_streams(hipStream_t st) {
        // one event per internal stream: re-recording a single event before the caller's stream
        // has consumed the first wait must never be able to drop the side stream from the join
        HIPCHK(hipEventRecord(ev_join, side));
        HIPCHK(hipEventRecord(ev_join_main, main_st));
        HIPCHK(hipStreamWaitEvent(st, ev_join, 0));
        HIPCHK(hipStreamWaitEvent(st, ev_join_main, 0));
        HIPCHK(hipGetLastError());
    }

    RaygenArgs raygen_args(uint32_t N, float4 *L, uint32_t *count, bool first) const {
        RaygenArgs rg{};
        rg.cam = cam;
        rg.pixel = d_pixel.p;
        rg.n = N;
        rg.seed = d_seed.p;
        rg.L = L;
        rg.ray_out = d_ray0.p;
        rg.state_out = d_state0.p;
        rg.slot_out = d_slot0.p;
        rg.count_out = count;
        rg.first_pass = first;
        return rg;
    }

    uint64_t render(const akr_pt_params &p, const akr_rect *tiles, int32_t n_tiles, hipStream_t st) {
        if (p.spp < 0 || p.max_depth < 0) throw std::runtime_error("spp and max_depth must be >= 0");
        if (p.max_depth > 1000) throw std::runtime_error("max_depth too large");
        // counters per pass, each on its own 128-B line (atomics on one line serialise):
        // D ray-queue counts, D shadow-queue counts, 2 trace launches x kTraceWords per bounce;
        // two sets, alternating by pass, since consecutive passes overlap
        const int D = p.max_depth + 2;
        const size_t n_count_words = 2 * (size_t)D * kWorkStride + 2 * (size_t)D * kTraceWords;
        last_passes = 0;
        last_form = AKR_FORM_NONE;
        last_ordered = 0;
        form_pending = pilot_sum_pending = false;
        probe_ok = false;
        probe_n = 0;
        const uint64_t N = setup_pixels(tiles, n_tiles, n_count_words, st);
        if (N == 0) return 0;
        if (unchecked_render) {  // a fault raised by an earlier render_device that ran without "verify"
            unchecked_render = false;
            if (done_recorded) HIPCHK(hipEventSynchronize(ev_done));
            check_fault("the previous render_device call (run without verify; reported by the next render)");
        }
        hipStream_t ms = main_st;
        uint4 *probe_p = nullptr;  // option "pixel_probe"
        if (probe) {
            d_probe.reserve(N);
            HIPCHK(hipMemsetAsync(d_probe.p, 0, N * sizeof(uint4), ms));
            probe_p = d_probe.p;
            probe_n = N;
            probe_ok = true;
        }
        const SceneDev sd = scene_dev();
        const bool tight = !(exact_cull || (p.flags & AKR_PT_EXACT_CULL));
    // Persistent path kernel: every sample of every pixel in one launch.  It
        // runs the lean wide traversal only; the reference cull, the BVH2 kernel and a wide view whose
        // frames exceed the lean test's bounds keep the wavefront form.
        // auto: the persistent kernel for scenes whose shading is constant Diffuse / Emissive; Glossy,
        // Mix or image textures diverge inside the traversal waves, and the wavefront's separate shade
        // kernel measured faster there (textured hall 11.5 vs 16.0 ms per 4K spp)
        const bool use_path = path_kernel == 1 || (path_kernel == 2 && (int64_t)N <= path_auto_pixels &&
                                                   (simple_shading || path_auto_complex));
        if (use_path && tight && wide && trace_args(nullptr).lean) {
            if (p.spp > 0) {
                HIPCHK(hipMemsetAsync(d_counts.p, 0, kWorkWords * sizeof(uint32_t), ms));
                PathArgs pa{};
                pa.t = trace_args(nullptr);
                pa.sc = sd;
                pa.cam = cam;
                pa.pixel = d_pixel.p;
                pa.film = d_film.p;
                pa.work = d_counts.p;
                pa.n_pix = (uint32_t)N;
                pa.spp = (uint32_t)p.spp;
                pa.max_depth = p.max_depth;
                pa.ray_clamp = p.ray_clamp;
                pa.prof = count ? d_pprof.p : nullptr;
                if (count && count_lines) {
                    auto span = [](const void *p, size_t bytes) {
                        const uint64_t a = (uint64_t)p;
                        return (uint32_t)(bytes ? ((a + bytes - 1) >> 7) - (a >> 7) + 1 : 0);
                    };
                    lines_span[0] = 0;
                    lines_span[1] = span(d_wnodes.p, d_wnodes.n * sizeof(akr_bvh4_node));
                    lines_span[2] = lines_span[1] + span(d_wleaves.p, d_wleaves.n * sizeof(float4));
                    lines_span[3] = lines_span[2] + span(d_shade_tri.p, d_shade_tri.n * sizeof(ShadeTri));
                    d_lines.reserve(lines_span[3] / 32 + 1);
                    HIPCHK(hipMemsetAsync(d_lines.p, 0, (lines_span[3] / 32 + 1) * sizeof(uint32_t), ms));
                    pa.lines = d_lines.p;
                    for (int r = 0; r < 4; r++) pa.lines_span[r] = lines_span[r];
                }
                pa.probe = probe_p;
                pa.fault = d_fault_host;
                pa.fault_test = fault_test ? 1u : 0u;
                pa.probe_clock = probe_clock ? 1u : 0u;
                pa.spec_depth = (uint32_t)path_spec_depth;
                // the shading's material / light / CDF tables in LDS when they fit
                const bool tab = path_tab && path_tab_fits(n_mats, n_lights);
                // pixels per resident lane of k_path (the occupancy query's grid)
                const uint64_t lanes = std::max<uint64_t>(1, (uint64_t)path_grid[PATH_PLAIN][tab] *
                                                                 (uint64_t)path_grid_pct / 100) * kTraceBlock;
                const int64_t ppl1000 = (int64_t)((N * 1000 + lanes / 2) / lanes);
                last_ppl1000 = ppl1000;
                last_pilot_rays = last_pilot_steps = -1;
                form_pending = pilot_sum_pending = false;
                // the first persistent render of a context runs the pilot once on a few pixels: its
                // kernels (and rocPRIM's) are loaded then, not inside a later ordered render
                if (path_order != 0 && !order_warm) {
                    pixel_order((uint32_t)std::min<uint64_t>(N, 64), ms);
                    order_warm = true;
                }
                const int order_min_spp = (int64_t)N <= path_order_share_pixels
                                              ? std::min(path_order_share_min_spp, path_order_min_spp)
                                              : path_order_min_spp;
                pa.min_wait = (uint32_t)(path_min_wait > 0 ? path_min_wait : 40);
                const bool forced = path_spec == 1 || path_defer != 2;
                // the pilot can rank pixels for every form (path_order 2), or for k_path only (1)
                const bool pilot = path_order != 0 && p.spp >= order_min_spp && N >= 2 &&
                                   (path_order == 2 || (!forced || (path_spec != 1 && path_defer == 0)));
                const bool path_pilot = pilot && path_order_pilot_spp > 0;
                // the rule: its size and scene tests, then the camera-ray pilot's mean steps
                const bool size_ok = ppl1000 <= path_tail_ppl10 * 100;
                const bool tris_ok = path_defer_min_tris == 0 || (int64_t)n_tris() >= path_defer_min_tris;
                // the BVH's device bytes against the Infinity Cache share: a cache-resident
                // tree takes k_path_defer at any size, a larger one k_path_spec up to path_tail_ppl10
                const uint64_t bvh_bytes = bvh_dev_bytes;
                const bool cache_resident = path_spec != 1 && p.max_depth <= 8 && bvh_bytes <= (uint64_t)path_cache_mb << 20;
                const bool size_tail = path_spec == 2 ? (path_spec_pixels > 0 ? (int64_t)N <= path_spec_pixels : size_ok)
                                                      : (path_defer_pixels > 0 ? (int64_t)N <= path_defer_pixels : size_ok);
                const bool want_steps = !forced && path_order == 2 && pilot && !path_pilot && tris_ok && (cache_resident || size_tail);
                if (pilot) {
                    if (path_pilot)
                        timed("pilot", ms, [&] { pixel_order_path(pa, tab, (uint32_t)N, path_order_pilot_spp, ms); });
                    else
                        timed("pilot", ms, [&] { pixel_order((uint32_t)N, ms, want_steps); });
                    pa.order = d_oidx[1].p;
                }
                // The rule's tail test reads the pilot's step sum, which is on the device: no host wait
                // inside the render.  k_pick_form writes a gate word from the sum, and both
                // candidate kernels are launched back to back, each exiting at once unless the gate
                // names it; the form that ran is read back only when akr_hip_render_form asks.
                const int tail_kind = cache_resident ? PATH_DEFER
                                                     : (path_spec == 2 ? PATH_SPEC : (p.max_depth <= 8 ? PATH_DEFER : PATH_PLAIN));
                const bool gated = want_steps && tail_kind != PATH_PLAIN;
                int kind = PATH_PLAIN;
                if (path_spec == 1) kind = PATH_SPEC;
                else if (path_defer == 1 && p.max_depth <= 8) kind = PATH_DEFER;
                // one candidate's launch arguments and grid
                auto configure = [&](int k, PathArgs &x) {
                    const uint64_t resident = (uint64_t)path_grid[k][tab] * (uint64_t)path_grid_pct / 100;
                    const uint32_t grid = (uint32_t)std::max<uint64_t>(
                        1, std::min<uint64_t>(resident, (N + kTraceBlock - 1) / kTraceBlock));
                    if (k == PATH_DEFER) {
                        d_contrib.reserve((size_t)18 * grid * kTraceBlock);  // 16 NEE slots + the waiting ray
                        x.contrib = d_contrib.p;
                        x.mix = path_mix ? 1u : 0u;
                    }
                    if (x.order && !(k == PATH_PLAIN || path_order == 2)) x.order = nullptr;  // path_order 1
                    if (x.order) {
                        const bool small = ppl1000 <= 1500;  // at most 1.5 pixels per resident lane (8-way share)
                        const bool pair = path_order_pair == 3 ||
                                          (k != PATH_PLAIN && (path_order_pair == 1 || (path_order_pair == 2 && small)));
                        x.order_mode = pair ? 2u : 0u;  // FETCH_PAIR / FETCH_LINEAR
                        // k_path_spec: every wave takes pixels from the whole cost order (FETCH_STRIDE), so
                        // each has cheap pixels whose lanes turn helpers early (option path_spec_fetch)
                        if (k == PATH_SPEC && path_spec_fetch >= 0 &&
                            (path_spec_fetch_pixels > 0 ? (int64_t)N <= path_spec_fetch_pixels : small))
                            x.order_mode = (uint32_t)path_spec_fetch;
                        x.prio = (uint32_t)path_prio;
                    }
                    return grid;
                };
                auto form_of = [](int k) {
                    return k == PATH_SPEC ? AKR_FORM_PATH_SPEC : (k == PATH_DEFER ? AKR_FORM_PATH_DEFER : AKR_FORM_PATH);
                };
                if (want_steps) last_pilot_rays = (int64_t)(((uint64_t)N + (1u << path_order_sub) - 1) >> path_order_sub);
                if (gated) {
                    launch_pick_form(d_steps_sum.p, (unsigned long long)path_tail_steps * (uint64_t)last_pilot_rays,
                                     d_gate.p, ms);
                    PathArgs p0 = pa, p1 = pa;
                    const uint32_t g0 = configure(PATH_PLAIN, p0), g1 = configure(tail_kind, p1);
                    p0.gate = p1.gate = d_gate.p;
                    p0.gate_want = 0u;
                    p1.gate_want = 1u;
                    timed("path", ms, [&] {  // one timed record: the launch that exits at once adds microseconds
                        launch_path(count, PATH_PLAIN, tab, p0, g0, ms);
                        launch_path(count, tail_kind, tab, p1, g1, ms);
                    });
                    HIPCHK(hipGetLastError());
                    gate_forms[0] = form_of(PATH_PLAIN);
                    gate_forms[1] = form_of(tail_kind);
                    form_pending = true;
                    last_form = AKR_FORM_NONE;
                    pa.order = p0.order;
                } else {
                    if (want_steps) pilot_sum_pending = true;  // the step sum is read back on request
                    const uint32_t grid = configure(kind, pa);
                    timed("path", ms, [&] { launch_path(count, kind, tab, pa, grid, ms); });
                    HIPCHK(hipGetLastError());
                    last_form = form_of(kind);
                }
                last_ordered = pa.order ? 1 : 0;
            }
            last_passes = 1;
            join_streams(st);
            return N;
        }
        if (p.spp > 0) last_form = AKR_FORM_WAVEFRONT;
        const int nb = p.max_depth == 0 ? 1 : p.max_depth;  // the trace at depth == max_depth can
                                                             // add nothing: skipped
        int64_t g = 0;  // bounce index over all passes: shadow queues alternate by its parity
        const uint32_t *worder = nullptr;  // the cost order of the camera rays (option wave_order)
        {
            const int order_min_spp = (int64_t)N <= path_order_share_pixels
                                          ? std::min(path_order_share_min_spp, path_order_min_spp)
                                          : path_order_min_spp;
            if (wave_order && path_order != 0 && p.spp >= order_min_spp && N >= 2) {
                if (!order_warm) {
                    pixel_order((uint32_t)std::min<uint64_t>(N, 64), ms);
                    order_warm = true;
                }
                timed("pilot", ms, [&] { pixel_order((uint32_t)N, ms); });
                worder = d_oidx[1].p;
            }
            last_ordered = worder ? 1 : 0;
        }
        for (int s = 0; s < p.spp; s++) {
            const int ps = s & 1;
            last_passes++;
            uint32_t *cnt = d_counts.p + (size_t)ps * n_count_words;
            auto qcount = [&](int b) { return cnt + (size_t)b * kWorkStride; };
            auto scount = [&](int b) { return cnt + (size_t)(D + b) * kWorkStride; };
            auto work = [&](int b, int k) { return cnt + 2 * (size_t)D * kWorkStride + (size_t)(2 * b + k) * kTraceWords; };
            float4 *L = d_L[ps].p;
            // L[ps] and the counter set were last used by pass s - 2, whose splat ends its side-stream work
            if (s >= 2) HIPCHK(hipStreamWaitEvent(ms, ev_splat[ps], 0));
            HIPCHK(hipMemsetAsync(cnt, 0, n_count_words * sizeof(uint32_t), ms));
            RaygenArgs rg = raygen_args((uint32_t)N, L, qcount(0), s == 0);
            rg.probe = probe_p;
            rg.order = worder;
            timed("raygen", ms, [&] { launch_raygen(rg, ms); });
            for (int b = 0; b < nb; b++, g++) {
                const bool odd = b & 1;
                const int sq = (int)(g & 1);
                TraceArgs t = trace_args(work(b, 0));
                t.rays = odd ? d_ray1.p : d_ray0.p;
                t.count = qcount(b);
                t.hits = d_hit.p;
                timed("trace_closest", ms, [&] { trace_launch(TRACE_CLOSEST, tight, t, N, ms); });
                // shade refills shadow queue g % 2: the shadow trace of bounce g - 2 must be done
                if (g >= 2) HIPCHK(hipStreamWaitEvent(ms, ev_shadow[sq], 0));
                ShadeArgs sh{};
                sh.sc = sd;
                sh.ray_in = odd ? d_ray1.p : d_ray0.p;
                sh.state_in = odd ? d_state1.p : d_state0.p;
                sh.slot_in = odd ? d_slot1.p : d_slot0.p;
                sh.hit_in = d_hit.p;
                sh.count_in = qcount(b);
                sh.ray_out = odd ? d_ray0.p : d_ray1.p;
                sh.state_out = odd ? d_state0.p : d_state1.p;
                sh.slot_out = odd ? d_slot0.p : d_slot1.p;
                sh.count_out = qcount(b + 1);
                sh.shadow_ray = d_sray[sq].p;
                sh.shadow_color = d_scolor[sq].p;
                sh.shadow_count = scount(b);
                sh.seed = d_seed.p;
                sh.L = L;  // written at depth 0 only, before any shadow trace of the pass
                sh.depth = b;
                sh.max_depth = p.max_depth;
                sh.last = b == nb - 1;
                sh.probe = probe_p;
                timed("shade", ms, [&] { launch_shade(sh, (uint32_t)N, ms); });
                HIPCHK(hipEventRecord(ev_shade[sq], ms));
                HIPCHK(hipStreamWaitEvent(side, ev_shade[sq], 0));
                if (b < p.max_depth) {
                    TraceArgs ts = trace_args(work(b, 1));
                    ts.stack_ovf = d_ovf_side.p;  // concurrent with a main-stream trace
                    ts.rays = d_sray[sq].p;
                    ts.count = scount(b);
                    ts.shadow_color = d_scolor[sq].p;
                    ts.L = L;
                    // option serial_shadow (measurement): on the main stream, so the launch is timed alone
                    hipStream_t sst = serial_shadow ? ms : side;
                    timed("trace_shadow", sst, [&] { trace_launch(TRACE_SHADOW, tight, ts, N, sst); });
                }
                if (serial_shadow) {
                    HIPCHK(hipEventRecord(ev_shadow[sq], ms));
                    HIPCHK(hipStreamWaitEvent(side, ev_shadow[sq], 0));
                } else {
                    HIPCHK(hipEventRecord(ev_shadow[sq], side));
                }
            }
            // Tile::add_sample on the side stream, after the pass's last shadow trace: the next
            // pass (its own L and counters) proceeds on the main stream meanwhile
            SplatArgs sp{};
            sp.L = L;
            sp.film = d_film.p;
            sp.n = (uint32_t)N;
            sp.ray_clamp = p.ray_clamp;
            timed("splat", side, [&] { launch_splat(sp, (uint32_t)N, side); });
            HIPCHK(hipEventRecord(ev_splat[ps], side));
        }
        // the last shade of every pass ran on the main stream and left each slot's sampler state
        if (probe_p && p.spp > 0) launch_probe_seed(d_seed.p, (uint32_t)N, probe_p, ms);
        join_streams(st);
        return N;
    }

    // cpu::AmbientOcclusion::render (kernel/integrators/cpu/integrator.cpp:40-87) as one wavefront
    // pass per sample: raygen -> closest-hit trace -> k_ao_shade on the main stream, then the AO
    // rays and splat on the side stream (overlapping the next pass, as in render()).  occlude = +inf
    // makes "closest hit with t < occlude" plain occlusion (any hit in (Eps, inf)): a shadow-mode
    // trace adds 1 to L when unoccluded.  Any other occlude traces the AO rays closest-hit and
    // compares t (an any-hit trace bounded by tmax = occlude could differ from the reference by
    // float rounding in the box tests near t = occlude).
    uint64_t render_ao(const akr_ao_params &p, const akr_rect *tiles, int32_t n_tiles, hipStream_t st) {
        if (p.spp < 0) throw std::runtime_error("spp must be >= 0");
        // per pass: camera-queue count, AO-queue count, then 2 trace launches x kTraceWords
        const size_t n_count_words = 2 * (size_t)kWorkStride + 2 * (size_t)kTraceWords;
        probe_ok = false;
        probe_n = 0;
        const uint64_t N = setup_pixels(tiles, n_tiles, n_count_words, st);
        if (N == 0) return 0;
        const bool shadow_mode = std::isinf(p.occlude) && p.occlude > 0;
        if (!shadow_mode)
            for (int k = 0; k < 2; k++) d_ao_slot[k].reserve(N);
        hipStream_t ms = main_st;
        const bool tight = !(exact_cull || (p.flags & AKR_PT_EXACT_CULL));
        for (int s = 0; s < p.spp; s++) {
            const int ps = s & 1;
            uint32_t *cnt = d_counts.p + (size_t)ps * n_count_words;
            uint32_t *qcount = cnt, *acount = cnt + kWorkStride;
            uint32_t *work0 = cnt + 2 * kWorkStride, *work1 = work0 + kTraceWords;
            float4 *L = d_L[ps].p;
            // L[ps], the AO queue ps and the counter set were last used by pass s - 2 (ends with its splat)
            if (s >= 2) HIPCHK(hipStreamWaitEvent(ms, ev_splat[ps], 0));
            HIPCHK(hipMemsetAsync(cnt, 0, n_count_words * sizeof(uint32_t), ms));
            const RaygenArgs rg = raygen_args((uint32_t)N, L, qcount, s == 0);
            timed("raygen", ms, [&] { launch_raygen(rg, ms); });
            TraceArgs t = trace_args(work0);
            t.rays = d_ray0.p;
            t.count = qcount;
            t.hits = d_hit.p;
            timed("trace_closest", ms, [&] { trace_launch(TRACE_CLOSEST, tight, t, N, ms); });
            AoShadeArgs sh{};
            sh.tri = d_shade_tri.p;
            sh.hit_in = d_hit.p;
            sh.slot_in = d_slot0.p;
            sh.state_in = d_state0.p;
            sh.count_in = qcount;
            sh.seed = d_seed.p;
            sh.ray_out = d_sray[ps].p;
            sh.color_out = shadow_mode ? d_scolor[ps].p : nullptr;
            sh.slot_out = shadow_mode ? nullptr : d_ao_slot[ps].p;
            sh.count_out = acount;
            timed("ao_shade", ms, [&] { launch_ao_shade(sh, (uint32_t)N, ms); });
            HIPCHK(hipEventRecord(ev_shade[ps], ms));
            HIPCHK(hipStreamWaitEvent(side, ev_shade[ps], 0));
            TraceArgs ts = trace_args(work1);
            ts.stack_ovf = d_ovf_side.p;  // concurrent with the next pass's main-stream trace
            ts.rays = d_sray[ps].p;
            ts.count = acount;
            if (shadow_mode) {
                ts.shadow_color = d_scolor[ps].p;
                ts.L = L;
                timed("trace_shadow", side, [&] { trace_launch(TRACE_SHADOW, tight, ts, N, side); });
            } else {
                ts.hits = d_scolor[ps].p;  // the colour queue is free in this mode: AO hits
                timed("trace_ao_closest", side, [&] { trace_launch(TRACE_CLOSEST, tight, ts, N, side); });
                AoResolveArgs rs{d_scolor[ps].p, d_ao_slot[ps].p, acount, L, p.occlude};
                timed("ao_resolve", side, [&] { launch_ao_resolve(rs, (uint32_t)N, side); });
            }
            SplatArgs sp{};
            sp.L = L;
            sp.film = d_film.p;
            sp.n = (uint32_t)N;
            sp.ray_clamp = 0.0f;  // Tile::add_sample(p, L, 1) unclamped (integrator.cpp:78)
            timed("splat", side, [&] { launch_splat(sp, (uint32_t)N, side); });
            HIPCHK(hipEventRecord(ev_splat[ps], side));
        }
        join_streams(st);
        return N;
    }
};

namespace {

template <class F>
int guard(akr_hip_ctx *ctx, F &&f) {
    if (!ctx) return -1;
    try {
        HIPCHK(hipSetDevice(ctx->device));
        f();
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -1;
    } catch (...) {
        ctx->err = "unknown error";
        return -1;
    }
}

}  // namespace

extern "C" {

int akr_hip_api_version(void) { return AKR_HIP_API_VERSION; }

int akr_hip_device_count(int *n) {
    if (!n) return -1;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return 0;
}

int akr_hip_create(int device, akr_hip_ctx **out) {
    if (!out) return -1;
    *out = nullptr;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || device < 0 || device >= c) return -2;
    std::unique_ptr<akr_hip_ctx> ctx(new (std::nothrow) akr_hip_ctx());
    if (!ctx) return -1;
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess) return -1;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) return -1;
    if (hipEventCreateWithFlags(&ctx->ev_done, hipEventDisableTiming) != hipSuccess) return -1;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ctx->n_cu = prop.multiProcessorCount;
    *out = ctx.release();
    return 0;
}

int akr_hip_destroy(akr_hip_ctx *ctx) {
    delete ctx;
    return 0;
}

const char *akr_hip_last_error(const akr_hip_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int akr_hip_set_option(akr_hip_ctx *ctx, const char *key, int64_t value) {
    return guard(ctx, [&] {
        std::string k = key ? key : "";
        if (k == "stats") {  // 1: every kernel; 2: the dominant kernel (trace_closest, or path) only
            ctx->stats = value != 0;
            ctx->stats_closest_only = value == 2;
        } else if (k == "exact_cull") {
            ctx->exact_cull = value != 0;
        } else if (k == "count_tests") {
            ctx->count = value != 0;
        } else if (k == "count_lines") {  // with count_tests: k_path marks the 128-B lines it reads
            ctx->count_lines = value != 0;
        } else if (k == "ray_steps") {
            ctx->ray_steps = value != 0;
        } else if (k == "wide") {
            ctx->wide = value != 0;
        } else if (k == "lean") {
            ctx->lean = value != 0;
        } else if (k == "shadow_grid_pct") {
            if (value < 1 || value > 100) throw std::runtime_error("shadow_grid_pct must be in [1, 100]");
            ctx->shadow_grid_pct = (int)value;
        } else if (k == "path") {
            if (value < 0 || value > 2) throw std::runtime_error("path must be 0 (wavefront), 1 (path kernel) or 2 (auto)");
            ctx->path_kernel = (int)value;
        } else if (k == "path_auto_complex") {
            ctx->path_auto_complex = value != 0;
        } else if (k == "path_auto_pixels") {
            if (value < 0) throw std::runtime_error("path_auto_pixels must be >= 0");
            ctx->path_auto_pixels = value;
        } else if (k == "serial_shadow") {
            ctx->serial_shadow = value != 0;
        } else if (k == "any_far_first") {
            ctx->any_far_first = value != 0;
        } else if (k == "path_defer") {
            if (value < 0 || value > 2) throw std::runtime_error("path_defer must be 0, 1 or 2 (auto)");
            ctx->path_defer = (int)value;
        } else if (k == "path_defer_min_tris") {
            if (value < 0) throw std::runtime_error("path_defer_min_tris must be >= 0");
            ctx->path_defer_min_tris = value;
        } else if (k == "path_defer_pixels") {
            if (value < 0) throw std::runtime_error("path_defer_pixels must be >= 0");
            ctx->path_defer_pixels = value;
        } else if (k == "path_order") {
            if (value < 0 || value > 2) throw std::runtime_error("path_order must be 0, 1 or 2");
            ctx->path_order = (int)value;
        } else if (k == "path_order_min_spp") {
            if (value < 0) throw std::runtime_error("path_order_min_spp must be >= 0");
            ctx->path_order_min_spp = (int)std::min<int64_t>(value, INT32_MAX);
        } else if (k == "path_order_share_pixels") {
            if (value < 0) throw std::runtime_error("path_order_share_pixels must be >= 0");
            ctx->path_order_share_pixels = value;
        } else if (k == "path_order_share_min_spp") {
            if (value < 0) throw std::runtime_error("path_order_share_min_spp must be >= 0");
            ctx->path_order_share_min_spp = (int)std::min<int64_t>(value, INT32_MAX);
        } else if (k == "path_order_cap") {
            if (value < 0 || value > INT32_MAX) throw std::runtime_error("path_order_cap must be in [0, 2^31)");
            ctx->path_order_cap = (int)value;
        } else if (k == "path_order_sub") {
            if (value < 0 || value > 5) throw std::runtime_error("path_order_sub must be in [0, 5]");
            ctx->path_order_sub = (int)value;
        } else if (k == "path_order_classes") {
            if (value < 1 || value > 32) throw std::runtime_error("path_order_classes must be in [1, 32]");
            ctx->path_order_classes = (int)value;
        } else if (k == "path_order_shift") {
            if (value < 0 || value > 31) throw std::runtime_error("path_order_shift must be in [0, 31]");
            ctx->path_order_shift = (int)value;
        } else if (k == "path_order_pair") {
            if (value < 0 || value > 3)
                throw std::runtime_error("path_order_pair must be 0, 1, 2 (auto) or 3 (both persistent kernels)");
            ctx->path_order_pair = (int)value;
        } else if (k == "path_prio") {
            if (value < 0 || value > 256) throw std::runtime_error("path_prio must be in [0, 256]");
            ctx->path_prio = (int)value;
        } else if (k == "path_mix") {
            ctx->path_mix = value != 0;
        } else if (k == "path_tab") {
            ctx->path_tab = value != 0;
        } else if (k == "path_spec") {
            if (value < 0 || value > 2) throw std::runtime_error("path_spec must be 0, 1 or 2");
            ctx->path_spec = (int)value;
        } else if (k == "wave_order") {
            ctx->wave_order = value != 0;
        } else if (k == "path_order_pilot_spp") {
            if (value < 0 || value > 64) throw std::runtime_error("path_order_pilot_spp must be in [0, 64]");
            ctx->path_order_pilot_spp = (int)value;
        } else if (k == "path_spec_depth") {
            if (value < 1 || value > 3) throw std::runtime_error("path_spec_depth must be in [1, 3]");
            ctx->path_spec_depth = (int)value;
        } else if (k == "path_spec_fetch_pixels") {
            if (value < 0) throw std::runtime_error("path_spec_fetch_pixels must be >= 0");
            ctx->path_spec_fetch_pixels = value;
        } else if (k == "path_spec_fetch") {
            if (value < -1 || value > 3) throw std::runtime_error("path_spec_fetch must be in [-1, 3]");
            ctx->path_spec_fetch = (int)value;
        } else if (k == "path_tail_ppl10") {
            if (value < 0) throw std::runtime_error("path_tail_ppl10 must be >= 0");
            ctx->path_tail_ppl10 = value;
        } else if (k == "leaf_align") {
            if (value != 1 && value != 2 && value != 4 && value != 8) throw std::runtime_error("leaf_align must be 1, 2, 4 or 8");
            ctx->leaf_align = (int)value;
        } else if (k == "path_cache_mb") {
            if (value < 0) throw std::runtime_error("path_cache_mb must be >= 0");
            ctx->path_cache_mb = value;
        } else if (k == "path_tail_steps") {
            if (value < 0 || value > 4096) throw std::runtime_error("path_tail_steps must be in [0, 4096]");
            ctx->path_tail_steps = (int)value;
        } else if (k == "path_spec_pixels") {
            if (value < 0) throw std::runtime_error("path_spec_pixels must be >= 0");
            ctx->path_spec_pixels = value;
        } else if (k == "path_grid_pct") {
            if (value < 1 || value > 100) throw std::runtime_error("path_grid_pct must be in [1, 100]");
            ctx->path_grid_pct = (int)value;
        } else if (k == "path_min_wait") {
            if (value < 0 || value > 64) throw std::runtime_error("path_min_wait must be in [0, 64] (0: per kernel)");
            ctx->path_min_wait = (int)value;
        } else if (k == "pixel_probe") {
            ctx->probe = value != 0;
            ctx->probe_clock = value == 2;
        } else if (k == "fault_test") {
            ctx->fault_test = value != 0;
        } else if (k == "verify") {
            ctx->verify = value != 0;
        } else if (k == "rays_per_lane") {
            if (value < 1 || value > 64) throw std::runtime_error("rays_per_lane must be in [1, 64]");
            ctx->rays_per_lane = (int)value;
        } else {
            throw std::runtime_error("unknown option '" + k + "'");
        }
    });
}

int akr_hip_upload_mesh(akr_hip_ctx *ctx, const float *vertices, uint64_t n_vertices, const int32_t *indices,
                        const float *normals, const float *texcoords, const int32_t *material_indices,
                        uint64_t n_triangles, const int32_t *material_slots, int32_t n_slots, int32_t *geom_id) {
    return guard(ctx, [&] {
        if (n_triangles && (!vertices || !indices || !normals || !texcoords || !material_indices))
            throw std::runtime_error("null mesh array");
        if (ctx->n_tris() + n_triangles >= (1ull << 31)) throw std::runtime_error("scene too large");
        const uint64_t vb = ctx->verts.size() / 3;
        for (uint64_t i = 0; i < 3 * n_triangles; i++)
            if (indices[i] < 0 || (uint64_t)indices[i] >= n_vertices) throw std::runtime_error("vertex index out of range");
        for (uint64_t t = 0; t < n_triangles; t++) {
            int32_t m = material_indices[t];
            if (m >= n_slots) throw std::runtime_error("material index beyond the mesh's material list");
        }
        ctx->verts.insert(ctx->verts.end(), vertices, vertices + 3 * n_vertices);
        for (uint64_t i = 0; i < 3 * n_triangles; i++) ctx->idx.push_back((int32_t)(indices[i] + vb));
        ctx->normals.insert(ctx->normals.end(), normals, normals + 9 * n_triangles);
        ctx->texcoords.insert(ctx->texcoords.end(), texcoords, texcoords + 6 * n_triangles);
        for (uint64_t t = 0; t < n_triangles; t++) {
            int32_t m = material_indices[t];
            ctx->matid.push_back(m < 0 ? -1 : material_slots[m]);  // -1: no material (scene.h:73-76)
        }
        if (geom_id) *geom_id = (int32_t)ctx->mesh_base.size() - 1;
        ctx->mesh_base.push_back((uint32_t)ctx->n_tris());
        ctx->scene_dirty = true;
        ctx->accel_built = false;
    });
}

int akr_hip_upload_images(akr_hip_ctx *ctx, const float *rgba, const int32_t *widths, const int32_t *heights,
                          int32_t n_images) {
    return guard(ctx, [&] {
        ctx->images.clear();
        ctx->img_off.clear();
        ctx->img_w.clear();
        ctx->img_h.clear();
        int64_t off = 0;
        for (int i = 0; i < n_images; i++) {
            if (widths[i] <= 0 || heights[i] <= 0) throw std::runtime_error("empty image");
            ctx->img_off.push_back(off);
            ctx->img_w.push_back(widths[i]);
            ctx->img_h.push_back(heights[i]);
            off += 4 * (int64_t)widths[i] * heights[i];
        }
        ctx->images.assign(rgba, rgba + off);
        ctx->scene_dirty = true;
    });
}

int akr_hip_upload_textures(akr_hip_ctx *ctx, const akr_texture *textures, int32_t n) {
    return guard(ctx, [&] {
        ctx->texs.assign(textures, textures + n);
        ctx->scene_dirty = true;
    });
}

int akr_hip_upload_materials(akr_hip_ctx *ctx, const akr_material *materials, int32_t n) {
    return guard(ctx, [&] {
        ctx->mats.assign(materials, materials + n);
        ctx->scene_dirty = true;
    });
}

int akr_hip_upload_lights(akr_hip_ctx *ctx, const akr_area_light *lights, int32_t n, const float *power) {
    return guard(ctx, [&] {
        if (n < 0 || (n > 0 && (!lights || !power))) throw std::runtime_error("invalid light list");
        ctx->lights.assign(lights, lights + n);
        ctx->power.assign(power, power + n);
        ctx->scene_dirty = true;
    });
}

namespace {
// An imported tree's triangle records must be this scene's triangles: each record equals the one
// the builders write for its gid (v0 and the f32 edges v1 - v0, v2 - v0, instance.h:49-50, bit for
// bit), and every scene triangle is referenced by some leaf.  Shading reads the context's own
// vertices, so a tree shared from another scene would otherwise render wrong geometry without an
// error.  O(n_tris) on `n_threads` threads.
void check_tris_match_mesh(const akr_hip_ctx *ctx, const akr_bvh_tri *tr, uint64_t n, int n_threads) {
    const uint64_t nt = ctx->n_tris();
    // relaxed atomics: several threads may mark the same triangle (SBVH duplicates), ADVICE r4
    std::unique_ptr<std::atomic<uint8_t>[]> covered(new std::atomic<uint8_t>[nt]);
    for (uint64_t g = 0; g < nt; g++) covered[g].store(0, std::memory_order_relaxed);
    const int T = n_threads > 0 ? std::min(n_threads, 64)
                                : (int)std::min(64u, std::max(1u, std::thread::hardware_concurrency()));
    std::vector<uint64_t> bad(T, UINT64_MAX);
    run_on_threads(T, [&](int t) {
        const uint64_t r0 = n * t / T, r1 = n * (t + 1) / T;
        for (uint64_t r = r0; r < r1; r++) {
            const uint32_t g = tr[r].gid;  // < nt: checked by validate_bvh2
            const float *v0 = &ctx->verts[3 * (size_t)ctx->idx[3 * (size_t)g + 0]];
            const float *v1 = &ctx->verts[3 * (size_t)ctx->idx[3 * (size_t)g + 1]];
            const float *v2 = &ctx->verts[3 * (size_t)ctx->idx[3 * (size_t)g + 2]];
            float want[9];
            for (int k = 0; k < 3; k++) {
                want[k] = v0[k];
                want[3 + k] = v1[k] - v0[k];
                want[6 + k] = v2[k] - v0[k];
            }
            const float got[9] = {tr[r].v0[0], tr[r].v0[1], tr[r].v0[2], tr[r].e1[0], tr[r].e1[1],
                                  tr[r].e1[2], tr[r].e2[0], tr[r].e2[1], tr[r].e2[2]};
            if (std::memcmp(want, got, sizeof(want)) != 0) {
                bad[t] = r;
                return;
            }
            covered[g].store(1, std::memory_order_relaxed);
        }
    });
    for (uint64_t r : bad)
        if (r != UINT64_MAX)
            throw std::runtime_error("imported BVH: triangle record " + std::to_string(r) + " (gid " +
                                     std::to_string(tr[r].gid) + ") does not match this scene's triangle");
    for (uint64_t g = 0; g < nt; g++)
        if (!covered[g].load(std::memory_order_relaxed))
            throw std::runtime_error("imported BVH: scene triangle " + std::to_string(g) + " is in no leaf");
}

// After the BVH2 of ctx->bvh exists (built or imported): the wide view, its device copy, the BVH2
// itself for the exact lane path, the accel info, and the scene's shading records.
void finish_accel(akr_hip_ctx *ctx, int n_threads) {
        auto &b = ctx->bvh;
        ctx->accel_built = false;  // set again only once every buffer below holds the new tree
        {
            Bvh4Output w;
            build_bvh4(b.nodes, w, n_threads, ctx->wide_collapse);
            if (w.nodes.size() >= kMaxWideNodes)
                throw std::runtime_error("scene too large: the wide view needs fewer than 2^26 nodes (about 100 M triangles)");
            ctx->bvh4 = std::move(w);
        }
        ctx->d_nodes.upload(b.nodes.data(), b.nodes.size(), ctx->stream);
        // Device copy of the wide view: each leaf record is followed by its triangles in one blob, so
        // the leaf phase fetches the exact box and the first triangle in one batch; leaf refs in the
        // wide nodes become float4 offsets into the blob.
        // Offsets by a serial prefix sum, then the records and their triangles are copied on
        // `n_threads` threads (the blob is ~1 GB on C3).
        const auto &leaves = ctx->bvh4.leaves;
        std::vector<uint32_t> leaf_off(leaves.size());
        size_t words = 0;
        const size_t align = (size_t)std::max(1, ctx->leaf_align);
        for (size_t i = 0; i < leaves.size(); i++) {
            words = (words + align - 1) / align * align;
            if (words >= AKR_CHILD_LEAF) break;
            leaf_off[i] = (uint32_t)words;
            words += 2 + 3 * (size_t)leaves[i].count;
        }
        if (words >= AKR_CHILD_LEAF) throw std::runtime_error("BVH too large for the wide leaf blob");
        // zero float4 of padding behind the last leaf: a leaf phase fetches the second triangle
        // record with the header whatever the leaf's count (kernels.hip path_leaf)
        const size_t pad = 3;
        std::unique_ptr<float4[]> blob(new float4[words + pad]);
        if (align > 1) std::memset(static_cast<void *>(blob.get()), 0, sizeof(float4) * (words + pad));  // the gaps
        else std::memset(static_cast<void *>(blob.get() + words), 0, sizeof(float4) * pad);
        const float4 *tri4 = reinterpret_cast<const float4 *>(b.tris.data());
        std::vector<akr_bvh4_node> wn = ctx->bvh4.nodes;
        auto remap = [&](uint32_t r) {
            return (r != AKR_CHILD_EMPTY && (r & AKR_CHILD_LEAF)) ? (AKR_CHILD_LEAF | leaf_off[r & 0x7FFFFFFFu]) : r;
        };
        const int nt = n_threads > 0 ? std::min(n_threads, 64)
                                       : (int)std::min(64u, std::max(1u, std::thread::hardware_concurrency()));
        auto fill = [&](int t) {
            const size_t l0 = leaves.size() * t / nt, l1 = leaves.size() * (t + 1) / nt;
            for (size_t i = l0; i < l1; i++) {
                const akr_bvh_leaf &l = leaves[i];
                float4 *o = blob.get() + leaf_off[i];
                float4 h0, h1;
                h0.x = l.lo[0], h0.y = l.lo[1], h0.z = l.lo[2], h0.w = l.hi[0];
                uint32_t fc[2] = {l.first, l.count};
                h1.x = l.hi[1], h1.y = l.hi[2];
                std::memcpy(&h1.z, &fc[0], 4);
                std::memcpy(&h1.w, &fc[1], 4);
                o[0] = h0;
                o[1] = h1;
                std::memcpy(o + 2, tri4 + 3 * (size_t)l.first, sizeof(float4) * 3 * (size_t)l.count);
            }
            const size_t n0 = wn.size() * t / nt, n1 = wn.size() * (t + 1) / nt;
            for (size_t i = n0; i < n1; i++)
                for (auto &c : wn[i].child) c = remap(c);
        };
        run_on_threads(nt, fill);
        ctx->wide_root_dev = remap(ctx->bvh4.root_ref);
        ctx->d_wnodes.reserve(1);  // never a null pointer, even for an empty scene
        ctx->d_wleaves.reserve(1);
        ctx->d_wnodes.upload(wn.data(), wn.size(), ctx->stream);
        ctx->d_wleaves.upload(blob.get(), words + pad, ctx->stream);
        // the uploaded tree's bytes (the DBufs' capacities only grow), for the form rule
        ctx->bvh_dev_bytes = (uint64_t)wn.size() * sizeof(akr_bvh4_node) + (uint64_t)(words + pad) * sizeof(float4);
        HIPCHK(hipStreamSynchronize(ctx->stream));  // before the host staging vectors go away
        ctx->d_tris.upload(reinterpret_cast<const float4 *>(b.tris.data()), 3 * b.tris.size(), ctx->stream);
        HIPCHK(hipStreamSynchronize(ctx->stream));
        ctx->info.n_nodes = b.nodes.size();
        ctx->info.n_tris = b.tris.size();
        ctx->info.max_depth = b.max_depth;
        ctx->info.max_leaf = b.max_leaf;
        ctx->info.build_ms = b.build_ms;
        ctx->info.sah_cost = b.sah_cost;
        ctx->accel_built = true;
        ctx->commit_scene();
}
}  // namespace

int akr_hip_build_accel(akr_hip_ctx *ctx, const akr_build_params *params) {
    return guard(ctx, [&] {
        akr_build_params p{};
        p.max_leaf_size = 4;
        p.n_bins = 32;
        p.traversal_cost = 1.0f;
        p.intersect_cost = 4.0f;
        if (params) p = *params;
        BvhInput in{ctx->verts.data(), ctx->idx.data(), ctx->n_tris()};
        ctx->accel_built = false;  // until the new tree is on the device (a failure below leaves none)
        if (p.builder == AKR_BUILDER_LBVH) build_lbvh_gpu(in, ctx->bvh, ctx->stream);
        else if (p.builder == AKR_BUILDER_SAH || p.builder == AKR_BUILDER_SBVH) build_bvh(in, p, ctx->bvh);
        else throw std::runtime_error("unknown builder");
        if (p.wide_collapse != AKR_COLLAPSE_SAH && p.wide_collapse != AKR_COLLAPSE_BALANCED)
            throw std::runtime_error("unknown wide_collapse");
        ctx->wide_collapse = p.wide_collapse;
        finish_accel(ctx, p.n_threads);
    });
}

int akr_hip_import_accel(akr_hip_ctx *ctx, const void *nodes, uint64_t n_nodes, const void *tris, uint64_t n_tris,
                         int32_t n_threads) {
    return guard(ctx, [&] {
        if (!nodes || n_nodes == 0 || (n_tris && !tris)) throw std::runtime_error("null or empty BVH arrays");
        const auto *nd = reinterpret_cast<const akr_bvh_node *>(nodes);
        const auto *tr = reinterpret_cast<const akr_bvh_tri *>(tris);
        int max_leaf = 0;
        const int depth = validate_bvh2(nd, n_nodes, tr, n_tris, ctx->n_tris(), max_leaf);  // throws on bad input
        check_tris_match_mesh(ctx, tr, n_tris, n_threads);  // the records are this scene's triangles
        ctx->accel_built = false;  // until the new tree is on the device (a failure below leaves none)
        BvhOutput &b = ctx->bvh;
        b.nodes.assign(nd, nd + n_nodes);
        b.tris.assign(tr, tr + n_tris);
        b.max_depth = depth;
        b.max_leaf = max_leaf;
        b.sah_cost = 0.0;  // not known for an imported tree
        b.build_ms = 0.0;
        ctx->wide_collapse = AKR_COLLAPSE_SAH;
        finish_accel(ctx, n_threads);
    });
}

int akr_hip_accel_info(akr_hip_ctx *ctx, akr_accel_info *info) {
    return guard(ctx, [&] {
        if (!ctx->accel_built) throw std::runtime_error("acceleration structure not built");
        *info = ctx->info;
    });
}

int akr_hip_accel_export(akr_hip_ctx *ctx, void *nodes, uint64_t node_bytes, void *tris, uint64_t tri_bytes) {
    return guard(ctx, [&] {
        if (!ctx->accel_built) throw std::runtime_error("acceleration structure not built");
        uint64_t nb = ctx->bvh.nodes.size() * sizeof(akr_bvh_node), tb = ctx->bvh.tris.size() * sizeof(akr_bvh_tri);
        if (node_bytes < nb || tri_bytes < tb) throw std::runtime_error("export buffers too small");
        std::memcpy(nodes, ctx->bvh.nodes.data(), nb);
        std::memcpy(tris, ctx->bvh.tris.data(), tb);
    });
}

int akr_hip_set_camera(akr_hip_ctx *ctx, const akr_camera *camera) {
    return guard(ctx, [&] {
        if (!camera) throw std::runtime_error("null camera");
        ctx->cam = make_camera(*camera);
        ctx->cam_set = true;
    });
}

int akr_hip_trace(akr_hip_ctx *ctx, const akr_ray *rays, uint64_t n, akr_hit *hits, int any_hit) {
    return guard(ctx, [&] {
        if (n == 0) return;
        if (!rays || !hits) throw std::runtime_error("null ray or hit buffer");
        static_assert(sizeof(akr_ray) == 2 * sizeof(float4), "akr_ray layout");
        ctx->d_trace_rays.upload(reinterpret_cast<const float4 *>(rays), 2 * n, ctx->stream);
        ctx->d_trace_hits.reserve(n);
        ctx->trace(ctx->d_trace_rays.p, n, ctx->d_trace_hits.p, any_hit, ctx->stream);
        HIPCHK(hipMemcpyAsync(hits, ctx->d_trace_hits.p, n * sizeof(akr_hit), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
    });
}

int akr_hip_trace_device(akr_hip_ctx *ctx, const void *d_rays, uint64_t n, void *d_hits, int any_hit, void *stream) {
    return guard(ctx, [&] {
        if (n == 0) return;
        if (!d_rays || !d_hits) throw std::runtime_error("null ray or hit buffer");
        hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
        ctx->trace(reinterpret_cast<const float4 *>(d_rays), n, reinterpret_cast<akr_hit *>(d_hits), any_hit, st);
    });
}

int akr_hip_render_node(akr_hip_ctx *const *ctxs, int32_t n_ctx, const akr_pt_params *params, const akr_rect *tiles,
                        int32_t n_tiles, float *radiance, float *weight) {
    if (!ctxs || n_ctx < 1) return -1;
    for (int32_t k = 0; k < n_ctx; k++)
        if (!ctxs[k]) return -1;
    akr_hip_ctx *lead = ctxs[0];
    if (!params || !radiance || !weight || n_tiles < 0 || (n_tiles > 0 && !tiles)) {
        lead->err = "null or invalid argument";
        return -1;
    }
    for (int32_t k = 0; k < n_ctx; k++)
        for (int32_t j = 0; j < k; j++)
            if (ctxs[j] == ctxs[k]) {  // the per-context render threads would share one context
                lead->err = "a context is listed twice";
                return -1;
            }
    // tile j -> context j % n_ctx (interleaved, like the multi-process split of akari_amd/dist.py);
    // one host thread per context, each bound to its device by guard()
    std::vector<std::vector<akr_rect>> part(n_ctx);
    for (int32_t j = 0; j < n_tiles; j++) part[j % n_ctx].push_back(tiles[j]);
    std::vector<uint64_t> npix(n_ctx, 0);
    std::vector<int> status(n_ctx, 0);
    run_on_threads(n_ctx, [&](int k) {
        akr_hip_ctx *c = ctxs[k];
        status[k] = guard(c, [&] {
            hipStream_t st = c->stream;
            const uint64_t N = c->render(*params, part[k].data(), (int32_t)part[k].size(), st);
            c->verify_weights(st, N, params->spp);  // joins the render into st and checks it
            if (!c->verify) {
                c->join_streams(st);
                HIPCHK(hipStreamSynchronize(st));
                c->check_fault();
            }
            c->mark_done(st);
            npix[k] = N;
        });
    });
    for (int32_t k = 0; k < n_ctx; k++)
        if (status[k] != 0) {
            if (k) lead->err = "context " + std::to_string(k) + ": " + ctxs[k]->err;
            return -1;
        }
    // Gather on the lead device (Film::merge_tile, core/film.h:85-95).  Every other context pushes its
    // packed film and pixel list into its own staging buffers on the lead device from its own stream
    // (device-to-device peer copies, over xGMI between GPUs), so the copies of all contexts run at
    // once; the lead stream waits for each context's copy event and k_merge_film adds the films into
    // the frame in context order (the host loop's order).  No host synchronisation until the frame
    // goes back to the host.
    return guard(lead, [&] {
        const int W = lead->cam.width, H = lead->cam.height;
        const uint64_t F = (uint64_t)W * (uint64_t)H;
        hipStream_t st = lead->stream;
        for (int32_t k = 1; k < n_ctx; k++)
            if (ctxs[k]->device != lead->device) {
                const hipError_t e = hipDeviceEnablePeerAccess(ctxs[k]->device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
                (void)hipGetLastError();
            }
        lead->d_frame.reserve(4 * F);
        float *frad = lead->d_frame.p, *fw = lead->d_frame.p + 3 * F;
        HIPCHK(hipMemcpyAsync(frad, radiance, 3 * F * sizeof(float), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(fw, weight, F * sizeof(float), hipMemcpyHostToDevice, st));
        // a pixel listed r times by one context (overlapping tiles) goes to its r-th launch, so the
        // adds of a pixel stay in list order and no launch adds one pixel twice
        std::vector<uint32_t> seen(F, 0), all_order;
        std::vector<std::vector<std::pair<size_t, uint32_t>>> launches(n_ctx);  // (offset, count) per rank
        for (int32_t k = 0; k < n_ctx; k++) {
            const uint64_t N = npix[k];
            if (N == 0) continue;
            std::fill(seen.begin(), seen.end(), 0u);
            std::vector<std::vector<uint32_t>> rank;
            const std::vector<uint32_t> &pl = ctxs[k]->host_pixels();
            for (uint64_t i = 0; i < N; i++) {
                const uint32_t px = pl[i];
                const uint64_t p = (uint64_t)(px & 0xFFFFu) + (uint64_t)(px >> 16) * W;
                const uint32_t r = seen[p]++;
                if (r >= rank.size()) rank.emplace_back();
                rank[r].push_back((uint32_t)i);
            }
            if (rank.size() == 1) {
                launches[k].push_back({SIZE_MAX, (uint32_t)N});  // identity order
                continue;
            }
            for (auto &ord : rank) {
                launches[k].push_back({all_order.size(), (uint32_t)ord.size()});
                all_order.insert(all_order.end(), ord.begin(), ord.end());
            }
        }
        if (!all_order.empty()) lead->d_gorder.upload(all_order.data(), all_order.size(), st);
        // the peer pushes: one staging pair per context on the lead device, each copy on its
        // context's stream after that context's render
        if (lead->g_film.size() < (size_t)n_ctx) {
            lead->g_film.resize(n_ctx);
            lead->g_pix.resize(n_ctx);
        }
        for (int32_t k = 1; k < n_ctx; k++) {
            akr_hip_ctx *c = ctxs[k];
            const uint64_t N = npix[k];
            if (N == 0 || c == lead) continue;
            if (!lead->g_film[k]) {
                lead->g_film[k].reset(new DBuf<float4>());
                lead->g_pix[k].reset(new DBuf<uint32_t>());
            }
            lead->g_film[k]->reserve(N);  // on the lead device (current)
            lead->g_pix[k]->reserve(N);
            HIPCHK(hipSetDevice(c->device));
            if (!c->ev_gather) HIPCHK(hipEventCreateWithFlags(&c->ev_gather, hipEventDisableTiming));
            HIPCHK(hipMemcpyPeerAsync(lead->g_film[k]->p, lead->device, c->d_film.p, c->device, N * sizeof(float4),
                                      c->stream));
            HIPCHK(hipMemcpyPeerAsync(lead->g_pix[k]->p, lead->device, c->d_pixel.p, c->device, N * sizeof(uint32_t),
                                      c->stream));
            HIPCHK(hipEventRecord(c->ev_gather, c->stream));
            c->mark_done(c->stream);  // the context's film is not reused before the copy is done
            HIPCHK(hipSetDevice(lead->device));
        }
        for (int32_t k = 0; k < n_ctx; k++) {
            akr_hip_ctx *c = ctxs[k];
            if (npix[k] == 0) continue;
            const float4 *film = c->d_film.p;
            const uint32_t *pix = c->d_pixel.p;
            if (c != lead) {
                HIPCHK(hipStreamWaitEvent(st, c->ev_gather, 0));
                film = lead->g_film[k]->p;
                pix = lead->g_pix[k]->p;
            }
            for (const auto &l : launches[k])
                launch_merge_film(film, pix, l.first == SIZE_MAX ? nullptr : lead->d_gorder.p + l.first, l.second, W,
                                  frad, fw, st);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipMemcpyAsync(radiance, frad, 3 * F * sizeof(float), hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(weight, fw, F * sizeof(float), hipMemcpyDeviceToHost, st));
        lead->mark_done(st);
        HIPCHK(hipStreamSynchronize(st));
        for (int32_t k = 1; k < n_ctx; k++)  // a context's next call orders after its copy anyway
            if (ctxs[k] != lead && npix[k]) {
                HIPCHK(hipSetDevice(ctxs[k]->device));
                HIPCHK(hipStreamSynchronize(ctxs[k]->stream));
            }
        HIPCHK(hipSetDevice(lead->device));
    });
}

namespace {
// Film::merge_tile (core/film.h:85-95) of the context's packed film into full-frame host buffers
void merge_film(akr_hip_ctx *ctx, uint64_t N, int spp, float *radiance, float *weight) {
    hipStream_t st = ctx->stream;
    if (N == 0) {
        ctx->mark_done(st);
        return;
    }
    // the render's last splat runs on the internal side stream: wait for both internal streams on
    // the host before the copy, rather than trusting the DMA engine to honour the caller stream's
    // cross-stream event waits (two flaky short-weight reads were seen, never reproduced)
    ctx->host_join();
    HIPCHK(hipStreamSynchronize(st));
    ctx->check_fault();
    ctx->verify_weights(st, N, spp);
    std::vector<float4> film(N);
    HIPCHK(hipMemcpyAsync(film.data(), ctx->d_film.p, N * sizeof(float4), hipMemcpyDeviceToHost, st));
    ctx->mark_done(st);
    HIPCHK(hipStreamSynchronize(st));
    if (ctx->verify) {  // the read-back itself: every copied slot holds spp samples
        uint64_t bad = 0;
        for (uint64_t k = 0; k < N; k++) bad += film[k].w != (float)spp;
        if (bad) throw std::runtime_error("film read-back: " + std::to_string(bad) + " of " + std::to_string(N) +
                                          " pixels do not hold " + std::to_string(spp) + " samples");
    }
    const int W = ctx->cam.width;
    const std::vector<uint32_t> &pl = ctx->host_pixels();
    for (uint64_t k = 0; k < N; k++) {
        uint32_t px = pl[k];
        uint64_t pix = (uint64_t)(px & 0xFFFFu) + (uint64_t)(px >> 16) * W;
        radiance[3 * pix + 0] += film[k].x;
        radiance[3 * pix + 1] += film[k].y;
        radiance[3 * pix + 2] += film[k].z;
        weight[pix] += film[k].w;
    }
}
}  // namespace

int akr_hip_render(akr_hip_ctx *ctx, const akr_pt_params *params, const akr_rect *tiles, int32_t n_tiles,
                   float *radiance, float *weight) {
    return guard(ctx, [&] {
        if (!params || !radiance || !weight) throw std::runtime_error("null argument");
        merge_film(ctx, ctx->render(*params, tiles, n_tiles, ctx->stream), params->spp, radiance, weight);
    });
}

int akr_hip_render_ao(akr_hip_ctx *ctx, const akr_ao_params *params, const akr_rect *tiles, int32_t n_tiles,
                      float *radiance, float *weight) {
    return guard(ctx, [&] {
        if (!params || !radiance || !weight) throw std::runtime_error("null argument");
        merge_film(ctx, ctx->render_ao(*params, tiles, n_tiles, ctx->stream), params->spp, radiance, weight);
    });
}

int akr_hip_render_device(akr_hip_ctx *ctx, const akr_pt_params *params, const akr_rect *tiles, int32_t n_tiles,
                          float *d_radiance, float *d_weight, void *stream, uint64_t *n_pixels) {
    return guard(ctx, [&] {
        if (!params || !d_radiance || !d_weight) throw std::runtime_error("null argument");
        hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
        uint64_t N = ctx->render(*params, tiles, n_tiles, st);
        if (n_pixels) *n_pixels = N;
        ctx->timed("unpack", st, [&] { launch_unpack(ctx->d_film.p, (uint32_t)N, d_radiance, d_weight, st); });
        HIPCHK(hipGetLastError());
        ctx->verify_weights(st, N, params->spp);
        ctx->unchecked_render = !ctx->verify;
        ctx->mark_done(st);
    });
}

struct akr_bvh_host {
    BvhOutput out;
    Bvh4Output wide;
    bool wide_built = false;
    int n_threads = 0;  // the build's thread count, used by the wide collapse too
    int collapse = AKR_COLLAPSE_SAH;
};

int akr_bvh_host_build(const float *vertices, uint64_t n_vertices, const int32_t *indices, uint64_t n_triangles,
                       const akr_build_params *params, akr_bvh_host **out, akr_accel_info *info) {
    if (!out) return -1;
    *out = nullptr;
    try {
        for (uint64_t i = 0; i < 3 * n_triangles; i++)
            if (indices[i] < 0 || (uint64_t)indices[i] >= n_vertices) return -1;
        akr_build_params p{};
        p.max_leaf_size = 4;
        p.n_bins = 32;
        p.traversal_cost = 1.0f;
        p.intersect_cost = 4.0f;
        if (params) p = *params;
        std::unique_ptr<akr_bvh_host> h(new akr_bvh_host());
        h->n_threads = p.n_threads;
        if (p.wide_collapse != AKR_COLLAPSE_SAH && p.wide_collapse != AKR_COLLAPSE_BALANCED) return -1;
        h->collapse = p.wide_collapse;
        BvhInput in{vertices, indices, n_triangles};
        build_bvh(in, p, h->out);
        if (info) {
            info->n_nodes = h->out.nodes.size();
            info->n_tris = h->out.tris.size();
            info->max_depth = h->out.max_depth;
            info->max_leaf = h->out.max_leaf;
            info->build_ms = h->out.build_ms;
            info->sah_cost = h->out.sah_cost;
        }
        *out = h.release();
        return 0;
    } catch (...) {
        return -1;
    }
}
const void *akr_bvh_host_nodes(const akr_bvh_host *h) { return h ? h->out.nodes.data() : nullptr; }
const void *akr_bvh_host_tris(const akr_bvh_host *h) { return h ? h->out.tris.data() : nullptr; }
void akr_bvh_host_free(akr_bvh_host *h) { delete h; }

int akr_bvh_validate(const void *nodes, uint64_t n_nodes, const void *tris, uint64_t n_tris, uint64_t n_scene_tris,
                     int32_t *max_depth) {
    try {
        if (!nodes || (n_tris && !tris)) return -1;
        int max_leaf = 0;
        const int d = validate_bvh2(reinterpret_cast<const akr_bvh_node *>(nodes), n_nodes,
                                    reinterpret_cast<const akr_bvh_tri *>(tris), n_tris, n_scene_tris, max_leaf);
        if (max_depth) *max_depth = d;
        return 0;
    } catch (...) {
        return -1;
    }
}

int akr_bvh_host_wide(akr_bvh_host *h, uint64_t *n_nodes, uint64_t *n_leaves, uint32_t *root_ref) {
    if (!h) return -1;
    try {
        if (!h->wide_built) {
            build_bvh4(h->out.nodes, h->wide, h->n_threads, h->collapse);
            h->wide_built = true;
        }
        if (n_nodes) *n_nodes = h->wide.nodes.size();
        if (n_leaves) *n_leaves = h->wide.leaves.size();
        if (root_ref) *root_ref = h->wide.root_ref;
        return 0;
    } catch (...) {
        return -1;
    }
}
const void *akr_bvh_host_wide_nodes(const akr_bvh_host *h) { return h ? h->wide.nodes.data() : nullptr; }
const void *akr_bvh_host_wide_leaves(const akr_bvh_host *h) { return h ? h->wide.leaves.data() : nullptr; }

int akr_hip_ray_steps(akr_hip_ctx *ctx, uint32_t *out, uint64_t n) {
    return guard(ctx, [&] {
        if (!ctx->ray_steps || n > ctx->n_steps) throw std::runtime_error("no per-ray steps recorded for that many rays");
        if (n == 0) return;
        if (!out) throw std::runtime_error("null output");
        HIPCHK(hipMemcpyAsync(out, ctx->d_steps.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
    });
}

int akr_hip_kernel_stats(akr_hip_ctx *ctx, akr_kernel_stat *out, int32_t max_n, int32_t *n) {
    return guard(ctx, [&] {
        ctx->flush_stats();
        int32_t k = 0;
        for (auto &kv : ctx->stat) {
            if (k < max_n && out) {
                akr_kernel_stat &s = out[k];
                std::memset(&s, 0, sizeof(s));
                std::strncpy(s.name, kv.first.c_str(), sizeof(s.name) - 1);
                s.launches = kv.second.launches;
                s.total_ms = kv.second.total;
                s.min_ms = kv.second.launches ? kv.second.mn : 0;
                s.max_ms = kv.second.mx;
            }
            k++;
        }
        if (n) *n = k;
    });
}

int akr_hip_trace_counts(akr_hip_ctx *ctx, akr_trace_counts *out) {
    return guard(ctx, [&] {
        std::memset(out, 0, sizeof(*out));
        if (!ctx->d_counters.p) return;
        HIPCHK(hipDeviceSynchronize());
        TraceCounters c[3];
        HIPCHK(hipMemcpy(c, ctx->d_counters.p, sizeof(c), hipMemcpyDeviceToHost));
        out->rays = c[0].rays + c[1].rays + c[2].rays;
        out->box_tests = c[0].box + c[1].box + c[2].box;
        out->tri_tests = c[0].tri + c[1].tri + c[2].tri;
        out->closest_rays = c[0].rays;
        out->shadow_rays = c[1].rays + c[2].rays;
        for (int m = 0; m < 3; m++) {
            out->per_mode[m][0] = c[m].rays;
            out->per_mode[m][1] = c[m].box;
            out->per_mode[m][2] = c[m].tri;
            out->lane_slots[m][0] = c[m].slots_trav;
            out->lane_slots[m][1] = c[m].slots_leaf;
            out->lane_slots[m][2] = c[m].slots_tri;
            out->lane_slots[m][3] = c[m].visits;
            out->deep_rays[m] = c[m].deep;
            out->leaf_tests[m] = c[m].leaves;
        }
    });
}

int akr_hip_path_profile(akr_hip_ctx *ctx, uint64_t *out, int32_t n) {
    return guard(ctx, [&] {
        if (!out || n < 0) throw std::runtime_error("null output");
        PathProfile q{};
        if (ctx->d_pprof.p) HIPCHK(hipMemcpy(&q, ctx->d_pprof.p, sizeof(q), hipMemcpyDeviceToHost));
        uint64_t v[] = {q.waves, q.outer, q.procs, q.trav_iters, q.t_proc, q.t_trav, q.t_leaf, q.t_total, q.t_max,
                        q.lanes_proc, q.t_shade, q.spec_started, q.spec_aborted, q.tv_issue, q.tv_wait,
                        q.tv_comp, q.tl_issue, q.tl_wait, q.tl_comp, q.tp_park, q.tp_next, q.tp_begin, q.tp_load,
                        q.leaf_phases, q.leaf_holders, 0, 0, 0};
        // out[25..27]: distinct 128-B lines of the wide nodes, the leaf blob and the shading records the
        // last render with count_lines read (k_path)
        if (n > 25 && ctx->count_lines && ctx->d_lines.p && ctx->lines_span[3]) {
            std::vector<uint32_t> m(ctx->lines_span[3] / 32 + 1);
            HIPCHK(hipMemcpy(m.data(), ctx->d_lines.p, m.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
            for (int r = 0; r < 3; r++)
                for (uint32_t b = ctx->lines_span[r]; b < ctx->lines_span[r + 1]; b++)
                    v[25 + r] += (m[b >> 5] >> (b & 31u)) & 1u;
        }
        for (int32_t k = 0; k < n && k < (int32_t)(sizeof(v) / sizeof(v[0])); k++) out[k] = v[k];
    });
}

int akr_hip_render_info(akr_hip_ctx *ctx, int32_t *lanes, int32_t *passes) {
    return guard(ctx, [&] {
        if (lanes) *lanes = 1;  // one sample per pixel in flight (the lookahead lanes are gone)
        if (passes) *passes = ctx->last_passes;
    });
}

int akr_hip_render_form(akr_hip_ctx *ctx, int32_t *form, int32_t *ordered) {
    return guard(ctx, [&] {
        ctx->resolve_form();
        if (form) *form = ctx->last_form;
        if (ordered) *ordered = ctx->last_ordered;
    });
}

int akr_hip_render_form_inputs(akr_hip_ctx *ctx, int64_t *pixels_per_lane_x1000, int64_t *pilot_rays,
                               int64_t *pilot_steps) {
    return guard(ctx, [&] {
        ctx->resolve_form();
        if (pixels_per_lane_x1000) *pixels_per_lane_x1000 = ctx->last_ppl1000;
        if (pilot_rays) *pilot_rays = ctx->last_pilot_rays;
        if (pilot_steps) *pilot_steps = ctx->last_pilot_steps;
    });
}

int akr_hip_reset_stats(akr_hip_ctx *ctx) {
    return guard(ctx, [&] {
        HIPCHK(hipDeviceSynchronize());
        ctx->flush_stats();
        ctx->stat.clear();
        if (ctx->d_counters.p) HIPCHK(hipMemset(ctx->d_counters.p, 0, 3 * sizeof(TraceCounters)));
        if (ctx->d_pprof.p) HIPCHK(hipMemset(ctx->d_pprof.p, 0, sizeof(PathProfile)));
    });
}

int akr_hip_synchronize(akr_hip_ctx *ctx) {
    return guard(ctx, [&] {
        HIPCHK(hipStreamSynchronize(ctx->stream));
        HIPCHK(hipDeviceSynchronize());
        ctx->check_fault();
    });
}

int akr_hip_pixel_probe(akr_hip_ctx *ctx, akr_pixel_probe *out, uint64_t n) {
    return guard(ctx, [&] {
        if (!ctx->probe_ok || n > ctx->probe_n)
            throw std::runtime_error("no pixel probe recorded for that many slots (option pixel_probe, path renders only)");
        if (n == 0) return;
        if (!out) throw std::runtime_error("null output");
        static_assert(sizeof(akr_pixel_probe) == sizeof(uint4), "akr_pixel_probe layout");
        ctx->host_join();
        HIPCHK(hipStreamSynchronize(ctx->stream));
        HIPCHK(hipMemcpyAsync(out, ctx->d_probe.p, n * sizeof(uint4), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
    });
}

}  // extern "C"
