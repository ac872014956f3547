// Calibration of the L2 -> fabric read counters on the traversal's own access widths.
//
// MI355X_MICROARCH.md §HBM validates "2 x FETCH_SIZE = bytes read" only for 16-B-per-lane streaming reads.
// The path kernel's reads are random gathers of 64-B wide nodes (4 x 16-B loads of one lane), 32-B leaf
// headers, 48-B triangle records and the leaf phase's 128-B batch (header + two triangles) at any 16-B
// alignment.  This program reads each of those shapes from a 2 GiB table (8x the 256-MiB Infinity Cache),
// every record exactly once, in a scattered order (a bijection i -> i * P mod N), independently (all of a
// lane's loads issued together) and as dependent chains (the next record's index is in the record read).
// Records sit 256 B apart, so no two records share a 128-B line and the bytes each launch must move are
// known exactly: the record bytes, the 64-B sectors and the 128-B lines the records cover.  The packed
// pattern (two 64-B nodes per line, both read at different times) shows what a line read twice costs.
//
// Each pattern is its own kernel instantiation (calib<PATTERN>), so the rocprofv3 counter csv of a pass
// attributes counters by kernel name; a flush kernel streams a separate 1 GiB buffer between patterns so
// no pattern finds the previous one's lines in L2 or the Infinity Cache.  Output: one JSON line per
// pattern with its known byte counts and its time (HIP events); tools/fetch_calib.py joins them with
// the counter passes of tools/fetch_calib.sh into profiles/<tag>_fetch_calib.json.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr uint64_t TABLE = 2ull << 30;           // 2 GiB
constexpr uint32_t STRIDE = 256;                 // one record per 256 B: no two records share a line
constexpr uint32_t NREC = TABLE / STRIDE;        // 8 M records
constexpr uint32_t PERM = 0x9E3779B1u;           // odd: i -> i * PERM mod 2^k is a bijection
constexpr int THREADS = 256;

enum Pattern : int {
    STREAM16 = 0,     // 16 B per lane, coalesced, the whole table once
    NODE64_IND, NODE64_DEP,      // 64 B at line offset 0
    LEAF32_IND, LEAF32_DEP,      // 32 B at line offset 0
    TRI48_IND, TRI48_DEP,        // 48 B at line offset 32 (crosses a 64-B sector, not a line)
    BATCH128_IND, BATCH128_DEP,  // 128 B at a 16-B offset (r * 16) mod 144 of its 256-B slot: crosses a line unless 0 / 128
    NODE64_PACKED,               // 64-B records packed two per line, every record once (each line read twice)
    NPAT
};

struct PatInfo { const char *name; int width; int dep; };
static const PatInfo INFO[NPAT] = {
    {"stream16", 16, 0},
    {"node64_ind", 64, 0}, {"node64_dep", 64, 1},
    {"leaf32_ind", 32, 0}, {"leaf32_dep", 32, 1},
    {"tri48_ind", 48, 0}, {"tri48_dep", 48, 1},
    {"batch128_ind", 128, 0}, {"batch128_dep", 128, 1},
    {"node64_packed", 64, 0},
};

__host__ __device__ inline uint32_t rec_offset(int pat, uint32_t r) {   // byte offset of record r in its slot
    switch (pat) {
    case TRI48_IND: case TRI48_DEP: return 32;
    case BATCH128_IND: case BATCH128_DEP: return ((r * 7u) % 9u) * 16u;   // 0, 16, ..., 128
    default: return 0;
    }
}

__host__ __device__ inline uint32_t scatter(uint32_t i, uint32_t n) { return (uint32_t)((uint64_t)i * PERM & (n - 1)); }

// Dependent chains: record scatter(p) holds scatter(p + 1) in its first dword (its first 16-B load), so
// a lane that starts at position p0 reads scatter(p0), scatter(p0 + 1), ... one after another.
__global__ void init_chain(uint32_t *table, int pat, uint32_t n) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        uint32_t r = scatter(p, n), nx = scatter(p + 1 == n ? 0 : p + 1, n);
        table[((uint64_t)r * STRIDE + rec_offset(pat, r)) / 4] = nx;
    }
}

template <int W>
__device__ inline uint32_t read_rec(const uint4 *__restrict__ base, uint64_t byte_off, uint32_t &first) {
    const uint4 *p = base + byte_off / 16;
    uint4 v[W / 16];
#pragma unroll
    for (int k = 0; k < W / 16; ++k) v[k] = p[k];
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < W / 16; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    first = v[0].x;
    return acc;
}

template <int PAT>
__global__ __launch_bounds__(THREADS) void calib(const uint4 *__restrict__ table, uint32_t *__restrict__ sink,
                                                 uint32_t per_lane) {
    constexpr int W = PAT == STREAM16 ? 16 : (PAT == LEAF32_IND || PAT == LEAF32_DEP) ? 32
                    : (PAT == TRI48_IND || PAT == TRI48_DEP) ? 48 : (PAT == BATCH128_IND || PAT == BATCH128_DEP) ? 128 : 64;
    constexpr bool DEP = PAT == NODE64_DEP || PAT == LEAF32_DEP || PAT == TRI48_DEP || PAT == BATCH128_DEP;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nthr = gridDim.x * blockDim.x;
    uint32_t acc = 0, first = 0;
    if constexpr (PAT == STREAM16) {
        const uint64_t n16 = TABLE / 16;
        for (uint64_t i = tid; i < n16; i += nthr) { uint4 v = table[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    } else if constexpr (PAT == NODE64_PACKED) {
        const uint32_t n = TABLE / 64;
        for (uint32_t k = 0; k < per_lane; ++k) {
            uint32_t i = tid + k * nthr;
            if (i < n) acc ^= read_rec<64>(table, (uint64_t)scatter(i, n) * 64, first);
        }
    } else if constexpr (DEP) {
        uint32_t r = scatter(tid * per_lane, NREC);          // this lane's chain covers positions [tid * per_lane, +per_lane)
        for (uint32_t k = 0; k < per_lane; ++k) {
            acc ^= read_rec<W>(table, (uint64_t)r * STRIDE + rec_offset(PAT, r), first);
            r = first;
        }
    } else {
        for (uint32_t k = 0; k < per_lane; ++k) {           // all of a lane's loads independent of each other
            uint32_t r = scatter(tid + k * nthr, NREC);
            acc ^= read_rec<W>(table, (uint64_t)r * STRIDE + rec_offset(PAT, r), first);
        }
    }
    sink[tid] = acc;
}

__global__ void flush(const uint4 *__restrict__ buf, uint64_t n16, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) {
        uint4 v = buf[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int PAT>
static float run(const uint4 *table, uint32_t *sink, uint32_t grid, uint32_t per_lane, hipEvent_t a, hipEvent_t b) {
    CHECK(hipEventRecord(a));
    calib<PAT><<<grid, THREADS>>>(table, sink, per_lane);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 1;
    uint4 *table, *fbuf;
    uint32_t *sink;
    const uint64_t fbytes = 1ull << 30;
    CHECK(hipMalloc(&table, TABLE));
    CHECK(hipMalloc(&fbuf, fbytes));
    CHECK(hipMalloc(&sink, 64u << 20));
    CHECK(hipMemset(fbuf, 1, fbytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    // Independent and packed: 256 CUs x 8 workgroups, each lane reading its share in per_lane rounds.
    // Dependent: one chain per lane, 32 records long (NREC / 32 lanes = 1024 workgroups of 256).
    const uint32_t grid_ind = 2048, lanes_ind = grid_ind * THREADS;
    const uint32_t per_ind = NREC / lanes_ind, per_packed = (uint32_t)(TABLE / 64) / lanes_ind;
    const uint32_t dep_len = 32, grid_dep = NREC / dep_len / THREADS;
    for (int rep = 0; rep < reps; ++rep) {
        for (int pat = 0; pat < NPAT; ++pat) {
            CHECK(hipMemset(table, 0, TABLE));
            if (INFO[pat].dep) {
                init_chain<<<4096, 256>>>((uint32_t *)table, pat, NREC);
                CHECK(hipGetLastError());
            }
            flush<<<4096, 256>>>(fbuf, fbytes / 16, sink);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            float ms = 0;
            uint64_t recs = NREC, rbytes = 0, sectors = 0, lines = 0;
            switch (pat) {
            case STREAM16: ms = run<STREAM16>(table, sink, grid_ind, 0, a, b); recs = TABLE / 16; break;
            case NODE64_IND: ms = run<NODE64_IND>(table, sink, grid_ind, per_ind, a, b); break;
            case NODE64_DEP: ms = run<NODE64_DEP>(table, sink, grid_dep, dep_len, a, b); break;
            case LEAF32_IND: ms = run<LEAF32_IND>(table, sink, grid_ind, per_ind, a, b); break;
            case LEAF32_DEP: ms = run<LEAF32_DEP>(table, sink, grid_dep, dep_len, a, b); break;
            case TRI48_IND: ms = run<TRI48_IND>(table, sink, grid_ind, per_ind, a, b); break;
            case TRI48_DEP: ms = run<TRI48_DEP>(table, sink, grid_dep, dep_len, a, b); break;
            case BATCH128_IND: ms = run<BATCH128_IND>(table, sink, grid_ind, per_ind, a, b); break;
            case BATCH128_DEP: ms = run<BATCH128_DEP>(table, sink, grid_dep, dep_len, a, b); break;
            case NODE64_PACKED: ms = run<NODE64_PACKED>(table, sink, grid_ind, per_packed, a, b); recs = TABLE / 64; break;
            }
            // Known bytes: record bytes, and the distinct 64-B sectors / 128-B lines the records cover.
            const int w = INFO[pat].width;
            if (pat == STREAM16 || pat == NODE64_PACKED) {
                rbytes = TABLE; sectors = TABLE / 64; lines = TABLE / 128;
            } else {
                for (uint32_t r = 0; r < NREC; ++r) {
                    uint32_t o = rec_offset(pat, r);
                    sectors += (o + w - 1) / 64 - o / 64 + 1;
                    lines += (o + w - 1) / 128 - o / 128 + 1;
                }
                rbytes = (uint64_t)NREC * w;
            }
            printf("{\"pattern\": \"%s\", \"kernel\": \"calib<%d>\", \"rep\": %d, \"width\": %d, \"dependent\": %d, "
                   "\"records\": %llu, \"record_bytes\": %llu, \"sector64_bytes\": %llu, \"line128_bytes\": %llu, "
                   "\"ms\": %.4f, \"record_GBps\": %.1f, \"line_GBps\": %.1f}\n",
                   INFO[pat].name, pat, rep, w, INFO[pat].dep, (unsigned long long)recs, (unsigned long long)rbytes,
                   (unsigned long long)(sectors * 64), (unsigned long long)(lines * 128), ms,
                   rbytes / (ms * 1e6), lines * 128.0 / (ms * 1e6));
            fflush(stdout);
        }
    }
    CHECK(hipFree(table));
    CHECK(hipFree(fbuf));
    CHECK(hipFree(sink));
    return 0;
}
