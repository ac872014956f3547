// scenegen.cpp — synthetic triangle-soup generator, built as
// libakr_scenegen.so.  Workload data only: it is not on the render path.
//
// Soup definition: PCG32 sampler (src/akari/kernel/sampler.h:28-53) with
// set_sample_index(seed); per triangle 12 next1d() draws in this order: centroid x, y, z, then
// for vertex k = 0..2 the offsets x, y, z; coordinate = c + (2u - 1) * r, c = 2u - 1.
// Per-face normals = normalize(cross(v1 - v0, v2 - v0)) and texcoords (v > 0, v % 2 == 0) as
// the OBJ importer writes them when the file has none (src/akari/cmd/akari-import.cpp:73-87).
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "bvh_build.h"

namespace {
struct Pcg {
    uint64_t state;
    static constexpr uint64_t mult = 6364136223846793005ull;
    static constexpr uint64_t inc = 1442695040888963407ull;
    uint32_t next() {
        uint64_t x = state;
        unsigned count = (unsigned)(x >> 59);
        state = x * mult + inc;
        x ^= x >> 18;
        uint32_t v = (uint32_t)(x >> 27);
        return v >> count | v << (-count & 31);
    }
    float next1d() { return (float)next() / (float)0xffffffffu; }
};
// state after k steps of the LCG x -> a x + c (jump-ahead, so threads can start mid-stream)
uint64_t lcg_jump(uint64_t state, uint64_t k) {
    uint64_t acc_mult = 1, acc_plus = 0, cur_mult = Pcg::mult, cur_plus = Pcg::inc;
    while (k) {
        if (k & 1) {
            acc_mult *= cur_mult;
            acc_plus = acc_plus * cur_mult + cur_plus;
        }
        cur_plus = (cur_mult + 1) * cur_plus;
        cur_mult *= cur_mult;
        k >>= 1;
    }
    return acc_mult * state + acc_plus;
}
void face(const float *v, float *n) {
    float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
    float e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
    float c[3] = {(e1[1] * e2[2]) - (e1[2] * e2[1]), (e1[2] * e2[0]) - (e1[0] * e2[2]), (e1[0] * e2[1]) - (e1[1] * e2[0])};
    float d = c[0] * c[0];
    d += c[1] * c[1];
    d += c[2] * c[2];
    float l = std::sqrt(d);
    for (int k = 0; k < 3; k++) n[k] = c[k] / l;
}
}  // namespace

extern "C" {

// vertices[9n] (3 unique vertices per triangle), normals[9n], texcoords[6n].
int akr_gen_soup(uint64_t n, uint64_t seed, float r, float *vertices, float *normals, float *texcoords, int n_threads) {
    Pcg p0;
    p0.state = seed + Pcg::inc;  // pcg32_init: state = seed + inc; pcg32()
    (void)p0.next();
    int T = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    if (T < 1) T = 1;
    uint64_t chunk = (n + T - 1) / T;
    // every started thread is joined even if creating a later one fails (bvh_build.h run_on_threads)
    akr::run_on_threads(T, [&](int t) {
        const uint64_t b = (uint64_t)t * chunk, e = std::min<uint64_t>(n, b + chunk);
        if (b >= e) return;
        {
            Pcg p;
            p.state = lcg_jump(p0.state, 12 * b);
            for (uint64_t i = b; i < e; i++) {
                float c[3];
                for (int k = 0; k < 3; k++) c[k] = 2.0f * p.next1d() - 1.0f;
                float *v = vertices + 9 * i;
                for (int j = 0; j < 3; j++)
                    for (int k = 0; k < 3; k++) v[3 * j + k] = c[k] + (2.0f * p.next1d() - 1.0f) * r;
                float nn[3];
                face(v, nn);
                for (int j = 0; j < 3; j++)
                    for (int k = 0; k < 3; k++) normals[9 * i + 3 * j + k] = nn[k];
                for (int j = 0; j < 3; j++) {
                    texcoords[6 * i + 2 * j + 0] = (float)(j > 0);
                    texcoords[6 * i + 2 * j + 1] = (float)(j % 2 == 0);
                }
            }
        }
    });
    return 0;
}

}  // extern "C"
