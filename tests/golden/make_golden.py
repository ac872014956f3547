"""Generate tests/golden/kat.json: known-answer vectors computed in pure Python integer / numpy f32
arithmetic straight from the reference formulas (independent of oracle/ and of the HIP library).

  lcg        LCGSampler::next1d, src/akari/kernel/sampler.h:60-63 (u32 wrap, float(seed)/float(2^32-1))
  pcg        PCGSampler, sampler.h:28-53 (set_sample_index(seed) then next1d)
  dist       Distribution1D + upper_bound, common/distribution.h:32-102
  mt         Moller-Trumbore MeshInstance::intersect, kernel/instance.h:42-80
Run: python tests/golden/make_golden.py
"""
import json
from pathlib import Path

import numpy as np

F = np.float32
M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF


def lcg(seed, n):
    out, s = [], seed & M32
    for _ in range(n):
        s = (1103515245 * s + 12345) & M32
        out.append(float(F(s) / F(4294967295)))   # (float)seed / (float)0xFFFFFFFF
    return out, s


def pcg(seed, n):
    mult, inc = 6364136223846793005, 1442695040888963407

    def step(st):
        x = st
        count = x >> 59
        st = (x * mult + inc) & M64
        x ^= x >> 18
        v = (x >> 27) & M32
        return st, ((v >> count) | (v << ((-count) & 31))) & M32

    st = (seed + inc) & M64
    st, _ = step(st)
    out = []
    for _ in range(n):
        st, v = step(st)
        out.append(float(F(v) / F(4294967295)))
    return out


def dist(func, us):
    n = len(func)
    f = [F(x) for x in func]
    cdf = [F(0)] * (n + 1)
    for i in range(n):
        cdf[i + 1] = F(cdf[i] + F(f[i] / F(n)))
    fi = cdf[n]
    if fi == 0:
        cdf = [F(0)] + [F(F(i) / F(n)) for i in range(1, n + 1)]
    else:
        cdf = [cdf[0]] + [F(c / fi) for c in cdf[1:]]
    res = []
    for u in us:
        lo, hi = 0, n + 1
        while lo < hi:
            mid = (lo + hi) // 2
            if cdf[mid] <= F(u):
                lo = mid + 1
            else:
                hi = mid
        i = min(max(hi - 1, 0), n - 1)
        with np.errstate(invalid="ignore"):   # all-zero power: pdf = 0 / 0 as in the reference
            res.append([i, float(F(f[i] / F(fi * F(n))))])
    return res


def slab(lo, hi, o, d, tmin, tmax):
    rmin = lambda a, b: b if b < a else a          # std::min
    rmax = lambda a, b: b if a < b else a          # std::max
    with np.errstate(divide="ignore", invalid="ignore"):
        o, d = np.array(o, F), np.array(d, F)
        invd = F(1) / d
        t0 = (lo - o) * invd
        t1 = (hi - o) * invd
    mn = [rmin(t0[k], t1[k]) for k in range(3)]
    mx = [rmax(t0[k], t1[k]) for k in range(3)]
    m0 = rmax(rmax(mn[0], mn[1]), mn[2])
    m1 = rmin(rmin(mx[0], mx[1]), mx[2])
    if m0 <= m1:
        t = rmax(F(tmin), m0)
        return -1.0 if t >= F(tmax) else float(t)
    return -1.0


def main():
    kat = {"lcg": {}, "pcg": {}, "dist": [], "mt": []}
    for seed in (0, 1, 1919, 2 ** 32 - 1, 123456789):
        vals, last = lcg(seed, 16)
        kat["lcg"][str(seed)] = {"values": vals, "final_state": last}
    for seed in (0, 42):
        kat["pcg"][str(seed)] = pcg(seed, 16)
    for func, us in (([1, 2, 3, 4], [0.0, 0.05, 0.1, 0.1000001, 0.3, 0.6, 0.99, 1.0]),
                     ([1.1149462, 1.1149462], [0.0, 0.25, 0.5, 0.75, 1.0]),
                     ([0, 0, 0], [0.0, 0.4, 0.9]),
                     ([5.0], [0.0, 0.5, 1.0])):
        kat["dist"].append({"func": func, "u": us, "expect": dist(func, us)})
    # Moller-Trumbore known answers on the unit right triangle (0,0,0), (1,0,0), (0,1,0)
    tri = [[0, 0, 0], [1, 0, 0], [0, 1, 0]]
    cases = [
        ([0.25, 0.25, 1.0], [0, 0, -1], 1e-3, float("inf"), True, 1.0, 0.25, 0.25),
        ([0.25, 0.25, -1.0], [0, 0, 1], 1e-3, float("inf"), True, 1.0, 0.25, 0.25),   # back face: two-sided
        ([0.6, 0.6, 1.0], [0, 0, -1], 1e-3, float("inf"), False, 0, 0, 0),          # u + v > 1
        ([-0.1, 0.5, 1.0], [0, 0, -1], 1e-3, float("inf"), False, 0, 0, 0),         # u < 0
        ([0.25, 0.25, 1.0], [1, 0, 0], 1e-3, float("inf"), False, 0, 0, 0),         # parallel: |det| < 1e-6
        ([0.25, 0.25, 1.0], [0, 0, -1], 1e-3, 1.0, False, 0, 0, 0),                 # t == tmax: strict
        ([0.25, 0.25, 1.0], [0, 0, -1], 1.0, 5.0, False, 0, 0, 0),                  # t == tmin: strict
        ([0.25, 0.25, 1.0], [0, 0, -1], 1e-3, 1.0000001, True, 1.0, 0.25, 0.25),
        ([0.0, 0.0, 2.0], [0, 0, -1], 1e-3, float("inf"), True, 2.0, 0.0, 0.0),    # vertex hit (u = v = 0)
        ([0.5, 0.5, 2.0], [0, 0, -1], 1e-3, float("inf"), True, 2.0, 0.5, 0.5),    # edge hit (u + v = 1)
    ]
    for o, d, tmin, tmax, hit, t, u, v in cases:
        # the reference traversal also needs the triangle's box to pass intersectAABB
        # (bvh-accelerator.h:89-103, std::min/max NaN semantics): (lo - o) * (1/0) is NaN when o
        # lies on a box plane whose direction component is 0, and the box is then missed.
        lo = np.min(np.array(tri, F), axis=0)
        hi = np.max(np.array(tri, F), axis=0)
        kat["mt"].append({"tri": tri, "o": o, "d": d, "tmin": tmin, "tmax": tmax if tmax != float("inf") else "inf",
                          "hit": hit, "bvh_hit": hit and slab(lo, hi, o, d, tmin, tmax) >= 0,
                          "t": t, "u": u, "v": v})
    out = Path(__file__).with_name("kat.json")
    out.write_text(json.dumps(kat, indent=1))
    print("wrote", out)


if __name__ == "__main__":
    main()
