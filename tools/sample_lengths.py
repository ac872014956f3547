"""Per-sample draw counts of the C3 soup's pixels (CPU restatement, oracle/): how predictable is the
length of a pixel's next sample from its earlier ones?  A sample consumes 4 + 6k LCG draws for k
scattering events (+2 per zero-pdf BSDF sample; pathtracer.h:96-164), so the sampler state a sample
starts from is known only once the previous sample has ended (cpu/integrator.cpp:124-134).  Any
speculative run of sample s+1 must guess that count; this tool measures how often simple guesses
are right.

The render is repeated at spp = 1..S over a strided subset of the frame; the final sampler state
after s samples (the pixel probe) gives the cumulative draw count D(s), so n_s = D(s) - D(s-1).
Usage: python tools/sample_lengths.py [--spp 16] [--stride 16] [--tris 10000000]"""
import argparse
import collections
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

A, C = 1103515245, 12345


def lcg_distance(s0, s1, cap=4096):
    """n with LCG^n(s0) == s1 (elementwise), -1 if none within cap."""
    out = np.full(s0.shape, -1, np.int64)
    s = s0.astype(np.uint64)
    t = s1.astype(np.uint64)
    for n in range(cap):
        hit = (s == t) & (out < 0)
        out[hit] = n
        if (out >= 0).all():
            break
        s = (s * A + C) & 0xFFFFFFFF
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--stride", type=int, default=16, help="every n-th 32x32 tile of the frame")
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--save", default="", help="write the [pixels, spp] draw counts (and x, y) to this .npz")
    args = ap.parse_args()
    from akari_amd import capi, dist, scene
    import py_oracle
    W, H = 1920, 1080
    t0 = time.time()
    cs = scene.compile_scene(scene.soup_scene(n_tris=args.tris, resolution=(W, H)))
    nodes, tris, _ = capi.build_bvh_host(cs.vertices, cs.indices, n_threads=args.threads)
    orc = py_oracle.OracleScene(cs, nodes, tris, capi)
    print(f"scene + BVH {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    tiles = dist.tiles_for_rank(W, H, 32, 0, args.stride)
    mask = np.zeros((H, W), bool)
    for x0, y0, x1, y1 in tiles:
        mask[y0:y1, x0:x1] = True
    ys, xs = np.nonzero(mask)
    seed0 = (xs + ys * W).astype(np.uint64)
    prev = seed0
    lengths = []
    for s in range(1, args.spp + 1):
        _, _, _, pr = orc.render(s, 5, tiles=tiles, n_threads=args.threads, probe=True)
        cur = pr["seed"][ys, xs].astype(np.uint64)
        n = lcg_distance(prev, cur)
        assert (n >= 0).all()
        lengths.append(n)
        prev = cur
        print(f"spp {s} done ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
    L = np.stack(lengths, 1)                       # [pixels, spp]
    if args.save:
        np.savez_compressed(args.save, L=L, x=xs, y=ys)
    soup = (L > 4).any(1)                          # pixels whose camera rays hit something in S samples
    Ls = L[soup]
    hist = collections.Counter(Ls.reshape(-1).tolist())
    tot = Ls.size
    # guess policies for sample s from samples < s (s >= 1)
    pol = {}
    mode_all = max(hist, key=hist.get)
    pol["global_mode"] = np.mean(Ls[:, 1:] == mode_all)
    pol["previous_length"] = np.mean(Ls[:, 1:] == Ls[:, :-1])
    acc = []
    for s in range(1, Ls.shape[1]):                # the pixel's own running mode
        m = np.array([collections.Counter(r.tolist()).most_common(1)[0][0] for r in Ls[:, :s]])
        acc.append(np.mean(Ls[:, s] == m))
    pol["own_running_mode"] = float(np.mean(acc))
    top2 = [k for k, _ in hist.most_common(2)]
    pol["global_top2"] = np.mean(np.isin(Ls[:, 1:], top2))
    top3 = [k for k, _ in hist.most_common(3)]
    pol["global_top3"] = np.mean(np.isin(Ls[:, 1:], top3))
    out = {"pixels": int(L.shape[0]), "soup_pixels": int(soup.sum()), "spp": args.spp,
           "draws_hist_soup": {int(k): round(v / tot, 4) for k, v in sorted(hist.items())},
           "guess_accuracy_soup": {k: round(float(v), 4) for k, v in pol.items()},
           "mean_draws_soup": round(float(Ls.mean()), 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
