"""Secondary benchmark: the ambient-occlusion integrator (akr_hip_render_ao)
on the C3 scene (10M-triangle soup, 1920x1080).  Not the headline metric: prints one JSON line with
Msamples/s of render_ao(spp) over the full frame (host-buffer API, so the 2M-pixel film copy and
merge are inside the timed call) and the per-kernel event times of one timed call.

Usage: python tools/ao_bench.py [--spp 16] [--occlude inf] [--tris 10000000]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--occlude", type=float, default=float("inf"))
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    args = ap.parse_args()
    from akari_amd import capi, scene

    W, H = args.width, args.height
    cs = scene.compile_scene(scene.soup_scene(n_tris=args.tris, resolution=(W, H)))
    with capi.HipContext(0) as ctx:
        scene.upload_scene(ctx, cs, max_leaf_size=4, intersect_cost=4.0, n_threads=16)
        tiles = [(0, 0, W, H)]
        rad = np.zeros((H, W, 3), np.float32)
        wt = np.zeros((H, W), np.float32)
        ctx.render_ao(1, tiles, W, H, occlude=args.occlude, radiance=rad, weight=wt)   # warmup
        best = float("inf")
        for _ in range(args.reps):
            rad[:] = 0
            wt[:] = 0
            t0 = time.perf_counter()
            ctx.render_ao(args.spp, tiles, W, H, occlude=args.occlude, radiance=rad, weight=wt)
            best = min(best, time.perf_counter() - t0)
        ao_mean = float(rad[..., 0].sum() / wt.sum())
        ctx.set_option("stats", 1)
        ctx.reset_stats()
        ctx.render_ao(args.spp, tiles, W, H, occlude=args.occlude)
        ks = ctx.kernel_stats()
        ctx.set_option("stats", 0)
    samples = W * H * args.spp
    print(json.dumps({"metric": "AO Msamples/s, 10M-tri soup 1080p", "value": samples / best / 1e6,
                      "spp": args.spp, "occlude": args.occlude, "seconds": best, "ao_mean": ao_mean,
                      "kernels_ms": {k: round(v["total_ms"], 3) for k, v in ks.items()}}))


if __name__ == "__main__":
    main()
