"""Cost-balanced rank partition: does giving each rank tiles of
equal estimated cost, instead of tile k -> rank k % world, shorten the slowest rank?

A pilot render of the whole frame (counting build, per-pixel probe: closest-hit + shadow rays of
the first S samples) gives each tile's cost; tiles are assigned longest-first to the rank with the
least cost so far (LPT), ties by tile index, so every rank computes the same partition.  Then every
rank's share is timed at --spp for both partitions, alternating.

Usage (GPU box): python tools/balance_probe.py [--world 8] [--spp 1040] [--pilot-spp 4] [--repeat 2]"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--spp", type=int, default=1040)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--pilot-spp", type=int, default=4)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--tile", type=int, default=32)
    args = ap.parse_args()
    import torch
    from akari_amd import capi, dist, scene
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    cs = scene.compile_scene(scene.soup_scene(n_tris=args.tris, resolution=(W, H)))
    ctx = capi.HipContext(0)
    t0 = time.time()
    scene.upload_scene(ctx, cs, builder=capi.BUILDER_SBVH, n_threads=16)
    print(f"built in {time.time() - t0:.1f} s", flush=True)
    grid = dist.tile_grid(W, H, args.tile)
    n_all = dist.n_pixels(grid)
    film = torch.zeros(4 * n_all, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    # pilot: rays per tile over the first pilot-spp samples
    ctx.set_option("count_tests", 1)
    ctx.set_option("pixel_probe", 1)
    t = time.perf_counter()
    ctx.render_device(args.pilot_spp, 5, grid, film[:3 * n_all].data_ptr(), film[3 * n_all:].data_ptr(), stream)
    torch.cuda.synchronize(dev)
    pilot_ms = (time.perf_counter() - t) * 1e3
    pr = ctx.pixel_probe(n_all)
    ctx.set_option("pixel_probe", 0)
    ctx.set_option("count_tests", 0)
    rays = pr["closest_rays"].astype(np.int64) + pr["shadow_rays"]
    sizes = np.array([(x1 - x0) * (y1 - y0) for x0, y0, x1, y1 in grid])
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    tile_cost = np.add.reduceat(rays, starts)

    def lpt(cost, world):
        order = sorted(range(len(cost)), key=lambda k: (-int(cost[k]), k))
        load = [0] * world
        own = [[] for _ in range(world)]
        for k in order:
            r = min(range(world), key=lambda q: (load[q], q))
            load[r] += int(cost[k])
            own[r].append(k)
        return [[grid[k] for k in sorted(o)] for o in own], load

    bal, bal_load = lpt(tile_cost, args.world)
    inter = [dist.tiles_for_rank(W, H, args.tile, r, args.world) for r in range(args.world)]
    inter_load = [int(sum(tile_cost[k] for k in range(len(grid)) if k % args.world == r)) for r in range(args.world)]
    print(json.dumps({"pilot_ms": round(pilot_ms, 2), "pilot_spp": args.pilot_spp,
                      "interleaved_cost": inter_load, "balanced_cost": bal_load,
                      "interleaved_pixels": [dist.n_pixels(x) for x in inter],
                      "balanced_pixels": [dist.n_pixels(x) for x in bal]}), flush=True)

    def share_ms(tiles, spp):
        n = dist.n_pixels(tiles)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        ctx.render_device(spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / spp * 1e3

    res = {"interleaved": [[] for _ in range(args.world)], "balanced": [[] for _ in range(args.world)]}
    share_ms(inter[0], args.warmup)
    for rep in range(args.repeat):
        for r in range(args.world):
            for name, part in (("interleaved", inter), ("balanced", bal)):
                res[name][r].append(share_ms(part[r], args.spp))
        print(f"repeat {rep} done", flush=True)
    for name in res:
        per = [min(x) for x in res[name]]
        print(json.dumps({"partition": name, "world": args.world, "spp": args.spp,
                          "rank_ms": [round(x, 4) for x in per], "max_ms": round(max(per), 4),
                          "mean_ms": round(sum(per) / len(per), 4),
                          "imbalance": round(max(per) * len(per) / sum(per), 4)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
