"""Per-pixel chain profile of a persistent render (diagnostic): with the counting
build and option "pixel_probe" 2 every pixel records its committed rays (closest-hit + shadow, all
samples) and the wall clock at which its last sample was committed.  A share of a tile split ends
when its last pixel does; this shows whether the last pixels are the costliest chains (the sampler
chain is the floor) or ordinary ones (the waves are).

Usage (GPU box): python tools/chain_profile.py [--split 8] [--spp 128] [--configs "" "path_spec=0"]"""
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
    ap.add_argument("--split", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--configs", nargs="+", default=["", "path_spec=0"])
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
    tiles = dist.tile_grid(W, H, 32) if args.split == 1 else dist.tiles_for_rank(W, H, 32, args.rank, args.split)
    n = dist.n_pixels(tiles)
    film = torch.zeros(4 * n, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    base = {}
    for cfg in args.configs:
        opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in cfg.split(",") if kv)
        for k, v in opts.items():
            base.setdefault(k, None)
            ctx.set_option(k, v)
        ctx.set_option("count_tests", 1)
        ctx.set_option("pixel_probe", 2)
        ctx.reset_stats()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        ctx.render_device(args.spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:].data_ptr(), stream)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t
        pr = ctx.pixel_probe(n)
        q = ctx.path_profile()
        ctx.set_option("pixel_probe", 0)
        ctx.set_option("count_tests", 0)
        rays = (pr["closest_rays"].astype(np.int64) + pr["shadow_rays"]) / args.spp
        tick = (pr["flags"] >> 8).astype(np.int64)
        assert (pr["flags"] & 4).all(), "completion clock not recorded (counting build of a persistent kernel?)"
        tick = (tick - tick.min()) * 16 / 100.0   # us (100 MHz wall clock, recorded / 16)
        end = tick.max()
        order = np.argsort(-rays)
        last = np.argsort(-tick)[: max(1, n // 100)]
        out = {"config": cfg or "(defaults)", "form": ctx.render_form(), "split": args.split, "pixels": n,
               "spp": args.spp, "wall_ms": round(wall * 1e3, 2),
               "completion_us_pct": {p: round(float(np.percentile(tick, p)), 1) for p in (1, 10, 50, 90, 99, 100)},
               "rays_per_sample_pct": {p: round(float(np.percentile(rays, p)), 2) for p in (1, 10, 50, 90, 99, 100)},
               "corr_rays_completion": round(float(np.corrcoef(rays, tick)[0, 1]), 3),
               "costliest_1pct": {"rays": round(float(rays[order[: n // 100]].mean()), 2),
                                  "completion_frac_of_end": round(float(tick[order[: n // 100]].mean() / end), 3)},
               "last_1pct_completed": {"rays": round(float(rays[last].mean()), 2),
                                       "rays_rank_pct": round(float(np.mean([np.searchsorted(np.sort(rays), rays[i]) for i in last]) / n * 100), 1)},
               "spec": {"started_per_sample": round(q["spec_started"] / n / args.spp, 4),
                        "dropped": round(q["spec_aborted"] / max(1, q["spec_started"]), 4)},
               "waves": {"mean_us": round(q["t_total"] / max(1, q["waves"]) / 100.0, 1), "longest_us": round(q["t_max"] / 100.0, 1)}}
        # completion time against cost: mean completion per cost decile
        dec = np.array_split(order[::-1], 10)
        out["completion_frac_by_cost_decile"] = [round(float(tick[d].mean() / end), 3) for d in dec]
        print(json.dumps(out), flush=True)
        for k in opts:   # back to the library's defaults for the next configuration
            ctx.set_option(k, {"path_spec": 2, "path_defer": 2, "path_order": 2, "path_order_pair": 2}.get(k, 0))
    ctx.close()


if __name__ == "__main__":
    main()
