"""Load balance of the interleaved tile split: every rank's share of an N-way split of
the C3 frame rendered on this one GPU, one after another, with the library's default (auto) form.
The N-rank bench step is the slowest rank's, so the max over ranks is the projected step.

Usage (GPU box): python tools/rank_shares.py [--splits 2,4,8] [--steps 20] [--warmup 5] [--repeat 2]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", default="2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--opts", default="", help="library options 'key=v;key2=v'")
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
    for kv in (x for x in args.opts.split(";") if x):
        k, _, v = kv.partition("=")
        ctx.set_option(k, int(v))
    film = torch.zeros(4 * W * H, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step_ms(tiles, spp):
        n = dist.n_pixels(tiles)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        ctx.render_device(spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / spp * 1e3

    full = dist.tile_grid(W, H, args.tile)
    step_ms(full, args.warmup)
    runs = [step_ms(full, args.steps) for _ in range(args.repeat)]
    whole, whole_avg = min(runs), sum(runs) / len(runs)
    print(json.dumps({"split": 1, "ms_per_step": round(whole, 3), "ms_per_step_avg": round(whole_avg, 3),
                      "form": ctx.render_form()}), flush=True)
    for n in (int(x) for x in args.splits.split(",")):
        per, per_avg = [], []
        for r in range(n):
            tiles = dist.tiles_for_rank(W, H, args.tile, r, n)
            step_ms(tiles, args.warmup)
            runs = [step_ms(tiles, args.steps) for _ in range(args.repeat)]
            per.append(min(runs))
            per_avg.append(sum(runs) / len(runs))
        worst, worst_avg = max(per), max(per_avg)
        # best-of-repeats per rank, and the average over repeats (what one N-rank run sees on average)
        print(json.dumps({"split": n, "rank_ms": [round(x, 3) for x in per], "max_ms": round(worst, 3),
                          "mean_ms": round(sum(per) / n, 3), "imbalance": round(worst * n / sum(per), 3),
                          "projected_speedup": round(whole / worst, 2),
                          "rank_ms_avg": [round(x, 3) for x in per_avg], "max_ms_avg": round(worst_avg, 3),
                          "projected_speedup_avg": round(whole_avg / worst_avg, 2), "form": ctx.render_form()}),
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
