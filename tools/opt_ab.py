"""A/B of library runtime options on the C3 frame (or one rank's share of an N-way split) at the
driver's spp: one context per configuration (each adopts the first context's BVH through
akr_hip_import_accel, so every configuration runs on the same tree and starts from the library's
defaults), renders alternating between configurations, `--repeat` rounds.

Usage (GPU box): python tools/opt_ab.py --spp 1040 [--split 8 --rank 0] --configs "" "path_order=0" "path_order_classes=2,path_order_shift=3"
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


BUILD_OPTS = {"leaf_align"}   # options read when the BVH is built or imported


def parse(cfg: str):
    out = {}
    for kv in (x for x in cfg.split(",") if x):
        k, _, v = kv.partition("=")
        out[k] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=1040)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--split", type=int, default=1, help="1: whole frame; N: rank --rank's share of an N-way split")
    ap.add_argument("--ranks", default="0", help="ranks of the split to time (comma list; 'all')")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--tile", type=int, default=64, help="tile size of the split (bench.py's default; 32 before r20)")
    ap.add_argument("--configs", nargs="+", default=[""])
    ap.add_argument("--kstats", type=int, default=0,
                    help="N > 0: after the timed rounds, one N-spp render per config with HIP events on every "
                         "launch, printing the per-kernel launch counts and average ms")
    ap.add_argument("--scene", choices=["soup", "cornell", "hall"], default="soup",
                    help="cornell: the C2 box at 1080p; hall: the C4 stand-in at 4K (ADVICE r4: wave_order there)")
    args = ap.parse_args()
    import torch
    from akari_amd import capi, dist, scene
    W, H = (3840, 2160) if args.scene == "hall" else (1920, 1080)
    dev = torch.device("cuda", 0)
    if args.scene == "cornell":
        sc = scene.cornell_scene(ROOT / "tests" / "golden" / "CornellBox-Original.obj.mesh", resolution=(W, H))
    elif args.scene == "hall":
        sc = scene.hall_scene(resolution=(W, H))
    else:
        sc = scene.soup_scene(n_tris=args.tris, resolution=(W, H))
    cs = scene.compile_scene(sc)
    ctxs = []
    t0 = time.time()
    base = capi.HipContext(0)
    for key, v in parse(args.configs[0]).items():   # build-time options take effect at the upload
        if key in BUILD_OPTS:
            base.set_option(key, v)
    scene.upload_scene(base, cs, builder=capi.BUILDER_SBVH, n_threads=16)
    nodes, tris = base.accel_export()
    print(f"built in {time.time() - t0:.1f} s", flush=True)
    for k, cfg in enumerate(args.configs):
        c = base if k == 0 else capi.HipContext(0)
        if k:
            for key, v in parse(cfg).items():
                if key in BUILD_OPTS:
                    c.set_option(key, v)
            scene.upload_scene(c, cs, bvh=(nodes, tris), n_threads=16)
        for key, v in parse(cfg).items():
            c.set_option(key, v)
        ctxs.append(c)
    del nodes, tris
    film = torch.zeros(4 * W * H, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ranks = list(range(args.split)) if args.ranks == "all" else [int(r) for r in args.ranks.split(",")]
    shares = {r: (dist.tile_grid(W, H, args.tile) if args.split == 1 else dist.tiles_for_rank(W, H, args.tile, r, args.split))
              for r in ranks}

    def run(c, tiles, spp):
        n = dist.n_pixels(tiles)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        c.render_device(spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / spp * 1e3

    for c in ctxs:
        for r in ranks:
            run(c, shares[r], args.warmup)
    res = {cfg: {r: [] for r in ranks} for cfg in args.configs}
    for rep in range(args.repeat):
        for cfg, c in zip(args.configs, ctxs):
            for r in ranks:
                ms = run(c, shares[r], args.spp)
                res[cfg][r].append(ms)
                print(json.dumps({"config": cfg or "(defaults)", "split": args.split, "rank": r, "rep": rep,
                                  "ms_per_spp": round(ms, 4), "form": c.render_form()}), flush=True)
    print("summary (ms per spp: min over repeats per rank; max over ranks)", flush=True)
    for cfg in args.configs:
        per = {r: min(v) for r, v in res[cfg].items()}
        print(json.dumps({"config": cfg or "(defaults)", "split": args.split, "spp": args.spp,
                          "per_rank_min": {r: round(x, 4) for r, x in per.items()},
                          "max_over_ranks": round(max(per.values()), 4),
                          "all": {r: [round(x, 4) for x in v] for r, v in res[cfg].items()}}), flush=True)
    if args.kstats:
        for cfg, c in zip(args.configs, ctxs):
            c.reset_stats()
            c.set_option("stats", 1)
            ms = run(c, shares[ranks[0]], args.kstats)
            ks = c.kernel_stats()
            c.set_option("stats", 0)
            print(json.dumps({"kstats": cfg or "(defaults)", "spp": args.kstats, "ms_per_spp_with_events": round(ms, 4),
                              "kernels": {k: {"launches": v["launches"], "avg_ms": round(v["total_ms"] / v["launches"], 4),
                                              "ms_per_spp": round(v["total_ms"] / args.kstats, 4)}
                                          for k, v in ks.items()}}), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
