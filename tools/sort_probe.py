"""The wavefront's ray reordering (tools/experiments/wave_sort.patch: option wave_sort; run with
AKR_HIP_LIB=tools/experiments/lib/libakr_hip_wave_sort.so) measured per scene:
for each configuration, one context at a time (one context per process time: several live contexts share
the process's four hardware queues and serialise their streams), the BVH imported from one SBVH build,
ms per spp of a render in the production stream layout, then a 1-spp counting pass for the traversal
loop's lane utilisation and the node visits per ray.  --no-count with one configuration is the form for a
rocprofv3 --pmc pass around it (tools/sort_pmc.py sums the trace kernels' counters).

Usage (GPU box): python tools/sort_probe.py --scene soup [--spp 32] [--split 8 --rank 0]
                 --configs path=0 path=0,wave_sort=3 ..."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


def parse(cfg):
    out = {}
    for kv in (x for x in cfg.split(",") if x):
        k, _, v = kv.partition("=")
        out[k] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", choices=["soup", "hall", "cornell"], default="soup")
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--split", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--configs", nargs="+", default=["path=0", "path=0,wave_sort=3"])
    ap.add_argument("--no-count", action="store_true", help="skip the counting pass (PMC runs)")
    ap.add_argument("--kstats", type=int, default=0, help="N > 0: per-kernel ms per spp of an N-spp render with HIP events")
    args = ap.parse_args()
    import torch
    from akari_amd import capi, dist, scene
    W, H = (3840, 2160) if args.scene == "hall" else (1920, 1080)
    if args.scene == "soup":
        sc = scene.soup_scene(n_tris=args.tris, resolution=(W, H))
    elif args.scene == "hall":
        sc = scene.hall_scene(resolution=(W, H))
    else:
        sc = scene.cornell_scene(ROOT / "tests" / "golden" / "CornellBox-Original.obj.mesh", resolution=(W, H))
    cs = scene.compile_scene(sc)
    t0 = time.time()
    nodes, tris, _ = capi.build_bvh_host(cs.vertices, cs.indices, builder=capi.BUILDER_SBVH, n_threads=16)
    print(f"SBVH built in {time.time() - t0:.1f} s", flush=True)
    dev = torch.device("cuda", 0)
    tiles = dist.tile_grid(W, H, 64) if args.split == 1 else dist.tiles_for_rank(W, H, 64, args.rank, args.split)
    n = dist.n_pixels(tiles)
    film = torch.zeros(4 * n, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def render(c, spp):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        c.render_device(spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:].data_ptr(), stream)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / spp * 1e3

    for cfg in args.configs:
        with capi.HipContext(0) as c:
            scene.upload_scene(c, cs, bvh=(nodes, tris), n_threads=16)
            for k, v in parse(cfg).items():
                c.set_option(k, v)
            render(c, 2)
            ms = [render(c, args.spp) for _ in range(args.repeat)]
            rec = {"scene": args.scene, "split": args.split, "rank": args.rank, "pixels": n, "config": cfg,
                   "spp": args.spp, "ms_per_spp": [round(x, 4) for x in ms], "form": c.render_form()["form"]}
            if not args.no_count:
                c.set_option("count_tests", 1)
                c.reset_stats()
                render(c, 1)
                tc = c.trace_counts()["per_mode"]
                c.set_option("count_tests", 0)
                for m in ("closest", "shadow"):
                    x = tc[m]
                    rec[m] = {"rays": x["rays"], "visits_per_ray": round(x["visits"] / max(1, x["rays"]), 2),
                              "tri_per_ray": round(x["tri_tests"] / max(1, x["rays"]), 2),
                              "lane_util_traversal": round(x["visits"] / max(1, x["slots_traversal"]), 4),
                              "holding_ray": round(x["slots_busy"] / max(1, x["slots_traversal"]), 4),
                              "lane_util_triangles": round(x["tri_tests"] / max(1, x["slots_tri"]), 4)}
            if args.kstats:
                c.reset_stats()
                c.set_option("stats", 1)
                render(c, args.kstats)
                c.set_option("stats", 0)
                rec["kstats"] = {k: [v["launches"], round(v["total_ms"] / args.kstats, 4)] for k, v in c.kernel_stats().items()}
            print("SORT " + json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
