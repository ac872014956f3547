"""Fixed and per-sample cost of a render (C3 soup): times the whole frame and one rank's share of
an N-way tile split at several spp in one process, fits time = F + spp * x per share, and prints
the library's per-kernel HIP-event breakdown of one render per point (kernel_stats).  F is what a
render pays regardless of its length: pilot and sort, launch ramp, the tail of the longest pixel
chain beyond the mean, film check and unpack.

Usage (GPU box): python tools/spp_fit.py [--spps 1,2,5,10,20,64] [--splits 1,8] [--reps 2]"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spps", default="1,2,5,10,20,64")
    ap.add_argument("--splits", default="1,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--opts", default="", help="library options 'key=v;key2=v'")
    ap.add_argument("--profile-spp", type=int, default=20, help="counted phase profile at this spp (0: none)")
    ap.add_argument("--sweep", default="", help="one library option swept in-process: 'key=v1,v2,...'")
    args = ap.parse_args()
    import numpy as np
    import torch
    from akari_amd import capi, dist, scene
    dev = torch.device("cuda", 0)
    W, H = 1920, 1080
    sc = scene.soup_scene(n_tris=args.tris, resolution=(W, H))
    cs = scene.compile_scene(sc)
    ctx = capi.HipContext(0)
    t0 = time.time()
    scene.upload_scene(ctx, cs, builder=capi.BUILDER_SBVH, n_threads=16)
    print(f"built in {time.time() - t0:.1f} s", flush=True)
    for kv in (x for x in args.opts.split(";") if x):
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    ctx.set_option("stats", 1)  # HIP events around every launch (kernel_stats)
    film = torch.zeros(4 * W * H, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    spps = [int(x) for x in args.spps.split(",")]
    sweep = [(args.sweep.split("=")[0], int(v)) for v in args.sweep.split("=")[1].split(",")] if args.sweep else [None]
    for n_split, sw in ((n, sw) for n in (int(x) for x in args.splits.split(",")) for sw in sweep):
        if sw:
            ctx.set_option(*sw)
            print(f"-- {sw[0]} = {sw[1]}", flush=True)
        tiles = dist.tile_grid(W, H, 32) if n_split == 1 else dist.tiles_for_rank(W, H, 32, 0, n_split)
        n = dist.n_pixels(tiles)
        rt = capi.rect_array(tiles)  # as the bench passes it

        def render(spp):
            ctx.render_device(spp, 5, rt, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)

        render(2)
        torch.cuda.synchronize(dev)
        xs, ys = [], []
        for spp in spps:
            for _ in range(args.reps):
                ctx.reset_stats()
                torch.cuda.synchronize(dev)
                t = time.perf_counter()
                render(spp)
                torch.cuda.synchronize(dev)
                ms = (time.perf_counter() - t) * 1e3
                ks = ctx.kernel_stats()
                form = ctx.render_form()
                xs.append(spp)
                ys.append(ms)
                kt = ", ".join(f"{k} {v['total_ms']:.3f}" for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["total_ms"])
                               if v["launches"])
                print(f"{n_split}-way share ({n} px) spp {spp}: {ms:.3f} ms ({ms / spp:.3f} ms/spp) form {form}; "
                      f"kernels [ms]: {kt}", flush=True)
        A = np.vstack([np.ones(len(xs)), np.array(xs, float)]).T
        (F, x), *_ = np.linalg.lstsq(A, np.array(ys), rcond=None)
        print(f"== {n_split}-way share: time = {F:.3f} ms + spp x {x:.4f} ms  (fit over spp {spps})", flush=True)
        if args.profile_spp:
            ctx.set_option("count_tests", 1)
            ctx.reset_stats()
            render(args.profile_spp)
            torch.cuda.synchronize(dev)
            q = ctx.path_profile()
            ctx.set_option("count_tests", 0)
            w = max(1, q["waves"])
            print(f"   counted {args.profile_spp} spp: waves {q['waves']}, mean wave {q['t_total'] / w / 100:.0f} us, "
                  f"longest {q['t_max'] / 100:.0f} us ({q['t_max'] * w / max(1, q['t_total']):.2f}x the mean)", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
