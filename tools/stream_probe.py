"""The streaming wavefront (option wave_stream) beside the classic wavefront and the persistent form
on one scene: ms per spp of a whole-frame render (best of --repeat after a warm render), the form
that ran and, for the streaming form, the closest-hit launches it took.

Usage (GPU box): python tools/stream_probe.py [--scene soup|cornell|hall] [--spp 64] [--repeat 2]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="soup")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--forms", default="path,wave,stream")
    ap.add_argument("--opts", default="")
    args = ap.parse_args()
    import torch
    from akari_amd import capi, dist, scene
    if args.scene == "cornell":
        W, H = 1920, 1080
        sc = scene.cornell_scene(ROOT / "tests" / "golden" / "CornellBox-Original.obj.mesh", resolution=(W, H))
    elif args.scene == "hall":
        W, H = 3840, 2160
        sc = scene.hall_scene(resolution=(W, H))
    else:
        W, H = 1920, 1080
        sc = scene.soup_scene(n_tris=args.tris, resolution=(W, H))
    cs = scene.compile_scene(sc)
    ctx = capi.HipContext(0)
    t0 = time.time()
    scene.upload_scene(ctx, cs, builder=capi.BUILDER_SBVH, n_threads=16)
    print(f"{args.scene}: {cs.n_tris} triangles, BVH in {time.time() - t0:.1f} s", flush=True)
    for kv in (x for x in args.opts.split(",") if x):
        k, _, v = kv.partition("=")
        ctx.set_option(k, int(v))
    dev = torch.device("cuda", 0)
    film = torch.zeros(4 * W * H, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    tiles = dist.tile_grid(W, H, 64)
    n = dist.n_pixels(tiles)
    settings = {"path": {"path": 2, "wave_stream": 0}, "wave": {"path": 0, "wave_stream": 0},
                "stream": {"path": 0, "wave_stream": 1}}
    out = {"scene": args.scene, "spp": args.spp}
    for name in args.forms.split(","):
        for k, v in settings[name].items():
            ctx.set_option(k, v)
        ctx.render_device(4, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
        torch.cuda.synchronize(dev)
        best = None
        for _ in range(args.repeat):
            t = time.perf_counter()
            ctx.render_device(args.spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t) / args.spp * 1e3
            best = ms if best is None else min(best, ms)
        w = film[3 * n:4 * n]
        assert int(w.min().item()) == args.spp and int(w.max().item()) == args.spp
        out[name] = {"ms_per_spp": round(best, 4), "form": ctx.render_form()["form"],
                     "Msamples_per_s": round(n / best / 1e3, 1)}
        print(json.dumps({name: out[name]}), flush=True)
    print("STREAM " + json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
