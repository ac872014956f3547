"""Which persistent form wins where: for the Cornell box and soups
of 100K / 1M / 10M triangles at 1920x1080, rank 0's share of a 1- (whole frame), 2-, 4- and 8-way
interleaved 64x64 tile split rendered in each persistent form and in the library's automatic choice,
with the rule's inputs (pixels per resident lane, the cost-ordering pilot's mean steps per camera ray).

Usage (GPU box): python tools/form_probe.py [--spp 128] [--scenes cornell,soup100k,soup1m,soup10m]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))

FORMS = {"k_path": dict(path=1, path_spec=0, path_defer=0), "k_path_spec": dict(path=1, path_spec=1, path_defer=0),
         "k_path_defer": dict(path=1, path_spec=0, path_defer=1), "auto": dict(path=2, path_spec=2, path_defer=2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--scenes", default="cornell,soup100k,soup1m,soup10m")
    ap.add_argument("--splits", default="1,2,4,8")
    args = ap.parse_args()
    import torch
    from akari_amd import capi, dist, scene
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    film = torch.zeros(4 * W * H, device=dev)
    for name in args.scenes.split(","):
        if name == "cornell":
            sc = scene.cornell_scene(ROOT / "tests" / "golden" / "CornellBox-Original.obj.mesh", resolution=(W, H))
        else:
            n = {"soup100k": 100_000, "soup1m": 1_000_000, "soup10m": 10_000_000}[name]
            sc = scene.soup_scene(n_tris=n, resolution=(W, H))
        cs = scene.compile_scene(sc)
        with capi.HipContext(0) as ctx:
            t0 = time.time()
            scene.upload_scene(ctx, cs, builder=capi.BUILDER_SBVH, n_threads=16)
            print(f"{name}: {cs.n_tris} tris, built in {time.time() - t0:.1f} s", flush=True)
            for split in (int(x) for x in args.splits.split(",")):
                tiles = dist.tiles_for_rank(W, H, 64, 0, split)
                npx = dist.n_pixels(tiles)
                row = {"scene": name, "split": split, "pixels": npx}
                for form, opts in FORMS.items():
                    for k, v in opts.items():
                        ctx.set_option(k, v)
                    ctx.render_device(16, 5, tiles, film[:3 * npx].data_ptr(), film[3 * npx:4 * npx].data_ptr(), stream)
                    best = None
                    for _ in range(2):
                        torch.cuda.synchronize(dev)
                        t = time.perf_counter()
                        ctx.render_device(args.spp, 5, tiles, film[:3 * npx].data_ptr(), film[3 * npx:4 * npx].data_ptr(),
                                          stream)
                        torch.cuda.synchronize(dev)
                        ms = (time.perf_counter() - t) / args.spp * 1e3
                        best = ms if best is None else min(best, ms)
                    row[form] = round(best, 4)
                    if form == "auto":
                        row["auto_form"] = ctx.render_form()["form"]
                        row["inputs"] = ctx.render_form_inputs()
                row["best"] = min(FORMS, key=lambda f: row[f] if f != "auto" else 1e9)
                print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
