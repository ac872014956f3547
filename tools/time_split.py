"""Time split of the persistent path kernels: the counting build's
wave clocks over a C3 render — processing phases, the traversal phase split into issuing the wide
node's loads / waiting for them / the dependent work after them, the leaf phase likewise — for the
whole 1080p frame and an 8-way rank share, in the forms the library runs there.

Usage (GPU box): python tools/time_split.py [--spp 32] [--forms k_path,k_path_spec]"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))
sys.path.insert(0, str(ROOT))

FORM_OPTS = {"k_path": dict(path=1, path_spec=0, path_defer=0), "k_path_spec": dict(path=1, path_spec=1, path_defer=0),
             "k_path_defer": dict(path=1, path_spec=0, path_defer=1), "auto": dict(path=2, path_spec=2, path_defer=2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--forms", default="k_path,k_path_spec")
    ap.add_argument("--tris", type=int, default=10_000_000)
    args = ap.parse_args()
    import torch
    import bench
    from akari_amd import capi, dist, scene
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    cs = scene.compile_scene(scene.soup_scene(n_tris=args.tris, resolution=(W, H)))
    ctx = capi.HipContext(0)
    scene.upload_scene(ctx, cs, builder=capi.BUILDER_SBVH, n_threads=16)
    film = torch.zeros(4 * W * H, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    shares = {"whole": dist.tile_grid(W, H, 64), "8-way rank 0": dist.tiles_for_rank(W, H, 64, 0, 8)}
    for share, tiles in shares.items():
        n = dist.n_pixels(tiles)
        for form in args.forms.split(","):
            for k, v in FORM_OPTS[form].items():
                ctx.set_option(k, v)
            ctx.set_option("count_tests", 1)
            ctx.render_device(1, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
            torch.cuda.synchronize(dev)
            ctx.reset_stats()
            ctx.render_device(args.spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
            torch.cuda.synchronize(dev)
            split = bench.time_split(ctx.path_profile(), ctx.trace_counts())
            ctx.set_option("count_tests", 0)
            print(json.dumps({"share": share, "pixels": n, "spp": args.spp, "form": ctx.render_form()["form"],
                              "split": split}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
