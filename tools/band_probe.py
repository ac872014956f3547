"""Locality probe for the rank partition: the C3 frame's 8-way split rendered as the
bench's interleaved 64x64 tiles (tile k -> rank k % 8) and as contiguous row bands (rank r: rows
[r H / 8, (r + 1) H / 8), cut into 64-pixel-wide column tiles), each share one after another on this
GPU with the library's default form, beside the whole frame.  An interleaved share spreads its pixels
over the whole soup surface, so each XCD's L2 sees 1/8 of the pixel density of a whole frame; a band
keeps a rank's paths in 1/8 of the surface.  Sum over bands < whole frame = locality gain.

Usage (GPU box): python tools/band_probe.py [--spp 256] [--repeat 2]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


def band_tiles(W, y0, y1, tw=64):
    return [(x, y0, min(W, x + tw), y1) for x in range(0, W, tw)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--tris", type=int, default=10_000_000)
    args = ap.parse_args()
    import torch
    from akari_amd import capi, dist, scene
    W, H, N = 1920, 1080, args.world
    dev = torch.device("cuda", 0)
    cs = scene.compile_scene(scene.soup_scene(n_tris=args.tris, resolution=(W, H)))
    ctx = capi.HipContext(0)
    t0 = time.time()
    scene.upload_scene(ctx, cs, builder=capi.BUILDER_SBVH, n_threads=16)
    print(f"built in {time.time() - t0:.1f} s", flush=True)
    film = torch.zeros(4 * W * H, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def ms_per_spp(tiles, spp):
        n = dist.n_pixels(tiles)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        ctx.render_device(spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / spp * 1e3

    def measure(name, shares):
        rows = []
        for tiles in shares:
            ms_per_spp(tiles, 16)
            best = min(ms_per_spp(tiles, args.spp) for _ in range(args.repeat))
            inp, form = ctx.render_form_inputs(), ctx.render_form()
            rows.append({"px": dist.n_pixels(tiles), "ms": round(best, 4), "form": form["form"],
                         "pilot_mean_steps": inp["pilot_mean_steps"]})
        ms = [r["ms"] for r in rows]
        print(json.dumps({"partition": name, "max_ms": max(ms), "sum_ms": round(sum(ms), 3),
                          "mean_ms": round(sum(ms) / len(ms), 4), "shares": rows}), flush=True)
        return ms

    whole = measure("whole", [dist.tile_grid(W, H, 64)])[0]
    inter = measure("interleaved64", [dist.tiles_for_rank(W, H, 64, r, N) for r in range(N)])
    bands = measure("bands", [band_tiles(W, r * H // N, (r + 1) * H // N) for r in range(N)])
    print(json.dumps({"whole_ms": whole, "interleaved_speedup": round(whole / max(inter), 3),
                      "band_sum_over_whole": round(sum(bands) / whole, 3),
                      "interleaved_sum_over_whole": round(sum(inter) / whole, 3),
                      "balanced_band_bound_speedup": round(whole * N / sum(bands), 3)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
