"""Per-bounce drain of the wavefront form: where its 1.17x over k_path
goes.  `run` (under rocprofv3 --kernel-trace) renders the C3 frame in the wavefront form: counting
renders at max_depth 1..5 first (the closest-hit rays of bounce b = rays(depth b+1) - rays(depth b)),
then `--spp` timed passes.  `summarize <dir>` reads the kernel trace: per bounce the closest-hit
launch's mean duration, the shade launch's, and the main stream's gaps; a least-squares fit
duration = a * rays + d over the five bounces gives each launch's fixed part d (ramp + drain: the
launch lasts as long as its slowest rays).

Usage (GPU box): rocprofv3 --kernel-trace --output-format csv -d gpurun_out/drain -o run -- python3 tools/wave_drain.py run
                 python3 tools/wave_drain.py summarize gpurun_out/drain"""
import csv
import glob
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))
W, H = 1920, 1080


def run(spp=4):
    import torch
    from akari_amd import capi, dist, scene
    cs = scene.compile_scene(scene.soup_scene(n_tris=10_000_000, resolution=(W, H)))
    ctx = capi.HipContext(0)
    scene.upload_scene(ctx, cs, builder=capi.BUILDER_SBVH, n_threads=16)
    ctx.set_option("path", 0)
    dev = torch.device("cuda", 0)
    film = torch.zeros(4 * W * H, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    tiles = dist.tile_grid(W, H, 64)
    n = dist.n_pixels(tiles)
    rays = []
    for d in range(1, 6):
        ctx.set_option("count_tests", 1)
        ctx.reset_stats()
        ctx.render_device(1, d, tiles, film[:3 * n].data_ptr(), film[3 * n:].data_ptr(), st)
        torch.cuda.synchronize(dev)
        rays.append(ctx.trace_counts()["per_mode"]["closest"]["rays"])
    ctx.set_option("count_tests", 0)
    per_bounce = [rays[0]] + [rays[k] - rays[k - 1] for k in range(1, 5)]
    ctx.render_device(2, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:].data_ptr(), st)   # warm
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    ctx.render_device(spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:].data_ptr(), st)
    torch.cuda.synchronize(dev)
    t = time.perf_counter() - t
    print("WAVE " + json.dumps({"closest_rays_per_bounce": per_bounce, "spp": spp, "ms_per_spp": t / spp * 1e3}),
          flush=True)
    ctx.close()


def summarize(d, log=None):
    ops = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ops.sort()
    info = None
    for l in open(log or os.path.join(d, "run.log")):
        if l.startswith("WAVE "):
            info = json.loads(l[5:])
    spp = info["spp"]
    is_closest = lambda k: "k_trace<0, false, true, true>" in k
    # the timed render's passes: the last spp raygen launches and what follows each
    raygen = [i for i, o in enumerate(ops) if "k_raygen" in o[2]]
    starts = raygen[-spp:]
    per_b = [[] for _ in range(5)]
    shade_b = [[] for _ in range(5)]
    pass_ms = []
    for k, i0 in enumerate(starts):
        i1 = starts[k + 1] if k + 1 < len(starts) else len(ops)
        seq = ops[i0:i1]
        cl = [o for o in seq if is_closest(o[2])]
        sh = [o for o in seq if "k_shade" in o[2]]
        for b, o in enumerate(cl[:5]):
            per_b[b].append((o[1] - o[0]) / 1e6)
        for b, o in enumerate(sh[:5]):
            shade_b[b].append((o[1] - o[0]) / 1e6)
        if k + 1 < len(starts):
            pass_ms.append((ops[i1][0] - ops[i0][0]) / 1e6)
    mean = lambda v: sum(v) / len(v) if v else float("nan")
    dur = [mean(v) for v in per_b]
    rays = info["closest_rays_per_bounce"]
    # least squares dur = a * rays + d
    n = len(dur)
    mx, my = sum(rays) / n, sum(dur) / n
    a = sum((x - mx) * (y - my) for x, y in zip(rays, dur)) / sum((x - mx) ** 2 for x in rays)
    dfix = my - a * mx
    out = {"ms_per_spp": info["ms_per_spp"], "pass_ms_trace": mean(pass_ms),
           "closest_ms_per_bounce": [round(x, 4) for x in dur], "shade_ms_per_bounce": [round(mean(v), 4) for v in shade_b],
           "closest_rays_per_bounce": rays, "fit_ms_per_mray": round(a * 1e6, 4), "fit_fixed_ms_per_launch": round(dfix, 4),
           "fixed_ms_per_pass": round(5 * dfix, 4),
           "main_stream_ms_per_pass": round(sum(dur) + sum(mean(v) for v in shade_b), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 4)
    else:
        summarize(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
