"""A/B of library builds (tools/experiments/build.sh <name>: tools/experiments/lib/libakr_hip_<name>.so) on
the C3 frame: the SBVH is built once (the product library) and saved under /tmp, then every build runs
in its own process (AKR_HIP_LIB; one library per process, so no symbol of one build can bind to
another's), adopting that BVH through akr_hip_import_accel, alternating builds for --repeat rounds.
Each process times the whole frame and the given rank shares of an N-way split at --spp.

A library may carry options of its own after an "@" (path@key=v,key=v), added to --opts.
Usage (GPU box): python tools/lib_ab.py --libs akarirender-1_amd/libakr_hip.so tools/experiments/lib/libakr_hip_x.so
                 [--spp 520] [--split 8 --ranks 0,5] [--repeat 2] [--opts key=v,...]"""
import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))
W, H = 1920, 1080


def worker(args):
    import numpy as np
    import torch
    from akari_amd import capi, dist, scene
    cs = scene.compile_scene(scene.soup_scene(n_tris=args.tris, resolution=(W, H)))
    ctx = capi.HipContext(0)
    for kv in (x for x in args.opts.split(",") if x):
        k, _, v = kv.partition("=")
        ctx.set_option(k, int(v))
    nodes, tris = np.load(args.bvh + "_nodes.npy", mmap_mode="r"), np.load(args.bvh + "_tris.npy", mmap_mode="r")
    scene.upload_scene(ctx, cs, bvh=(nodes, tris), n_threads=16)
    dev = torch.device("cuda", 0)
    film = torch.zeros(4 * W * H, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    shares = {"whole": dist.tile_grid(W, H, 64)}
    for r in (int(x) for x in args.ranks.split(",") if x):
        shares[f"{args.split}-way r{r}"] = dist.tiles_for_rank(W, H, 64, r, args.split)
    out = {}
    for name, tiles in shares.items():
        n = dist.n_pixels(tiles)
        ctx.render_device(20, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        ctx.render_device(args.spp, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
        torch.cuda.synchronize(dev)
        out[name] = round((time.perf_counter() - t) / args.spp * 1e3, 4)
        out[name + " form"] = ctx.render_form()["form"] + " ppl %.2f" % ctx.render_form_inputs()["pixels_per_lane"]
        if args.count:   # a 1-spp counting pass: lane utilisation of the loops, lanes holding a leaf per leaf phase
            ctx.set_option("count_tests", 1)
            ctx.reset_stats()
            ctx.render_device(1, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
            torch.cuda.synchronize(dev)
            ctx.set_option("count_tests", 0)
            cl, sh = (ctx.trace_counts()["per_mode"][m] for m in ("closest", "shadow"))
            pp = ctx.path_profile()
            out[name + " lanes"] = {
                "traversal": round((cl["visits"] + sh["visits"]) / max(1, cl["slots_traversal"]), 4),
                "triangles": round((cl["tri_tests"] + sh["tri_tests"]) / max(1, cl["slots_tri"]), 4),
                "holders_per_leaf_phase": round(pp["leaf_holders"] / max(1, pp["leaf_phases"]), 2),
                "holding_ray": round(cl["slots_busy"] / max(1, cl["slots_traversal"]), 4)}
            ctx.reset_stats()
        if args.kstats:   # one more render with HIP events on every launch: per-kernel ms per spp
            ctx.reset_stats()
            ctx.set_option("stats", 1)
            ctx.render_device(args.kstats, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
            torch.cuda.synchronize(dev)
            ctx.set_option("stats", 0)
            out[name + " kstats"] = {k: [v["launches"], round(v["total_ms"] / args.kstats, 4)]
                                     for k, v in ctx.kernel_stats().items()}
    ctx.close()
    print("RESULT " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=False, default=[])
    ap.add_argument("--spp", type=int, default=520)
    ap.add_argument("--split", type=int, default=8)
    ap.add_argument("--ranks", default="0")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--opts", default="")
    ap.add_argument("--kstats", type=int, default=0, help="N > 0: per-kernel launches and ms per spp of an N-spp render")
    ap.add_argument("--count", action="store_true", help="also a 1-spp counting pass (lane utilisation)")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--bvh", default="/tmp/akr_lib_ab_bvh")
    args = ap.parse_args()
    if args.worker:
        return worker(args)
    import numpy as np
    from akari_amd import capi, scene
    t0 = time.time()
    cs = scene.compile_scene(scene.soup_scene(n_tris=args.tris, resolution=(W, H)))
    nodes, tris, info = capi.build_bvh_host(cs.vertices, cs.indices, builder=capi.BUILDER_SBVH, n_threads=16)
    np.save(args.bvh + "_nodes.npy", nodes)
    np.save(args.bvh + "_tris.npy", tris)
    del nodes, tris
    print(f"SBVH built and saved in {time.time() - t0:.1f} s", flush=True)
    res = {lib: [] for lib in args.libs}
    try:
        for rep in range(args.repeat):
            for lib in args.libs:
                path, _, own = lib.partition("@")
                env = dict(os.environ, AKR_HIP_LIB=str(Path(path).resolve()))
                opts = ",".join(x for x in (args.opts, own) if x)
                cmd = [sys.executable, __file__, "--worker", "--spp", str(args.spp), "--split", str(args.split),
                       "--ranks", args.ranks, "--tris", str(args.tris), "--opts", opts, "--bvh", args.bvh,
                       "--kstats", str(args.kstats)] + (["--count"] if args.count else [])
                p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
                line = next((l for l in p.stdout.splitlines() if l.startswith("RESULT ")), None)
                if p.returncode != 0 or line is None:
                    print(p.stdout[-2000:], p.stderr[-3000:], flush=True)
                    raise SystemExit(f"{lib}: worker failed with {p.returncode}")
                r = json.loads(line[7:])
                res[lib].append(r)
                print(json.dumps({"lib": lib, "rep": rep, **r}), flush=True)
    finally:
        for suf in ("_nodes.npy", "_tris.npy"):
            Path(args.bvh + suf).unlink(missing_ok=True)
    print("summary (min over repeats, ms per spp)", flush=True)
    for lib, rs in res.items():
        keys = [k for k in rs[0] if not k.endswith((" form", " kstats", " lanes"))]
        print(json.dumps({"lib": lib, **{k: min(r[k] for r in rs) for k in keys}}), flush=True)


if __name__ == "__main__":
    main()
