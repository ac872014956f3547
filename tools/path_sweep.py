"""Tuning sweep of the persistent path kernel (k_path) on C3: per library build (AKR_HIP_LIB variants
or the product lib) and per runtime setting, the full-frame step (N = 1) and the step of one rank's
share of an 8-way tile split.  One scene generation per process, one BVH build per library.

Usage (GPU box): python tools/path_sweep.py [--libs a.so,b.so] [--min-wait 16,32,48] [--steps 8]"""
import argparse
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default=str(ROOT / "akarirender-1_amd" / "libakr_hip.so"))
    ap.add_argument("--min-wait", default="0", help="0: the per-kernel default (comma list)")
    ap.add_argument("--path", default="1")
    ap.add_argument("--far-first", default="0", help="occlusion rays far slots first (comma list)")
    ap.add_argument("--defer", default="2", help="path_defer: 0 k_path, 1 k_path_defer at every size, 2 the library's choice (comma list; r18 sweeps ran with 1, EXPERIMENTS.md §9 caveat)")
    ap.add_argument("--mix", default="1", help="scrambled pixel fetch in k_path_defer (comma list)")
    ap.add_argument("--grid-pct", default="100", help="persistent path grid, %% of resident (comma list)")
    ap.add_argument("--tab", default="1", help="scene tables in LDS (comma list)")
    ap.add_argument("--order", default="2", help="cost-ordered pixel fetch: 0 off, 1 k_path, 2 both forms (comma list)")
    ap.add_argument("--order-shift", default="2", help="pilot-step classes of 2^shift (comma list)")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--builder", default="sbvh")
    ap.add_argument("--scene", choices=["soup", "hall", "cornell"], default="soup")
    ap.add_argument("--profile", type=int, default=0, help="also print the counted k_path phase profile")
    ap.add_argument("--splits", default="8", help="emulated ranks of the tile split to time besides the full frame")
    ap.add_argument("--opts", default="", help="extra library options to sweep: 'key=v1,v2;key2=v1,v2' (cartesian)")
    ap.add_argument("--collapse", default="0", help="wide_collapse build parameter(s): one context each (comma list)")
    args = ap.parse_args()
    libs = args.libs.split(",")
    if len(libs) > 1:
        # one child process per library: the product binding loads the library RTLD_GLOBAL, so a
        # second library in the same process would have its internal calls bound to the first one's
        # kernels.  This parent never touches the GPU.
        import subprocess
        rc = 0
        for lib in libs:
            argv = [a for a in sys.argv[1:]]
            k = argv.index("--libs")
            argv[k + 1] = lib
            rc = rc or subprocess.run([sys.executable, "-u", __file__, *argv]).returncode
        sys.exit(rc)
    import torch
    from akari_amd import dist
    dev = torch.device("cuda", 0)
    W, H = (3840, 2160) if args.scene == "hall" else (1920, 1080)
    full = dist.tile_grid(W, H, 32)
    splits = [int(x) for x in args.splits.split(",")]
    shares = {n: dist.tiles_for_rank(W, H, 32, 0, n) for n in splits}
    share = shares[splits[-1]]
    film = torch.zeros(4 * W * H, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for lib in libs:
        os.environ["AKR_HIP_LIB"] = lib
        import akari_amd.capi as capi
        import akari_amd.scene as scene
        if args.scene == "hall":
            sc = scene.hall_scene(resolution=(W, H))
        elif args.scene == "cornell":
            sc = scene.cornell_scene(Path(__file__).resolve().parent.parent / "tests" / "golden" / "CornellBox-Original.obj.mesh",
                                     resolution=(W, H))
        else:
            sc = scene.soup_scene(n_tris=args.tris, resolution=(W, H))
        cs = scene.compile_scene(sc)  # this module's types
        for collapse in (int(x) for x in args.collapse.split(",")):
            ctx = capi.HipContext(0)
            t0 = time.time()
            scene.upload_scene(ctx, cs, builder={"sah": capi.BUILDER_SAH, "sbvh": capi.BUILDER_SBVH,
                                                 "lbvh": capi.BUILDER_LBVH}[args.builder], n_threads=16,
                               wide_collapse=collapse)
            print(f"== {Path(lib).name} wide_collapse={collapse}: built in {time.time() - t0:.1f} s, "
                  f"BVH2 nodes {ctx.accel_info().n_nodes}", flush=True)
            combos = [(p, f, d, m, t, o, osh) for p in (int(x) for x in args.path.split(",")) for f in (int(x) for x in args.far_first.split(","))
                      for d in (int(x) for x in args.defer.split(",")) for m in (int(x) for x in args.mix.split(","))
                      for t in (int(x) for x in args.tab.split(",")) for o in (int(x) for x in args.order.split(","))
                      for osh in (int(x) for x in args.order_shift.split(","))]
            import itertools
            extra = [(kv.split("=")[0], [int(x) for x in kv.split("=")[1].split(",")]) for kv in args.opts.split(";") if kv]
            extra_combos = list(itertools.product(*[[(k, v) for v in vs] for k, vs in extra])) or [()]
            combos = [c + (e,) for c in combos for e in extra_combos]
            for path, ff, dfr, mx, tab, order, osh, ex in combos:
                for k, v in ex:
                    ctx.set_option(k, v)
                ctx.set_option("path_order", order)
                ctx.set_option("path_order_shift", osh)
                ctx.set_option("path_tab", tab)
                ctx.set_option("path", path)
                ctx.set_option("any_far_first", ff)
                ctx.set_option("path_defer", dfr)
                ctx.set_option("path_mix", mx)
                for mw, gp in ((m, g) for m in (int(x) for x in args.min_wait.split(",")) for g in (int(x) for x in args.grid_pct.split(","))):
                    ctx.set_option("path_min_wait", mw)
                    ctx.set_option("path_grid_pct", gp)
                    res = []
                    for tiles in [full] + [shares[n] for n in splits]:
                        n = dist.n_pixels(tiles)
                        ctx.render_device(2, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
                        torch.cuda.synchronize(dev)
                        t = time.perf_counter()
                        ctx.render_device(args.steps, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
                        torch.cuda.synchronize(dev)
                        res.append((time.perf_counter() - t) / args.steps * 1e3)
                    print(f"   path={path} far_first={ff} defer={dfr} mix={mx} tab={tab} order={order}/{osh} min_wait={mw} grid={gp}%"
                          f"{''.join(f' {k}={v}' for k, v in ex)}: full {res[0]:.3f} ms/step ({W * H / res[0] / 1e3:.1f} Msamples/s)"
                          + "".join(f", {n}-way rank {r:.3f} ms/step (projected {res[0] / r:.2f}x, {W * H / r / 1e3:.0f} Msamples/s)"
                                    for n, r in zip(splits, res[1:])), flush=True)
                    if args.profile and path:
                        for name, tiles in (("full", full), ("8-way", share)):
                            n = dist.n_pixels(tiles)
                            ctx.set_option("count_tests", 1)
                            ctx.reset_stats()
                            ctx.render_device(args.steps, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:4 * n].data_ptr(), stream)
                            torch.cuda.synchronize(dev)
                            q = ctx.path_profile()
                            c = ctx.trace_counts()
                            ctx.set_option("count_tests", 0)
                            w = max(1, q["waves"])
                            us = lambda t: t / 100.0   # 100 MHz ticks -> us
                            print(f"     {name} counted: waves {q['waves']}, mean wave {us(q['t_total'] / w):.0f} us, longest "
                                  f"{us(q['t_max']):.0f} us; per wave: outer {q['outer'] / w:.0f}, proc {q['procs'] / w:.0f} "
                                  f"({q['lanes_proc'] / max(1, q['procs']):.1f} lanes each), trav iters {q['trav_iters'] / w:.0f}; "
                                  f"time proc {q['t_proc'] / max(1, q['t_total']):.3f} trav {q['t_trav'] / max(1, q['t_total']):.3f} "
                                  f"leaf {q['t_leaf'] / max(1, q['t_total']):.3f}; us per trav iter "
                                  f"{us(q['t_trav']) / max(1, q['trav_iters']):.3f}, per proc {us(q['t_proc']) / max(1, q['procs']):.2f} "
                                  f"(results/shading {us(q['t_shade']) / max(1, q['procs']):.2f}), "
                                  f"per outer leaf {us(q['t_leaf']) / max(1, q['outer']):.3f}; rays/px closest "
                                  f"{c['per_mode']['closest']['rays'] / n / args.steps:.2f} shadow "
                                  f"{c['per_mode']['shadow']['rays'] / n / args.steps:.2f}; speculative samples "
                                  f"{q['spec_started'] / n / args.steps:.3f} per sample, dropped "
                                  f"{q['spec_aborted'] / max(1, q['spec_started']):.3f}", flush=True)
            ctx.close()


if __name__ == "__main__":
    main()
