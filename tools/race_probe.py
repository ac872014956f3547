"""Repeat small renders and count film mismatches against the first render of each mode (the
results are deterministic, so any difference is a race).  Usage: python tools/race_probe.py [reps]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "akarirender-1_amd"), str(ROOT / "tests")]
from akari_amd import capi, scene  # noqa: E402
from helpers import cornell  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
tiles = [(0, 0, 16, 16), (24, 8, 40, 24), (30, 0, 64, 64), (5, 5, 5, 9)]
modes = {"classic": dict(lookahead=1), "la3": dict(lookahead=3), "la3_noexit": dict(lookahead=3, la_early_exit=0),
         "la64": dict(lookahead=64), "ao": dict(lookahead=1)}
with capi.HipContext(0) as ctx:
    scene.upload_scene(ctx, scene.compile_scene(cornell((40, 24))))
    for name, opts in modes.items():
        for k, v in opts.items():
            ctx.set_option(k, v)
        bad_w = bad_r = 0
        ref = None
        for i in range(reps):
            spp, depth = (9, 2) if i % 2 else (13, 5)
            if name == "ao":
                r, w = ctx.render_ao(spp, tiles, 40, 24)
            else:
                r, w = ctx.render(spp, depth, tiles, 40, 24)
            key = i % 2
            if ref is None:
                ref = {}
            if key not in ref:
                ref[key] = (r, w)
                continue
            if not np.array_equal(w, ref[key][1]):
                bad_w += 1
                d = np.argwhere(w != ref[key][1])
                print(f"  {name} rep {i}: {len(d)} weights differ, e.g. {d[:3].tolist()} {w[tuple(d[0])]} vs {ref[key][1][tuple(d[0])]}",
                      ctx.render_info() if name != "ao" else "", flush=True)
            elif not np.array_equal(r, ref[key][0]):
                bad_r += 1
                print(f"  {name} rep {i}: radiance differs", flush=True)
        ctx.set_option("la_early_exit", 1)
        print(f"{name}: {reps} renders, weight mismatches {bad_w}, radiance mismatches {bad_r}", flush=True)
