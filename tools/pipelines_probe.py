"""Probe: one frame rendered by one context vs split over two (or more) contexts on the SAME GPU
(akr_hip_render_node), i.e. independent pipelines whose launch tails can overlap.  Timing only.
Usage: python tools/pipelines_probe.py [steps] [n_ctx...]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))
from akari_amd import capi, scene  # noqa: E402
from akari_amd.dist import tiles_for_rank  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 16
counts = [int(x) for x in sys.argv[2:]] or [1, 2, 3]
W, H = 1920, 1080
cs = scene.compile_scene(scene.soup_scene(resolution=(W, H)))
ctxs = []
for k in range(max(counts)):
    c = capi.HipContext(0)
    scene.upload_scene(c, cs, n_threads=16)
    ctxs.append(c)
tiles = tiles_for_rank(W, H, 32, 0, 1)
for opts in ({"path": 0}, {"path": 0, "shadow_grid_pct": 50}, {"path": 2}):
    for c in ctxs:
        c.set_option("path", opts.get("path", 2))   # 0: the wavefront (north_star's layout)
        c.set_option("rays_per_lane", opts.get("rays_per_lane", 1))
        c.set_option("shadow_grid_pct", opts.get("shadow_grid_pct", 100))
    for n in counts:
        capi.render_node(ctxs[:n], 1, 5, tiles, W, H)   # warm
        t = time.perf_counter()
        capi.render_node(ctxs[:n], K, 5, tiles, W, H)
        dt = time.perf_counter() - t
        print(f"{opts} contexts {n}: {dt / K * 1e3:.3f} ms/step  {W * H * K / dt / 1e6:.1f} Msamples/s", flush=True)
