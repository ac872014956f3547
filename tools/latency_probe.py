"""Traversal latency probe on the C3 soup: per-ray step distributions (option "ray_steps") and
closest-hit launch time against batch size, for camera rays, first-bounce rays and shadow rays.
Answers: is a small launch bound by its slowest rays (a heavy tail of steps) or by the per-step
latency of every ray?  Prints JSON lines.

Usage: python tools/latency_probe.py [--tris 10000000]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))


def camera_rays(W, H, pos, fov_deg, rng):
    s = np.tan(np.radians(fov_deg) / 2)   # approximate pinhole (shape of the workload only)
    y, x = np.mgrid[0:H, 0:W].astype(np.float32)
    x = x + rng.random(x.shape, np.float32)
    y = y + rng.random(y.shape, np.float32)
    px = (2 * x / W - 1) * s * W / H
    py = (1 - 2 * y / H) * s
    d = np.stack([px, py, -np.ones_like(px)], -1).reshape(-1, 3)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros(d.shape[0], [("o", np.float32, 3), ("tmin", np.float32), ("d", np.float32, 3), ("tmax", np.float32)])
    r["o"] = pos
    r["tmin"] = 1e-3
    r["d"] = d
    r["tmax"] = np.inf
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from akari_amd import capi, scene

    W, H = 1920, 1080
    rng = np.random.default_rng(1)
    cs = scene.compile_scene(scene.soup_scene(n_tris=args.tris, resolution=(W, H)))
    V = cs.vertices
    I = cs.indices.reshape(-1, 3)
    with capi.HipContext(0) as ctx:
        scene.upload_scene(ctx, cs, max_leaf_size=4, intersect_cost=4.0, n_threads=16)

        def launch_ms(rays, any_hit):
            ctx.set_option("stats", 1)
            ctx.reset_stats()
            for _ in range(args.reps):
                ctx.trace(rays, any_hit=any_hit)
            st = ctx.kernel_stats()["trace_any" if any_hit else "trace_closest"]
            ctx.set_option("stats", 0)
            return st["min_ms"]

        def steps_of(rays, any_hit):
            ctx.set_option("ray_steps", 1)
            hits = ctx.trace(rays, any_hit=any_hit)
            s = ctx.ray_steps(rays.shape[0])
            ctx.set_option("ray_steps", 0)
            return hits, s

        def report(name, rays, any_hit):
            hits, s = steps_of(rays, any_hit)
            ok = s != 0xFFFFFFFF
            sv = s[ok].astype(np.int64)
            q = np.percentile(sv, [50, 90, 99, 99.9, 99.99]).tolist() if sv.size else []
            sizes = [rays.shape[0], 1 << 20, 259_200, 65_536, 16_384, 4_096, 1_024, 64]
            times = {}
            for n in sizes:
                if n > rays.shape[0]:
                    continue
                sub = rays[rng.choice(rays.shape[0], n, replace=False)] if n < rays.shape[0] else rays
                times[n] = round(launch_ms(sub, any_hit), 4)
            order = np.argsort(sv)
            slow = rays[ok][order[-1024:]]
            fast = rays[ok][order[:1024]]
            print(json.dumps({"set": name, "n": int(rays.shape[0]), "exact_fallback": int((~ok).sum()),
                              "steps_mean": float(sv.mean()), "steps_pct_50_90_99_999_9999": q,
                              "steps_max": int(sv.max()), "launch_ms_by_n": times,
                              "slowest1024_ms": round(launch_ms(slow, any_hit), 4),
                              "fastest1024_ms": round(launch_ms(fast, any_hit), 4)}), flush=True)
            return hits

        cam = camera_rays(W, H, np.array([0, 0, 4], np.float32), 40.0, rng)
        h = report("camera", cam, False)
        hit = h["prim_id"] >= 0
        # first-bounce rays: cosine-ish directions about the hit triangle's normal
        gid = h["prim_id"][hit]
        p = cam["o"][hit] + h["t"][hit, None] * cam["d"][hit]
        tri = V[I[gid]]
        n = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
        n /= np.linalg.norm(n, axis=1, keepdims=True) + 1e-30
        n *= np.where(np.sum(n * cam["d"][hit], 1) > 0, -1, 1)[:, None]
        w = rng.normal(size=n.shape).astype(np.float32)
        w /= np.linalg.norm(w, axis=1, keepdims=True)
        w = n + w
        w /= np.linalg.norm(w, axis=1, keepdims=True) + 1e-30
        b = np.zeros(p.shape[0], cam.dtype)
        b["o"] = p
        b["tmin"] = 1e-3
        b["d"] = w
        b["tmax"] = np.inf
        report("bounce1", b, False)
        # shadow rays: light point -> hit point (the NEE direction convention, light.h:68-69)
        lp = np.stack([rng.uniform(-1, 1, p.shape[0]), np.full(p.shape[0], 1.5), rng.uniform(-1, 1, p.shape[0])],
                      -1).astype(np.float32)
        dv = p - lp
        dist = np.linalg.norm(dv, axis=1)
        s = np.zeros(p.shape[0], cam.dtype)
        s["o"] = lp
        s["tmin"] = 1e-3
        s["d"] = dv / dist[:, None]
        s["tmax"] = dist * (1 - 1e-4)
        report("shadow", s, True)


if __name__ == "__main__":
    main()
