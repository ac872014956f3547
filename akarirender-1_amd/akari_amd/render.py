"""SceneNode::render (core/nodes/scene.cpp:112-160) on the HIP path: upload the scene through the
C-ABI, run the scene's integrator node on the GPU, and write the film.

The integrator node picks the C-ABI call the reference's compile_gpu would have produced
(core/nodes/integrator.cpp:26-84):
  Path -> akr_hip_render (gpu::PathTracer: spp, max_depth, tile_size, ray_clamp)
  AO   -> akr_hip_render_ao (AmbientOcclusion: spp, occlude)
The reference's GPU AO adds acc/spp once per pixel with weight 1 (gpu/cuda/integrator.cpp:83-90),
its CPU AO adds every sample with weight 1 (cpu/integrator.cpp:78); both resolve to the same
image acc/spp, and this film holds the CPU form (radiance = acc, weight = spp).

Usage: python -m akari_amd.render scene.akari [--out image.png|.pfm] [--gpus N]
"""
from __future__ import annotations

import argparse
import math
import sys
import time
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import capi, film, scene
from .dist import tile_grid


def _tiles(sc: scene.Scene, tile_size: int) -> List[Tuple[int, int, int, int]]:
    w, h = (int(v) for v in sc.camera.resolution)
    return tile_grid(w, h, max(1, int(tile_size)))


def render_scene(sc: scene.Scene, devices: Sequence[int] = (0,), **build_kw) -> Tuple[np.ndarray, np.ndarray]:
    """Render `sc` with its integrator node; returns the film (radiance [H,W,3], weight [H,W])."""
    cs = scene.compile_scene(sc)
    w, h = (int(v) for v in sc.camera.resolution)
    it = sc.integrator
    ctxs = [capi.HipContext(d) for d in devices]
    try:
        for c in ctxs:
            scene.upload_scene(c, cs, **build_kw)
        if isinstance(it, scene.AOIntegrator):
            if len(ctxs) != 1:
                raise ValueError("the AO integrator renders on one device")
            return ctxs[0].render_ao(it.spp, _tiles(sc, 16), w, h, occlude=it.occlude)
        if isinstance(it, scene.PathIntegrator):
            tiles = _tiles(sc, it.tile_size)
            if len(ctxs) == 1:
                return ctxs[0].render(it.spp, it.max_depth, tiles, w, h, ray_clamp=it.ray_clamp)
            return capi.render_node(ctxs, it.spp, it.max_depth, tiles, w, h, ray_clamp=it.ray_clamp)
        raise ValueError(f"integrator {type(it).__name__} is not supported on gpu")
    finally:
        for c in ctxs:
            c.close()


def write_film(path: str, radiance: np.ndarray, weight: np.ndarray) -> None:
    """Film::write_image (core/film.h:97-113): PNG is sRGB 8-bit, PFM keeps linear floats."""
    if path.lower().endswith(".pfm"):
        film.write_pfm(path, radiance, weight)
    else:
        film.write_png(path, radiance, weight)


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="akari_amd.render", description=__doc__.splitlines()[0])
    ap.add_argument("scene")
    ap.add_argument("--out", default=None, help="output image (default: the scene's `output` field)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--spp", type=int, default=None, help="override the integrator's spp")
    args = ap.parse_args(argv)
    sc = scene.load_scene_file(args.scene)
    if args.spp is not None:
        sc.integrator.spp = args.spp
    t0 = time.time()
    rad, wt = render_scene(sc, devices=list(range(args.gpus)))
    out = args.out or sc.output
    write_film(out, rad, wt)
    print(f"{type(sc.integrator).__name__} {sc.camera.resolution[0]}x{sc.camera.resolution[1]} "
          f"spp {sc.integrator.spp}: {time.time() - t0:.2f}s -> {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
