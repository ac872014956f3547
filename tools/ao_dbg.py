import sys
from pathlib import Path
import numpy as np
ROOT = Path("/root/repo")
sys.path[:0] = [str(ROOT / "akarirender-1_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import py_oracle
from akari_amd import capi, scene
from helpers import cornell
with capi.HipContext(0) as ctx:
    cs = scene.compile_scene(cornell((40, 24)))
    scene.upload_scene(ctx, cs)
    nodes, tris = ctx.accel_export()
    orc = py_oracle.OracleScene(cs, nodes, tris, capi)
    tiles = [(0, 0, 16, 16), (24, 8, 40, 24), (30, 0, 64, 64), (5, 5, 5, 9)]
    for rep in range(3):
        for occlude in (float("inf"), 1e30, 1.0, 0.0, -1.0, float("nan")):
            rad, w = ctx.render_ao(3, tiles, 40, 24, occlude=occlude)
            orad, ow, _ = orc.render_ao(3, tiles=tiles, occlude=occlude)
            bw = np.argwhere(w != ow)
            br = np.argwhere(np.any(rad != orad, axis=-1)) if rad.ndim == 3 else np.argwhere(rad != orad)
            print(rep, occlude, "w bad", len(bw), bw[:4].tolist(), [ (w[tuple(b)], ow[tuple(b)]) for b in bw[:4]], "rad bad", len(br), flush=True)
