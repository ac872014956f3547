"""Debug: cooperative-tail traces vs the oracle on the LBVH 100K soup (small batches, many seeds)."""
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "akarirender-1_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import py_oracle
from akari_amd import capi, scene
from helpers import hits_to_gid, random_rays, small_soup

with capi.HipContext(0) as ctx:
    cs = scene.compile_scene(small_soup(100_000))
    scene.upload_scene(ctx, cs, builder=capi.BUILDER_LBVH)
    nodes, tris = ctx.accel_export()
    orc = py_oracle.OracleScene(cs, nodes, tris, capi)
    for coop in ([int(x) for x in sys.argv[1:]] or (0, 1, 2)):
        ctx.set_option("coop", coop)
        bad = 0
        tot = 0
        for seed in range(40):
            n = [1, 7, 64, 200, 1000, 4096][seed % 6]
            rays = random_rays(n, 100 + seed, -1.3, 1.3)
            gh = ctx.trace(rays, any_hit=False)
            oh, _, _ = orc.trace(rays, any_hit=False)
            ok = (gh["geom_id"] >= -1) & (gh["geom_id"] < len(cs.mesh_base) - 1)
            gh["geom_id"][~ok] = -1
            g = hits_to_gid(gh, cs.mesh_base)
            diff = np.nonzero((g != oh["gid"]) | ((oh["gid"] != 0xFFFFFFFF) & (gh["t"] != oh["t"])))[0]
            tot += n
            bad += diff.size
            for i in diff[:3]:
                print("coop", coop, "seed", seed, "ray", i, "o", rays["o"][i], "d", rays["d"][i], "gpu", g[i], gh["t"][i], "orc", oh["gid"][i], oh["t"][i], flush=True)
        rad, w = ctx.render(2, 5, [(0, 0, 96, 54)], 96, 54)
        orad, ow, _ = orc.render(2, 5, tiles=[(0, 0, 96, 54)])
        print("coop", coop, "trace bad", bad, "of", tot, "render bad", int((rad != orad).sum()), flush=True)
