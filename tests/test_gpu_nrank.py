"""The HIP N-rank path end to end: bench.py --gpus 2 spawns two ranks under
torch.distributed.run, rank 0 builds the SBVH and shares it, rank 1 adopts it through
akr_hip_import_accel, each rank renders its interleaved tile share with the HIP library, the films
are all-gathered, and rank 0 checks the assembled frame bit for bit against one whole-frame render
of its own context.  On the one-GPU test box both ranks use device 0 and the gather runs over gloo
(--rehearse-one-gpu); on a multi-GPU node the same code runs over RCCL (bench.py).  Reference:
pixels are independent (sampler seeded x + y*W, cpu/integrator.cpp:124), SURVEY.md §8e."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


# (ranks, triangles, width, height, tile, steps, frame spp): toy frames at 2 and 3 ranks, and the
# driver's 8-way split of a 1080p frame in 64x64 tiles: each rank's share is the
# size the 8-GPU bench renders, so the form each rank picks from its own pilot is the one it runs there
CASES = {2: (50_000, 200, 120, 16, 2, 6), 3: (50_000, 200, 120, 16, 2, 6), 8: (1_000_000, 1920, 1080, 64, 1, 4)}


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 3, 8])
def test_nrank_hip_tile_split_gather_bit_exact(ranks):
    tris, width, height, tile, steps, spp = CASES[ranks]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", str(ranks), "--rehearse-one-gpu", "--verify-frame",
           "--tris", str(tris), "--width", str(width), "--height", str(height), "--tile", str(tile), "--steps",
           str(steps), "--frame-spp", str(spp), "--warmup", "1", "--cpu-baseline", "0", "--wavefront-spp", "0",
           "--side-legs", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = lines[0]
    assert line["n_gpus"] == ranks and "REHEARSAL" in line["data"]
    assert line["config"]["spp"] == spp and line["config"]["parallelism"] == f"tile-split x{ranks}"
    fc = line["frame_check"]
    assert fc["weights_equal"], fc
    assert fc["bit_exact"], fc
    assert fc["mean_radiance"] > 0.0
    assert fc["adopted_bvh"] == [False] + [True] * (ranks - 1), fc
