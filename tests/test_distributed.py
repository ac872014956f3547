"""Tile-split across ranks + frame-end gather, rehearsed with gloo (world size 2, CPU).

Each rank renders only its interleaved tiles (akari_amd.dist.tiles_for_rank) — here with the CPU
restatement standing in for the device renderer, since the partition and the gather are the logic
under test — and the all-gather assembles the frame, which must equal the single-process render
bit for bit (pixels are independent: sampler seeded x + y*W, cpu/integrator.cpp:124)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from akari_amd import dist


def test_tile_partition_is_exact_cover():
    W, H, T = 70, 45, 16
    grid = dist.tile_grid(W, H, T)
    for world in (1, 2, 3, 8):
        parts = [dist.tiles_for_rank(W, H, T, r, world) for r in range(world)]
        cover = np.zeros((H, W), np.int32)
        for p in parts:
            for x0, y0, x1, y1 in p:
                cover[y0:y1, x0:x1] += 1
        assert np.all(cover == 1)
        assert sum(len(p) for p in parts) == len(grid)
        sizes = [dist.n_pixels(p) for p in parts]
        assert max(sizes) - min(sizes) <= T * T
        assert dist.max_pixels_per_rank(W, H, T, world) == max(sizes)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, T, out):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    for p in (root / "akarirender-1_amd", root / "oracle", root / "tests"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as tdist
    import py_oracle as O
    from akari_amd import capi, dist as D, scene
    from helpers import cornell
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    cs = scene.compile_scene(cornell((W, H)))
    nodes, tris, _ = capi.build_bvh_host(cs.vertices, cs.indices)
    orc = O.OracleScene(cs, nodes, tris, capi)
    tiles = D.tiles_for_rank(W, H, T, rank, world)
    cap = D.max_pixels_per_rank(W, H, T, world)
    rad, wt, _ = orc.render(3, 5, tiles=tiles, n_threads=2)
    film = np.zeros(4 * cap, np.float32)          # packed [rgb * cap | w * cap], tiles in order
    k = 0
    for x0, y0, x1, y1 in tiles:
        n = (x1 - x0) * (y1 - y0)
        film[3 * k:3 * (k + n)] = rad[y0:y1, x0:x1].reshape(-1)
        film[3 * cap + k:3 * cap + k + n] = wt[y0:y1, x0:x1].reshape(-1)
        k += n
    frame, fw = D.gather_frame(torch.from_numpy(film), W, H, T)
    if rank == 0:
        np.save(out, np.concatenate([frame.reshape(-1), fw.reshape(-1)]))
    tdist.destroy_process_group()


def test_gloo_tile_split_gather_equals_single_render(tmp_path):
    import py_oracle as O
    from akari_amd import capi, scene
    from helpers import cornell
    W, H, T = 40, 28, 16
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(2, _free_port(), W, H, T, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    cs = scene.compile_scene(cornell((W, H)))
    nodes, tris, _ = capi.build_bvh_host(cs.vertices, cs.indices)
    rad, wt, _ = O.OracleScene(cs, nodes, tris, capi).render(3, 5)
    assert np.array_equal(got, np.concatenate([rad.reshape(-1), wt.reshape(-1)]))
