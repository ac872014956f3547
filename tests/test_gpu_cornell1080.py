"""BASELINE.json configs[1] (C2) at its own size: the reference's Cornell box (resources/data/
cornell_box/scene.akari:3-21, the .mesh fixture) at 1920x1080, max_depth 5.

The closed box keeps every path alive to max_depth (a camera ray always hits), so this is the
integrator's shading, NEE and bounce code at full frame, not the soup's traversal.  The oracle renders
the whole frame at 2 spp in seconds, so the bar is the whole frame bit-exact in radiance and weights
in the library's default form, and the strided tile subset bit-exact with the per-pixel fingerprint
(final sampler state, closest-hit and shadow rays per pixel) in every render form."""
import numpy as np
import pytest

import py_oracle
from akari_amd import capi, dist, scene
from conftest import CORNELL_MESH
from helpers import check_probe

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

W, H, TILE = 1920, 1080, 64


@pytest.fixture(scope="module")
def cornell1080(hip_ctx_factory):
    ctx = hip_ctx_factory(0)
    cs = scene.compile_scene(scene.cornell_scene(CORNELL_MESH, resolution=(W, H)))
    scene.upload_scene(ctx, cs)
    nodes, tris = ctx.accel_export()
    orc = py_oracle.OracleScene(cs, nodes, tris, capi)
    yield ctx, cs, orc
    ctx.close()


def test_cornell_1080p_full_frame_bit_exact(cornell1080):
    """The whole 1080p frame, 2 spp, through render_device in the library's default form: every pixel
    holds 2 samples (the in-band check runs as well) and equals the oracle bit for bit."""
    import torch
    ctx, cs, orc = cornell1080
    tiles = dist.tile_grid(W, H, TILE)
    n = dist.n_pixels(tiles)
    assert n == W * H
    dev = torch.device("cuda", 0)
    film = torch.zeros(4 * n, device=dev)
    ctx.render_device(2, 5, tiles, film[:3 * n].data_ptr(), film[3 * n:].data_ptr(),
                      torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    form = ctx.render_form()
    packed = film.cpu().numpy()
    assert np.all(packed[3 * n:] == 2.0), "a pixel does not hold 2 samples"
    rad = np.zeros((H, W, 3), np.float32)
    w = np.zeros((H, W), np.float32)
    dist.unpack_to_frame(packed, tiles, W, H, rad, w)
    orad, ow, st = orc.render(2, 5, n_threads=16)
    assert np.array_equal(w, ow)
    diff = np.abs(rad - orad).max()
    assert np.array_equal(rad, orad), f"{form}: radiance differs from the oracle (max abs diff {diff})"
    # the box is lit and the paths bounce: NEE and multi-bounce radiance reach the film
    assert st["shadow_rays"] > n and st["extension_rays"] > 4 * n
    assert orad.mean() > 0.05


FORMS = [
    ("k_path", dict(path=1, path_defer=0, path_spec=0, path_order=0)),
    ("k_path ordered", dict(path=1, path_defer=0, path_spec=0, path_order=1)),
    ("k_path_defer ordered", dict(path=1, path_defer=1, path_spec=0, path_order=2)),
    ("k_path_spec ordered", dict(path=1, path_defer=0, path_spec=1, path_order=2)),
    ("wavefront", dict(path=0, path_defer=2, path_spec=2, path_order=2)),
]
DEFAULTS = dict(path=2, path_defer=2, path_spec=2, path_order=2, path_order_min_spp=16, count_tests=0, pixel_probe=0)


def test_cornell_1080p_tile_subset_every_form(cornell1080):
    """Every 16th 64x64 tile, 2 spp, each render form (persistent ones also in the counting build):
    radiance and weights bit-exact, and the per-pixel fingerprint equal to the oracle's."""
    ctx, cs, orc = cornell1080
    tiles = dist.tiles_for_rank(W, H, TILE, 3, 16)
    orad, ow, _, opr = orc.render(2, 5, tiles=tiles, n_threads=16, probe=True)
    counted = []
    try:
        ctx.set_option("pixel_probe", 1)
        ctx.set_option("path_order_min_spp", 0)
        for name, opts in FORMS:
            for count in ((0, 1) if opts["path"] == 1 else (0,)):
                for k, v in opts.items():
                    ctx.set_option(k, v)
                ctx.set_option("count_tests", count)
                what = f"{name}{' (counting build)' if count else ''}"
                rad, w = ctx.render(2, 5, tiles, W, H)
                assert np.array_equal(w, ow), f"{what}: weights differ"
                assert np.array_equal(rad, orad), f"{what}: radiance differs (max {np.abs(rad - orad).max()})"
                if check_probe(ctx.pixel_probe(dist.n_pixels(tiles)), opr, tiles, W, H, what):
                    counted.append(what)
    finally:
        for k, v in DEFAULTS.items():
            ctx.set_option(k, v)
        ctx.reset_stats()
    assert len(counted) == 5, counted


def test_cornell_8way_share_takes_k_path(cornell1080):
    """The form rule: the Cornell box's 8-way share (64x64 tiles,
    16 spp, default options) has about one pixel per resident lane like the soup's, but its rays are a
    few traversal steps long (a 36-triangle scene), so a freed lane has no long fetch chain to overlap
    and the library runs k_path (measured faster there than the tail forms);
    bit-exact against the oracle."""
    ctx, cs, orc = cornell1080
    share = dist.tiles_for_rank(W, H, TILE, 0, 8)
    rad, w = ctx.render(16, 5, share, W, H)
    form, inp = ctx.render_form(), ctx.render_form_inputs()
    assert form == {"form": "k_path", "ordered": True}, (form, inp)
    assert 0.5 < inp["pixels_per_lane"] < 1.5 and inp["pilot_mean_steps"] < 12, inp
    assert inp["pilot_rays"] == dist.n_pixels(share)
    orad, ow, _ = orc.render(16, 5, tiles=share, n_threads=16)
    assert np.array_equal(w, ow)
    assert np.array_equal(rad, orad), f"radiance differs (max abs diff {np.abs(rad - orad).max()})"
