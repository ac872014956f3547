"""The headline configuration at full size (BASELINE.json configs[2]): the
10,000,002-triangle soup with the SBVH the bench builds, 1920x1080, max_depth 5.

Bar: bit-exact against the oracle walking the same exported BVH2 with the reference algorithm
(bvh-accelerator.h:488-547; pathtracer.h:61-164) — seeded closest-hit and any-hit traces (camera-like
rays from the bench camera and rays from inside the soup), a strided tile subset of the frame
rendered at 2 spp, and the deep-stack path: the counting kernel must see rays whose traversal stack
went past the LDS-resident entries into the global overflow area.  At the full frame, where the
oracle would take minutes, size-independent properties: every pixel holds exactly spp samples, and
the frame is the same bit for bit whether rendered whole or as one rank's share of an 8-way split
(pixels are independent, cpu/integrator.cpp:124).
"""
import dataclasses

import numpy as np
import pytest

import py_oracle
from akari_amd import capi, dist, scene
from helpers import check_probe, hits_to_gid, random_rays

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

W, H, TILE = 1920, 1080, 32


@pytest.fixture(scope="module")
def c3(hip_ctx_factory):
    ctx = hip_ctx_factory(0)
    cs = scene.compile_scene(scene.soup_scene(n_tris=10_000_000, resolution=(W, H)))
    assert cs.n_tris == 10_000_002
    info = scene.upload_scene(ctx, cs, builder=capi.BUILDER_SBVH, n_threads=16)
    nodes, tris = ctx.accel_export()
    assert len(tris) > cs.n_tris, "the SBVH duplicates references on the soup"
    orc = py_oracle.OracleScene(cs, nodes, tris, capi)
    yield ctx, cs, orc, info
    ctx.close()


def _camera_rays(cs, n, seed):
    """Rays from the bench camera (0, 0, 4) through random points of the soup's bounding cube."""
    rng = np.random.default_rng(seed)
    r = np.zeros(n, capi.RAY_DTYPE)
    o = np.asarray(cs.camera.position, np.float32)
    target = rng.uniform(-1.01, 1.01, (n, 3)).astype(np.float32)
    d = target - o
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    r["o"] = o
    r["d"] = d
    r["tmin"] = np.float32(1e-3)
    r["tmax"] = np.float32(np.inf)
    return r


def _check(ctx, orc, cs, rays, any_hit, exact=False):
    ctx.set_option("exact_cull", int(exact))
    gh = ctx.trace(rays, any_hit=any_hit)
    oh, _, _ = orc.trace(rays, any_hit=any_hit, exact_cull=exact, n_threads=16)
    ctx.set_option("exact_cull", 0)
    ggid = hits_to_gid(gh, cs.mesh_base)
    bad = np.count_nonzero(ggid != oh["gid"])
    assert bad == 0, f"{bad} of {len(rays)} hit ids differ"
    hit = oh["gid"] != 0xFFFFFFFF
    assert np.array_equal(gh["t"][hit], oh["t"][hit])
    if not any_hit:
        assert np.array_equal(gh["u"][hit], oh["u"][hit]) and np.array_equal(gh["v"][hit], oh["v"][hit])
    return hit.mean()


@pytest.mark.parametrize("any_hit", [False, True])
def test_c3_trace_bit_exact(c3, any_hit):
    ctx, cs, orc, _ = c3
    n = 1 << 17
    frac_cam = _check(ctx, orc, cs, _camera_rays(cs, n, 100 + any_hit), any_hit)
    frac_in = _check(ctx, orc, cs, random_rays(n, 200 + any_hit, -1.0, 1.0), any_hit)
    assert frac_cam > 0.5 and frac_in > 0.5   # the rays really run through the soup


def test_c3_trace_reference_cull_bit_exact(c3):
    """The reference's own intersectAABB (AKR_PT_EXACT_CULL: no behind-origin cull, ~10x the box
    tests) on a smaller batch."""
    ctx, cs, orc, _ = c3
    _check(ctx, orc, cs, random_rays(1 << 12, 300, -1.0, 1.0), False, exact=True)
    _check(ctx, orc, cs, _camera_rays(cs, 1 << 12, 301), True, exact=True)


def test_c3_deep_stack_overflow_path(c3):
    """Rays whose traversal stack spills past the LDS entries (the global overflow area) are
    present in the parity batches above and come out bit-exact."""
    ctx, cs, orc, _ = c3
    rays = np.concatenate([_camera_rays(cs, 1 << 16, 400), random_rays(1 << 16, 401, -1.0, 1.0)])
    ctx.set_option("count_tests", 1)
    ctx.reset_stats()
    try:
        _check(ctx, orc, cs, rays, False)
        deep = ctx.trace_counts()["per_mode"]["closest"]["deep_rays"]
        ctx.reset_stats()
        _check(ctx, orc, cs, rays, True)
        deep_any = ctx.trace_counts()["per_mode"]["any"]["deep_rays"]
    finally:
        ctx.set_option("count_tests", 0)
        ctx.reset_stats()
    assert deep > 0, "no closest-hit ray reached the overflow stack"
    print(f"deep-stack rays: closest {deep}, any-hit {deep_any} of {len(rays)}")


def test_c3_render_tile_subset_bit_exact(c3):
    """Every 64th 32x32 tile of the 1080p frame, 2 spp, max_depth 5, through the C-ABI."""
    ctx, cs, orc, _ = c3
    tiles = dist.tiles_for_rank(W, H, TILE, 0, 64)
    rad, w = ctx.render(2, 5, tiles, W, H)
    orad, ow, st = orc.render(2, 5, tiles=tiles, n_threads=16)
    assert np.array_equal(w, ow)
    assert (ow > 0).sum() == dist.n_pixels(tiles)
    diff = np.abs(rad - orad).max()
    assert np.array_equal(rad, orad), f"radiance differs (max abs diff {diff})"
    # NEE runs (shadow rays are traced), though the 1-cm mean free path of the soup occludes the
    # emitter above it from everything the camera sees: the C3 frame is dark by construction
    assert st["shadow_rays"] > 0 and st["extension_rays"] > 0
    # the cost-ordered pixel fetch (on by default from 16 spp) forced on at 2 spp,
    # for k_path and for the deferred form this subset runs with by default
    try:
        for order, defer in ((1, 0), (2, 2)):
            ctx.set_option("path_order", order)
            ctx.set_option("path_order_min_spp", 0)
            ctx.set_option("path_defer", defer)
            rad2, w2 = ctx.render(2, 5, tiles, W, H)
            assert np.array_equal(w2, ow) and np.array_equal(rad2, orad), f"path_order={order} differs"
    finally:
        ctx.set_option("path_order", 2)
        ctx.set_option("path_order_min_spp", 16)
        ctx.set_option("path_defer", 2)


def test_c3_full_frame_split_invariance(c3):
    """Full 1080p frame at 1 spp on the device (cost-ordered fetch forced on): every pixel holds one
    sample (the library's in-band check runs too), and rank 3's share of an 8-way tile split renders the same bits as the same
    pixels of the whole frame."""
    import torch
    ctx, cs, orc, _ = c3
    dev = torch.device("cuda", 0)
    full = dist.tile_grid(W, H, TILE)
    n = dist.n_pixels(full)
    film = torch.zeros(4 * n, device=dev)
    ctx.set_option("path_order_min_spp", 0)  # the whole frame with the cost-ordered fetch (§3.10)
    try:
        ctx.render_device(1, 5, full, film[:3 * n].data_ptr(), film[3 * n:].data_ptr(),
                          torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
    finally:
        ctx.set_option("path_order_min_spp", 16)
    packed = film.cpu().numpy()
    assert np.all(packed[3 * n:] == 1.0)
    frame = np.zeros((H, W, 3), np.float32)
    fw = np.zeros((H, W), np.float32)
    dist.unpack_to_frame(packed, full, W, H, frame, fw)
    share = dist.tiles_for_rank(W, H, TILE, 3, 8)
    m = dist.n_pixels(share)
    sfilm = torch.zeros(4 * m, device=dev)
    ctx.render_device(1, 5, share, sfilm[:3 * m].data_ptr(), sfilm[3 * m:].data_ptr(),
                      torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    sframe = np.zeros((H, W, 3), np.float32)
    sw = np.zeros((H, W), np.float32)
    dist.unpack_to_frame(sfilm.cpu().numpy(), share, W, H, sframe, sw)
    sel = sw > 0
    assert sel.sum() == m
    assert np.array_equal(sframe[sel], frame[sel])


# Every render form of the library, as set_option values: (path, path_defer, path_order, count_tests).
# The persistent kernels record per-pixel ray counts in their counting build only; the seed always.
FORMS = [
    ("k_path", dict(path=1, path_defer=0, path_order=0)),
    ("k_path ordered", dict(path=1, path_defer=0, path_order=1)),
    ("k_path_defer scrambled", dict(path=1, path_defer=1, path_order=0)),
    ("k_path_defer ordered", dict(path=1, path_defer=1, path_order=2, path_order_pair=0)),
    ("k_path_defer ordered, paired", dict(path=1, path_defer=1, path_order=2, path_order_pair=1)),
    ("k_path_spec", dict(path=1, path_defer=0, path_spec=1, path_order=0)),
    ("k_path_spec ordered, paired", dict(path=1, path_defer=0, path_spec=1, path_order=2, path_order_pair=1)),
    ("wavefront", dict(path=0, path_defer=2, path_order=2)),
]
DEFAULTS = dict(path=2, path_defer=2, path_spec=0, path_order=2, path_order_pair=2, path_order_min_spp=16,
                count_tests=0, pixel_probe=0)


def _render_forms(ctx, orc_rad, orc_w, orc_probe, tiles, spp, depth):
    """Render `tiles` in every form (persistent ones also counted), each bit-exact in radiance and
    weights, and in the per-pixel probe (final sampler state = every path length and RNG draw; ray
    counts = every bounce and NEE decision) against the oracle.  Returns the forms whose ray counts
    were compared."""
    counted = []
    try:
        ctx.set_option("pixel_probe", 1)
        ctx.set_option("path_order_min_spp", 0)
        for name, opts in FORMS:
            for count in ((0, 1) if opts["path"] == 1 else (0,)):
                for k, v in dict(dict(path_spec=0), **opts).items():
                    ctx.set_option(k, v)
                ctx.set_option("count_tests", count)
                what = f"{name}{' (counting build)' if count else ''}"
                rad, w = ctx.render(spp, depth, tiles, W, H)
                assert np.array_equal(w, orc_w), f"{what}: weights differ"
                diff = np.abs(rad - orc_rad).max()
                assert np.array_equal(rad, orc_rad), f"{what}: radiance differs (max abs diff {diff})"
                pr = ctx.pixel_probe(dist.n_pixels(tiles))
                if check_probe(pr, orc_probe, tiles, W, H, what):
                    counted.append(what)
    finally:
        for k, v in DEFAULTS.items():
            ctx.set_option(k, v)
        ctx.reset_stats()
    return counted


def test_c3_integrator_probe_bit_exact(c3):
    """Integrator parity on the headline scene that can fail on a shading bug: per pixel of the
    strided subset, the final LCG state (its draw count encodes every path length, BSDF-pdf
    rejection and light sample, sampler.h:54-67) and the closest-hit / shadow rays traced
    (pathtracer.h:69-91, 133-164) equal the oracle's, for k_path and k_path_defer with and without the
    cost-ordered fetch and for the wavefront."""
    ctx, cs, orc, _ = c3
    tiles = dist.tiles_for_rank(W, H, TILE, 0, 64)
    orad, ow, st, opr = orc.render(2, 5, tiles=tiles, n_threads=16, probe=True)
    ys, xs = np.nonzero(ow)
    # the paths really bounce and sample lights here: the fingerprint is not trivially equal
    assert opr["shadow_rays"][ys, xs].sum() > 0 and (opr["closest_rays"][ys, xs] > 2).mean() > 0.2
    counted = _render_forms(ctx, orad, ow, opr, tiles, 2, 5)
    assert len(counted) == 8, counted


LIT_CAMERA = dict(position=(0.0, 1.4, 1.6), rotation=(0.0, -40.0, 0.0), fov=70.0)


def test_c3_lit_view_render_bit_exact(c3):
    """A lit test-only view of the same 10M-triangle SBVH soup: the camera sits under the emitter
    (y = 1.5, facing down) looking down at the soup's top face, which the emitter lights, so NEE
    contributions, emission at depth 0 and multi-bounce radiance all reach the film.  Strided tile
    subset at 2 spp, every render form, bit-exact in radiance and in the per-pixel probe."""
    ctx, cs, orc, _ = c3
    cam = scene.PerspectiveCamera(resolution=(W, H), **LIT_CAMERA)
    lit = dataclasses.replace(cs, camera=cam)
    orc_lit = py_oracle.OracleScene(lit, orc.nodes, orc.tris, capi)
    tiles = dist.tiles_for_rank(W, H, TILE, 5, 64)
    ctx.set_camera(cam.position, cam.rotation, cam.fov, cam.resolution)
    try:
        orad, ow, st, opr = orc_lit.render(2, 5, tiles=tiles, n_threads=16, probe=True)
        sel = ow > 0
        L = orad.sum(-1)[sel] / 2
        assert L.mean() > 0.2 and (L > 0).mean() > 0.15, f"view not lit: mean {L.mean()}, lit {(L > 0).mean()}"
        counted = _render_forms(ctx, orad, ow, opr, tiles, 2, 5)
        assert len(counted) == 8, counted
    finally:
        c = cs.camera
        ctx.set_camera(c.position, c.rotation, c.fov, c.resolution)


def test_c3_8way_share_takes_k_path_spec(c3):
    """The form rule on the headline scene: an 8-way share of the 1080p frame (64x64
    tiles, as the bench) at 16 spp under the default options runs k_path_spec in cost order — about
    one pixel per resident lane, and the cost-ordering pilot's camera rays take long traversals — and
    equals the oracle bit for bit.  The Cornell box's share takes k_path (test_gpu_cornell1080)."""
    ctx, cs, orc, _ = c3
    share = dist.tiles_for_rank(W, H, 64, 0, 8)
    for k, v in dict(path=2, path_defer=2, path_spec=2, path_order=2, path_order_min_spp=16).items():
        ctx.set_option(k, v)
    try:
        rad, w = ctx.render(16, 5, share, W, H)
        form, inp = ctx.render_form(), ctx.render_form_inputs()
    finally:
        for k, v in DEFAULTS.items():
            ctx.set_option(k, v)
    assert form == {"form": "k_path_spec", "ordered": True}, (form, inp)
    assert 0.5 < inp["pixels_per_lane"] < 1.5 and inp["pilot_rays"] == dist.n_pixels(share), inp
    assert inp["pilot_mean_steps"] >= 12, inp
    orad, ow, _ = orc.render(16, 5, tiles=share, n_threads=16)
    assert np.array_equal(w, ow)
    assert np.array_equal(rad, orad), f"radiance differs (max abs diff {np.abs(rad - orad).max()})"
