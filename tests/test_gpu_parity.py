"""HIP path (libakr_hip.so through the C-ABI) against the CPU restatement, on device 0.

Bar: bit-exact.  The oracle traverses the same BVH arrays with the reference's own algorithm
(bvh-accelerator.h:488-547), so hit ids, t and barycentrics must match exactly; renders must
match exactly because every f32 operation is kept in the reference's order on both sides
(DESIGN.md §4).  Tolerances appear only where the reference itself is builder-dependent.
"""
import numpy as np
import pytest

import py_oracle
from akari_amd import capi, scene
from helpers import check_bvh, cornell, edge_rays, hits_to_gid, mixed_scene, random_rays, small_soup, textured_scene

pytestmark = pytest.mark.gpu


def _setup(ctx, sc, **kw):
    cs = scene.compile_scene(sc)
    scene.upload_scene(ctx, cs, **kw)
    nodes, tris = ctx.accel_export()
    return cs, py_oracle.OracleScene(cs, nodes, tris, capi)


def _check_trace(ctx, orc, cs, rays, any_hit, exact=False):
    ctx.set_option("exact_cull", int(exact))
    gh = ctx.trace(rays, any_hit=any_hit)
    oh, _, _ = orc.trace(rays, any_hit=any_hit, exact_cull=exact)
    ggid = hits_to_gid(gh, cs.mesh_base)
    assert np.array_equal(ggid, oh["gid"]), f"{np.count_nonzero(ggid != oh['gid'])} hit ids differ"
    hit = oh["gid"] != 0xFFFFFFFF
    assert np.array_equal(gh["t"][hit], oh["t"][hit])
    assert np.all(np.isinf(gh["t"][~hit]))
    if not any_hit:
        assert np.array_equal(gh["u"][hit], oh["u"][hit]) and np.array_equal(gh["v"][hit], oh["v"][hit])
    assert np.all(gh["geom_id"][~hit] == -1) and np.all(gh["prim_id"][~hit] == -1)
    return gh, oh


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("any_hit", [False, True])
def test_trace_cornell(hip_ctx_factory, any_hit, exact):
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell())
        rays = random_rays(1 << 16, 1, -0.9, 0.9)
        rays["o"][:, 1] += 1.0          # the box spans y in [0, 2]
        _check_trace(ctx, orc, cs, rays, any_hit, exact)
        _check_trace(ctx, orc, cs, edge_rays((0.0, 1.0, 0.0)), any_hit, exact)


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("any_hit", [False, True])
def test_trace_soup(hip_ctx_factory, any_hit, exact):
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, small_soup(100_000))
        rays = random_rays(1 << 17, 2, -1.2, 1.2)
        _check_trace(ctx, orc, cs, rays, any_hit, exact)
        _check_trace(ctx, orc, cs, edge_rays(), any_hit, exact)


def test_tight_cull_same_hits_as_reference_cull(hip_ctx_factory):
    """The default slab test (behind-origin boxes culled) returns the reference cull's hits."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, small_soup(100_000))
        rays = random_rays(1 << 17, 6, -1.2, 1.2)
        ctx.set_option("exact_cull", 0)
        a = ctx.trace(rays)
        ctx.set_option("exact_cull", 1)
        b = ctx.trace(rays)
        assert (hits_to_gid(a, cs.mesh_base) == hits_to_gid(b, cs.mesh_base)).mean() >= 0.9999
        assert np.array_equal(a["t"], b["t"])


def test_trace_builder_independent(hip_ctx_factory):
    """Closest hits agree with a BVH-free brute force (builder independence, >= 99.99 %)."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, small_soup(20_000))
        rays = random_rays(1 << 13, 3, -1.1, 1.1)
        gh = ctx.trace(rays)
        bh = orc.trace_brute(rays)
        same = hits_to_gid(gh, cs.mesh_base) == bh["gid"]
        assert same.mean() >= 0.9999
        both = same & (bh["gid"] != 0xFFFFFFFF)
        assert np.array_equal(gh["t"][both], bh["t"][both])


@pytest.mark.parametrize("leaf,align", [(1, 1), (2, 1), (8, 1), (1, 8), (4, 4), (8, 8)])
def test_trace_leaf_sizes(hip_ctx_factory, leaf, align):
    """Leaves of 1, 2 and up to 8 triangles: the leaf phases fetch the second triangle record with the
    header whatever the count (a one-triangle leaf reads into the next leaf, the alignment gap or the
    blob's padding), and read the third and later ones in the loop; leaf records packed or aligned to
    64 / 128 B (option leaf_align); closest-hit and any-hit traces, and renders through the three
    persistent kernels (final sampler states too)."""
    with hip_ctx_factory(0) as ctx:
        ctx.set_option("leaf_align", align)
        cs, orc = _setup(ctx, small_soup(30_000), max_leaf_size=leaf)
        assert ctx.accel_info().max_leaf <= leaf
        _check_trace(ctx, orc, cs, random_rays(1 << 14, 4, -1.1, 1.1), False)
        _check_trace(ctx, orc, cs, random_rays(1 << 14, 5, -1.1, 1.1), True)
        ctx.set_option("path", 1)
        for defer in (0, 1, 2):   # k_path, k_path_defer, k_path_spec
            ctx.set_option("path_defer", 1 if defer == 1 else 0)
            ctx.set_option("path_spec", 1 if defer == 2 else 0)
            _check_render(ctx, orc, 2, 5, [(0, 0, 96, 54), (40, 20, 75, 50)], 96, 54, probe=True)


@pytest.mark.parametrize("n_tris", [1, 2, 37, 100_000])
def test_gpu_lbvh_builder(hip_ctx_factory, n_tris):
    """The GPU LBVH builder (lbvh.hip): a valid BVH2 in the same format, and
    hits / renders bit-exact against the oracle walking that BVH with the reference algorithm."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, small_soup(n_tris), builder=capi.BUILDER_LBVH)
        nodes, tris = ctx.accel_export()
        check_bvh(cs, nodes, tris, 1)
        assert ctx.accel_info().max_leaf == 1
        _check_trace(ctx, orc, cs, random_rays(1 << 14, 8, -1.2, 1.2), False)
        _check_trace(ctx, orc, cs, random_rays(1 << 14, 9, -1.2, 1.2), True)
        _check_trace(ctx, orc, cs, edge_rays(), False)
        if n_tris >= 37:
            _check_render(ctx, orc, 2, 5, [(0, 0, 96, 54)], 96, 54)


def test_gpu_lbvh_duplicates_and_cornell(hip_ctx_factory):
    """Identical triangles (equal Morton codes, split by index) and the Cornell box."""
    with hip_ctx_factory(0) as ctx:
        sc = small_soup(500)
        m = sc.shapes[0]
        m.vertices[3 * 100:3 * 200] = np.tile(m.vertices[0:3], (100, 1))  # triangles 100..199 = triangle 0
        cs, orc = _setup(ctx, sc, builder=capi.BUILDER_LBVH)
        nodes, tris = ctx.accel_export()
        check_bvh(cs, nodes, tris, 1)
        _check_trace(ctx, orc, cs, random_rays(1 << 12, 10, -1.2, 1.2), False)
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell((32, 32)), builder=capi.BUILDER_LBVH)
        _check_render(ctx, orc, 4, 5, [(0, 0, 32, 32)], 32, 32)


def test_trace_empty_and_device_batch(hip_ctx_factory):
    torch = pytest.importorskip("torch")
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell())
        assert ctx.trace(np.zeros(0, capi.RAY_DTYPE)).shape == (0,)
        rays = random_rays(4096, 5, -0.9, 0.9)
        rays["o"][:, 1] += 1.0
        d_r = torch.from_numpy(rays.view(np.uint8).copy()).to("cuda:0")
        d_h = torch.zeros(4096 * 32, dtype=torch.uint8, device="cuda:0")
        ctx.trace_device(d_r.data_ptr(), 4096, d_h.data_ptr(), any_hit=False)
        ctx.synchronize()
        gh = d_h.cpu().numpy().view(capi.HIT_DTYPE)
        oh, _, _ = orc.trace(rays)
        assert np.array_equal(hits_to_gid(gh, cs.mesh_base), oh["gid"])


@pytest.mark.parametrize("n", [1, 63, 65, 1000, 100_003])
def test_trace_each_ray_once(hip_ctx_factory, n):
    """The persistent kernels' dynamic fetch hands every queued ray to exactly one lane."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, small_soup(20_000))
        rays = random_rays(n, 7, -1.1, 1.1)
        ctx.set_option("count_tests", 1)
        ctx.set_option("path_spec", 0)   # (k_path_spec's dropped samples trace rays too; its
        for any_hit in (False, True):    # committed rays are checked per pixel by the probe tests)
            ctx.reset_stats()
            ctx.trace(rays, any_hit=any_hit)
            assert ctx.trace_counts()["per_mode"]["any" if any_hit else "closest"]["rays"] == n
        # a one-bounce render traces exactly one camera ray per pixel sample
        ctx.reset_stats()
        ctx.render(3, 1, [(0, 0, 96, 54)], 96, 54)
        c = ctx.trace_counts()["per_mode"]
        assert c["closest"]["rays"] == 3 * 96 * 54
        assert 0 < c["shadow"]["rays"] <= 3 * 96 * 54


def _check_render(ctx, orc, spp, depth, tiles, W, H, clamp=0.0, exact=False, probe=False):
    """Render through the C-ABI and compare with the oracle bit for bit; with `probe`, also the
    per-pixel fingerprint (final sampler state; ray counts where the form records them).  Returns
    (radiance, weight), plus whether ray counts were compared when `probe`."""
    if probe:
        ctx.set_option("pixel_probe", 1)
    rad, w = ctx.render(spp, depth, tiles, W, H, ray_clamp=clamp, exact_cull=exact)
    out = orc.render(spp, depth, tiles=tiles, ray_clamp=clamp, exact_cull=exact, probe=probe)
    orad, ow = out[0], out[1]
    assert np.array_equal(w, ow)
    bad = rad != orad
    assert not bad.any(), f"{bad.sum()} radiance values differ, max {np.abs(rad - orad).max()}"
    if probe:
        from helpers import slot_pixels, check_probe
        ctx.set_option("pixel_probe", 0)
        n = len(slot_pixels(tiles, W, H)[0])
        return rad, w, check_probe(ctx.pixel_probe(n), out[3], tiles, W, H)
    return rad, w


@pytest.mark.parametrize("path", [0, 2])
@pytest.mark.parametrize("exact", [False, True])
def test_render_cornell_bit_exact(hip_ctx_factory, exact, path):
    """The Cornell box in the wavefront form (path 0) and the library's choice (path 2)."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell((64, 64)))
        ctx.set_option("path", path)
        rad, w = _check_render(ctx, orc, 16, 5, [(0, 0, 64, 64)], 64, 64, exact=exact)
        assert np.all(w == 16) and rad.mean() > 0
        info = ctx.render_info()
        assert info["lanes"] == 1 and info["passes"] == (16 if path == 0 or exact else 1)


def test_render_soup_and_node_mixed_forms(hip_ctx_factory):
    """A soup in both forms, and render_node over two contexts that run different forms: the same image."""
    with hip_ctx_factory(0) as ctx, hip_ctx_factory(0) as other:
        cs, orc = _setup(ctx, small_soup(50_000, (64, 36)))
        for path in (0, 2):
            ctx.set_option("path", path)
            _check_render(ctx, orc, 12, 5, [(0, 0, 64, 36)], 64, 36)
        scene.upload_scene(other, cs)
        other.set_option("path", 0)
        tiles = [(x, y, x + 16, y + 12) for y in range(0, 36, 12) for x in range(0, 64, 16)]
        ref, wref = ctx.render(7, 5, tiles, 64, 36)
        rad, w = capi.render_node([ctx, other], 7, 5, tiles, 64, 36)
        assert np.array_equal(w, wref) and np.array_equal(rad, ref)


def test_render_tiles_depths_clamp(hip_ctx_factory):
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell((40, 24)))
        tiles = [(0, 0, 16, 16), (24, 8, 40, 24), (30, 0, 64, 64), (5, 5, 5, 9)]   # ragged, clipped, empty
        for depth in (0, 1, 2, 5):
            _check_render(ctx, orc, 3, depth, tiles, 40, 24)
        _check_render(ctx, orc, 4, 5, tiles, 40, 24, clamp=10.0)
        rad, w = ctx.render(0, 5, tiles, 40, 24)
        assert not w.any() and not rad.any()
        rad, w = ctx.render(2, 5, [], 40, 24)
        assert not w.any()


@pytest.mark.parametrize("exact", [False, True])
def test_render_soup_bit_exact(hip_ctx_factory, exact):
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, small_soup(50_000, (64, 36)))
        _check_render(ctx, orc, 4, 5, [(0, 0, 64, 36)], 64, 36, exact=exact)


@pytest.mark.parametrize("mk", ["cornell", "big_soup"])
def test_sbvh_trace_and_render_bit_exact(hip_ctx_factory, mk):
    """The SBVH builder's clipped, duplicated references through the wide traversal: traces and
    renders bit-exact against the oracle walking the same BVH (and hits equal to the binned-SAH
    BVH's up to ties)."""
    sc = cornell((48, 48)) if mk == "cornell" else small_soup(30_000, (64, 36), r=0.2)
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, sc, builder=capi.BUILDER_SBVH)
        if mk == "big_soup":
            assert ctx.accel_info().n_tris > cs.n_tris   # spatial splits happened
        lo, hi = (-0.9, 0.9) if mk == "cornell" else (-1.1, 1.1)
        rays = random_rays(20_000, 5, lo, hi)
        for any_hit in (False, True):
            _check_trace(ctx, orc, cs, rays, any_hit)
        W, H = cs.camera.resolution
        _check_render(ctx, orc, 4, 5, [(0, 0, W, H)], W, H)


def test_render_glossy_mix_bit_exact(hip_ctx_factory):
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, mixed_scene((48, 48)))
        _check_render(ctx, orc, 8, 5, [(0, 0, 48, 48)], 48, 48)


def test_render_hall_bit_exact(hip_ctx_factory):
    """The C4 stand-in (scene.hall_scene: tessellated, image-textured Diffuse / Glossy / Mix, six
    one-sided ceiling lights), coarse tessellation, against the oracle."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, scene.hall_scene((64, 36), detail=0.1), builder=capi.BUILDER_SBVH)
        rad, w = _check_render(ctx, orc, 4, 5, [(0, 0, 64, 36)], 64, 36)
        assert rad.mean() > 0


def test_render_image_textures_bit_exact(hip_ctx_factory):
    """ImageTexture (texture.h:39-57, View lookup image.hpp:83-99) on diffuse colour, glossy
    roughness, mix fraction and emission, with texcoords outside [0, 1]."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, textured_scene((40, 40)))
        assert len(cs.images) == 6
        rad, w = _check_render(ctx, orc, 6, 5, [(0, 0, 40, 40)], 40, 40)
        assert rad.mean() > 0


def test_render_node_matches_single_context(hip_ctx_factory):
    """akr_hip_render_node (two contexts on device 0 here; one per GPU in production) splits the
    tiles between contexts and gives the single-context image bit for bit."""
    with hip_ctx_factory(0) as a, hip_ctx_factory(0) as b:
        sc = cornell((48, 32))
        cs, orc = _setup(a, sc)
        scene.upload_scene(b, cs)
        tiles = [(x, y, x + 16, y + 16) for y in range(0, 32, 16) for x in range(0, 48, 16)]
        ref, wref = a.render(4, 5, tiles, 48, 32)
        rad, w = capi.render_node([a, b], 4, 5, tiles, 48, 32)
        assert np.array_equal(w, wref) and np.array_equal(rad, ref)
        orad, ow, _ = orc.render(4, 5, tiles=tiles)
        assert np.array_equal(rad, orad)


def test_render_node_overlapping_tiles_prefilled(hip_ctx_factory):
    """render_node with three contexts, overlapping and repeated tiles (a pixel listed up to 8 times,
    several times by one context: the gather's per-rank merge launches) into pre-filled host
    buffers: the single-context result bit for bit, and the oracle's."""
    with hip_ctx_factory(0) as a, hip_ctx_factory(0) as b, hip_ctx_factory(0) as c:
        sc = cornell((40, 24))
        cs, orc = _setup(a, sc)
        scene.upload_scene(b, cs)
        scene.upload_scene(c, cs)
        t = (4, 2, 20, 14)
        tiles = [t, (0, 0, 40, 24), t, (10, 5, 30, 20), t, t, (16, 0, 32, 8), t, (-5, -5, 3, 3)]
        rng = np.random.default_rng(7)
        pre_r = rng.uniform(0, 3, (24, 40, 3)).astype(np.float32)
        pre_w = rng.integers(0, 5, (24, 40)).astype(np.float32)
        ref, wref = a.render(3, 5, tiles, 40, 24, radiance=pre_r.copy(), weight=pre_w.copy())
        rad, w = capi.render_node([a, b, c], 3, 5, tiles, 40, 24, radiance=pre_r.copy(), weight=pre_w.copy())
        assert np.array_equal(w, wref) and np.array_equal(rad, ref)
        orad, ow, _ = orc.render(3, 5, tiles=tiles, radiance=pre_r.copy(), weight=pre_w.copy())
        assert np.array_equal(w, ow) and np.array_equal(rad, orad)
        assert (w - pre_w)[5, 16] == 8 * 3   # listed 8 times: t x 5, the frame, two more tiles
        with pytest.raises(capi.AkrError):   # one context listed twice would race with itself
            capi.render_node([a, b, a], 3, 5, tiles, 40, 24)


def test_import_accel_bit_exact(hip_ctx_factory):
    """akr_hip_import_accel: a context that adopts another context's exported BVH2 (the ranks of a
    node build once, bench.py) traces and renders bit for bit like the context that built it, and a
    malformed tree is refused with a status, not adopted."""
    sc = small_soup(100_000, (64, 36))
    with hip_ctx_factory(0) as a, hip_ctx_factory(0) as b:
        cs, orc = _setup(a, sc, builder=capi.BUILDER_SBVH, n_threads=8)
        nodes, tris = a.accel_export()
        info = scene.upload_scene(b, cs, bvh=(nodes, tris), n_threads=8)
        ia = a.accel_info()
        assert (info.n_nodes, info.n_tris, info.max_depth, info.max_leaf) == (ia.n_nodes, ia.n_tris, ia.max_depth,
                                                                              ia.max_leaf)
        rays = random_rays(1 << 14, 77, -1.0, 1.0)
        for any_hit in (False, True):
            ha, hb = a.trace(rays, any_hit), b.trace(rays, any_hit)
            assert ha.tobytes() == hb.tobytes()
        _check_render(b, orc, 3, 5, [(0, 0, 64, 36)], 64, 36)
        bad = nodes.copy()
        bad[3]["child"][0] = len(nodes) + 10
        with pytest.raises(capi.AkrError, match="BVH"):
            b.import_accel(bad, tris)
        # records that are not this scene's triangles, or a scene triangle in no leaf
        moved = tris.copy()
        moved[5]["v0"][1] += 1e-3
        with pytest.raises(capi.AkrError, match="does not match"):
            b.import_accel(nodes, moved)
        relabelled = tris.copy()
        g = relabelled["gid"]
        relabelled["gid"] = np.where(g == g[0], g[1], g)   # triangle g[0] vanishes from every leaf
        with pytest.raises(capi.AkrError, match="does not match|in no leaf"):
            b.import_accel(nodes, relabelled)
        # a refused import leaves the previous tree in place, consistent with the device
        _check_render(b, orc, 1, 5, [(0, 0, 64, 36)], 64, 36)


def test_hang_guard_fault_is_reported(hip_ctx_factory):
    """The persistent kernel's hang guard raises a fault word in mapped host memory that the host
    checks after every render whatever "verify" says: with the test option that raises
    it, a synchronous render fails, a render_device with verify on fails, and one with verify off
    returns and reports it at akr_hip_synchronize.  Renders after that succeed again."""
    torch = pytest.importorskip("torch")
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell((32, 32)))
        ctx.set_option("path", 1)
        ctx.set_option("path_defer", 1)
        tiles = [(0, 0, 32, 32)]
        ctx.set_option("fault_test", 1)
        with pytest.raises(capi.AkrError, match="hang guard"):
            ctx.render(2, 5, tiles, 32, 32)
        rad = torch.zeros(1024 * 3, device="cuda:0")
        wt = torch.zeros(1024, device="cuda:0")
        with pytest.raises(capi.AkrError, match="hang guard"):
            ctx.render_device(2, 5, tiles, rad.data_ptr(), wt.data_ptr())
        ctx.set_option("verify", 0)
        ctx.render_device(2, 5, tiles, rad.data_ptr(), wt.data_ptr())
        with pytest.raises(capi.AkrError, match="hang guard"):
            ctx.synchronize()
        # an unverified render's fault found by the next render names the earlier call
        ctx.render_device(2, 5, tiles, rad.data_ptr(), wt.data_ptr())
        ctx.set_option("fault_test", 0)
        with pytest.raises(capi.AkrError, match="previous render_device"):
            ctx.render_device(2, 5, tiles, rad.data_ptr(), wt.data_ptr())
        ctx.set_option("fault_test", 1)
        ctx.set_option("verify", 1)
        ctx.set_option("fault_test", 0)
        _check_render(ctx, orc, 2, 5, tiles, 32, 32)


def test_render_device_packed(hip_ctx_factory):
    torch = pytest.importorskip("torch")
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell((32, 32)))
        tiles = [(16, 0, 32, 16), (0, 16, 16, 32)]
        rad = torch.zeros(512 * 3, device="cuda:0")
        wt = torch.zeros(512, device="cuda:0")
        n = ctx.render_device(4, 5, tiles, rad.data_ptr(), wt.data_ptr())
        ctx.synchronize()
        assert n == 512
        orad, ow, _ = orc.render(4, 5, tiles=tiles)
        k = 0
        r = rad.cpu().numpy().reshape(-1, 3)
        for (x0, y0, x1, y1) in tiles:
            blk = orad[y0:y1, x0:x1].reshape(-1, 3)
            assert np.array_equal(r[k:k + blk.shape[0]], blk)
            k += blk.shape[0]


def _check_ao(ctx, orc, spp, tiles, W, H, occlude=float("inf"), exact=False):
    rad, w = ctx.render_ao(spp, tiles, W, H, occlude=occlude, exact_cull=exact)
    orad, ow, _ = orc.render_ao(spp, tiles=tiles, occlude=occlude, exact_cull=exact)
    assert np.array_equal(w, ow)
    bad = rad != orad
    assert not bad.any(), f"{bad.sum()} AO values differ (occlude={occlude})"
    return rad, w


@pytest.mark.parametrize("occlude", [float("inf"), 0.5])
def test_render_ao_cornell_bit_exact(hip_ctx_factory, occlude):
    """cpu::AmbientOcclusion (integrator.cpp:40-87): +inf runs the AO rays as a shadow-mode
    occlusion trace, a finite distance as a closest-hit trace compared against occlude."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell((48, 40)))
        rad, w = _check_ao(ctx, orc, 16, [(0, 0, 48, 40)], 48, 40, occlude=occlude)
        assert np.all(w == 16) and 0 < rad.mean() < 16


@pytest.mark.parametrize("exact", [False, True])
def test_render_ao_soup_bit_exact(hip_ctx_factory, exact):
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, small_soup(50_000, (64, 36)))
        for occlude in (float("inf"), 0.05):
            _check_ao(ctx, orc, 4, [(0, 0, 64, 36)], 64, 36, occlude=occlude, exact=exact)


def test_render_ao_edges(hip_ctx_factory):
    """Ragged / clipped / empty tiles, spp 0, an empty tile list, and the degenerate occlude
    values (0, negative, NaN: t < occlude never holds, every camera hit scores 1)."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell((40, 24)))
        tiles = [(0, 0, 16, 16), (24, 8, 40, 24), (30, 0, 64, 64), (5, 5, 5, 9)]
        for occlude in (float("inf"), 1e30, 1.0, 0.0, -1.0, float("nan")):
            _check_ao(ctx, orc, 3, tiles, 40, 24, occlude=occlude)
        a, _ = ctx.render_ao(3, tiles, 40, 24)
        b, _ = ctx.render_ao(3, tiles, 40, 24, occlude=1e30)   # closest-hit path, same answer
        assert np.array_equal(a, b)
        rad, w = ctx.render_ao(0, tiles, 40, 24)
        assert not w.any() and not rad.any()
        rad, w = ctx.render_ao(2, [], 40, 24)
        assert not w.any()
        # the path tracer after AO on the same context still matches its oracle
        _check_render(ctx, orc, 2, 5, tiles, 40, 24)


def test_scene_file_render_ao_and_path(tmp_path):
    """SceneNode::render on the HIP path (akari_amd.render): a .akari scene with an AO node, then
    a Path node, each through its C-ABI integrator, the AO image bit-exact against the oracle."""
    from akari_amd import film, render
    from conftest import CORNELL_MESH
    sdl = f"""
let grey = DiffuseMaterial {{ color: [0.725, 0.71, 0.68] }}
export scene = Scene {{
    camera: PerspectiveCamera {{ fov: 15, position: [0, 1, 9], resolution: [40, 24] }},
    integrator: AO {{ spp: 5, occlude: 0.75 }},
    output: "{tmp_path / 'ao.pfm'}",
    shapes: [ AkariMesh {{ path: "{CORNELL_MESH}", materials: [$grey, $grey, $grey, $grey, $grey, $grey, $grey,
                                                                 EmissiveMaterial {{ color: [17, 12, 4] }}] }} ]
}}
"""
    path = tmp_path / "ao.akari"
    path.write_text(sdl)
    assert render.main([str(path)]) == 0
    raw = (tmp_path / "ao.pfm").read_bytes()
    img = np.frombuffer(raw[raw.index(b"-1.0\n") + 5:], np.float32).reshape(24, 40, 3)[::-1]
    sc = scene.load_scene_file(path)
    cs = scene.compile_scene(sc)
    with capi.HipContext(0) as ctx:
        scene.upload_scene(ctx, cs)
        nodes, tris = ctx.accel_export()
    orc = py_oracle.OracleScene(cs, nodes, tris, capi)
    orad, ow, _ = orc.render_ao(5, occlude=np.float32(0.75))
    assert np.array_equal(img, film.resolve(orad, ow))
    path.write_text(sdl.replace("AO { spp: 5, occlude: 0.75 }", "Path { spp: 3, max_depth: 4, tile_size: 16 }"))
    rad, w = render.render_scene(scene.load_scene_file(path))
    orad, ow, _ = orc.render(3, 4, tiles=render._tiles(sc, 16), ray_clamp=10.0)
    assert np.array_equal(rad, orad) and np.array_equal(w, ow)


def test_trace_small_batches_and_grazing(hip_ctx_factory):
    """Launches far smaller than the persistent grid (one ray, one wave, ragged) and grazing rays
    aimed along the faces of the 100K-triangle soup, on the wide lean traversal."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, small_soup(100_000))
        for n, seed in ((1, 31), (64, 32), (777, 33), (1 << 16, 34)):
            _check_trace(ctx, orc, cs, random_rays(n, seed, -1.3, 1.3), False)
        rays = random_rays(4096, 35, -1.05, 1.05)
        rays["o"][:, 2] = -3.0
        d = rays["d"]
        d[:, 2] = np.abs(d[:, 2]) + 0.2
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rays["d"] = d.astype(np.float32)
        _check_trace(ctx, orc, cs, rays, False)
        _check_trace(ctx, orc, cs, rays, True)


def test_kernel_stats_modes(hip_ctx_factory):
    """"stats" 1 times every kernel, 2 only the dominant one (bench.py's timed region at a split):
    trace_closest in the wavefront form, the one persistent launch in the path-kernel form; the
    image does not depend on either."""
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, cornell((32, 32)))
        ref, _ = ctx.render(3, 5, [(0, 0, 32, 32)], 32, 32)
        cases = ((0, 1, {"raygen", "trace_closest", "shade", "trace_shadow", "splat"}, "trace_closest", 15),
                 (0, 2, {"trace_closest"}, "trace_closest", 15), (1, 1, {"path"}, "path", 1), (1, 2, {"path"}, "path", 1))
        for path, mode, expect, key, launches in cases:
            ctx.set_option("path", path)
            ctx.reset_stats()
            ctx.set_option("stats", mode)
            rad, _ = ctx.render(3, 5, [(0, 0, 32, 32)], 32, 32)
            assert np.array_equal(rad, ref)
            ks = ctx.kernel_stats()
            assert set(ks) == expect and ks[key]["launches"] == launches
        # shadow traces serialised on the main stream (the bench's isolated timing): same image
        ctx.set_option("path", 0)
        ctx.set_option("serial_shadow", 1)
        rad, _ = ctx.render(3, 5, [(0, 0, 32, 32)], 32, 32)
        assert np.array_equal(rad, ref)
        ctx.set_option("serial_shadow", 0)
        # auto (the default): the path kernel up to path_auto_pixels pixels, the wavefront above
        ctx.set_option("path", 2)
        ctx.set_option("stats", 2)
        for limit, key in ((1 << 20, "path"), (1000, "trace_closest")):
            ctx.set_option("path_auto_pixels", limit)
            ctx.reset_stats()
            rad, _ = ctx.render(3, 5, [(0, 0, 32, 32)], 32, 32)
            assert np.array_equal(rad, ref) and set(ctx.kernel_stats()) == {key}
        ctx.set_option("stats", 0)


@pytest.mark.parametrize("defer", [0, 1, 2])
def test_path_pilot_order_bit_exact(hip_ctx_factory, defer):
    """The path pilot (option path_order_pilot_spp): slots ranked by the rays of
    their first samples in a counting k_path render, which must leave nothing behind: the ordered
    render of every persistent form equals the oracle bit for bit, film, weights, sampler states and
    (counting build) ray counts per pixel."""
    with hip_ctx_factory(0) as ctx:
        ctx.set_option("path", 1)
        ctx.set_option("path_defer", 1 if defer == 1 else 0)
        ctx.set_option("path_spec", 1 if defer == 2 else 0)
        ctx.set_option("path_order", 2)
        ctx.set_option("path_order_min_spp", 0)
        ctx.set_option("path_order_share_min_spp", 0)
        ctx.set_option("path_order_pilot_spp", 2)
        cs, orc = _setup(ctx, small_soup(20_000, (48, 27)))
        for spp, depth in ((1, 5), (6, 5), (3, 2)):
            _check_render(ctx, orc, spp, depth, [(0, 0, 48, 27), (5, 3, 19, 11)], 48, 27, probe=True)
            assert ctx.render_form()["ordered"]
        try:
            ctx.set_option("count_tests", 1)
            *_, rays = _check_render(ctx, orc, 4, 5, [(0, 0, 48, 27)], 48, 27, probe=True)
            assert rays
        finally:
            ctx.set_option("count_tests", 0)


def test_count_lines_bitmap(hip_ctx_factory):
    """Option count_lines (bench.py roofline.lines_per_pass): k_path's counting build
    marks the 128-B lines it reads.  The render stays bit-exact; every region has lines marked; a 64-B
    node lies in one line, so the node lines are at most the node visits; every hit reads one 80-B
    shading record (at most two lines); a render of a sub-tile marks no more lines than the whole frame."""
    with hip_ctx_factory(0) as ctx:
        for k, v in (("path", 1), ("path_defer", 0), ("path_spec", 0), ("path_order", 0)):
            ctx.set_option(k, v)
        cs, orc = _setup(ctx, small_soup(20_000, (48, 27)))
        got = []
        try:
            ctx.set_option("count_tests", 1)
            ctx.set_option("count_lines", 1)
            for tiles in ([(0, 0, 48, 27)], [(5, 3, 13, 9)]):
                ctx.reset_stats()
                _check_render(ctx, orc, 1, 5, tiles, 48, 27)
                got.append((ctx.path_profile(), ctx.trace_counts()["per_mode"]))
        finally:
            ctx.set_option("count_lines", 0)
            ctx.set_option("count_tests", 0)
        (full, fc), (sub, _) = got
        for k in ("lines_nodes", "lines_leaves", "lines_shading"):
            assert 0 < sub[k] <= full[k], (k, sub[k], full[k])
        assert full["lines_nodes"] <= fc["closest"]["visits"] + fc["shadow"]["visits"]
        assert full["lines_shading"] <= 2 * fc["closest"]["rays"]
        assert full["lines_shading"] * 128 <= cs.n_tris * 80 + 256


def test_spec_and_order_options_are_validated(hip_ctx_factory):
    """The speculative form's and the cost order's options reject values outside their ranges
    (akr_hip_set_option returns an error and leaves the option as it was), and accept their ends."""
    with hip_ctx_factory(0) as ctx:
        for key, good, bad in (("path_spec_depth", (1, 3), (0, 4)), ("path_spec_fetch", (-1, 3), (-2, 5)),
                               ("path_order_pilot_spp", (0, 64), (-1, 65)), ("path_spec_fetch_pixels", (0, 1 << 40), (-1,)),
                               ("path_tail_ppl10", (0, 1 << 40), (-1,)), ("path_tail_steps", (0, 4096), (-1, 4097)), ("path_cache_mb", (0, 1 << 20), (-1,)),
                               ("leaf_align", (1, 8), (0, 3, 16)),
                               ("wave_order", (0, 1), ())):
            for v in good:
                ctx.set_option(key, v)
            for v in bad:
                with pytest.raises(capi.AkrError, match=key):
                    ctx.set_option(key, v)
        with pytest.raises(capi.AkrError):
            ctx.set_option("no_such_option", 1)


def test_auto_form_by_shading(hip_ctx_factory):
    """Auto dispatch: constant Diffuse / Emissive scenes render with the persistent
    kernel, scenes with Glossy / Mix materials or image textures with the wavefront (whose shade
    kernel measured faster there), unless path_auto_complex asks for the persistent kernel; every
    form gives the oracle's image."""
    for sc, simple in ((cornell((32, 32)), True), (mixed_scene((32, 32)), False), (textured_scene((32, 32)), False)):
        with hip_ctx_factory(0) as ctx:
            cs, orc = _setup(ctx, sc)
            ctx.set_option("stats", 2)
            for complex_ok in (0, 1):
                ctx.set_option("path_auto_complex", complex_ok)
                ctx.reset_stats()
                _check_render(ctx, orc, 3, 5, [(0, 0, 32, 32)], 32, 32)
                want = "path" if (simple or complex_ok) else "trace_closest"
                assert set(ctx.kernel_stats()) == {want}, (sc, complex_ok, ctx.kernel_stats())
                # 3 spp: no pilot, so the constant-shading scene takes k_path
                assert ctx.render_form()["form"] == ("k_path" if (simple or complex_ok) else "wavefront")
    # the persistent form by the pilot rule: for a scene whose camera rays take long
    # traversals (the cost-ordering pilot's mean steps), k_path_defer when the BVH is cache-resident,
    # else k_path_spec (k_path_defer with path_spec 0) for a render of few pixels per resident lane;
    # k_path otherwise, and without a pilot
    with hip_ctx_factory(0) as ctx:
        cs, orc = _setup(ctx, small_soup(20_000, (48, 27)))
        tiles = [(0, 0, 48, 27)]
        _check_render(ctx, orc, 3, 5, tiles, 48, 27)     # below the order's 16-spp floor: no pilot
        assert ctx.render_form() == {"form": "k_path", "ordered": False}
        assert ctx.render_form_inputs()["pilot_rays"] == -1
        ctx.set_option("path_tail_steps", 1)   # a bar every camera ray of the soup clears
        _check_render(ctx, orc, 16, 5, tiles, 48, 27)
        inp = ctx.render_form_inputs()
        assert inp["pilot_rays"] == 48 * 27 and inp["pilot_mean_steps"] >= 1, inp
        assert 0 < inp["pixels_per_lane"] < 0.01
        assert ctx.render_form() == {"form": "k_path_defer", "ordered": True}   # a 20K soup's BVH: cache-resident
        ctx.set_option("path_cache_mb", 0)     # as if it were not
        _check_render(ctx, orc, 16, 5, tiles, 48, 27)
        assert ctx.render_form() == {"form": "k_path_spec", "ordered": True}
        ctx.set_option("path_spec", 0)    # the rule's tail form is then the deferred one
        _check_render(ctx, orc, 16, 5, tiles, 48, 27)
        assert ctx.render_form() == {"form": "k_path_defer", "ordered": True}
        ctx.set_option("path_spec", 2)
        ctx.set_option("path_tail_steps", 4096)   # camera rays too short: k_path
        _check_render(ctx, orc, 16, 5, tiles, 48, 27)
        assert ctx.render_form() == {"form": "k_path", "ordered": True}
        ctx.set_option("path_tail_steps", 1)
        ctx.set_option("path_tail_ppl10", 0)        # too many pixels per lane: k_path, the pilot not read
        _check_render(ctx, orc, 16, 5, tiles, 48, 27)
        assert ctx.render_form() == {"form": "k_path", "ordered": True}
        assert ctx.render_form_inputs()["pilot_rays"] == -1
        ctx.set_option("path_tail_ppl10", 60)
        ctx.set_option("path_spec_pixels", 1000)    # the explicit size override (1296 pixels > 1000)
        _check_render(ctx, orc, 16, 5, tiles, 48, 27)
        assert ctx.render_form()["form"] == "k_path"
        ctx.set_option("path_spec_pixels", 0)
        ctx.set_option("path_defer_min_tris", 10 ** 9)
        _check_render(ctx, orc, 16, 5, tiles, 48, 27)
        assert ctx.render_form()["form"] == "k_path"
        ctx.set_option("path_defer_min_tris", 0)
        # a render of at most path_order_share_pixels pixels takes the order from path_order_share_min_spp
        # (16) samples even when the general floor is higher; without the order, no tail form
        ctx.set_option("path_order_min_spp", 64)
        _check_render(ctx, orc, 16, 5, tiles, 48, 27)
        assert ctx.render_form() == {"form": "k_path_spec", "ordered": True}
        ctx.set_option("path_order_share_pixels", 1000)
        _check_render(ctx, orc, 16, 5, tiles, 48, 27)
        assert ctx.render_form() == {"form": "k_path", "ordered": False}
        # forced forms ignore the rule
        ctx.set_option("path_spec", 1)
        _check_render(ctx, orc, 3, 5, tiles, 48, 27)
        assert ctx.render_form() == {"form": "k_path_spec", "ordered": False}
        ctx.set_option("path_spec", 2)
        ctx.set_option("path_defer", 1)
        _check_render(ctx, orc, 3, 5, tiles, 48, 27)
        assert ctx.render_form() == {"form": "k_path_defer", "ordered": False}


def _tab_fits(cs):
    """The persistent kernels' LDS copy of the scene tables holds the scene (kernels.hip kTabBytes:
    96-B lights, 48-B materials, the light CDF)."""
    nl, nm = len(cs.lights), len(cs.materials)
    return nl * 96 + nm * 48 + (nl + 1) * 4 <= 1024


def test_form_rule_reads_the_uploaded_tree_size(hip_ctx_factory):
    """The rule's cache-resident test sizes the tree the context holds now: after a
    rebuild into a smaller tree the render takes the cache-resident form, whatever the device buffers'
    capacities kept from the larger tree."""
    cs = scene.compile_scene(small_soup(200_000, (48, 27)))

    def dev_bytes(builder):   # wide nodes + leaf blob as the library uploads them (align 1, 3 float4 of padding)
        *_, (wn, lv, _) = capi.build_bvh_host(cs.vertices, cs.indices, builder=builder, n_threads=1, wide=True)
        return len(wn) * 64 + (int(np.sum(2 + 3 * lv["count"].astype(np.int64))) + 3) * 16

    big, small = dev_bytes(capi.BUILDER_SBVH), dev_bytes(capi.BUILDER_SAH)   # SBVH references are duplicated
    mib = (small >> 20) + 1                  # a cache share between the two trees
    assert small <= mib << 20 < big, (small, big)
    with hip_ctx_factory(0) as ctx:
        scene.upload_scene(ctx, cs, builder=capi.BUILDER_SBVH, n_threads=1)
        ctx.set_option("path_tail_steps", 1)
        ctx.set_option("path_cache_mb", mib)
        tiles = [(0, 0, 48, 27)]
        ctx.render(16, 5, tiles, 48, 27)
        assert ctx.render_form()["form"] == "k_path_spec"     # the large tree: not cache-resident
        ctx.build_accel(builder=capi.BUILDER_SAH, n_threads=1)
        ctx.render(16, 5, tiles, 48, 27)
        assert ctx.render_form()["form"] == "k_path_defer"    # the small one is


@pytest.mark.parametrize("path,defer,mix,tab,order", [(0, 0, 0, 1, 0), (0, 0, 0, 1, 1), (1, 0, 0, 0, 0), (1, 0, 0, 1, 0),
                                                      (1, 0, 0, 1, 1), (1, 1, 0, 1, 0), (1, 1, 1, 0, 0),
                                                      (1, 1, 1, 1, 0), (1, 1, 1, 1, 2), (1, 0, 0, 1, 2),
                                                      (1, 2, 0, 1, 0), (1, 2, 0, 0, 2), (1, 2, 0, 1, 2),
                                                      (1, 4, 0, 0, 0)])
def test_render_path_kernel_and_wavefront_bit_exact(hip_ctx_factory, path, defer, mix, tab, order):
    """The persistent path kernel (k_path), its deferred-NEE form (k_path_defer,
    §3.9: shadow rays handed to idle lanes of the wave, contributions added when the sample closes,
    scrambled or tile-order pixel fetch; defer = 1), its speculative-sample form (k_path_spec, §3.11:
    idle lanes run a busy pixel's next sample from a guessed sampler state, committed in order only
    when the guess was the true state; defer = 2, 4 with one sample beyond the head) and the wavefront kernels give the oracle's image bit for
    bit: ragged / clipped / empty tiles, depths 0-9 (above 8 the deferred form falls back to
    k_path), the clamp, Glossy + Mix + two-sided emitter, image textures, a soup whose rays take the
    deep stack, and a tile list smaller than one workgroup (fewer pixels than lanes); with the
    scene's material / light / CDF tables read from HBM or from the kernels' LDS copy (tab); with the
    cost-ordered pixel fetch (order, §3.10; the wavefront's camera-ray queue, option wave_order)
    forced on at every spp, or off."""
    def opts(ctx):
        ctx.set_option("path", path)
        ctx.set_option("path_defer", 1 if defer == 1 else 0)
        ctx.set_option("path_spec", 1 if defer >= 2 else 0)
        ctx.set_option("path_spec_depth", 1 if defer == 4 else 3)
        ctx.set_option("path_mix", mix)
        ctx.set_option("path_tab", tab)
        ctx.set_option("path_order", order)
        # paired cost order (§3.10): k_path_defer's (1), or k_path's too (3, an A/B option)
        ctx.set_option("path_order_pair", (1 if defer else 3) if order == 2 else 0)
        ctx.set_option("path_order_min_spp", 0 if order else 64)
        ctx.set_option("path_order_shift", 0)
    with hip_ctx_factory(0) as ctx:
        opts(ctx)
        cs, orc = _setup(ctx, cornell((40, 24)))
        assert _tab_fits(cs)
        tiles = [(0, 0, 16, 16), (24, 8, 40, 24), (30, 0, 64, 64), (5, 5, 5, 9)]
        for spp, depth in ((3, 0), (2, 1), (3, 2), (5, 5), (3, 8), (2, 9)):
            _check_render(ctx, orc, spp, depth, tiles, 40, 24)
        _check_render(ctx, orc, 4, 5, tiles, 40, 24, clamp=10.0)
        _check_render(ctx, orc, 7, 5, [(3, 3, 10, 8)], 40, 24)
    for sc in (mixed_scene((48, 48)), textured_scene((40, 40)), small_soup(100_000, (64, 36))):
        with hip_ctx_factory(0) as ctx:   # one scene per context (uploads append meshes)
            opts(ctx)
            cs, orc = _setup(ctx, sc)
            assert _tab_fits(cs)
            W, H = cs.camera.resolution
            _check_render(ctx, orc, 5, 5, [(0, 0, W, H)], W, H)
            _check_render(ctx, orc, 9, 3, [(0, 0, W, H)], W, H)
            # the per-pixel fingerprint (akr_pixel_probe): seeds always, ray counts from the
            # wavefront and from the persistent kernels' counting build
            try:
                for count in (0, 1):
                    ctx.set_option("count_tests", count)
                    *_, rays = _check_render(ctx, orc, 3, 5, [(0, 0, W, H), (3, 1, 17, 9)], W, H, probe=True)
                    assert rays == (path == 0 or count == 1)
            finally:
                ctx.set_option("count_tests", 0)


@pytest.mark.parametrize("spp", [16, 32])
def test_cornell_gpu_render_matches_reference_ref_png(hip_ctx_factory, spp):
    """Statistical pin of the HIP render on the reference's own output image (ref.png, 512^2,
    settings unknown; golden block statistics in tests/golden/ref_png_blocks.json): per-block
    z-test of the grey level (helpers.refpng_ztest), |z| <= 3 on >= 99 % of the blocks outside
    the light gap; in the gap (block row 2, columns 11-20) ref.png is brighter (its estimator
    differs there)."""
    import json
    from conftest import GOLDEN
    from helpers import refpng_verdict, refpng_ztest
    g = json.loads((GOLDEN / "ref_png_blocks.json").read_text())
    with hip_ctx_factory(0) as ctx:
        scene.upload_scene(ctx, scene.compile_scene(cornell((512, 512))))
        rad, w = ctx.render(spp, 5, [(0, 0, 512, 512)], 512, 512)
    frac, fails, gap_darker = refpng_verdict(refpng_ztest(rad, w, g))
    print(f"ref.png z-test at {spp} spp: {frac:.4f} within 3 sigma outside the gap; failing {fails}; "
          f"gap blocks darker: {gap_darker}/10")
    assert frac >= 0.99, fails
    assert gap_darker >= 8
