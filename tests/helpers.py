"""Shared test inputs: seeded ray batches and small scenes."""
import numpy as np

from akari_amd import capi, scene


def random_rays(n, seed, lo, hi, tmin=1e-3, tmax=np.inf):
    """Origins uniform in the box [lo, hi]^3, directions uniform on the sphere (normalised in f32)."""
    rng = np.random.default_rng(seed)
    r = np.zeros(n, capi.RAY_DTYPE)
    r["o"] = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    r["d"] = d
    r["tmin"] = np.float32(tmin)
    r["tmax"] = np.float32(tmax)
    return r


def edge_rays(center=(0.0, 0.0, 0.0)):
    """Axis-aligned directions (zero components -> inf/NaN slabs), degenerate intervals, +-0."""
    c = np.asarray(center, np.float32)
    dirs = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1), (-0.0, -1, 0.0),
            (0.5, 0.5, 0.0), (0, 0.5, -0.5), (1e-30, 1, 0)]
    rays = []
    for d in dirs:
        d = np.asarray(d, np.float32)
        d = d / np.float32(np.sqrt(np.float32(np.dot(d, d))))
        for tmin, tmax in ((1e-3, np.inf), (0.0, np.inf), (1e-3, 1e-3), (5.0, 1.0), (1e-3, 0.5)):
            r = np.zeros(1, capi.RAY_DTYPE)
            r["o"], r["d"], r["tmin"], r["tmax"] = c, d, tmin, tmax
            rays.append(r)
    return np.concatenate(rays)


def cornell(resolution=(64, 64)):
    from conftest import CORNELL_MESH
    return scene.cornell_scene(CORNELL_MESH, resolution=resolution)


def small_soup(n_tris=20000, resolution=(96, 54), seed=42, r=0.01):
    return scene.soup_scene(n_tris=n_tris, resolution=resolution, seed=seed, r=r)


def check_sbvh(cs, nodes, tris, max_leaf, budget=0.5, samples=6):
    """Invariants of an SBVH export (references may be clipped and duplicated): every triangle in
    at least one leaf and at most budget * n extra records, records equal to the mesh, child boxes
    inside their parents, and every triangle covered by the union of its leaf boxes (a barycentric
    grid of points, in f64, each inside at least one of the triangle's leaf boxes)."""
    n = cs.n_tris
    g = tris["gid"].astype(np.int64)
    assert set(g.tolist()) == set(range(n)) and len(g) <= n + int(budget * n) + 1
    v = cs.vertices[cs.indices]
    assert np.array_equal(tris["v0"], v[g, 0])
    assert np.array_equal(tris["e1"], (v[g, 1] - v[g, 0]).astype(np.float32))
    assert np.array_equal(tris["e2"], (v[g, 2] - v[g, 0]).astype(np.float32))
    leaf_lo = np.zeros((len(g), 3), np.float64)
    leaf_hi = np.zeros((len(g), 3), np.float64)
    root_lo = np.array([nodes[0]["bxy0"][0], nodes[0]["bxy0"][2], nodes[0]["bz"][0]], np.float32)
    root_hi = np.array([nodes[0]["bxy0"][1], nodes[0]["bxy0"][3], nodes[0]["bz"][1]], np.float32)
    stack = [(int(nodes[0]["child"][0]), root_lo, root_hi, root_lo, root_hi, 1)]
    while stack:
        ref, lo, hi, plo, phi, depth = stack.pop()
        assert depth <= 64 and np.all(lo >= plo) and np.all(hi <= phi)
        if ref & 0x80000000:
            first, cnt = (ref & 0x7FFFFFFF) >> 3, (ref & 7) + 1
            assert cnt <= max_leaf
            leaf_lo[first:first + cnt] = lo
            leaf_hi[first:first + cnt] = hi
        else:
            nd = nodes[ref]
            for k, (bxy, bz) in enumerate(((nd["bxy0"], nd["bz"][:2]), (nd["bxy1"], nd["bz"][2:]))):
                clo = np.array([bxy[0], bxy[2], bz[0]], np.float32)
                chi = np.array([bxy[1], bxy[3], bz[1]], np.float32)
                stack.append((int(nd["child"][k]), clo, chi, lo, hi, depth + 1))
    vd = v.astype(np.float64)
    bary = [(a / samples, b / samples) for a in range(samples + 1) for b in range(samples + 1 - a)]
    order = np.argsort(g, kind="stable")
    starts = np.searchsorted(g[order], np.arange(n + 1))
    for tri in range(n):
        idx = order[starts[tri]:starts[tri + 1]]
        lo, hi = leaf_lo[idx], leaf_hi[idx]
        for a, b in bary:
            p = (1 - a - b) * vd[tri, 0] + a * vd[tri, 1] + b * vd[tri, 2]
            eps = 1e-12 * (1.0 + np.abs(p))   # f64 rounding of the combination, far below an f32 ulp
            assert np.any(np.all((p >= lo - eps) & (p <= hi + eps), axis=1)), f"triangle {tri} point {a, b} not covered"
    return len(g) - n


def mixed_scene(resolution=(48, 48)):
    """Cornell geometry with Glossy / Mix materials and a two-sided emitter (BSDF coverage)."""
    sc = cornell(resolution)
    m = sc.shapes[0]
    ct = scene.ConstantTexture
    glossy = scene.GlossyMaterial(ct([0.9, 0.8, 0.7]), ct([0.4, 0.4, 0.4]))
    mix = scene.MixMaterial(ct([0.3, 0.3, 0.3]), scene.DiffuseMaterial(ct([0.2, 0.7, 0.2])), glossy)
    m.materials[5] = glossy       # short box
    m.materials[6] = mix          # tall box
    m.materials[7] = scene.EmissiveMaterial(ct([17.0, 12.0, 4.0]), double_sided=True)
    return sc


def textured_scene(resolution=(48, 48)):
    """Cornell geometry with image textures on diffuse, glossy roughness, mix fraction and emitter
    colour (a15); texcoords stretched to [-1, 2] so the fmod wrap and the clamp are exercised."""
    sc = mixed_scene(resolution)
    m = sc.shapes[0]
    rng = np.random.default_rng(11)
    img = lambda h, w: scene.ImageTexture(rng.random((h, w, 4), dtype=np.float32))
    m.texcoords = (np.asarray(m.texcoords, np.float32) * np.float32(3.0) - np.float32(1.0)).astype(np.float32)
    ct = scene.ConstantTexture
    m.materials[0] = scene.DiffuseMaterial(img(23, 37))                       # floor
    m.materials[2] = scene.GlossyMaterial(img(5, 7), img(9, 4))               # back wall: roughness image
    m.materials[6] = scene.MixMaterial(img(16, 16), scene.DiffuseMaterial(img(3, 3)),
                                       scene.GlossyMaterial(ct([0.8, 0.8, 0.8]), ct([0.3, 0.3, 0.3])))
    m.materials[7] = scene.EmissiveMaterial(scene.ImageTexture(rng.random((4, 6, 4), dtype=np.float32) * 20),
                                            double_sided=False)
    return sc


def hits_to_gid(hits, mesh_base):
    gid = np.full(hits.shape[0], 0xFFFFFFFF, np.uint32)
    ok = hits["geom_id"] >= 0
    gid[ok] = mesh_base[hits["geom_id"][ok]] + hits["prim_id"][ok].astype(np.uint32)
    return gid


def check_bvh(cs, nodes, tris, max_leaf):
    """Invariants of an exported BVH2: every triangle in exactly one leaf, leaf records equal to
    the mesh (e1, e2 as f32 subtractions), child boxes containing their subtrees, depth <= 64."""
    n = cs.n_tris
    assert sorted(tris["gid"].tolist()) == list(range(n)), "every triangle in exactly one leaf"
    v = cs.vertices[cs.indices]
    g = tris["gid"]
    assert np.array_equal(tris["v0"], v[g, 0])
    assert np.array_equal(tris["e1"], (v[g, 1] - v[g, 0]).astype(np.float32))
    assert np.array_equal(tris["e2"], (v[g, 2] - v[g, 0]).astype(np.float32))
    # walk: child boxes contain their subtree's triangles, depth bounded, leaf sizes bounded
    stack = [(int(nodes[0]["child"][0]), nodes[0]["bxy0"], nodes[0]["bz"][:2], 1)]
    seen = 0
    while stack:
        ref, bxy, bz, depth = stack.pop()
        assert depth <= 64
        lo = np.array([bxy[0], bxy[2], bz[0]], np.float32)
        hi = np.array([bxy[1], bxy[3], bz[1]], np.float32)
        if ref & 0x80000000:
            first, cnt = (ref & 0x7FFFFFFF) >> 3, (ref & 7) + 1
            assert cnt <= max_leaf
            pts = v[tris["gid"][first:first + cnt]].reshape(-1, 3)
            assert np.all(pts >= lo) and np.all(pts <= hi)
            seen += cnt
        else:
            nd = nodes[ref]
            assert nd["axis"] < 3
            stack.append((int(nd["child"][0]), nd["bxy0"], nd["bz"][:2], depth + 1))
            stack.append((int(nd["child"][1]), nd["bxy1"], nd["bz"][2:], depth + 1))
    assert seen == n


# ref.png blocks where the reference's image was made by a different estimator: the
# ceiling strip in the 1-cm gap above the one-sided light (y 1.98 vs ceiling 1.99), block row 2.
REFPNG_LIGHT_GAP = [(2, c) for c in range(11, 21)]


def refpng_ztest(rad, w, golden):
    """Per-block z statistic of the grey level (channel mean of the sRGB8 image, 16x16 blocks)
    against the reference's ref.png, z = (ours - ref) / sqrt((var_ours + var_ref) / 256), each
    variance the image's own within-block pixel variance (per-block z-test; spatial
    variation inside a block only inflates sigma).  Returns z [32, 32]."""
    from akari_amd import film
    grey = film.to_srgb8(rad, w).astype(np.float64).mean(axis=2).reshape(32, 16, 32, 16)
    mo, vo = grey.mean(axis=(1, 3)), grey.var(axis=(1, 3), ddof=1)
    mr, vr = np.asarray(golden["grey_mean"]), np.asarray(golden["grey_var"])
    return (mo - mr) / np.sqrt((vo + vr) / 256.0 + 1e-12)


def refpng_verdict(z):
    """(fraction of blocks outside the light gap with |z| <= 3, failing blocks outside the gap,
    gap blocks where ref.png is brighter by more than 3 sigma)."""
    gap = np.zeros(z.shape, bool)
    for r, c in REFPNG_LIGHT_GAP:
        gap[r, c] = True
    ok = np.abs(z) <= 3
    outside = ~gap
    fails = [(int(r), int(c), round(float(z[r, c]), 1)) for r, c in np.argwhere(outside & ~ok)]
    gap_darker = int(np.count_nonzero(gap & (z < -3)))
    return ok[outside].mean(), fails, gap_darker


def slot_pixels(tiles, width, height):
    """(ys, xs) of every film slot in packed tile order (tiles clipped to the frame, row-major
    inside a tile): the order of akr_hip_render_device's output and of akr_hip_pixel_probe."""
    ys, xs = [], []
    for x0, y0, x1, y1 in tiles:
        x0, y0, x1, y1 = max(0, x0), max(0, y0), min(width, x1), min(height, y1)
        if x1 <= x0 or y1 <= y0:
            continue
        yy, xx = np.mgrid[y0:y1, x0:x1]
        ys.append(yy.reshape(-1))
        xs.append(xx.reshape(-1))
    if not ys:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    return np.concatenate(ys), np.concatenate(xs)


def check_probe(gpu, orc_frame, tiles, width, height, what=""):
    """Compare a device pixel probe (slot order) with the oracle's frame-indexed probe: the final
    sampler state always, the ray counts when the device recorded them.  Returns whether it
    compared ray counts."""
    ys, xs = slot_pixels(tiles, width, height)
    exp = orc_frame[ys, xs]
    assert len(gpu) == len(exp)
    assert np.all(gpu["flags"] & capi.PROBE_SEED), f"{what}: seeds not recorded"
    bad = np.count_nonzero(gpu["seed"] != exp["seed"])
    assert bad == 0, f"{what}: {bad} of {len(exp)} final sampler states differ from the oracle"
    rays = bool(np.all(gpu["flags"] & capi.PROBE_RAYS))
    if rays:
        for k in ("closest_rays", "shadow_rays"):
            bad = np.count_nonzero(gpu[k] != exp[k])
            assert bad == 0, f"{what}: {bad} of {len(exp)} per-pixel {k} differ from the oracle"
    return rays
