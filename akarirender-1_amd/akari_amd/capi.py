"""ctypes binding of the C-ABI in include/akr_hip.h (libakr_hip.so, built in-tree).

The product path is the HIP library: if ``libakr_hip.so`` is missing this module raises on
import — there is no CPU fallback anywhere in the package.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent.parent          # .../akarirender-1_amd
PRODUCT_LIB = PKG_DIR / "libakr_hip.so"
# Timing experiments only (tools/experiments/: a patch applied to a copy of csrc, built beside it): the
# override is honoured for a library under tools/experiments/lib/, never for another path
EXPERIMENT_LIB_DIR = PKG_DIR.parent / "tools" / "experiments" / "lib"
LIB_PATH = Path(os.environ.get("AKR_HIP_LIB", PRODUCT_LIB))
if LIB_PATH != PRODUCT_LIB and LIB_PATH.resolve().parent != EXPERIMENT_LIB_DIR.resolve():
    raise ImportError(f"AKR_HIP_LIB={LIB_PATH}: only tools/experiments/lib/*.so may replace the product library")
GEN_PATH = PKG_DIR / "libakr_scenegen.so"


class AkrError(RuntimeError):
    """A non-zero status from the C-ABI (the reference's AKR_ASSERT_THROW convention)."""


class Ray(C.Structure):
    _fields_ = [("o", C.c_float * 3), ("tmin", C.c_float), ("d", C.c_float * 3), ("tmax", C.c_float)]


class Hit(C.Structure):
    _fields_ = [("t", C.c_float), ("u", C.c_float), ("v", C.c_float), ("geom_id", C.c_int32),
                ("prim_id", C.c_int32), ("_pad", C.c_int32 * 3)]


class Texture(C.Structure):
    _fields_ = [("type", C.c_int32), ("value", C.c_float * 3), ("image", C.c_int32), ("_pad", C.c_int32 * 3)]


class Material(C.Structure):
    _fields_ = [("type", C.c_int32), ("color", C.c_int32), ("roughness", C.c_int32), ("fraction", C.c_int32),
                ("first", C.c_int32), ("second", C.c_int32), ("double_sided", C.c_int32), ("_pad", C.c_int32)]


class AreaLight(C.Structure):
    _fields_ = [("geom_id", C.c_int32), ("prim_id", C.c_int32)]


class Camera(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("rotation_deg", C.c_float * 3), ("fov_deg", C.c_double),
                ("resolution", C.c_int32 * 2), ("_pad", C.c_int32 * 2)]


class PtParams(C.Structure):
    _fields_ = [("spp", C.c_int32), ("max_depth", C.c_int32), ("ray_clamp", C.c_float), ("flags", C.c_int32)]


class AoParams(C.Structure):
    _fields_ = [("spp", C.c_int32), ("occlude", C.c_float), ("flags", C.c_int32), ("_pad", C.c_int32)]


class Rect(C.Structure):
    _fields_ = [("x0", C.c_int32), ("y0", C.c_int32), ("x1", C.c_int32), ("y1", C.c_int32)]


def _arr_ptr(arr):
    return C.c_void_p(arr.ctypes.data) if isinstance(arr, np.ndarray) else C.cast(arr, C.c_void_p)


def rect_array(tiles) -> np.ndarray:
    """Tiles (x0, y0, x1, y1) as the akr_rect array the render calls take without a copy."""
    return np.ascontiguousarray(np.asarray(tiles, dtype=np.int32).reshape(-1, 4))


class BuildParams(C.Structure):
    _fields_ = [("max_leaf_size", C.c_int32), ("n_bins", C.c_int32), ("traversal_cost", C.c_float),
                ("intersect_cost", C.c_float), ("n_threads", C.c_int32), ("builder", C.c_int32),
                ("spatial_budget", C.c_float), ("wide_collapse", C.c_int32)]


class AccelInfo(C.Structure):
    _fields_ = [("n_nodes", C.c_uint64), ("n_tris", C.c_uint64), ("max_depth", C.c_int32), ("max_leaf", C.c_int32),
                ("build_ms", C.c_double), ("sah_cost", C.c_double)]


class KernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("launches", C.c_uint64), ("total_ms", C.c_double), ("min_ms", C.c_double),
                ("max_ms", C.c_double)]


class TraceCounts(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("box_tests", C.c_uint64), ("tri_tests", C.c_uint64),
                ("closest_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("per_mode", (C.c_uint64 * 3) * 3),
                ("lane_slots", (C.c_uint64 * 4) * 3), ("deep_rays", C.c_uint64 * 3),
                ("leaf_tests", C.c_uint64 * 3)]


class PixelProbe(C.Structure):
    _fields_ = [("seed", C.c_uint32), ("closest_rays", C.c_uint32), ("shadow_rays", C.c_uint32), ("flags", C.c_uint32)]


TEX_CONSTANT, TEX_IMAGE = 0, 1
PT_EXACT_CULL = 1
BUILDER_SAH, BUILDER_LBVH, BUILDER_SBVH = 0, 1, 2
COLLAPSE_SAH, COLLAPSE_BALANCED = 0, 1   # akr_build_params::wide_collapse
MAT_DIFFUSE, MAT_GLOSSY, MAT_EMISSIVE, MAT_MIX = 0, 1, 2, 3
PROBE_SEED, PROBE_RAYS = 1, 2
FORM_NAMES = {-1: None, 0: "wavefront", 2: "k_path", 3: "k_path_defer", 4: "k_path_spec"}

# numpy views of the POD structs (for vectorised ray/hit buffers)
RAY_DTYPE = np.dtype([("o", np.float32, 3), ("tmin", np.float32), ("d", np.float32, 3), ("tmax", np.float32)])
HIT_DTYPE = np.dtype([("t", np.float32), ("u", np.float32), ("v", np.float32), ("geom_id", np.int32),
                      ("prim_id", np.int32), ("_pad", np.int32, 3)])
NODE_DTYPE = np.dtype([("bxy0", np.float32, 4), ("bxy1", np.float32, 4), ("bz", np.float32, 4),
                       ("child", np.uint32, 2), ("axis", np.uint32), ("_pad", np.uint32)])
TRI_DTYPE = np.dtype([("v0", np.float32, 3), ("gid", np.uint32), ("e1", np.float32, 3), ("_p0", np.uint32),
                      ("e2", np.float32, 3), ("_p1", np.uint32)])
NODE4_DTYPE = np.dtype([("origin", np.float32, 3), ("meta", np.uint32), ("child", np.uint32, 4),
                        ("q", np.uint32, 6), ("order", np.uint32, 2)])
PROBE_DTYPE = np.dtype([("seed", np.uint32), ("closest_rays", np.uint32), ("shadow_rays", np.uint32),
                        ("flags", np.uint32)])
LEAF_DTYPE = np.dtype([("lo", np.float32, 3), ("hi", np.float32, 3), ("first", np.uint32), ("count", np.uint32)])
assert RAY_DTYPE.itemsize == 32 and HIT_DTYPE.itemsize == 32
assert NODE_DTYPE.itemsize == 64 and TRI_DTYPE.itemsize == 48
assert NODE4_DTYPE.itemsize == 64 and LEAF_DTYPE.itemsize == 32

# Every export of include/akr_hip.h: name -> (restype, argtypes)
_P = C.c_void_p
EXPORTS = {
    "akr_hip_api_version": (C.c_int, []),
    "akr_hip_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "akr_hip_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "akr_hip_destroy": (C.c_int, [_P]),
    "akr_hip_last_error": (C.c_char_p, [_P]),
    "akr_hip_set_option": (C.c_int, [_P, C.c_char_p, C.c_int64]),
    "akr_hip_upload_mesh": (C.c_int, [_P, _P, C.c_uint64, _P, _P, _P, _P, C.c_uint64, _P, C.c_int32,
                                      C.POINTER(C.c_int32)]),
    "akr_hip_upload_images": (C.c_int, [_P, _P, _P, _P, C.c_int32]),
    "akr_hip_upload_textures": (C.c_int, [_P, _P, C.c_int32]),
    "akr_hip_upload_materials": (C.c_int, [_P, _P, C.c_int32]),
    "akr_hip_upload_lights": (C.c_int, [_P, _P, C.c_int32, _P]),
    "akr_hip_build_accel": (C.c_int, [_P, C.POINTER(BuildParams)]),
    "akr_hip_import_accel": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint64, C.c_int32]),
    "akr_bvh_validate": (C.c_int, [_P, C.c_uint64, _P, C.c_uint64, C.c_uint64, C.POINTER(C.c_int32)]),
    "akr_hip_accel_info": (C.c_int, [_P, C.POINTER(AccelInfo)]),
    "akr_hip_accel_export": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint64]),
    "akr_hip_set_camera": (C.c_int, [_P, C.POINTER(Camera)]),
    "akr_hip_trace": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_int]),
    "akr_hip_trace_device": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_int, _P]),
    "akr_hip_render": (C.c_int, [_P, C.POINTER(PtParams), _P, C.c_int32, _P, _P]),
    "akr_hip_render_ao": (C.c_int, [_P, C.POINTER(AoParams), _P, C.c_int32, _P, _P]),
    "akr_hip_ray_steps": (C.c_int, [_P, _P, C.c_uint64]),
    "akr_hip_render_device": (C.c_int, [_P, C.POINTER(PtParams), _P, C.c_int32, _P, _P, _P,
                                        C.POINTER(C.c_uint64)]),
    "akr_hip_kernel_stats": (C.c_int, [_P, _P, C.c_int32, C.POINTER(C.c_int32)]),
    "akr_hip_trace_counts": (C.c_int, [_P, C.POINTER(TraceCounts)]),
    "akr_hip_path_profile": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_int32]),
    "akr_hip_reset_stats": (C.c_int, [_P]),
    "akr_hip_render_info": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "akr_hip_synchronize": (C.c_int, [_P]),
    "akr_hip_render_form": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "akr_hip_render_form_inputs": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "akr_hip_pixel_probe": (C.c_int, [_P, _P, C.c_uint64]),
    "akr_bvh_host_build": (C.c_int, [_P, C.c_uint64, _P, C.c_uint64, C.POINTER(BuildParams), C.POINTER(_P),
                                     C.POINTER(AccelInfo)]),
    "akr_bvh_host_nodes": (_P, [_P]),
    "akr_bvh_host_tris": (_P, [_P]),
    "akr_bvh_host_free": (None, [_P]),
    "akr_hip_render_node": (C.c_int, [C.POINTER(_P), C.c_int32, C.POINTER(PtParams), _P, C.c_int32, _P, _P]),
    "akr_bvh_host_wide": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]),
    "akr_bvh_host_wide_nodes": (_P, [_P]),
    "akr_bvh_host_wide_leaves": (_P, [_P]),
}

_lib = None


def load_library() -> C.CDLL:
    """Load libakr_hip.so (raises if it has not been built — no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
        variant = LIB_PATH != PRODUCT_LIB  # an experiment build may predate newer exports
        for name, (res, args) in EXPORTS.items():
            if variant and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def device_count() -> int:
    n = C.c_int(0)
    load_library().akr_hip_device_count(C.byref(n))
    return n.value


def build_bvh_host(vertices, indices, max_leaf_size=4, n_bins=32, traversal_cost=1.0, intersect_cost=4.0,
                   n_threads=0, wide=False, builder=0, spatial_budget=0.0, wide_collapse=0):
    """Run the product BVH builder on the host (no device): returns (nodes, tris, info), plus
    (wide_nodes, leaves, root_ref) of the 4-wide traversal view when `wide` (wide_collapse:
    COLLAPSE_SAH or COLLAPSE_BALANCED).  builder: BUILDER_SAH
    or BUILDER_SBVH (the host builders)."""
    lib = load_library()
    v = np.ascontiguousarray(vertices, np.float32).reshape(-1)
    i = np.ascontiguousarray(indices, np.int32).reshape(-1)
    p = BuildParams(max_leaf_size, n_bins, traversal_cost, intersect_cost, n_threads, builder, spatial_budget,
                    wide_collapse)
    h = C.c_void_p()
    info = AccelInfo()
    st = lib.akr_bvh_host_build(_ptr(v), v.size // 3, _ptr(i), i.size // 3, C.byref(p), C.byref(h), C.byref(info))
    if st != 0:
        raise AkrError("akr_bvh_host_build failed (invalid indices or build error)")
    try:
        nodes = np.empty(info.n_nodes, NODE_DTYPE)
        tris = np.empty(info.n_tris, TRI_DTYPE)
        C.memmove(nodes.ctypes.data, lib.akr_bvh_host_nodes(h), nodes.nbytes)
        if tris.nbytes:
            C.memmove(tris.ctypes.data, lib.akr_bvh_host_tris(h), tris.nbytes)
        if wide:
            nn, nl, root = C.c_uint64(0), C.c_uint64(0), C.c_uint32(0)
            if lib.akr_bvh_host_wide(h, C.byref(nn), C.byref(nl), C.byref(root)) != 0:
                raise AkrError("akr_bvh_host_wide failed")
            wn = np.empty(nn.value, NODE4_DTYPE)
            lv = np.empty(nl.value, LEAF_DTYPE)
            if wn.nbytes:
                C.memmove(wn.ctypes.data, lib.akr_bvh_host_wide_nodes(h), wn.nbytes)
            if lv.nbytes:
                C.memmove(lv.ctypes.data, lib.akr_bvh_host_wide_leaves(h), lv.nbytes)
    finally:
        lib.akr_bvh_host_free(h)
    if wide:
        return nodes, tris, info, (wn, lv, root.value)
    return nodes, tris, info


def validate_bvh(nodes, tris, n_scene_tris):
    """Host check of a BVH2 (akr_bvh_validate): returns its depth, raises AkrError when malformed."""
    nodes = np.ascontiguousarray(nodes, NODE_DTYPE)
    tris = np.ascontiguousarray(tris, TRI_DTYPE)
    d = C.c_int32(0)
    if load_library().akr_bvh_validate(_ptr(nodes), nodes.shape[0], _ptr(tris), tris.shape[0], int(n_scene_tris),
                                       C.byref(d)) != 0:
        raise AkrError("malformed BVH")
    return d.value


def render_node(ctxs, spp, max_depth, tiles, width, height, ray_clamp=0.0, exact_cull=False, radiance=None,
                weight=None):
    """akr_hip_render_node: tile j on ctxs[j % len(ctxs)], one host thread per context; returns
    the full-frame (radiance, weight) accumulated like HipContext.render (into the given buffers)."""
    lib = load_library()
    if radiance is None:
        radiance = np.zeros((height, width, 3), np.float32)
    if weight is None:
        weight = np.zeros((height, width), np.float32)
    assert radiance.dtype == np.float32 and radiance.flags.c_contiguous and radiance.size == 3 * width * height
    assert weight.dtype == np.float32 and weight.flags.c_contiguous and weight.size == width * height
    arr = (Rect * max(1, len(tiles)))(*[Rect(*t) for t in tiles])
    hs = (C.c_void_p * len(ctxs))(*[c.h for c in ctxs])
    p = PtParams(int(spp), int(max_depth), float(ray_clamp), PT_EXACT_CULL if exact_cull else 0)
    if lib.akr_hip_render_node(hs, len(ctxs), C.byref(p), _arr_ptr(arr), len(tiles), _ptr(radiance),
                               _ptr(weight)) != 0:
        raise AkrError(lib.akr_hip_last_error(ctxs[0].h).decode() if ctxs else "no contexts")
    return radiance, weight


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class HipContext:
    """Owner of one akr_hip_ctx (one device, one stream)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        st = self.lib.akr_hip_create(int(device), C.byref(h))
        if st != 0:
            raise AkrError(f"akr_hip_create({device}) failed with status {st} (no HIP device?)")
        self.h = h
        self.device = device
        self._keep = []
        self._opts = {}   # options set through this object (the library has no getter)

    def close(self):
        if getattr(self, "h", None):
            self.lib.akr_hip_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, st: int):
        if st != 0:
            msg = self.lib.akr_hip_last_error(self.h)
            raise AkrError(msg.decode() if msg else f"status {st}")

    def set_option(self, key: str, value: int):
        self._check(self.lib.akr_hip_set_option(self.h, key.encode(), int(value)))
        self._opts[key] = int(value)

    def option_set(self, key: str):
        """The value this object last set for `key`, or None (the library's default is in effect)."""
        return self._opts.get(key)

    def upload_mesh(self, vertices, indices, normals, texcoords, material_indices, material_slots) -> int:
        v = np.ascontiguousarray(vertices, np.float32).reshape(-1)
        i = np.ascontiguousarray(indices, np.int32).reshape(-1)
        n = np.ascontiguousarray(normals, np.float32).reshape(-1)
        t = np.ascontiguousarray(texcoords, np.float32).reshape(-1)
        m = np.ascontiguousarray(material_indices, np.int32).reshape(-1)
        s = np.ascontiguousarray(material_slots, np.int32).reshape(-1)
        nt = m.size
        if i.size != 3 * nt or n.size != 9 * nt or t.size != 6 * nt or v.size % 3:
            raise ValueError("inconsistent mesh array sizes")
        gid = C.c_int32(-1)
        self._check(self.lib.akr_hip_upload_mesh(self.h, _ptr(v), v.size // 3, _ptr(i), _ptr(n), _ptr(t), _ptr(m),
                                                 nt, _ptr(s), s.size, C.byref(gid)))
        return gid.value

    def upload_textures(self, texs):
        arr = (Texture * max(1, len(texs)))(*texs)
        self._check(self.lib.akr_hip_upload_textures(self.h, _arr_ptr(arr), len(texs)))

    def upload_images(self, images):
        """images: list of float32 [h, w, 4] RGBA arrays."""
        if not images:
            self._check(self.lib.akr_hip_upload_images(self.h, None, None, None, 0))
            return
        flat = np.concatenate([np.ascontiguousarray(im, np.float32).reshape(-1) for im in images])
        w = np.array([im.shape[1] for im in images], np.int32)
        hh = np.array([im.shape[0] for im in images], np.int32)
        self._check(self.lib.akr_hip_upload_images(self.h, _ptr(flat), _ptr(w), _ptr(hh), len(images)))

    def upload_materials(self, mats):
        arr = (Material * max(1, len(mats)))(*mats)
        self._check(self.lib.akr_hip_upload_materials(self.h, _arr_ptr(arr), len(mats)))

    def upload_lights(self, lights, power):
        arr = (AreaLight * max(1, len(lights)))(*[AreaLight(g, p) for g, p in lights])
        pw = np.ascontiguousarray(power, np.float32)
        self._check(self.lib.akr_hip_upload_lights(self.h, _arr_ptr(arr), len(lights), _ptr(pw)))

    def build_accel(self, max_leaf_size=4, n_bins=32, traversal_cost=1.0, intersect_cost=4.0, n_threads=0,
                    builder=0, spatial_budget=0.0, wide_collapse=0):
        """builder: BUILDER_SAH (host binned SAH), BUILDER_LBVH (GPU Morton / Karras) or BUILDER_SBVH
        (host SBVH with the reference's spatial splits; spatial_budget = extra references / triangles).
        wide_collapse: COLLAPSE_SAH (default) or COLLAPSE_BALANCED, the traversal's 4-wide view."""
        p = BuildParams(max_leaf_size, n_bins, traversal_cost, intersect_cost, n_threads, builder, spatial_budget,
                    wide_collapse)
        self._check(self.lib.akr_hip_build_accel(self.h, C.byref(p)))
        return self.accel_info()

    def import_accel(self, nodes, tris, n_threads=0):
        """Adopt a BVH2 exported by another context (accel_export) instead of building one."""
        nodes = np.ascontiguousarray(nodes, NODE_DTYPE)
        tris = np.ascontiguousarray(tris, TRI_DTYPE)
        self._check(self.lib.akr_hip_import_accel(self.h, _ptr(nodes), nodes.shape[0], _ptr(tris), tris.shape[0],
                                                  int(n_threads)))
        return self.accel_info()

    def accel_info(self) -> AccelInfo:
        info = AccelInfo()
        self._check(self.lib.akr_hip_accel_info(self.h, C.byref(info)))
        return info

    def accel_export(self):
        info = self.accel_info()
        nodes = np.zeros(info.n_nodes, NODE_DTYPE)
        tris = np.zeros(info.n_tris, TRI_DTYPE)
        self._check(self.lib.akr_hip_accel_export(self.h, _ptr(nodes), nodes.nbytes, _ptr(tris), tris.nbytes))
        return nodes, tris

    def set_camera(self, position, rotation_deg, fov_deg, resolution):
        cam = Camera((C.c_float * 3)(*position), (C.c_float * 3)(*rotation_deg), float(fov_deg),
                     (C.c_int32 * 2)(*resolution))
        self._check(self.lib.akr_hip_set_camera(self.h, C.byref(cam)))

    def trace(self, rays: np.ndarray, any_hit: bool = False) -> np.ndarray:
        rays = np.ascontiguousarray(rays, RAY_DTYPE)
        hits = np.zeros(rays.shape[0], HIT_DTYPE)
        self._check(self.lib.akr_hip_trace(self.h, _ptr(rays), rays.shape[0], _ptr(hits), int(bool(any_hit))))
        return hits

    def trace_device(self, d_rays: int, n: int, d_hits: int, any_hit: bool = False, stream: int = 0):
        self._check(self.lib.akr_hip_trace_device(self.h, C.c_void_p(d_rays), n, C.c_void_p(d_hits),
                                                  int(bool(any_hit)), C.c_void_p(stream)))

    @staticmethod
    def _rects(tiles):
        """The tile list as the C-ABI's akr_rect array: an (n, 4) int32 array from rect_array()
        passes without a copy (the caller converts once, not per render: building 2,000 ctypes
        records took 0.8 ms per call)."""
        if isinstance(tiles, np.ndarray):
            if tiles.dtype != np.int32 or tiles.ndim != 2 or tiles.shape[1] != 4 or not tiles.flags.c_contiguous:
                raise ValueError("tile array must be a C-contiguous (n, 4) int32 array (capi.rect_array)")
            return tiles, len(tiles)
        arr = (Rect * max(1, len(tiles)))(*[Rect(*t) for t in tiles])
        return arr, len(tiles)

    def render(self, spp, max_depth, tiles, width, height, ray_clamp=0.0, radiance=None, weight=None,
               exact_cull=False):
        """Accumulate into full-frame host buffers (Film::merge_tile semantics)."""
        if radiance is None:
            radiance = np.zeros((height, width, 3), np.float32)
        if weight is None:
            weight = np.zeros((height, width), np.float32)
        assert radiance.dtype == np.float32 and radiance.flags.c_contiguous and radiance.size == 3 * width * height
        assert weight.dtype == np.float32 and weight.flags.c_contiguous and weight.size == width * height
        p = PtParams(int(spp), int(max_depth), float(ray_clamp), PT_EXACT_CULL if exact_cull else 0)
        arr, n = self._rects(tiles)
        self._check(self.lib.akr_hip_render(self.h, C.byref(p), _arr_ptr(arr), n, _ptr(radiance),
                                            _ptr(weight)))
        return radiance, weight

    def render_ao(self, spp, tiles, width, height, occlude=float("inf"), radiance=None, weight=None,
                  exact_cull=False):
        """Ambient occlusion (akr_hip_render_ao), accumulated like render()."""
        if radiance is None:
            radiance = np.zeros((height, width, 3), np.float32)
        if weight is None:
            weight = np.zeros((height, width), np.float32)
        assert radiance.dtype == np.float32 and radiance.flags.c_contiguous and radiance.size == 3 * width * height
        assert weight.dtype == np.float32 and weight.flags.c_contiguous and weight.size == width * height
        p = AoParams(int(spp), float(occlude), PT_EXACT_CULL if exact_cull else 0, 0)
        arr, n = self._rects(tiles)
        self._check(self.lib.akr_hip_render_ao(self.h, C.byref(p), _arr_ptr(arr), n, _ptr(radiance),
                                               _ptr(weight)))
        return radiance, weight

    def render_device(self, spp, max_depth, tiles, d_radiance: int, d_weight: int, stream: int = 0, ray_clamp=0.0):
        p = PtParams(int(spp), int(max_depth), float(ray_clamp), 0)
        arr, n = self._rects(tiles)
        npx = C.c_uint64(0)
        self._check(self.lib.akr_hip_render_device(self.h, C.byref(p), _arr_ptr(arr), n,
                                                   C.c_void_p(d_radiance), C.c_void_p(d_weight), C.c_void_p(stream),
                                                   C.byref(npx)))
        return npx.value

    def ray_steps(self, n: int) -> np.ndarray:
        """Per-ray traversal iterations of the last standalone trace (option "ray_steps")."""
        out = np.zeros(n, np.uint32)
        self._check(self.lib.akr_hip_ray_steps(self.h, _ptr(out), n))
        return out

    def kernel_stats(self) -> dict:
        n = C.c_int32(0)
        self._check(self.lib.akr_hip_kernel_stats(self.h, None, 0, C.byref(n)))
        arr = (KernelStat * max(1, n.value))()
        self._check(self.lib.akr_hip_kernel_stats(self.h, _arr_ptr(arr), n.value, C.byref(n)))
        return {arr[i].name.decode(): dict(launches=arr[i].launches, total_ms=arr[i].total_ms, min_ms=arr[i].min_ms,
                                           max_ms=arr[i].max_ms) for i in range(n.value)}

    def render_info(self) -> dict:
        """Lanes per pixel (always 1) and sample passes of the last render (1 for a persistent form)."""
        lanes, passes = C.c_int32(0), C.c_int32(0)
        self._check(self.lib.akr_hip_render_info(self.h, C.byref(lanes), C.byref(passes)))
        return {"lanes": lanes.value, "passes": passes.value}

    def render_form(self) -> dict:
        """The form that ran the last path render (FORM_NAMES) and whether its pixel fetch was
        cost-ordered."""
        f, o = C.c_int32(0), C.c_int32(0)
        self._check(self.lib.akr_hip_render_form(self.h, C.byref(f), C.byref(o)))
        return {"form": FORM_NAMES.get(f.value, str(f.value)), "ordered": bool(o.value)}

    def render_form_inputs(self) -> dict:
        """The last persistent render's form-choice inputs: pixels per resident lane,
        and the cost-ordering pilot's rays and mean traversal steps per ray (rays -1: not read)."""
        a, b, c = C.c_int64(0), C.c_int64(0), C.c_int64(0)
        self._check(self.lib.akr_hip_render_form_inputs(self.h, C.byref(a), C.byref(b), C.byref(c)))
        return {"pixels_per_lane": a.value / 1000, "pilot_rays": b.value,
                "pilot_mean_steps": c.value / b.value if b.value > 0 else None}

    def path_profile(self) -> dict:
        """k_path phase profile of the counted launches since reset_stats (ticks: 100 MHz)."""
        keys = ("waves", "outer", "procs", "trav_iters", "t_proc", "t_trav", "t_leaf", "t_total", "t_max", "lanes_proc",
                "t_shade", "spec_started", "spec_aborted", "tv_issue", "tv_wait", "tv_comp", "tl_issue", "tl_wait",
                "tl_comp", "tp_park", "tp_next", "tp_begin", "tp_load", "leaf_phases", "leaf_holders",
                # option count_lines (k_path): distinct 128-B lines the last such render read, per region
                "lines_nodes", "lines_leaves", "lines_shading")
        out = (C.c_uint64 * len(keys))()
        self._check(self.lib.akr_hip_path_profile(self.h, out, len(keys)))
        return dict(zip(keys, (int(v) for v in out)))

    def trace_counts(self) -> dict:
        c = TraceCounts()
        self._check(self.lib.akr_hip_trace_counts(self.h, C.byref(c)))
        modes = ("closest", "any", "shadow")
        per = {m: dict(rays=c.per_mode[k][0], box_tests=c.per_mode[k][1], tri_tests=c.per_mode[k][2],
                       slots_traversal=c.lane_slots[k][0], slots_busy=c.lane_slots[k][1],
                       slots_tri=c.lane_slots[k][2], visits=c.lane_slots[k][3], deep_rays=c.deep_rays[k],
                       leaf_tests=c.leaf_tests[k])
               for k, m in enumerate(modes)}
        return dict(rays=c.rays, box_tests=c.box_tests, tri_tests=c.tri_tests, per_mode=per)

    def pixel_probe(self, n: int) -> np.ndarray:
        """Test-only per-slot fingerprint of the last render (option "pixel_probe"): PROBE_DTYPE[n]
        in packed tile order (final sampler state, closest-hit and shadow traces)."""
        out = np.zeros(n, PROBE_DTYPE)
        self._check(self.lib.akr_hip_pixel_probe(self.h, _ptr(out), n))
        return out

    def reset_stats(self):
        self._check(self.lib.akr_hip_reset_stats(self.h))

    def synchronize(self):
        self._check(self.lib.akr_hip_synchronize(self.h))


_gen = None


def generate_soup(n_tris: int, seed: int = 42, r: float = 0.01, n_threads: int = 0):
    """Synthetic soup: returns (vertices [3n,3], normals [n,9], texcoords [n,6])."""
    global _gen
    if _gen is None:
        if not GEN_PATH.exists():
            raise ImportError(f"{GEN_PATH} is missing: run __graft_entry__.build()")
        _gen = C.CDLL(str(GEN_PATH))
        _gen.akr_gen_soup.restype = C.c_int
        _gen.akr_gen_soup.argtypes = [C.c_uint64, C.c_uint64, C.c_float, _P, _P, _P, C.c_int]
    v = np.empty((3 * n_tris, 3), np.float32)
    nn = np.empty((n_tris, 9), np.float32)
    t = np.empty((n_tris, 6), np.float32)
    _gen.akr_gen_soup(n_tris, seed, r, _ptr(v), _ptr(nn), _ptr(t), int(n_threads or min(16, os.cpu_count() or 1)))
    return v, nn, t
