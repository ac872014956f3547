"""Scene description, `.mesh` I/O, `.akari` loader and scene compilation.

Host-side mirror of the reference's scene graph (src/akari/core/nodes/*.cpp) reduced to what the
hot path consumes.  ``compile_scene`` restates ``SceneNode<C>::compile``
(src/akari/core/nodes/scene.cpp:43-95): it flattens meshes, numbers materials and textures, and
builds the emissive-triangle light list with the reference's power weights (float/double
arithmetic kept as written there, so Distribution1D selects the same light).
"""
from __future__ import annotations

import math
import os
import struct
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional, Sequence, Union

import numpy as np

from . import capi

MESH_MAGIC = b"AKARI_BINARY_MESH"   # core/mesh.cpp:27
F32 = np.float32


# ----------------------------------------------------------------------------- scene nodes
@dataclass(eq=False)
class ConstantTexture:          # ConstantTexture (kernel/texture.h:30-37)
    value: Sequence[float]


@dataclass(eq=False)
class ImageTexture:             # ImageTexture (kernel/texture.h:39-57)
    image: np.ndarray           # float32 [h, w, 4] RGBA, /255 without sRGB decode (core/image.cpp:105-119)


Texture = Union[ConstantTexture, ImageTexture]


@dataclass(eq=False)
class DiffuseMaterial:          # material.h:205-216
    color: Texture


@dataclass(eq=False)
class GlossyMaterial:           # material.h:217-231
    color: Texture
    roughness: Texture


@dataclass(eq=False)
class EmissiveMaterial:         # material.h:232-240
    color: Texture
    double_sided: bool = False


@dataclass(eq=False)
class MixMaterial:              # material.h:241-248 (first = material_A, second = material_B)
    fraction: Texture
    first: "MaterialT"
    second: "MaterialT"


MaterialT = Union[DiffuseMaterial, GlossyMaterial, EmissiveMaterial, MixMaterial]


@dataclass(eq=False)
class Mesh:                      # Mesh / AkariMesh (common/mesh.h, core/nodes/mesh.cpp)
    vertices: np.ndarray         # float32 [nv, 3]
    indices: np.ndarray          # int32 [nt, 3]
    normals: np.ndarray          # float32 [nt, 9] per face-vertex
    texcoords: np.ndarray        # float32 [nt, 6]
    material_indices: np.ndarray  # int32 [nt], -1 = none
    materials: List[Optional[MaterialT]] = field(default_factory=list)

    @property
    def n_tris(self) -> int:
        return int(self.material_indices.shape[0])


@dataclass
class PerspectiveCamera:        # core/nodes/camera.cpp:26-52 (fov default radians(80))
    position: Sequence[float] = (0.0, 0.0, 0.0)
    rotation: Sequence[float] = (0.0, 0.0, 0.0)   # degrees
    fov: float = 80.0                               # degrees
    resolution: Sequence[int] = (512, 512)


@dataclass
class PathIntegrator:           # core/nodes/integrator.cpp:50-84
    spp: int = 16
    max_depth: int = 5
    tile_size: int = 256
    ray_clamp: float = 10.0
    wavefront: bool = True


@dataclass
class AOIntegrator:             # core/nodes/integrator.cpp:26-49
    spp: int = 16
    occlude: float = math.inf


@dataclass
class Scene:                    # SceneNode (core/nodes/scene.h)
    camera: PerspectiveCamera
    shapes: List[Mesh]
    integrator: object = field(default_factory=PathIntegrator)
    output: str = "out.png"


# ----------------------------------------------------------------------------- .mesh I/O
def load_mesh(path) -> Mesh:
    """BinaryGeometry::load (core/mesh.cpp:48-85)."""
    data = Path(path).read_bytes()
    m = len(MESH_MAGIC)
    if data[:m] != MESH_MAGIC:
        raise ValueError(f"{path}: invalid format, expected {MESH_MAGIC!r}")
    nv, nt = struct.unpack_from("<QQ", data, m)
    off = m + 16

    def take(dtype, count):
        nonlocal off
        a = np.frombuffer(data, dtype, count, off).copy()
        off += a.nbytes
        return a

    v = take(np.float32, 3 * nv).reshape(nv, 3)
    n = take(np.float32, 9 * nt).reshape(nt, 9)
    t = take(np.float32, 6 * nt).reshape(nt, 6)
    i = take(np.int32, 3 * nt).reshape(nt, 3)
    mi = take(np.int32, nt)
    if data[off:off + m] != MESH_MAGIC:
        raise ValueError(f"{path}: invalid format (trailing magic)")
    return Mesh(v, i, n, t, mi)


def save_mesh(path, mesh: Mesh):
    """BinaryGeometry::save (core/mesh.cpp:28-47)."""
    with open(path, "wb") as f:
        f.write(MESH_MAGIC)
        f.write(struct.pack("<QQ", mesh.vertices.shape[0], mesh.n_tris))
        for a, dt in ((mesh.vertices, np.float32), (mesh.normals, np.float32), (mesh.texcoords, np.float32),
                      (mesh.indices, np.int32), (mesh.material_indices, np.int32)):
            f.write(np.ascontiguousarray(a, dt).tobytes())
        f.write(MESH_MAGIC)


# ----------------------------------------------------------------------------- compile
def _f32_dot(a, b):
    s = F32(a[0]) * F32(b[0])
    s = F32(s + F32(a[1]) * F32(b[1]))
    s = F32(s + F32(a[2]) * F32(b[2]))
    return F32(s)


def _f32_cross(a, b):
    a = [F32(x) for x in a]
    b = [F32(x) for x in b]
    return (F32(a[1] * b[2] - a[2] * b[1]), F32(a[2] * b[0] - a[0] * b[2]), F32(a[0] * b[1] - a[1] * b[0]))


def _f32_sub(a, b):
    return tuple(F32(F32(x) - F32(y)) for x, y in zip(a, b))


def _f32_length(a):
    return F32(np.sqrt(_f32_dot(a, a)))


LUMA = (F32(0.2126), F32(0.7152), F32(0.0722))   # color.h:52-55 (Color3f from double literals)


def luminance(rgb) -> np.float32:
    return _f32_dot(rgb, LUMA)


def texture_integral(tex: Texture) -> np.float32:
    """Texture::integral (texture.h:36, 49-55): sequential f32 sum of texel luminance / count."""
    if isinstance(tex, ConstantTexture):
        return luminance([F32(x) for x in tex.value])
    im = np.ascontiguousarray(tex.image, np.float32)
    rgb = im[..., :3].reshape(-1, 3)
    lum = (rgb[:, 0] * LUMA[0] + rgb[:, 1] * LUMA[1]).astype(np.float32) + (rgb[:, 2] * LUMA[2]).astype(np.float32)
    total = np.cumsum(lum.astype(np.float32), dtype=np.float32)[-1]
    return F32(total / F32(rgb.shape[0]))


@dataclass
class CompiledScene:
    """Flat render scene (Scene<C>, kernel/scene.h:50-91): meshes concatenated."""
    vertices: np.ndarray            # float32 [nv, 3]
    indices: np.ndarray             # int32 [nt, 3] global vertex ids
    normals: np.ndarray
    texcoords: np.ndarray
    matid: np.ndarray               # int32 [nt] global material id or -1
    mesh_base: np.ndarray           # uint32 [n_meshes + 1]
    mesh_slots: List[np.ndarray]    # per mesh: local material index -> global material id
    materials: List[capi.Material]
    textures: List[capi.Texture]
    images: List[np.ndarray]
    lights: List[tuple]             # (geom_id, prim_id) of emissive triangles
    light_gid: np.ndarray           # uint32
    power: np.ndarray               # float32
    camera: PerspectiveCamera
    meshes: List[Mesh]

    @property
    def n_tris(self) -> int:
        return int(self.matid.shape[0])


def compile_scene(scene: Scene) -> CompiledScene:
    tex_ids, mat_ids = {}, {}
    textures: List[capi.Texture] = []
    images: List[np.ndarray] = []
    materials: List[capi.Material] = []

    def tex_index(t: Texture) -> int:
        if id(t) in tex_ids:
            return tex_ids[id(t)]
        if isinstance(t, ConstantTexture):
            v = [float(F32(x)) for x in t.value]
            ct = capi.Texture(capi.TEX_CONSTANT, (capi.C.c_float * 3)(*v), -1)
        elif isinstance(t, ImageTexture):
            images.append(np.ascontiguousarray(t.image, np.float32))
            ct = capi.Texture(capi.TEX_IMAGE, (capi.C.c_float * 3)(0, 0, 0), len(images) - 1)
        else:
            raise TypeError(f"unsupported texture {type(t).__name__}")
        textures.append(ct)
        tex_ids[id(t)] = len(textures) - 1
        return tex_ids[id(t)]

    def mat_index(m: MaterialT) -> int:
        if id(m) in mat_ids:
            return mat_ids[id(m)]
        idx = len(materials)
        mat_ids[id(m)] = idx
        materials.append(capi.Material())
        cm = capi.Material(-1, -1, -1, -1, -1, -1, 0)
        if isinstance(m, DiffuseMaterial):
            cm.type, cm.color = capi.MAT_DIFFUSE, tex_index(m.color)
        elif isinstance(m, GlossyMaterial):
            cm.type, cm.color, cm.roughness = capi.MAT_GLOSSY, tex_index(m.color), tex_index(m.roughness)
        elif isinstance(m, EmissiveMaterial):
            cm.type, cm.color, cm.double_sided = capi.MAT_EMISSIVE, tex_index(m.color), int(bool(m.double_sided))
        elif isinstance(m, MixMaterial):
            cm.type, cm.fraction = capi.MAT_MIX, tex_index(m.fraction)
            cm.first = mat_index(m.first)
            cm.second = mat_index(m.second)
        else:
            raise TypeError(f"unsupported material {type(m).__name__}")
        materials[idx] = cm
        return idx

    verts, idxs, norms, tcs, mids, slots_all = [], [], [], [], [], []
    mesh_base = [0]
    vb = 0
    lights, light_gid, power = [], [], []
    for geom_id, mesh in enumerate(scene.shapes):
        slots = np.array([mat_index(m) if m is not None else -1 for m in mesh.materials], np.int32)
        mi = np.asarray(mesh.material_indices, np.int32)
        if mi.size and mi.max(initial=-1) >= len(slots):
            raise ValueError(f"mesh {geom_id}: material index beyond its material list")
        if slots.size:
            g = np.where(mi >= 0, slots[np.clip(mi, 0, None)], -1).astype(np.int32)
        else:
            g = np.full(mi.shape, -1, np.int32)
        verts.append(np.asarray(mesh.vertices, np.float32).reshape(-1, 3))
        idxs.append(np.asarray(mesh.indices, np.int32).reshape(-1, 3) + vb)
        norms.append(np.asarray(mesh.normals, np.float32).reshape(-1, 9))
        tcs.append(np.asarray(mesh.texcoords, np.float32).reshape(-1, 6))
        mids.append(g)
        slots_all.append(slots)
        # light list: every triangle whose material is Emissive (core/nodes/scene.cpp:51-67)
        for prim in np.nonzero(mi >= 0)[0]:
            m = mesh.materials[mi[prim]]
            if isinstance(m, EmissiveMaterial):
                lights.append((geom_id, int(prim)))
                light_gid.append(mesh_base[-1] + int(prim))
                power.append(_light_power(mesh, int(prim), m))
        vb += verts[-1].shape[0]
        mesh_base.append(mesh_base[-1] + mesh.n_tris)

    cat = lambda xs, shape, dt: np.concatenate(xs) if xs else np.zeros(shape, dt)
    return CompiledScene(
        vertices=cat(verts, (0, 3), np.float32), indices=cat(idxs, (0, 3), np.int32),
        normals=cat(norms, (0, 9), np.float32), texcoords=cat(tcs, (0, 6), np.float32),
        matid=cat(mids, (0,), np.int32), mesh_base=np.array(mesh_base, np.uint32), mesh_slots=slots_all,
        materials=materials, textures=textures, images=images, lights=lights,
        light_gid=np.array(light_gid, np.uint32), power=np.array(power, np.float32),
        camera=scene.camera, meshes=list(scene.shapes))


def _light_power(mesh: Mesh, prim: int, m: EmissiveMaterial) -> np.float32:
    """power = area * tc_area * I (core/nodes/scene.cpp:72-87), with its f32/f64 mix."""
    I = texture_integral(m.color)
    v = [mesh.vertices[mesh.indices[prim, k]] for k in range(3)]
    tc = [(F32(mesh.texcoords[prim, 2 * k]), F32(mesh.texcoords[prim, 2 * k + 1]), F32(0.0)) for k in range(3)]
    tc_area = float(_f32_length(_f32_cross(_f32_sub(tc[1], tc[0]), _f32_sub(tc[2], tc[0])))) * 0.5
    area = _f32_length(_f32_cross(_f32_sub(v[1], v[0]), _f32_sub(v[2], v[0])))
    return F32(float(area) * tc_area * float(I))


def upload_scene(ctx: "capi.HipContext", cs: CompiledScene, build: bool = True, bvh=None, **build_kw):
    """Upload a compiled scene through the C-ABI (the HipAccelerator adapter's commit).  With
    `bvh` = (nodes, tris) from another context's accel_export, that tree is adopted instead of
    building one (n_threads from build_kw is kept for the wide view)."""
    ctx.upload_images(cs.images)
    ctx.upload_textures(cs.textures)
    ctx.upload_materials(cs.materials)
    for geom_id, mesh in enumerate(cs.meshes):
        g = ctx.upload_mesh(mesh.vertices, mesh.indices, mesh.normals, mesh.texcoords, mesh.material_indices,
                            cs.mesh_slots[geom_id])
        assert g == geom_id
    ctx.upload_lights(cs.lights, cs.power)
    cam = cs.camera
    ctx.set_camera(cam.position, cam.rotation, cam.fov, cam.resolution)
    if bvh is not None:
        return ctx.import_accel(bvh[0], bvh[1], n_threads=build_kw.get("n_threads", 0))
    if build:
        return ctx.build_accel(**build_kw)
    return None


# ----------------------------------------------------------------------------- .akari loader
class SdlError(ValueError):
    pass


class _Module:
    def __init__(self, name):
        self.name = name
        self.exports, self.locals, self.submodules = {}, {}, {}


class _Obj:
    def __init__(self, type_, fields):
        self.type, self.fields = type_, fields


class SdlParser:
    """The reference's scene language (core/parser.cpp:150-363): import/let/export, objects,
    arrays, strings, numbers (parsed as n + frac / 10^k), true/false, $mod.var references."""

    def __init__(self):
        self.cache = {}

    def parse_file(self, path, name="main") -> _Module:
        path = Path(path).resolve()
        return self.parse_string(path.read_text(), path, name)

    def parse_string(self, src: str, path: Path, name="main") -> _Module:
        self.src, self.pos, self.path = src, 0, Path(path)
        mod = _Module(name)
        mod.dir = self.path.parent
        self.mod = mod
        while True:
            self._skip()
            if self.pos >= len(self.src):
                break
            if self._starts("import"):
                self._import()
            elif self._starts("let"):
                self.pos += 3
                var, val = self._binding()
                if var in mod.locals:
                    self._err(f"{var} is already defined")
                mod.locals[var] = val
            elif self._starts("export"):
                self.pos += 6
                var, val = self._binding()
                if var in mod.exports:
                    self._err(f"{var} is already defined")
                mod.exports[var] = val
            else:
                self._err(f"stray token {self.src[self.pos]!r}")
        return mod

    def _err(self, msg):
        line = self.src.count("\n", 0, self.pos) + 1
        raise SdlError(f"{self.path}:{line}: {msg}")

    def _starts(self, w):
        return self.src.startswith(w, self.pos)

    def _peek(self):
        return self.src[self.pos] if self.pos < len(self.src) else ""

    def _skip(self):
        while self.pos < len(self.src):
            c = self.src[self.pos]
            if c.isspace():
                self.pos += 1
            elif self.src.startswith("//", self.pos):
                e = self.src.find("\n", self.pos)
                self.pos = len(self.src) if e < 0 else e + 1
            else:
                break

    def _expect(self, s):
        if not self._starts(s):
            self._err(f"{s!r} expected")
        self.pos += len(s)

    def _ident(self):
        self._skip()
        b = self.pos
        while self.pos < len(self.src) and (self.src[self.pos].isalnum() or self.src[self.pos] == "_"):
            self.pos += 1
        if b == self.pos:
            self._err("identifier expected")
        return self.src[b:self.pos]

    def _binding(self):
        var = self._ident()
        self._skip()
        self._expect("=")
        self._skip()
        return var, self._value()

    def _import(self):
        self.pos += 6
        self._skip()
        fname = self._string()
        self._skip()
        self._expect("as")
        alias = self._ident()
        if alias in self.mod.submodules:
            self._err(f"{alias} is already defined")
        full = (self.mod.dir / fname).resolve()
        if not full.exists():
            self._err(f'module "{fname}" not found')
        saved = (self.src, self.pos, self.path, self.mod)
        sub = SdlParser().parse_file(full, alias)
        self.src, self.pos, self.path, self.mod = saved
        self.mod.submodules[alias] = sub

    def _string(self):
        self._expect('"')
        out = []
        while self._peek() and self._peek() != '"':
            c = self.src[self.pos]
            self.pos += 1
            if c == "\\":
                e = self.src[self.pos]
                self.pos += 1
                out.append({"\\": "\\", "n": "\n", '"': '"'}.get(e) or self._err("illegal escape sequence"))
            else:
                out.append(c)
        self._expect('"')
        return "".join(out)

    def _number(self):
        if self._peek() == "-":
            self.pos += 1
            return -self._number()
        if not self._peek().isdigit():
            self._err("digit expected")
        n = 0
        while self._peek().isdigit():
            n = n * 10 + int(self.src[self.pos])
            self.pos += 1
        frac, p = 0, 1.0
        if self._peek() == ".":
            self.pos += 1
            while self._peek().isdigit():
                frac = frac * 10 + int(self.src[self.pos])
                p *= 10
                self.pos += 1
        return n + frac / p                      # parser.cpp:338-363

    def _value(self):
        self._skip()
        c = self._peek()
        if c == "$":
            self.pos += 1
            path = [self._ident()]
            while self._peek() == ".":
                self.pos += 1
                path.append(self._ident())
            mod = self.mod
            for p in path[:-1]:
                if p not in mod.submodules:
                    self._err(f"module {mod.name} has no submodule named {p}")
                mod = mod.submodules[p]
            if len(path) == 1 and path[0] in self.mod.locals:
                return self.mod.locals[path[0]]
            if path[-1] not in mod.exports:
                self._err(f"module {mod.name} has no exported variable named {path[-1]}")
            return mod.exports[path[-1]]
        if c == "[":
            self.pos += 1
            arr = []
            self._skip()
            while self._peek() and self._peek() != "]":
                arr.append(self._value())
                self._skip()
                if self._peek() != "]":
                    self._expect(",")
                self._skip()
            self._expect("]")
            return arr
        if c == '"':
            return self._string()
        if c == "-" or c.isdigit():
            return self._number()
        if c.isalpha() or c == "_":
            if self._starts("true"):
                self.pos += 4
                return True
            if self._starts("false"):
                self.pos += 5
                return False
            t = self._ident()
            self._skip()
            self._expect("{")
            fields = {}
            self._skip()
            while self._peek() and self._peek() != "}":
                k = self._ident()
                if k in fields:
                    self._err(f"field {k} redefined")
                self._skip()
                self._expect(":")
                fields[k] = self._value()
                self._skip()
                if self._peek() != "}":
                    self._expect(",")
                self._skip()
            self._expect("}")
            return self._build(t, fields)
        self._err(f"stray token {c!r}")

    # object construction (core/nodes/*: object_field semantics)
    def _texture(self, v) -> Texture:
        if isinstance(v, list):
            if len(v) != 3:
                self._err("colour array must have 3 elements")
            return ConstantTexture([float(F32(x)) for x in v])
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            return ConstantTexture([float(F32(v))] * 3)
        if isinstance(v, str):
            return ImageTexture(load_image((self.path.parent / v)))
        if isinstance(v, (ConstantTexture, ImageTexture)):
            return v
        self._err("texture expected")

    def _build(self, t, f):
        if t == "PerspectiveCamera":
            cam = PerspectiveCamera()
            if "fov" in f:
                cam.fov = float(f["fov"])
            if "rotation" in f:
                cam.rotation = tuple(float(F32(x)) for x in f["rotation"])
            if "position" in f:
                cam.position = tuple(float(F32(x)) for x in f["position"])
            if "resolution" in f:
                cam.resolution = tuple(int(x) for x in f["resolution"])
            return cam
        if t == "DiffuseMaterial":
            return DiffuseMaterial(self._texture(f.get("color", 0.0)))
        if t == "GlossyMaterial":
            return GlossyMaterial(self._texture(f.get("color", 0.0)), self._texture(f.get("roughness", 0.0)))
        if t == "EmissiveMaterial":
            # the node never reads double_sided (core/nodes/material.cpp:145-160): always one-sided
            return EmissiveMaterial(self._texture(f.get("color", 0.0)), False)
        if t == "MixMaterial":
            return MixMaterial(self._texture(f.get("fraction", 0.5)), f["first"], f["second"])
        if t == "AkariMesh":
            mesh = load_mesh(self.path.parent / f["path"])
            mesh.materials = list(f.get("materials", []))
            return mesh
        if t == "Path":
            it = PathIntegrator()
            for k in ("spp", "max_depth", "tile_size"):
                if k in f:
                    setattr(it, k, int(f[k]))
            if "ray_clamp" in f:
                it.ray_clamp = float(F32(f["ray_clamp"]))
            if "wavefront" in f:
                it.wavefront = bool(f["wavefront"])
            if "megakernel" in f:
                it.wavefront = not bool(f["megakernel"])
            return it
        if t == "AO":
            return AOIntegrator(int(f.get("spp", 16)), float(f.get("occlude", math.inf)))
        if t == "Scene":
            return Scene(camera=f["camera"], shapes=list(f.get("shapes", [])),
                         integrator=f.get("integrator", PathIntegrator()), output=f.get("output", "out.png"))
        return _Obj(t, f)


def load_scene_file(path, export="scene") -> Scene:
    mod = SdlParser().parse_file(path)
    if export not in mod.exports:
        raise SdlError(f"{path}: no exported '{export}'")
    return mod.exports[export]


def load_image(path) -> np.ndarray:
    """Float RGBA image for ImageTexture: .npy (float [h,w,3|4]) or binary PPM/PFM."""
    path = Path(path)
    if path.suffix == ".npy":
        a = np.load(path)
    elif path.suffix.lower() in (".ppm",):
        raw = path.read_bytes()
        parts = raw.split(maxsplit=4)
        w, h, mx = int(parts[1]), int(parts[2]), int(parts[3])
        a = np.frombuffer(parts[4][:w * h * 3], np.uint8).reshape(h, w, 3).astype(np.float32) / F32(mx)
    else:
        raise SdlError(f"unsupported image format {path.suffix} (no image codec in this build)")
    a = np.asarray(a, np.float32)
    if a.shape[-1] == 3:
        a = np.concatenate([a, np.ones(a.shape[:2] + (1,), np.float32)], axis=-1)
    return np.ascontiguousarray(a)


# ----------------------------------------------------------------------------- built-in scenes
def cornell_scene(mesh_path, resolution=(512, 512), spp=16, max_depth=5) -> Scene:
    """The reference's Cornell box (resources/data/cornell_box/{scene,cornell_box}.akari): camera,
    material values and slot order restated; the geometry is the reference's own .mesh fixture."""
    mesh = load_mesh(mesh_path)
    grey = [0.725, 0.71, 0.68]
    d = lambda c: DiffuseMaterial(ConstantTexture([float(F32(x)) for x in c]))
    mesh.materials = [d([0.63, 0.065, 0.05]), d([0.14, 0.45, 0.091]), d(grey), d(grey), d(grey), d(grey), d(grey),
                      EmissiveMaterial(ConstantTexture([17.0, 12.0, 4.0]))]
    cam = PerspectiveCamera(position=(0.0, 1.0, 9.0), rotation=(0.0, 0.0, 0.0), fov=15.0, resolution=tuple(resolution))
    return Scene(camera=cam, shapes=[mesh], integrator=PathIntegrator(spp=spp, max_depth=max_depth, tile_size=1024))


def _grid(o, u, v, nu, nv, normal, uv_scale, mat):
    """A planar grid of nu x nv quads spanning o + [0,1] u + [0,1] v: (vertices [6q, 3], normals
    [2q, 9], texcoords [2q, 6], material ids [2q]); texcoords run over [0, uv_scale]."""
    o, u, v = (np.asarray(a, np.float64) for a in (o, u, v))
    a, b = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    a, b = a.reshape(-1, 1), b.reshape(-1, 1)
    p = lambda i, j: o + (i / nu) * u + (j / nv) * v
    c00, c10, c11, c01 = p(a, b), p(a + 1, b), p(a + 1, b + 1), p(a, b + 1)
    verts = np.stack([c00, c10, c11, c00, c11, c01], axis=1).reshape(-1, 3).astype(np.float32)
    t = lambda i, j: np.concatenate([i / nu * uv_scale[0], j / nv * uv_scale[1]], axis=1)
    tc = np.stack([t(a, b), t(a + 1, b), t(a + 1, b + 1), t(a, b), t(a + 1, b + 1), t(a, b + 1)], axis=1)
    q = nu * nv
    return (verts, np.tile(np.asarray(normal, np.float32), (2 * q, 3)), tc.reshape(-1, 6).astype(np.float32),
            np.full(2 * q, mat, np.int32))


def _pattern(h, w, seed, base, contrast):
    """A procedural RGBA texture: coloured checker tiles with per-tile noise, float32 [h, w, 4]."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    check = ((x // (w // 8) + y // (h // 8)) % 2).astype(np.float32)
    noise = rng.random((h, w)).astype(np.float32)
    img = np.empty((h, w, 4), np.float32)
    for c in range(3):
        img[..., c] = np.clip(base[c] * (1 - contrast + contrast * check) * (0.85 + 0.15 * noise), 0, 1)
    img[..., 3] = 1.0
    return img


def hall_scene(resolution=(3840, 2160), detail=1.0, spp=256, max_depth=5) -> Scene:
    """Config C4 stand-in (a Sponza-class textured scene; the reference ships none):
    a hall 20 x 8 x 8 with tessellated floor, ceiling and walls, two rows of columns, image-textured
    Diffuse, Glossy (image roughness) and Mix (image fraction) materials, and six emissive ceiling
    panels (area lights only: the reference has no HDRI light).  detail = 1 gives ~270K triangles."""
    n = lambda k: max(1, int(round(k * detail)))
    tex_floor = ImageTexture(_pattern(256, 256, 1, (0.8, 0.7, 0.55), 0.5))
    tex_rough = ImageTexture(_pattern(64, 64, 2, (0.6, 0.6, 0.6), 0.8))
    tex_wall = ImageTexture(_pattern(256, 256, 3, (0.75, 0.6, 0.5), 0.3))
    tex_frac = ImageTexture(_pattern(32, 32, 4, (0.7, 0.7, 0.7), 0.9))
    ct = ConstantTexture
    diffuse_floor = DiffuseMaterial(tex_floor)
    mats = [MixMaterial(tex_frac, diffuse_floor, GlossyMaterial(tex_floor, tex_rough)),   # 0 floor
            DiffuseMaterial(tex_wall),                                                     # 1 walls
            DiffuseMaterial(ct([0.7, 0.7, 0.68])),                                         # 2 ceiling
            GlossyMaterial(ct([0.8, 0.75, 0.7]), ct([0.35, 0.35, 0.35])),                  # 3 columns
            EmissiveMaterial(ct([12.0, 11.0, 9.0]))]                                       # 4 lights
    parts = [
        _grid((-10, 0, -4), (20, 0, 0), (0, 0, 8), n(256), n(128), (0, 1, 0), (10, 4), 0),     # floor
        _grid((-10, 8, -4), (0, 0, 8), (20, 0, 0), n(128), n(256), (0, -1, 0), (4, 10), 2),    # ceiling
        _grid((-10, 0, -4), (0, 8, 0), (20, 0, 0), n(64), n(256), (0, 0, 1), (3, 8), 1),       # wall z = -4
        _grid((-10, 0, 4), (20, 0, 0), (0, 8, 0), n(256), n(64), (0, 0, -1), (8, 3), 1),       # wall z = +4
        _grid((-10, 0, -4), (0, 0, 8), (0, 8, 0), n(128), n(128), (1, 0, 0), (3, 3), 1),      # wall x = -10
        _grid((10, 0, -4), (0, 8, 0), (0, 0, 8), n(128), n(128), (-1, 0, 0), (3, 3), 1),      # wall x = +10
    ]
    for zc in (-2.5, 2.5):
        for xc in np.arange(-8.0, 8.01, 2.0):
            w = 0.3
            x0, x1, z0, z1 = xc - w, xc + w, zc - w, zc + w
            parts += [_grid((x0, 0, z1), (x1 - x0, 0, 0), (0, 8, 0), n(4), n(48), (0, 0, 1), (1, 4), 3),
                      _grid((x1, 0, z0), (x0 - x1, 0, 0), (0, 8, 0), n(4), n(48), (0, 0, -1), (1, 4), 3),
                      _grid((x1, 0, z1), (0, 0, z0 - z1), (0, 8, 0), n(4), n(48), (1, 0, 0), (1, 4), 3),
                      _grid((x0, 0, z0), (0, 0, z1 - z0), (0, 8, 0), n(4), n(48), (-1, 0, 0), (1, 4), 3)]
    for xc in (-7.0, 0.0, 7.0):
        for zc in (-1.5, 1.5):
            # winding u x v = -y: the panel's geometric normal faces down (one-sided AreaLight)
            parts.append(_grid((xc - 1, 7.99, zc - 0.5), (2, 0, 0), (0, 0, 1), 1, 1, (0, -1, 0), (1, 1), 4))
    verts = np.concatenate([p[0] for p in parts])
    normals = np.concatenate([p[1] for p in parts])
    tcs = np.concatenate([p[2] for p in parts])
    mi = np.concatenate([p[3] for p in parts])
    idx = np.arange(verts.shape[0], dtype=np.int32).reshape(-1, 3)
    mesh = Mesh(verts, idx, normals, tcs, mi, mats)
    cam = PerspectiveCamera(position=(-9.0, 3.0, 0.0), rotation=(-90.0, -8.0, 0.0), fov=60.0,
                            resolution=tuple(resolution))
    return Scene(camera=cam, shapes=[mesh], integrator=PathIntegrator(spp=spp, max_depth=max_depth))


def soup_scene(n_tris=10_000_000, resolution=(1920, 1080), seed=42, r=0.01, spp=1024, max_depth=5) -> Scene:
    """Config C3: n_tris random triangles + a 2-triangle emissive quad."""
    v, n, t = capi.generate_soup(n_tris, seed, r)
    quad_v = np.array([[-1, 1.5, -1], [1, 1.5, -1], [1, 1.5, 1], [-1, 1.5, -1], [1, 1.5, 1], [-1, 1.5, 1]], np.float32)
    quad_n = np.tile(np.array([0, -1, 0], np.float32), (2, 3))
    quad_t = np.tile(np.array([0, 1, 1, 0, 1, 1], np.float32), (2, 1))
    verts = np.concatenate([v, quad_v])
    idx = np.arange(verts.shape[0], dtype=np.int32).reshape(-1, 3)
    mi = np.zeros(n_tris + 2, np.int32)
    mi[-2:] = 1
    mesh = Mesh(verts, idx, np.concatenate([n, quad_n]), np.concatenate([t, quad_t]), mi,
                [DiffuseMaterial(ConstantTexture([0.5, 0.5, 0.5])),
                 EmissiveMaterial(ConstantTexture([10.0, 10.0, 10.0]))])
    cam = PerspectiveCamera(position=(0.0, 0.0, 4.0), rotation=(0.0, 0.0, 0.0), fov=40.0, resolution=tuple(resolution))
    return Scene(camera=cam, shapes=[mesh], integrator=PathIntegrator(spp=spp, max_depth=max_depth))
