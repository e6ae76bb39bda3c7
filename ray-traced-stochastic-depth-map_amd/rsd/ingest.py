"""Scene ingest: mesh files -> the world-space triangle soup librsd uploads.

Reference: SceneBuilder (Scene/SceneBuilder.cpp) flattens static meshes into world space
(:1585-1640, vertices transformed by the node's object->world matrix), flips a mesh's winding
flag when that matrix mirrors (:1601-1603, negative determinant) and then unifies every mesh
to counter-clockwise front faces by swapping the first two indices of each triangle
(unifyTriangleWinding :1703-1725, flipTriangleWinding :1655-1673).  Per-instance flags then
come from the material: double-sided -> TriangleFacingCullDisable (Scene.cpp:3436-3452),
AlphaMode::Mask -> alpha tested (MaterialFactory.slang:124-151).  The importers live in
Source/plugins/importers/* (Assimp for OBJ/FBX/glTF, the Python importer for .pyscene).

Here: `SceneBuilder` with the same flattening rules (add_material / add_mesh /
add_instance / set_camera), `load_obj` (OBJ + MTL: polygons fan-triangulated, negative
indices, `d`/`Tr` constant alpha, `map_d` / the alpha channel of `map_Kd` as the alpha
texture) and `read_image` (PNG via zlib, binary/ASCII PGM/PPM/PAM, .npy) for alpha textures.
A material with an alpha texture or a constant alpha below 1 is AlphaMode::Mask (Falcor's
importers mark such materials Mask; the threshold defaults to 0.5, MaterialData.slang:99).
Binary FBX 7.x: rsd.fbx.load_fbx (the same SceneBuilder).  glTF, USD and PBRT are out of scope."""
from __future__ import annotations

import dataclasses
import struct
import zlib
from pathlib import Path

import numpy as np

from .scenes import FLAG_ALPHA_MASK, FLAG_DOUBLE_SIDED, NO_TEXTURE, AlphaMaterials, Scene


@dataclasses.dataclass
class Material:
    """The subset of StandardMaterial the hot path reads (MaterialHeader flags + base-colour alpha)."""
    name: str = "default"
    double_sided: bool = False
    alpha_mode_mask: bool = False       # AlphaMode::Mask
    alpha_threshold: float = 0.5
    alpha: float = 1.0                  # base colour alpha when there is no texture
    alpha_texture: np.ndarray | None = None  # uint8 [h, w]


@dataclasses.dataclass
class Mesh:
    positions: np.ndarray               # float32 [nv, 3], object space
    indices: np.ndarray                 # uint32 [nt, 3]
    texcoords: np.ndarray | None = None  # float32 [nv, 2]
    material: int = 0
    front_face_cw: bool = False         # TriangleMesh::getFrontFaceCW


class SceneBuilder:
    """Flattens meshes x instances into one world-space soup (SceneBuilder.cpp:1585-1725)."""

    def __init__(self):
        self.materials: list[Material] = []
        self.meshes: list[Mesh] = []
        self.instances: list[tuple[int, np.ndarray]] = []
        self.camera = {"pos": [0.0, 0.0, 5.0], "target": [0.0, 0.0, 0.0], "up": [0.0, 1.0, 0.0]}

    def add_material(self, m: Material) -> int:
        self.materials.append(m)
        return len(self.materials) - 1

    def add_mesh(self, mesh: Mesh) -> int:
        mesh.positions = np.asarray(mesh.positions, np.float32).reshape(-1, 3)
        mesh.indices = np.asarray(mesh.indices, np.uint32).reshape(-1, 3)
        if mesh.indices.size and int(mesh.indices.max()) >= len(mesh.positions):
            raise ValueError("mesh index out of range")
        if mesh.texcoords is not None:
            mesh.texcoords = np.asarray(mesh.texcoords, np.float32).reshape(-1, 2)
            if len(mesh.texcoords) != len(mesh.positions):
                raise ValueError("texcoords must be indexed like the positions")
        self.meshes.append(mesh)
        return len(self.meshes) - 1

    def add_instance(self, mesh_id: int, transform=None):
        t = np.eye(4, dtype=np.float32) if transform is None else np.asarray(transform, np.float32).reshape(4, 4)
        self.instances.append((mesh_id, t))

    def set_camera(self, pos, target, up=(0.0, 1.0, 0.0)):
        self.camera = {"pos": list(map(float, pos)), "target": list(map(float, target)), "up": list(map(float, up))}

    def build(self, name: str = "scene") -> Scene:
        if not self.materials:
            self.add_material(Material())
        pos, ind, flg, uv, mat = [], [], [], [], []
        nv = 0
        for mesh_id, T in self.instances:
            m = self.meshes[mesh_id]
            mt = self.materials[m.material]
            # object -> world in float32 (transformPoint)
            p = (m.positions @ T[:3, :3].T + T[:3, 3]).astype(np.float32)
            tri = m.indices.astype(np.int64)
            cw = m.front_face_cw != bool(np.linalg.det(T[:3, :3].astype(np.float64)) < 0.0)
            if cw:  # unifyTriangleWinding: counter-clockwise front faces everywhere
                tri = tri[:, [1, 0, 2]]
            pos.append(p)
            ind.append((tri + nv).astype(np.uint32))
            f = (FLAG_DOUBLE_SIDED if mt.double_sided else 0) | (FLAG_ALPHA_MASK if mt.alpha_mode_mask else 0)
            flg.append(np.full(len(tri), f, np.uint32))
            uv.append(m.texcoords if m.texcoords is not None else np.zeros((len(p), 2), np.float32))
            mat.append(np.full(len(tri), m.material, np.uint32))
            nv += len(p)
        if not pos:
            return Scene(name, np.zeros((0, 3), np.float32), np.zeros((0, 3), np.uint32), np.zeros(0, np.uint32),
                         self.camera)
        positions, indices, flags = np.concatenate(pos), np.concatenate(ind), np.concatenate(flg)
        alpha = None
        if any(m.alpha_mode_mask for m in self.materials):
            textures, tex_of = [], []
            for m in self.materials:
                if m.alpha_texture is not None:
                    textures.append(np.ascontiguousarray(m.alpha_texture, np.uint8))
                    tex_of.append(len(textures) - 1)
                else:
                    tex_of.append(NO_TEXTURE)
            alpha = AlphaMaterials(np.concatenate(uv).astype(np.float32), np.concatenate(mat),
                                   np.array([m.alpha_threshold for m in self.materials], np.float32),
                                   np.array([m.alpha for m in self.materials], np.float32),
                                   np.array(tex_of, np.uint32), textures)
        return Scene(name, positions, indices, flags, self.camera, alpha)


# ---------------------------------------------------------------------------------- images

def _png_decode(data: bytes) -> np.ndarray:
    """8-bit PNG (grey, grey+alpha, RGB, RGBA, palette (+tRNS)), non-interlaced -> uint8 [h, w, c]."""
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG file")
    pos, idat, plte, trns = 8, [], None, None
    w = h = depth = ctype = interlace = None
    while pos < len(data):
        n, kind = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if kind == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
        elif kind == b"IDAT":
            idat.append(body)
        elif kind == b"PLTE":
            plte = np.frombuffer(body, np.uint8).reshape(-1, 3)
        elif kind == b"tRNS":
            trns = np.frombuffer(body, np.uint8)
        elif kind == b"IEND":
            break
    if depth != 8 or interlace:
        raise ValueError("only 8-bit non-interlaced PNG is supported")
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), np.uint8).reshape(h, 1 + w * ch)
    out = np.zeros((h, w * ch), np.int32)
    prev = np.zeros(w * ch, np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        cur = np.zeros(w * ch, np.int32)
        if f == 0:
            cur = line
        elif f == 2:
            cur = (line + prev) & 255
        else:  # 1 sub, 3 average, 4 Paeth: sequential in x
            for i in range(w * ch):
                a = cur[i - ch] if i >= ch else 0
                b = prev[i]
                c = prev[i - ch] if i >= ch else 0
                if f == 1:
                    pr = a
                elif f == 3:
                    pr = (a + b) >> 1
                else:
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pr = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
                cur[i] = (line[i] + pr) & 255
        out[y] = cur
        prev = cur
    img = out.astype(np.uint8).reshape(h, w, ch)
    if ctype == 3:
        idx = img[..., 0]
        rgb = plte[idx]
        a = np.full(idx.shape, 255, np.uint8)
        if trns is not None:
            lut = np.full(256, 255, np.uint8)
            lut[:len(trns)] = trns
            a = lut[idx]
        img = np.concatenate([rgb, a[..., None]], -1)
    return img


def _pnm_decode(data: bytes) -> np.ndarray:
    """Netpbm P2/P5 (grey), P3/P6 (RGB), 8-bit."""
    toks, pos = [], 2
    while len(toks) < 3:
        while data[pos:pos + 1].isspace():
            pos += 1
        if data[pos:pos + 1] == b"#":
            while data[pos:pos + 1] not in (b"\n", b""):
                pos += 1
            continue
        start = pos
        while not data[pos:pos + 1].isspace():
            pos += 1
        toks.append(int(data[start:pos]))
    w, h, mx = toks
    if mx > 255:
        raise ValueError("only 8-bit netpbm is supported")
    magic = data[:2]
    ch = 1 if magic in (b"P2", b"P5") else 3
    if magic in (b"P5", b"P6"):
        px = np.frombuffer(data[pos + 1:pos + 1 + w * h * ch], np.uint8)
    else:
        px = np.array(data[pos:].split()[:w * h * ch], np.int64).astype(np.uint8)
    return px.reshape(h, w, ch)


def read_image(path) -> np.ndarray:
    """uint8 [h, w, c] from PNG, PGM/PPM or .npy."""
    path = Path(path)
    if path.suffix.lower() == ".npy":
        a = np.load(path)  # allow_pickle stays False
        return a.astype(np.uint8).reshape(a.shape[0], a.shape[1], -1)
    data = path.read_bytes()
    if data[:4] == b"\x89PNG":
        return _png_decode(data)
    if data[:1] == b"P" and data[1:2] in b"2356":
        return _pnm_decode(data)
    raise ValueError(f"{path}: unsupported image format (PNG, PGM/PPM or .npy)")


def alpha_channel(img: np.ndarray, grey_is_alpha: bool) -> np.ndarray | None:
    """The alpha plane of an image: its 2nd/4th channel, or the grey value of a 1-channel
    `map_d`; None when the image has no alpha (an opaque base colour)."""
    c = img.shape[2]
    if c in (2, 4):
        return np.ascontiguousarray(img[..., c - 1])
    if c == 1 and grey_is_alpha:
        return np.ascontiguousarray(img[..., 0])
    return None


# ---------------------------------------------------------------------------------- OBJ

def _parse_mtl(path: Path, double_sided: set, threshold: float) -> dict:
    mats, cur = {}, None
    for raw in path.read_text(errors="replace").splitlines():
        parts = raw.split("#", 1)[0].split()
        if not parts:
            continue
        key, args = parts[0], parts[1:]
        if key == "newmtl":
            name = " ".join(args)
            cur = mats[name] = Material(name=name, double_sided=name in double_sided, alpha_threshold=threshold)
        elif cur is None:
            continue
        elif key == "d" and args:
            cur.alpha = float(args[-1])
        elif key == "Tr" and args:
            cur.alpha = 1.0 - float(args[-1])
        elif key in ("map_d", "map_Kd") and args:
            tex = path.parent / args[-1].replace("\\", "/")
            if tex.exists():
                a = alpha_channel(read_image(tex), grey_is_alpha=(key == "map_d"))
                if a is not None and (key == "map_d" or cur.alpha_texture is None):
                    cur.alpha_texture = a
    for m in mats.values():
        # importers mark a material Mask when its opacity can cut holes
        m.alpha_mode_mask = m.alpha_texture is not None and bool((m.alpha_texture < 255).any()) or m.alpha < 1.0
        if not m.alpha_mode_mask:
            m.alpha_texture = None
    return mats


def load_obj(path, transform=None, double_sided=(), alpha_threshold: float = 0.5,
             builder: SceneBuilder | None = None) -> SceneBuilder:
    """Wavefront OBJ (+ MTL) into a SceneBuilder: one mesh per (object/group, material) run,
    vertices de-duplicated per (position, texcoord) pair, polygons fan-triangulated.
    `double_sided`: material names to treat as double-sided (OBJ has no such flag)."""
    path = Path(path)
    B = builder or SceneBuilder()
    V, VT = [], []
    mats: dict[str, Material] = {}
    mat_ids: dict[str, int] = {}
    runs: dict[tuple, list] = {}
    group, cur_mat = "", ""

    def material_id(name):
        if name not in mat_ids:
            m = mats.get(name) or Material(name=name or "default", double_sided=name in set(double_sided),
                                           alpha_threshold=alpha_threshold)
            mat_ids[name] = B.add_material(m)
        return mat_ids[name]

    for raw in path.read_text(errors="replace").splitlines():
        parts = raw.split("#", 1)[0].split()
        if not parts:
            continue
        key, args = parts[0], parts[1:]
        if key == "v":
            V.append([float(x) for x in args[:3]])
        elif key == "vt":
            VT.append([float(args[0]), float(args[1]) if len(args) > 1 else 0.0])
        elif key == "f":
            corners = []
            for a in args:
                s = a.split("/")
                vi = int(s[0])
                vi = vi - 1 if vi > 0 else len(V) + vi
                ti = -1
                if len(s) > 1 and s[1]:
                    ti = int(s[1])
                    ti = ti - 1 if ti > 0 else len(VT) + ti
                corners.append((vi, ti))
            run = runs.setdefault((group, cur_mat), [])
            for k in range(1, len(corners) - 1):
                run.append((corners[0], corners[k], corners[k + 1]))
        elif key in ("o", "g"):
            group = " ".join(args)
        elif key == "usemtl":
            cur_mat = " ".join(args)
        elif key == "mtllib":
            mp = path.parent / " ".join(args)
            if mp.exists():
                mats.update(_parse_mtl(mp, set(double_sided), alpha_threshold))
    Vn = np.asarray(V, np.float32).reshape(-1, 3)
    VTn = np.asarray(VT, np.float32).reshape(-1, 2)
    for (grp, mname), tris in runs.items():
        remap, pos, uv, ind = {}, [], [], []
        for tri in tris:
            row = []
            for c in tri:
                if c not in remap:
                    remap[c] = len(pos)
                    pos.append(Vn[c[0]])
                    # OBJ's v axis points up; textures are stored top row first
                    uv.append([VTn[c[1], 0], 1.0 - VTn[c[1], 1]] if c[1] >= 0 else [0.0, 0.0])
                row.append(remap[c])
            ind.append(row)
        mid = material_id(mname)
        mesh = Mesh(np.asarray(pos, np.float32), np.asarray(ind, np.uint32), np.asarray(uv, np.float32), mid)
        B.add_instance(B.add_mesh(mesh), transform)
    return B
