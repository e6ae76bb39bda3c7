"""Binary FBX 7.x geometry ingest ("a .pyscene/OBJ/FBX loader").

The reference reads FBX through Assimp (`Source/plugins/importers/AssimpImporter/AssimpImporter.cpp:1093-1175`,
`AssimpImporter.h:45`): the Assimp FBX reader, then the post-process preset
`aiProcessPreset_TargetRealtime_MaxQuality | aiProcess_FlipUVs` (AssimpImporter.cpp:1098-1107), then
`createMeshes` / `createSceneGraph` hand world-space triangle meshes to SceneBuilder, which flattens them
(Scene.cpp:2688-2830 builds the BLAS from those).  Assimp is a third-party dependency that is not vendored in
`/root/reference` (`external/CMakeLists.txt:192-206` links the `libassimp.so` of Falcor's packman package
`falcor_dependencies`; its version is pinned by that package, which is not in the container), so this module
restates the published behaviour this path depends on:

* the binary FBX container (Kaydara FBX Binary, versions 7100-7500): a 27-byte header, node records
  {end offset, property count, property bytes (u32 before 7500, u64 from 7500), name} with typed properties
  (Y C I F D L scalars, f d l i b c arrays -- raw or zlib, encoding 1 -- S strings, R raw bytes) and nested
  records closed by a null record;
* the object graph: `Objects` (Geometry "Mesh", Model, Material, Texture) joined by `Connections`
  ("OO" child -> parent object, "OP" child -> parent property), `Properties70` values falling back to the
  `Definitions` property templates of the object's type (how the FBX SDK and Assimp's FBX parser resolve an
  unset property);
* a Model's local transform (the FBX SDK's node-transform definition, which Assimp's
  `FBXConverter::GenerateTransformationNodeChain` follows):
  `T * Roff * Rp * Rpre * R * Rpost^-1 * Rp^-1 * Soff * Sp * S * Sp^-1` (Lcl Translation / Rotation / Scaling,
  RotationOffset / Pivot, PreRotation / PostRotation -- Euler XYZ --, ScalingOffset / Pivot), rotations in
  degrees composed in the node's `RotationOrder` (XYZ: Rz * Ry * Rx, the first letter applied first); the
  geometric transform `GT * GR * GS` applies to the node's own geometry only, not to its children; parents
  through the Model -> Model connections;
* a Geometry's polygons: `Vertices` (doubles, read as float32 like Assimp's aiVector3D), `PolygonVertexIndex`
  with a polygon's last index stored as ~index, `LayerElementUV` (ByPolygonVertex / ByVertice, Direct /
  IndexToDirect; `aiProcess_FlipUVs`: v -> 1 - v) and `LayerElementMaterial` (AllSame / ByPolygon), one mesh per
  (geometry, material) as Assimp splits them;
* `aiProcess_Triangulate`: a triangle as is; a quad fanned from its concave corner if it has one, else from
  corner 0 (Assimp's quad path); a larger polygon fanned from corner 0 (Assimp clips ears there: identical for
  the convex polygons an exporter writes, a librsd definition otherwise); degenerate faces kept
  (`aiProcess_FindDegenerates` is off, AssimpImporter.cpp:1101);
* materials (AssimpImporter.cpp:848-961): base-colour alpha = the FBX `Opacity` property, else
  1 - TransparencyFactor * mean(TransparentColor) when that differs from 1 (Assimp's opacity rule); a name
  token ".doubleSided" makes the material double-sided (:939-953); a `DiffuseColor` texture's alpha channel is
  the alpha texture; the alpha mode follows StandardMaterial (rsd.pyscene: Mask when the alpha can fall below
  the threshold).

Not restated (no effect on the SD trace's hit set): Assimp's vertex-cache reordering
(`aiProcess_ImproveCacheLocality`, which only permutes primitive ids), normals, tangents, skinning, cameras,
lights and animation.  Parity with an Assimp run is unpinned (no Assimp here); the tests pin the container
against the reference's own FBX fixture (`data/framework/meshes/sphere.fbx`, copied to tests/fixtures) and the
transform rules against FBX files written by the test helpers."""
from __future__ import annotations

import dataclasses
import math
import struct
import zlib
from pathlib import Path

import numpy as np

from . import ingest

MAGIC = b"Kaydara FBX Binary  \x00"


@dataclasses.dataclass
class Node:
    name: str
    props: list
    children: list

    def first(self, name: str) -> "Node | None":
        return next((c for c in self.children if c.name == name), None)

    def all(self, name: str) -> list:
        return [c for c in self.children if c.name == name]


_SCALAR = {ord("Y"): "<h", ord("C"): "<?", ord("I"): "<i", ord("F"): "<f", ord("D"): "<d", ord("L"): "<q"}
_ARRAY = {ord("f"): np.float32, ord("d"): np.float64, ord("l"): np.int64, ord("i"): np.int32,
          ord("b"): np.bool_, ord("c"): np.uint8}


class FbxError(ValueError):
    pass


def _prop(buf: bytes, p: int):
    t = buf[p]
    p += 1
    if t in _SCALAR:
        fmt = _SCALAR[t]
        n = struct.calcsize(fmt)
        return struct.unpack_from(fmt, buf, p)[0], p + n
    if t in _ARRAY:
        count, enc, clen = struct.unpack_from("<III", buf, p)
        p += 12
        raw = buf[p:p + clen]
        if len(raw) != clen:
            raise FbxError("truncated array property")
        if enc == 1:
            raw = zlib.decompress(raw)
        elif enc != 0:
            raise FbxError(f"unknown array encoding {enc}")
        a = np.frombuffer(raw, _ARRAY[t])
        if a.size != count:
            raise FbxError("array length mismatch")
        return a, p + clen
    if t in (ord("S"), ord("R")):
        n = struct.unpack_from("<I", buf, p)[0]
        p += 4
        return bytes(buf[p:p + n]), p + n
    raise FbxError(f"unknown property type {chr(t)!r} at byte {p - 1}")


def parse(data: bytes) -> Node:
    """The node tree of a binary FBX file (a root Node named '' holding the top-level records)."""
    try:
        return _parse(data)
    except (struct.error, IndexError, zlib.error, UnicodeDecodeError) as e:
        raise FbxError(f"malformed binary FBX ({e})") from e


def _parse(data: bytes) -> Node:
    if data[:21] != MAGIC:
        raise FbxError("not a binary FBX file (ASCII FBX is not supported)")
    version = struct.unpack_from("<I", data, 23)[0]
    wide = version >= 7500
    hdr = 25 if wide else 13

    def record(p: int):
        if wide:
            end, nprop, _plen = struct.unpack_from("<QQQ", data, p)
            p += 24
        else:
            end, nprop, _plen = struct.unpack_from("<III", data, p)
            p += 12
        nlen = data[p]
        p += 1
        if end == 0:
            return None, p
        if end > len(data):
            raise FbxError("record past the end of the file")
        name = data[p:p + nlen].decode("ascii", "replace")
        p += nlen
        props = []
        for _ in range(nprop):
            v, p = _prop(data, p)
            props.append(v)
        kids = []
        while p < end:
            if end - p == hdr and not any(data[p:end]):
                p = end  # the null record closing the child list
                break
            c, p = record(p)
            if c is None:
                break
            kids.append(c)
        return Node(name, props, kids), end

    root = Node("", [version], [])
    p = 27
    while p + hdr <= len(data):
        n, p = record(p)
        if n is None:
            break
        root.children.append(n)
    return root


def _s(v) -> str:
    return v.decode("utf-8", "replace") if isinstance(v, bytes) else str(v)


def _props70(node: Node | None) -> dict:
    out = {}
    if node is None:
        return out
    p70 = node.first("Properties70")
    for p in (p70.all("P") if p70 else []):
        if p.props:
            out[_s(p.props[0])] = p.props[4:]
    return out


class _Doc:
    def __init__(self, root: Node):
        self.root = root
        self.version = root.props[0]
        # Definitions: per object type (and template class) the default Properties70
        self.templates: dict[str, dict] = {}
        d = root.first("Definitions")
        for ot in (d.all("ObjectType") if d else []):
            t = ot.first("PropertyTemplate")
            if ot.props and t is not None:
                self.templates[_s(ot.props[0])] = _props70(t)
        self.objects: dict[int, Node] = {}
        objs = root.first("Objects")
        for o in (objs.children if objs else []):
            if o.props:
                self.objects[int(o.props[0])] = o
        # connections: child -> [(parent, property)], parent -> [(child, property)] in file order
        self.parents: dict[int, list] = {}
        self.children: dict[int, list] = {}
        con = root.first("Connections")
        for c in (con.all("C") if con else []):
            kind = _s(c.props[0])
            child, parent = int(c.props[1]), int(c.props[2])
            prop = _s(c.props[3]) if kind == "OP" and len(c.props) > 3 else None
            self.parents.setdefault(child, []).append((parent, prop))
            self.children.setdefault(parent, []).append((child, prop))
        gs = _props70(root.first("GlobalSettings"))
        self.unit_scale = float(gs.get("UnitScaleFactor", [1.0])[0])

    def prop(self, obj: Node, name: str, default):
        own = _props70(obj)
        if name in own:
            return own[name]
        t = self.templates.get(obj.name, {})
        return t.get(name, default)

    def vec3(self, obj: Node, name: str, default) -> np.ndarray:
        v = self.prop(obj, name, None)
        return np.array(default if v is None or len(v) < 3 else [float(x) for x in v[:3]], np.float64)

    def kids_of(self, oid: int, node_name: str) -> list[int]:
        return [c for c, _ in self.children.get(oid, []) if c in self.objects and self.objects[c].name == node_name]


def _tr(v) -> np.ndarray:
    m = np.eye(4)
    m[:3, 3] = v
    return m


def _sc(v) -> np.ndarray:
    return np.diag([v[0], v[1], v[2], 1.0])


def _rot_axis(axis: int, deg: float) -> np.ndarray:
    a = math.radians(deg)
    c, s = math.cos(a), math.sin(a)
    m = np.eye(4)
    i, j = [(1, 2), (2, 0), (0, 1)][axis]
    m[i, i], m[i, j], m[j, i], m[j, j] = c, -s, s, c
    return m


# RotationOrder enum (FbxEuler::EOrder): the axes in the order they are applied
_ORDERS = {0: (0, 1, 2), 1: (0, 2, 1), 2: (1, 2, 0), 3: (1, 0, 2), 4: (2, 0, 1), 5: (2, 1, 0), 6: (0, 1, 2)}


def euler(deg, order: int = 0) -> np.ndarray:
    """Rotation by Euler angles in degrees, the axes applied in `order` (XYZ: Rz @ Ry @ Rx)."""
    m = np.eye(4)
    for ax in _ORDERS.get(int(order), (0, 1, 2)):
        if deg[ax] != 0.0:
            m = _rot_axis(ax, float(deg[ax])) @ m
    return m


def model_local(doc: _Doc, model: Node) -> tuple[np.ndarray, np.ndarray]:
    """(node transform, geometric transform) of a Model, float64 4x4 column-vector matrices."""
    v = lambda name, d=(0.0, 0.0, 0.0): doc.vec3(model, name, d)  # noqa: E731
    order = doc.prop(model, "RotationOrder", [0])
    order = int(order[0]) if order else 0
    T, R, S = v("Lcl Translation"), v("Lcl Rotation"), v("Lcl Scaling", (1.0, 1.0, 1.0))
    Roff, Rp, Soff, Sp = v("RotationOffset"), v("RotationPivot"), v("ScalingOffset"), v("ScalingPivot")
    Rpre, Rpost = v("PreRotation"), v("PostRotation")
    local = (_tr(T) @ _tr(Roff) @ _tr(Rp) @ euler(Rpre) @ euler(R, order) @ np.linalg.inv(euler(Rpost)) @
             _tr(-Rp) @ _tr(Soff) @ _tr(Sp) @ _sc(S) @ _tr(-Sp))
    geo = _tr(v("GeometricTranslation")) @ euler(v("GeometricRotation"), order) @ \
        _sc(v("GeometricScaling", (1.0, 1.0, 1.0)))
    return local, geo


def model_world(doc: _Doc, mid: int, memo: dict | None = None) -> np.ndarray:
    memo = {} if memo is None else memo
    if mid in memo:
        return memo[mid]
    local, _ = model_local(doc, doc.objects[mid])
    parent = next((p for p, prop in doc.parents.get(mid, []) if prop is None and p in doc.objects and
                   doc.objects[p].name == "Model"), None)
    w = local if parent is None else model_world(doc, parent, memo) @ local
    memo[mid] = w
    return w


def _layer(geom: Node, layer: str, values: str, index: str, width: int, npv: int, poly_vertex: np.ndarray):
    """Per polygon-vertex values of a LayerElement (ByPolygonVertex / ByVertice / ByPolygon..., Direct /
    IndexToDirect); None when the geometry has no such layer."""
    el = geom.first(layer)
    if el is None or el.first(values) is None:
        return None
    mapping = _s(el.first("MappingInformationType").props[0]) if el.first("MappingInformationType") else "ByPolygonVertex"
    ref = _s(el.first("ReferenceInformationType").props[0]) if el.first("ReferenceInformationType") else "Direct"
    data = np.asarray(el.first(values).props[0], np.float64).reshape(-1, width)
    if ref == "IndexToDirect" and el.first(index) is not None:
        data = data[np.asarray(el.first(index).props[0], np.int64)]
    if mapping == "ByPolygonVertex":
        return data[:npv]
    if mapping in ("ByVertice", "ByVertex"):
        return data[poly_vertex]
    return None


def _triangulate(corners: np.ndarray, pos: np.ndarray) -> list[tuple[int, int, int]]:
    """Corner-position indices of one polygon's triangles (aiProcess_Triangulate, see the module docstring)."""
    n = len(corners)
    if n < 3:
        return []  # points and lines: dropped by aiProcess_SortByPType + Falcor's triangle-only meshes
    if n == 3:
        return [(0, 1, 2)]
    start = 0
    if n == 4:
        for i in range(4):
            v = pos[corners[i]].astype(np.float32)
            left = pos[corners[(i + 3) % 4]].astype(np.float32) - v
            diag = pos[corners[(i + 2) % 4]].astype(np.float32) - v
            right = pos[corners[(i + 1) % 4]].astype(np.float32) - v
            nl, nd, nr = (np.linalg.norm(x) for x in (left, diag, right))
            if nl == 0 or nd == 0 or nr == 0:
                continue
            cl = float(np.clip(np.dot(left / nl, diag / nd), -1.0, 1.0))
            cr = float(np.clip(np.dot(right / nr, diag / nd), -1.0, 1.0))
            if math.acos(cl) + math.acos(cr) > math.pi:
                start = i  # the concave corner
                break
        return [(start, (start + 1) % 4, (start + 2) % 4), (start, (start + 2) % 4, (start + 3) % 4)]
    return [(0, k, k + 1) for k in range(1, n - 1)]


def _material(doc: _Doc, mat: Node | None, base: Path, threshold: float) -> ingest.Material:
    if mat is None:
        return ingest.Material(name="default", alpha_threshold=threshold)
    name = _s(mat.props[1]).split("\x00")[0] if len(mat.props) > 1 else "material"
    m = ingest.Material(name=name, alpha_threshold=threshold)
    m.double_sided = any(t.lower() == "doublesided" for t in name.split(".")[1:])
    op = doc.prop(mat, "Opacity", None)
    if op:
        m.alpha = float(op[0])
    else:
        tc = doc.prop(mat, "TransparentColor", None)
        tf = doc.prop(mat, "TransparencyFactor", None)
        if tc and len(tc) >= 3:
            f = float(tf[0]) if tf else 1.0
            calc = 1.0 - f * (float(tc[0]) + float(tc[1]) + float(tc[2])) / 3.0
            if calc != 1.0:
                m.alpha = calc
    # a DiffuseColor texture's alpha channel (TextureSlot BaseColor)
    for tid, prop in doc.children.get(int(mat.props[0]), []):
        tex = doc.objects.get(tid)
        if tex is None or tex.name != "Texture" or prop not in ("DiffuseColor", "Maya|baseColor"):
            continue
        for key in ("RelativeFilename", "FileName"):
            f = tex.first(key)
            if f is None or not f.props:
                continue
            p = Path(_s(f.props[0]).replace("\\", "/"))
            cand = [p if p.is_absolute() else base / p, base / p.name]
            hit = next((c for c in cand if c.exists()), None)
            if hit is not None:
                try:
                    a = ingest.alpha_channel(ingest.read_image(hit), grey_is_alpha=False)
                except ValueError:
                    a = None
                m.alpha_texture = a
                break
    lo = float(m.alpha_texture.min()) / 255.0 if m.alpha_texture is not None else m.alpha
    m.alpha_mode_mask = lo < m.alpha_threshold
    if not m.alpha_mode_mask:
        m.alpha_texture = None
    return m


def load_fbx(path, transform=None, alpha_threshold: float = 0.5,
             builder: ingest.SceneBuilder | None = None) -> ingest.SceneBuilder:
    """A binary FBX file into a SceneBuilder: one mesh per (Geometry, material) of every Model that has a
    mesh, instanced with the Model's world transform (times `transform`), its geometric transform applied to
    the mesh's vertices."""
    path = Path(path)
    doc = _Doc(parse(path.read_bytes()))
    B = builder or ingest.SceneBuilder()
    T0 = np.eye(4) if transform is None else np.asarray(transform, np.float64).reshape(4, 4)
    mat_ids: dict[int, int] = {}
    memo: dict = {}

    def material_id(mat_oid: int | None) -> int:
        key = -1 if mat_oid is None else mat_oid
        if key not in mat_ids:
            mat_ids[key] = B.add_material(_material(doc, doc.objects.get(mat_oid) if mat_oid is not None else None,
                                                    path.parent, alpha_threshold))
        return mat_ids[key]

    for mid, model in doc.objects.items():
        if model.name != "Model":
            continue
        geoms = doc.kids_of(mid, "Geometry")
        mats = doc.kids_of(mid, "Material")
        if not geoms:
            continue
        world = T0 @ model_world(doc, mid, memo)
        _, geo_xf = model_local(doc, model)
        for gid in geoms:
            g = doc.objects[gid]
            if len(g.props) < 3 or _s(g.props[2]) != "Mesh" or g.first("Vertices") is None:
                continue
            P = np.asarray(g.first("Vertices").props[0], np.float64).reshape(-1, 3)
            # geometric transform in float64, then float32 vertices (Assimp's aiVector3D)
            P = (P @ geo_xf[:3, :3].T + geo_xf[:3, 3]).astype(np.float32)
            pvi = np.asarray(g.first("PolygonVertexIndex").props[0], np.int64) if g.first("PolygonVertexIndex") \
                else np.zeros(0, np.int64)
            ends = pvi < 0
            corner = np.where(ends, ~pvi, pvi)
            if corner.size and (corner.max() >= len(P) or corner.min() < 0):
                raise FbxError(f"{path.name}: polygon vertex index out of range")
            npv = len(corner)
            uv = _layer(g, "LayerElementUV", "UV", "UVIndex", 2, npv, corner)
            # polygons -> corner ranges
            stops = np.flatnonzero(ends) + 1
            starts = np.concatenate([[0], stops[:-1]]) if stops.size else np.zeros(0, np.int64)
            # per-polygon material (LayerElementMaterial: AllSame / ByPolygon)
            pm = np.zeros(len(starts), np.int64)
            lm = g.first("LayerElementMaterial")
            if lm is not None and lm.first("Materials") is not None:
                mv = np.asarray(lm.first("Materials").props[0], np.int64)
                mapping = _s(lm.first("MappingInformationType").props[0]) if lm.first("MappingInformationType") \
                    else "AllSame"
                if mapping == "ByPolygon" and mv.size >= len(starts):
                    pm = mv[:len(starts)]
                elif mv.size:
                    pm[:] = mv[0]
            runs: dict[int, list] = {}
            for k, (s0, s1) in enumerate(zip(starts, stops)):
                cs = np.arange(s0, s1)
                for a, b, c in _triangulate(corner[cs], P):
                    runs.setdefault(int(pm[k]), []).append((cs[a], cs[b], cs[c]))
            for slot, tris in runs.items():
                mat_oid = mats[slot] if 0 <= slot < len(mats) else (mats[0] if mats else None)
                t = np.asarray(tris, np.int64).reshape(-1, 3)
                # polygon vertices -> unique (position, uv) vertices (aiProcess_JoinIdenticalVertices)
                used = np.unique(t)
                keyp = corner[used]
                if uv is not None:
                    uvs = uv[used].astype(np.float32)
                    uvs[:, 1] = np.float32(1.0) - uvs[:, 1]  # aiProcess_FlipUVs
                    key = np.concatenate([keyp[:, None].astype(np.float64), uvs.astype(np.float64)], 1)
                else:
                    uvs = None
                    key = keyp[:, None].astype(np.float64)
                uniq, inv = np.unique(key, axis=0, return_inverse=True)
                remap = np.empty(npv, np.int64)
                remap[used] = inv.reshape(-1)
                pos = P[uniq[:, 0].astype(np.int64)]
                tex = uniq[:, 1:3].astype(np.float32) if uvs is not None else None
                mesh = ingest.Mesh(pos, remap[t].astype(np.uint32), tex, material_id(mat_oid))
                B.add_instance(B.add_mesh(mesh), world.astype(np.float32))
    return B
