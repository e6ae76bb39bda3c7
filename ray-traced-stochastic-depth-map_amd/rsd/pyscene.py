"""Falcor `.pyscene` ingest: a scene script executed against a SceneBuilder.

Reference: the Python importer (Source/plugins/importers/PythonImporter/PythonImporter.cpp) runs
the script with `sceneBuilder` bound to the active SceneBuilder and Falcor's script bindings in
scope.  The bindings this module mirrors, with the geometry they produce:

* `Transform` (Scene/Transform.cpp:33-115, binding :151-236): translation / scaling (number or
  float3) / rotationEuler / rotationEulerDeg / position+target+up (lookAt) / order; the matrix is
  T * R * S for the default ScaleRotateTranslate order, R from quatFromEulerAngles
  (Utils/Math/QuaternionMath.h:398-409) or quatFromLookAt (:468-481) via matrixFromQuat
  (MatrixMath.h:715-741).
* `TriangleMesh` (Scene/TriangleMesh.cpp:40-341): createQuad / createDisk / createCube /
  createSphere / createFromFile (OBJ only here), addVertex / addTriangle, frontFaceCW.
* `StandardMaterial` / `Material` (Material/StandardMaterial.cpp:210-225, Material.cpp:363-392,
  BasicMaterial.cpp:233-259,611-633): baseColor, doubleSided, alphaMode, alphaThreshold (stored as
  float16), loadTexture(MaterialTextureSlot.BaseColor, path); the alpha mode follows
  updateAlphaMode: Mask iff the conservative alpha range's minimum is below the threshold.
* `sceneBuilder` (Scene/SceneBuilder.cpp:2877-2907): importScene (OBJ via rsd.ingest.load_obj, binary FBX via rsd.fbx.load_fbx),
  addTriangleMesh, addMaterial, getMaterial, replaceMaterial, loadMaterialTexture, addNode
  (world = parent world * local), addMeshInstance, addCamera (the first camera is the scene's).

What the SD trace cannot see is accepted and dropped: lights, env maps, grid volumes, animations
and procedural geometry (SDF grids, custom primitives) -- the SD rays skip procedural primitives
(StochasticDepthMapRT.rt.slang:85 RAY_FLAG_SKIP_PROCEDURAL_PRIMITIVES).  glTF / USD / PBRT / ASCII FBX
imports raise (no importer for them in this image)."""
from __future__ import annotations

import enum
from pathlib import Path

import numpy as np

from . import fbx, ingest

F32 = np.float32
INVALID_ID = 0xFFFFFFFF  # NodeID::kInvalidID


# ------------------------------------------------------------------------------ vectors

class _Vec(np.ndarray):
    """float2/3/4 with .x .y .z .w (a float32 ndarray)."""

    def _get(self, i):
        return float(self[i])

    x = property(lambda s: s._get(0))
    y = property(lambda s: s._get(1))
    z = property(lambda s: s._get(2))
    w = property(lambda s: s._get(3))


def _vec(n, args):
    if len(args) == 1:
        a = np.asarray(args[0], F32).reshape(-1)
        v = np.full(n, a[0], F32) if a.size == 1 else a.astype(F32)
    else:
        v = np.array([float(x) for x in args], F32)
    if v.size != n:
        raise TypeError(f"float{n} takes 1 or {n} components, got {v.size}")
    return v.view(_Vec)


def float2(*a):
    return _vec(2, a)


def float3(*a):
    return _vec(3, a)


def float4(*a):
    return _vec(4, a)


def _f3(v):
    return np.full(3, F32(v), F32) if np.isscalar(v) else np.asarray(v, F32).reshape(3)


# ------------------------------------------------------------------------------ Transform

class CompositionOrder(enum.Enum):
    SRT = "SRT"
    STR = "STR"
    RST = "RST"
    RTS = "RTS"
    TRS = "TRS"
    TSR = "TSR"
    Default = "SRT"  # alias of ScaleRotateTranslate (Transform.h)


def _quat_from_euler(e):
    """QuaternionMath.h:398-409 in float32: (x, y, z, w)."""
    e = np.asarray(e, F32)
    c, s = np.cos(e * F32(0.5)), np.sin(e * F32(0.5))
    return np.array([s[0] * c[1] * c[2] - c[0] * s[1] * s[2],
                     c[0] * s[1] * c[2] + s[0] * c[1] * s[2],
                     c[0] * c[1] * s[2] - s[0] * s[1] * c[2],
                     c[0] * c[1] * c[2] + s[0] * s[1] * s[2]], F32)


def _quat_from_matrix(m):
    """QuaternionMath.h:415-457 (m[row][col])."""
    fx = m[0, 0] - m[1, 1] - m[2, 2]
    fy = m[1, 1] - m[0, 0] - m[2, 2]
    fz = m[2, 2] - m[0, 0] - m[1, 1]
    fw = m[0, 0] + m[1, 1] + m[2, 2]
    big, idx = fw, 0
    for k, f in ((1, fx), (2, fy), (3, fz)):
        if f > big:
            big, idx = f, k
    bv = np.sqrt(big + F32(1)) * F32(0.5)
    mult = F32(0.25) / bv
    if idx == 0:
        q = ((m[2, 1] - m[1, 2]) * mult, (m[0, 2] - m[2, 0]) * mult, (m[1, 0] - m[0, 1]) * mult, bv)
    elif idx == 1:
        q = (bv, (m[1, 0] + m[0, 1]) * mult, (m[0, 2] + m[2, 0]) * mult, (m[2, 1] - m[1, 2]) * mult)
    elif idx == 2:
        q = ((m[1, 0] + m[0, 1]) * mult, bv, (m[2, 1] + m[1, 2]) * mult, (m[0, 2] - m[2, 0]) * mult)
    else:
        q = ((m[0, 2] + m[2, 0]) * mult, (m[2, 1] + m[1, 2]) * mult, bv, (m[1, 0] - m[0, 1]) * mult)
    return np.array(q, F32)


def _normalize(v):
    return (v / np.sqrt(F32(np.dot(v, v)))).astype(F32)


def _quat_from_look_at(d, up):
    """QuaternionMath.h:468-481, right-handed: forward -> -Z."""
    m = np.zeros((3, 3), F32)
    m[:, 2] = -d
    m[:, 0] = _normalize(np.cross(up, m[:, 2]).astype(F32))
    m[:, 1] = np.cross(m[:, 2], m[:, 0]).astype(F32)
    return _quat_from_matrix(m)


def _matrix_from_quat(q):
    """MatrixMath.h:715-741."""
    x, y, z, w = (F32(v) for v in q)
    xx, yy, zz, xz, xy, yz, wx, wy, wz = x * x, y * y, z * z, x * z, x * y, y * z, w * x, w * y, w * z
    one, two = F32(1), F32(2)
    return np.array([[one - two * (yy + zz), two * (xy - wz), two * (xz + wy)],
                     [two * (xy + wz), one - two * (xx + zz), two * (yz - wx)],
                     [two * (xz - wy), two * (yz + wx), one - two * (xx + yy)]], F32)


class Transform:
    """Scene/Transform.cpp: translation, rotation (quaternion), scaling and a composition order."""

    def __init__(self, **kw):
        self._t = np.zeros(3, F32)
        self._s = np.ones(3, F32)
        self._q = np.array([0, 0, 0, 1], F32)
        self.order = CompositionOrder.SRT
        look = {}
        for k, v in kw.items():
            if k == "translation":
                self.translation = v
            elif k == "scaling":
                self.scaling = v
            elif k == "rotationEuler":
                self.rotationEuler = v
            elif k == "rotationEulerDeg":
                self.rotationEulerDeg = v
            elif k in ("position", "target", "up"):
                look[k] = _f3(v)
            elif k == "order":
                self.order = CompositionOrder(v.value if isinstance(v, CompositionOrder) else v)
        if len(look) == 3:
            self.lookAt(look["position"], look["target"], look["up"])

    translation = property(lambda s: s._t.copy().view(_Vec), lambda s, v: setattr(s, "_t", _f3(v)))
    scaling = property(lambda s: s._s.copy().view(_Vec), lambda s, v: setattr(s, "_s", _f3(v)))

    def _set_euler(self, v):
        self._q = _quat_from_euler(_f3(v))

    def _set_euler_deg(self, v):
        self._set_euler(_f3(v) * F32(np.pi / 180.0))

    rotationEuler = property(None, _set_euler)
    rotationEulerDeg = property(None, _set_euler_deg)

    def lookAt(self, position, target, up):
        self._t = _f3(position)
        self._q = _quat_from_look_at(_normalize(_f3(target) - self._t), _f3(up))

    @property
    def matrix(self) -> np.ndarray:
        """Transform::getMatrix (:80-115), float32 4x4 acting on column vectors."""
        T = np.eye(4, dtype=F32)
        T[:3, 3] = self._t
        R = np.eye(4, dtype=F32)
        R[:3, :3] = _matrix_from_quat(self._q)
        S = np.diag(np.append(self._s, F32(1))).astype(F32)
        o = self.order.value
        mats = {"T": T, "R": R, "S": S}
        # "SRT" = scale first, then rotate, then translate: M = T * R * S
        return (mats[o[2]] @ mats[o[1]] @ mats[o[0]]).astype(F32)


# ------------------------------------------------------------------------------ meshes

class TriangleMesh:
    """Scene/TriangleMesh.cpp: a vertex list (position, normal, texCoord) and an index list."""

    def __init__(self, positions=None, normals=None, uvs=None, indices=None, frontFaceCW=False):
        self.name = ""
        self._p = [] if positions is None else [np.asarray(p, F32) for p in positions]
        self._n = [] if normals is None else [np.asarray(n, F32) for n in normals]
        self._uv = [] if uvs is None else [np.asarray(t, F32) for t in uvs]
        self._i = [] if indices is None else [int(i) for i in indices]
        self.frontFaceCW = bool(frontFaceCW)

    @property
    def vertices(self):
        return [dict(position=p, normal=n, texCoord=t) for p, n, t in zip(self._p, self._n, self._uv)]

    @property
    def indices(self):
        return list(self._i)

    def addVertex(self, position, normal, texCoord):
        self._p.append(_f3(position))
        self._n.append(_f3(normal))
        self._uv.append(np.asarray(texCoord, F32).reshape(2))
        return len(self._p) - 1

    def addTriangle(self, i0, i1, i2):
        self._i += [int(i0), int(i1), int(i2)]

    @staticmethod
    def createQuad(size=None):
        """:57-76"""
        size = np.asarray(size if size is not None else (1.0, 1.0), F32).reshape(2)
        h = F32(0.5) * size
        n = (0.0, 1.0, 0.0)
        P = [(-h[0], 0, -h[1]), (h[0], 0, -h[1]), (-h[0], 0, h[1]), (h[0], 0, h[1])]
        UV = [(0, 0), (1, 0), (0, 1), (1, 1)]
        return TriangleMesh(P, [n] * 4, UV, [2, 1, 0, 1, 2, 3], bool(size[0] * size[1] < 0))

    @staticmethod
    def createDisk(radius=1.0, segments=32):
        """:78-99"""
        r, seg = F32(radius), int(segments)
        P, UV, I = [(0, 0, 0)], [(0.5, 0.5)], []
        for i in range(seg):
            phi = F32(i) / F32(seg) * F32(2) * F32(np.pi)
            c, s = np.cos(phi), -np.sin(phi)
            P.append((c * r, 0, s * r))
            UV.append((F32(0.5) + c * F32(0.5), F32(0.5) + s * F32(0.5)))
            I += [0, i + 1, (i + 1) % seg + 1]
        return TriangleMesh(P, [(0, 1, 0)] * len(P), UV, I, False)

    @staticmethod
    def createCube(size=None):
        """:101-148"""
        size = _f3(size if size is not None else 1.0)
        pos = [[(-.5, -.5, -.5), (-.5, -.5, .5), (.5, -.5, .5), (.5, -.5, -.5)],
               [(-.5, .5, .5), (-.5, .5, -.5), (.5, .5, -.5), (.5, .5, .5)],
               [(-.5, .5, -.5), (-.5, -.5, -.5), (.5, -.5, -.5), (.5, .5, -.5)],
               [(.5, .5, .5), (.5, -.5, .5), (-.5, -.5, .5), (-.5, .5, .5)],
               [(-.5, .5, .5), (-.5, -.5, .5), (-.5, -.5, -.5), (-.5, .5, -.5)],
               [(.5, .5, -.5), (.5, -.5, -.5), (.5, -.5, .5), (.5, .5, .5)]]
        nrm = [(0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1), (-1, 0, 0), (1, 0, 0)]
        uv = [(0, 0), (1, 0), (1, 1), (0, 1)]
        sign = np.where(size < 0, F32(-1), F32(1))
        m = TriangleMesh(frontFaceCW=bool(size[0] * size[1] * size[2] < 0))
        for f in range(6):
            b = len(m._p)
            m._i += [b, b + 2, b + 1, b, b + 3, b + 2]
            for j in range(4):
                m._p.append(np.asarray(pos[f][j], F32) * size)
                m._n.append(np.asarray(nrm[f], F32) * sign)
                m._uv.append(np.asarray(uv[j], F32))
        return m

    @staticmethod
    def createSphere(radius=1.0, segmentsU=32, segmentsV=32):
        """:150-193"""
        r, su, sv = F32(radius), int(segmentsU), int(segmentsV)
        m = TriangleMesh()
        for v in range(sv + 1):
            for u in range(su + 1):
                uvx, uvy = F32(u) / F32(su), F32(v) / F32(sv)
                theta, phi = uvx * F32(2) * F32(np.pi), uvy * F32(np.pi)
                d = np.array([np.cos(theta) * np.sin(phi), np.cos(phi), np.sin(theta) * np.sin(phi)], F32)
                m._p.append(d * r)
                m._n.append(d)
                m._uv.append(np.array([uvx, uvy], F32))
        for v in range(sv):
            for u in range(su):
                i0 = v * (su + 1) + u
                i1 = v * (su + 1) + (u + 1) % (su + 1)
                i2 = (v + 1) * (su + 1) + u
                i3 = (v + 1) * (su + 1) + (u + 1) % (su + 1)
                m._i += [i0, i1, i2, i2, i1, i3]
        return m

    @staticmethod
    def createFromFile(path, smoothNormals=False):
        """:195-273 (Assimp, pre-transformed, UVs flipped): OBJ (rsd.ingest) and binary FBX (rsd.fbx) files."""
        p = _resolve(path)
        if p is None:
            return None  # the reference logs a warning and returns nullptr
        if p.suffix.lower() not in (".obj", ".fbx"):
            raise NotImplementedError(f"TriangleMesh.createFromFile: {p.suffix} needs Assimp (OBJ / FBX here)")
        b = ingest.load_obj(p) if p.suffix.lower() == ".obj" else fbx.load_fbx(p)
        m = TriangleMesh()
        for mesh_id, T in b.instances:
            mm = b.meshes[mesh_id]
            base = len(m._p)
            m._p += list(mm.positions)
            m._n += [np.zeros(3, F32)] * len(mm.positions)
            m._uv += list(mm.texcoords if mm.texcoords is not None else np.zeros((len(mm.positions), 2), F32))
            m._i += [base + int(i) for i in mm.indices.reshape(-1)]
        return m

    def _to_ingest(self, material_id: int) -> ingest.Mesh:
        nv = len(self._p)
        pos = np.asarray(self._p, F32).reshape(nv, 3)
        uv = np.asarray(self._uv, F32).reshape(nv, 2) if len(self._uv) == nv else None
        return ingest.Mesh(pos, np.asarray(self._i, np.uint32).reshape(-1, 3), uv, material_id, self.frontFaceCW)


# ------------------------------------------------------------------------------ materials

class AlphaMode(enum.Enum):
    Opaque = 0
    Mask = 1


class MaterialTextureSlot(enum.Enum):
    BaseColor = 0
    Specular = 1
    Emissive = 2
    Normal = 3
    Transmission = 4
    Displacement = 5
    Index = 6


class ShadingModel(enum.Enum):
    MetalRough = 0
    SpecGloss = 1


def _half(x: float) -> float:
    return float(np.float16(x))  # MaterialHeader stores the threshold as float16


class StandardMaterial:
    """The material state the SD trace reads (MaterialHeader: double-sided, alpha mode and
    threshold; base-colour alpha and its texture); other properties are kept, unused."""

    def __init__(self, name="", model=ShadingModel.MetalRough, _wrap: ingest.Material | None = None):
        m = _wrap or ingest.Material(name=name or "")
        object.__setattr__(self, "_m", m)
        object.__setattr__(self, "_extra", {})
        object.__setattr__(self, "_base", np.array([1, 1, 1, m.alpha], F32))
        object.__setattr__(self, "_tex_alpha_min", None if m.alpha_texture is None
                           else float(m.alpha_texture.min()) / 255.0)
        if _wrap is None:
            self._update_alpha_mode()

    # BasicMaterial::updateAlphaMode (:611-633); optimizeTexture's narrowed range for textures
    def _update_alpha_mode(self):
        lo = self._tex_alpha_min if self._tex_alpha_min is not None else float(self._base[3])
        self._m.alpha_mode_mask = lo < self._m.alpha_threshold

    name = property(lambda s: s._m.name, lambda s, v: setattr(s._m, "name", str(v)))
    doubleSided = property(lambda s: s._m.double_sided, lambda s, v: setattr(s._m, "double_sided", bool(v)))

    @property
    def alphaMode(self):
        return AlphaMode.Mask if self._m.alpha_mode_mask else AlphaMode.Opaque

    @alphaMode.setter
    def alphaMode(self, v):
        self._m.alpha_mode_mask = (v == AlphaMode.Mask)

    @property
    def alphaThreshold(self):
        return self._m.alpha_threshold

    @alphaThreshold.setter
    def alphaThreshold(self, v):
        self._m.alpha_threshold = _half(v)
        self._update_alpha_mode()

    @property
    def baseColor(self):
        return self._base.copy().view(_Vec)

    @baseColor.setter
    def baseColor(self, v):
        object.__setattr__(self, "_base", np.asarray(v, F32).reshape(4).copy())
        self._m.alpha = float(self._base[3])
        self._update_alpha_mode()

    def loadTexture(self, slot, path, useSrgb=True):
        if slot != MaterialTextureSlot.BaseColor:
            return True  # other slots do not reach the SD trace
        p = _resolve(path)
        if p is None:
            return False
        a = ingest.alpha_channel(ingest.read_image(p), grey_is_alpha=False)
        self._m.alpha_texture = a
        object.__setattr__(self, "_tex_alpha_min", None if a is None else float(a.min()) / 255.0)
        self._update_alpha_mode()
        return True

    def clearTexture(self, slot):
        if slot == MaterialTextureSlot.BaseColor:
            self._m.alpha_texture = None
            object.__setattr__(self, "_tex_alpha_min", None)
            self._update_alpha_mode()

    def __setattr__(self, k, v):
        if hasattr(type(self), k):
            object.__setattr__(self, k, v)
        else:
            self._extra[k] = v  # roughness, metallic, emissive*, specularParams, ...

    def __getattr__(self, k):
        ex = object.__getattribute__(self, "_extra")
        if k in ex:
            return ex[k]
        raise AttributeError(k)


Material = StandardMaterial  # StandardMaterial.cpp:225


# ------------------------------------------------------------------------------ inert bindings

class _Inert:
    """Bindings whose objects never reach the SD trace (lights, env maps, volumes, SDF grids,
    animations, settings): attributes are stored, methods accept anything."""

    def __init__(self, *args, **kw):
        object.__setattr__(self, "_attrs", dict(kw))
        object.__setattr__(self, "_args", args)

    def __getattr__(self, k):
        a = object.__getattribute__(self, "_attrs")
        if k in a:
            return a[k]
        if k[:1].isupper():
            return _Inert()  # nested enums (GridVolume.GridSlot.Density, ...)
        return lambda *args, **kw: _Inert()

    def __setattr__(self, k, v):
        self._attrs[k] = v

    def __call__(self, *args, **kw):
        return _Inert()


class _InertType(type):
    def __getattr__(cls, k):
        return _Inert()  # static factories and enums: Grid.createSphere, GridVolume.GridSlot, ...


class _InertClass(_Inert, metaclass=_InertType):
    pass


def _inert(name):
    return _InertType(name, (_InertClass,), {})


class Camera:
    """The scene camera the SD trace starts from (Scene/Camera/Camera.cpp bindings)."""

    def __init__(self, name=""):
        self.name = name
        self.position = float3(0, 0, 1)
        self.target = float3(0, 0, 0)
        self.up = float3(0, 1, 0)
        self.focalLength = 21.0
        self.nearPlane, self.farPlane = 0.1, 1000.0


# ------------------------------------------------------------------------------ the builder

_SCRIPT_DIR: list[Path] = []


def _resolve(path) -> Path | None:
    """Falcor's data-directory search, reduced to: absolute, or relative to the script."""
    p = Path(str(path).replace("\\", "/"))
    if p.is_absolute():
        return p if p.exists() else None
    for d in reversed(_SCRIPT_DIR):
        if (d / p).exists():
            return d / p
    return p if p.exists() else None


class PySceneBuilder:
    """`sceneBuilder` inside a .pyscene script, over an rsd.ingest.SceneBuilder."""

    def __init__(self, builder: ingest.SceneBuilder | None = None):
        self._B = builder or ingest.SceneBuilder()
        self._mat_ids: dict[int, int] = {}       # id(StandardMaterial) -> material index
        self._materials: list[StandardMaterial] = []
        self._nodes: list[tuple[np.ndarray, int]] = []  # (local matrix, parent)
        self._cameras: list[Camera] = []
        self.envMap = None
        self.settings = _Inert()

    # -- materials
    def addMaterial(self, material: StandardMaterial) -> int:
        key = id(material)
        if key not in self._mat_ids:
            self._mat_ids[key] = self._B.add_material(material._m)
            self._materials.append(material)
        return self._mat_ids[key]

    def getMaterial(self, name):
        for m in self._materials:
            if m.name == name:
                return m
        return None

    def replaceMaterial(self, material, replacement):
        idx = self.addMaterial(material)
        self._B.materials[idx] = replacement._m
        self._mat_ids[id(replacement)] = idx
        self._materials[self._materials.index(material)] = replacement

    def loadMaterialTexture(self, material, slot, path):
        material.loadTexture(slot, path)

    def waitForMaterialTextureLoading(self):
        pass

    # -- geometry
    def importScene(self, path, dict=None):
        """SceneBuilder::import: OBJ through rsd.ingest.load_obj, binary FBX through rsd.fbx.load_fbx (the
        reference's AssimpImporter); their meshes are placed by the importer itself (world space, like
        Assimp's node transforms)."""
        p = _resolve(path)
        if p is None:
            raise FileNotFoundError(f"importScene: can't find '{path}'")
        if p.suffix.lower() not in (".obj", ".fbx"):
            raise NotImplementedError(f"importScene: no importer for '{p.suffix}' in this build (OBJ, FBX)")
        before = len(self._B.materials)
        (ingest.load_obj if p.suffix.lower() == ".obj" else fbx.load_fbx)(p, builder=self._B)
        for idx in range(before, len(self._B.materials)):
            w = StandardMaterial(_wrap=self._B.materials[idx])
            self._mat_ids[id(w)] = idx
            self._materials.append(w)

    def addTriangleMesh(self, triangleMesh: TriangleMesh, material: StandardMaterial) -> int:
        if triangleMesh is None:
            raise ValueError("addTriangleMesh: 'triangleMesh' is missing")
        return self._B.add_mesh(triangleMesh._to_ingest(self.addMaterial(material)))

    def addNode(self, name, transform: Transform | None = None, parent=INVALID_ID) -> int:
        if parent != INVALID_ID and not 0 <= parent < len(self._nodes):
            raise ValueError(f"addNode: parent {parent} does not exist")
        self._nodes.append(((transform or Transform()).matrix, parent))
        return len(self._nodes) - 1

    def addMeshInstance(self, nodeID, meshID):
        if not 0 <= nodeID < len(self._nodes) or not 0 <= meshID < len(self._B.meshes):
            raise ValueError("addMeshInstance: invalid node or mesh id")
        self._B.add_instance(meshID, self._world(nodeID))  # in call order, like importScene's

    def _world(self, node) -> np.ndarray:
        M, parent = self._nodes[node]
        return M if parent == INVALID_ID else (self._world(parent) @ M).astype(F32)

    # -- procedural geometry: invisible to the SD rays (RAY_FLAG_SKIP_PROCEDURAL_PRIMITIVES)
    def addSDFGrid(self, sdfGrid, material):
        self.addMaterial(material)
        return 0

    def addSDFGridInstance(self, nodeID, sdfGridID):
        pass

    def addCustomPrimitive(self, *args, **kw):
        pass

    # -- camera, lights, volumes, animation
    def addCamera(self, camera: Camera):
        self._cameras.append(camera)

    def addLight(self, light):
        return 0

    def getLight(self, name):
        return None

    def loadLightProfile(self, *a, **kw):
        pass

    def addGridVolume(self, gridVolume, nodeID=INVALID_ID):
        return 0

    addVolume = addGridVolume

    def getGridVolume(self, name):
        return None

    getVolume = getGridVolume

    def addAnimation(self, animation):
        pass

    def createAnimation(self, animatable, name, duration):
        return _Inert()

    def getSettings(self):
        return self.settings

    def finish(self) -> ingest.SceneBuilder:
        """Pick the first camera (the scene's default camera)."""
        if self._cameras:
            c = self._cameras[0]
            self._B.set_camera(np.asarray(c.position, F32), np.asarray(c.target, F32), np.asarray(c.up, F32))
        return self._B


def namespace(sb: PySceneBuilder) -> dict:
    """The names a .pyscene script sees (the falcor module's scene bindings)."""
    ns = dict(sceneBuilder=sb, float2=float2, float3=float3, float4=float4, Transform=Transform,
              CompositionOrder=CompositionOrder, TriangleMesh=TriangleMesh, StandardMaterial=StandardMaterial,
              Material=Material, AlphaMode=AlphaMode, MaterialTextureSlot=MaterialTextureSlot,
              ShadingModel=ShadingModel, Camera=Camera, NodeID=INVALID_ID)
    for name in ("EnvMap", "PointLight", "DirectionalLight", "DistantLight", "AnalyticAreaLight", "RectLight",
                 "DiscLight", "SphereLight", "GridVolume", "Grid", "SDFGrid", "Animation", "HairMaterial",
                 "ClothMaterial", "MERLMaterial", "PBRTDiffuseMaterial", "PBRTConductorMaterial",
                 "PBRTDielectricMaterial", "RGLMaterial", "SceneBuilderFlags", "Falcor"):
        ns[name] = _inert(name)
    return ns


def load_pyscene(path, builder: ingest.SceneBuilder | None = None) -> ingest.SceneBuilder:
    """Run a .pyscene script (the user's scene description, like Falcor's PythonImporter does)
    and return the populated rsd.ingest.SceneBuilder."""
    path = Path(path)
    sb = PySceneBuilder(builder)
    _SCRIPT_DIR.append(path.resolve().parent)
    try:
        code = compile(path.read_text(), str(path), "exec")
        exec(code, namespace(sb))  # noqa: S102 -- the importer's contract: the scene file is a script
    finally:
        _SCRIPT_DIR.pop()
    return sb.finish()


def load_scene_file(path, **kw) -> ingest.SceneBuilder:
    """.pyscene, .obj or .fbx by extension."""
    p = Path(path)
    if p.suffix.lower() == ".pyscene":
        return load_pyscene(p, **kw)
    if p.suffix.lower() == ".obj":
        return ingest.load_obj(p, **kw)
    if p.suffix.lower() == ".fbx":
        return fbx.load_fbx(p, **kw)
    raise NotImplementedError(f"{p.suffix}: no importer in this build (.pyscene, .obj, .fbx)")
