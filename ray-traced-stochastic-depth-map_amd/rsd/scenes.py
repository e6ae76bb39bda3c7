"""Seeded procedural stand-ins for the reference's benchmark scenes.

The reference benchmarks on Arcade, Sun Temple, Bistro Exterior and Emerald Square
(BASELINE.json configs).  Those assets are packman/ORCA downloads that are not in
the container (dependencies.xml:16-17), so every config uses a
deterministic procedural scene of comparable triangle count.  The scenes are
architectural on purpose: floors, walls, columns, stairs, boxes, spheres and
thin double-sided panels give the contact occlusion at AO radius 0.2 and the
depth complexity behind the first surface that the stochastic depth map exists
to capture.

A scene is a world-space triangle soup (Scene.cpp:2688-2830 flattens static
meshes the same way): positions float32[nv,3], indices uint32[nt,3] and one
flags word per triangle (bit0 double-sided -> TriangleFacingCullDisable,
bit1 front-face clockwise -> TriangleFrontCounterClockwise, Scene.cpp:3446-3452).
Winding is counter-clockwise seen from the front (Falcor's right-handed default).

Alpha-masked materials: with `alpha=True` the thin foliage cards become
alpha-masked (flag bit2, AlphaMode::Mask) and carry texture coordinates into procedural R8
leaf / lattice textures (AlphaMaterials); a few extra cards stand in the camera's view.
The geometry is otherwise identical to the opaque scene of the same name and seed.
"""
from __future__ import annotations

import dataclasses

import numpy as np

FLAG_DOUBLE_SIDED = 1
FLAG_FRONT_CW = 2
FLAG_ALPHA_MASK = 4


@dataclasses.dataclass
class AlphaMaterials:
    """rsd_alpha_desc in numpy: per-vertex texture coordinates, a material per triangle,
    per-material alpha threshold / constant alpha / texture, R8 textures (mip 0)."""
    texcoords: np.ndarray          # float32 [nv, 2]
    tri_material: np.ndarray       # uint32 [nt]
    thresholds: np.ndarray         # float32 [m]
    alphas: np.ndarray             # float32 [m]
    material_textures: np.ndarray  # uint32 [m], NO_TEXTURE = 0xffffffff
    textures: list                 # uint8 [h, w] each


NO_TEXTURE = 0xFFFFFFFF


def alpha_textures():
    """Procedural R8 alpha textures: 0 = leaves (soft-edged ellipses), 1 = lattice (bars),
    2 = a 3 x 5 odd-sized noise pattern (non-power-of-two mip chain)."""
    y, x = np.mgrid[0:64, 0:64].astype(np.float64) + 0.5
    leaf = np.zeros((64, 64))
    for cx, cy, rx, ry, a in ((20, 18, 14, 8, 0.5), (44, 40, 16, 7, -0.6), (18, 48, 9, 13, 0.2), (50, 12, 8, 6, 1.1)):
        c, s_ = np.cos(a), np.sin(a)
        u = ((x - cx) * c + (y - cy) * s_) / rx
        v = (-(x - cx) * s_ + (y - cy) * c) / ry
        leaf = np.maximum(leaf, np.clip((1.0 - (u * u + v * v)) * 3.0, 0.0, 1.0))
    y, x = np.mgrid[0:32, 0:32]
    lattice = np.where(((x % 8) < 2) | ((y % 8) < 3), 1.0, 0.0)
    noise = np.random.default_rng(77).integers(0, 256, (5, 3))
    return [np.round(leaf * 255).astype(np.uint8), np.round(lattice * 255).astype(np.uint8), noise.astype(np.uint8)]


# material table of the alpha scenes: (threshold, constant alpha, texture)
ALPHA_MATERIALS = [
    (0.5, 1.0, NO_TEXTURE),   # 0: opaque (everything that is not a card)
    (0.5, 1.0, 0),            # 1: leaves
    (0.5, 1.0, 1),            # 2: lattice
    (0.33, 1.0, 0),           # 3: leaves, threshold 0.33 (float16 0.33008)
    (0.5, 0.3, NO_TEXTURE),   # 4: constant alpha below the threshold: never visible
    (0.4, 1.0, 2),            # 5: odd-sized noise texture
]


@dataclasses.dataclass
class Scene:
    name: str
    positions: np.ndarray  # float32 [nv, 3]
    indices: np.ndarray    # uint32 [nt, 3]
    flags: np.ndarray      # uint32 [nt]
    camera: dict           # look-at camera: pos, target, up
    alpha: AlphaMaterials | None = None

    @property
    def triangle_count(self) -> int:
        return int(self.indices.shape[0])


class _Builder:
    def __init__(self):
        self.pos = []
        self.ind = []
        self.flg = []
        self.uv = []
        self.mat = []
        self.nv = 0

    def add(self, p, tri, flags=0, uv=None, mat=0):
        p = np.asarray(p, np.float32).reshape(-1, 3)
        tri = np.asarray(tri, np.int64).reshape(-1, 3) + self.nv
        self.pos.append(p)
        self.ind.append(tri.astype(np.uint32))
        self.flg.append(np.full(tri.shape[0], flags, np.uint32))
        self.uv.append(np.zeros((p.shape[0], 2), np.float32) if uv is None else np.asarray(uv, np.float32).reshape(-1, 2))
        self.mat.append(np.full(tri.shape[0], mat, np.uint32))
        self.nv += p.shape[0]

    def grid(self, origin, ex, ey, nx, ny, flags=0, uv_scale=None, uv_offset=(0.0, 0.0), mat=0):
        """Quad patch origin + s*ex + t*ey, nx*ny cells, CCW seen from ex x ey."""
        o, ex, ey = (np.asarray(v, np.float64) for v in (origin, ex, ey))
        s = np.linspace(0.0, 1.0, nx + 1)
        t = np.linspace(0.0, 1.0, ny + 1)
        S, T = np.meshgrid(s, t, indexing="xy")
        p = o + S[..., None] * ex + T[..., None] * ey
        i = np.arange((nx + 1) * (ny + 1)).reshape(ny + 1, nx + 1)
        a, b = i[:-1, :-1], i[:-1, 1:]
        c, d = i[1:, 1:], i[1:, :-1]
        tri = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
        uv = None
        if uv_scale is not None:
            uv = np.stack([S * uv_scale[0] + uv_offset[0], T * uv_scale[1] + uv_offset[1]], -1).reshape(-1, 2)
        self.add(p.reshape(-1, 3), tri, flags, uv, mat)

    def box(self, center, half, yaw=0.0, sub=1, flags=0):
        """Closed box with outward CCW faces, rotated by `yaw` about +y."""
        c = np.asarray(center, np.float64)
        h = np.asarray(half, np.float64)
        cy, sy = np.cos(yaw), np.sin(yaw)
        R = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
        faces = [  # (normal axis, sign)
            (0, 1), (0, -1), (1, 1), (1, -1), (2, 1), (2, -1)]
        for ax, sg in faces:
            u_ax, v_ax = (ax + 1) % 3, (ax + 2) % 3
            n = np.zeros(3); n[ax] = sg
            eu = np.zeros(3); eu[u_ax] = 2 * h[u_ax]
            ev = np.zeros(3); ev[v_ax] = 2 * h[v_ax]
            if sg < 0:
                eu, ev = ev, eu
            o = n * h - 0.5 * eu - 0.5 * ev
            s = np.linspace(0.0, 1.0, sub + 1)
            S, T = np.meshgrid(s, s, indexing="xy")
            p = o + S[..., None] * eu + T[..., None] * ev
            p = p.reshape(-1, 3) @ R.T + c
            i = np.arange((sub + 1) ** 2).reshape(sub + 1, sub + 1)
            a, b, cc, d = i[:-1, :-1], i[:-1, 1:], i[1:, 1:], i[1:, :-1]
            tri = np.concatenate([np.stack([a, b, cc], -1).reshape(-1, 3), np.stack([a, cc, d], -1).reshape(-1, 3)])
            self.add(p, tri, flags)

    def cylinder(self, base, radius, height, segs, rings, flags=0, caps=True):
        b = np.asarray(base, np.float64)
        ang = np.linspace(0.0, 2 * np.pi, segs, endpoint=False)
        ys = np.linspace(0.0, height, rings + 1)
        A, Y = np.meshgrid(ang, ys, indexing="xy")
        p = np.stack([radius * np.cos(A), Y, -radius * np.sin(A)], -1).reshape(-1, 3) + b
        i = np.arange((rings + 1) * segs).reshape(rings + 1, segs)
        j = np.roll(i, -1, axis=1)
        a, bb, c, d = i[:-1], j[:-1], j[1:], i[1:]
        tri = np.concatenate([np.stack([a, bb, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
        self.add(p, tri, flags)
        if caps:
            for y, up in ((height, True), (0.0, False)):
                ring = np.stack([radius * np.cos(ang), np.full(segs, y), -radius * np.sin(ang)], -1) + b
                ctr = b + np.array([0.0, y, 0.0])
                p = np.concatenate([ctr[None], ring])
                k = np.arange(segs)
                tri = np.stack([np.zeros(segs, np.int64), 1 + k, 1 + (k + 1) % segs], -1)
                if not up:
                    tri = tri[:, [0, 2, 1]]
                self.add(p, tri, flags)

    def sphere(self, center, radius, segs, rings, flags=0):
        c = np.asarray(center, np.float64)
        th = np.linspace(0.0, np.pi, rings + 1)
        ph = np.linspace(0.0, 2 * np.pi, segs, endpoint=False)
        TH, PH = np.meshgrid(th, ph, indexing="ij")
        p = np.stack([radius * np.sin(TH) * np.cos(PH), radius * np.cos(TH), -radius * np.sin(TH) * np.sin(PH)], -1)
        p = p.reshape(-1, 3) + c
        i = np.arange((rings + 1) * segs).reshape(rings + 1, segs)
        j = np.roll(i, -1, axis=1)
        a, b, cc, d = i[:-1], i[1:], j[1:], j[:-1]
        tri = np.concatenate([np.stack([a, b, cc], -1).reshape(-1, 3), np.stack([a, cc, d], -1).reshape(-1, 3)])
        # drop the degenerate pole triangles
        keep = (tri[:, 0] != tri[:, 1]) & (tri[:, 1] != tri[:, 2])
        self.add(p, tri[keep], flags)

    def build(self, name, camera, alpha=False):
        pos = np.concatenate(self.pos).astype(np.float32)
        ind = np.concatenate(self.ind).astype(np.uint32)
        flg = np.concatenate(self.flg).astype(np.uint32)
        am = None
        if alpha:
            m = np.array(ALPHA_MATERIALS, dtype=np.float64)
            am = AlphaMaterials(np.concatenate(self.uv).astype(np.float32), np.concatenate(self.mat).astype(np.uint32),
                                m[:, 0].astype(np.float32), m[:, 1].astype(np.float32),
                                np.array([t for _, _, t in ALPHA_MATERIALS], np.uint32), alpha_textures())
        return Scene(name, pos, ind, flg, camera, am)


def _card(B, arng, x, y, z, ex, ey, nx, ny):
    """An alpha-masked double-sided card (material, uv repeat and offset from `arng`)."""
    mat = int(arng.choice([1, 1, 2, 3, 4, 5]))
    rep = arng.uniform(0.5, 3.0, 2)
    off = arng.uniform(-2.0, 2.0, 2)
    B.grid((x, y, z), ex, ey, nx, ny, FLAG_DOUBLE_SIDED | FLAG_ALPHA_MASK, rep, off, mat)


def _architecture(rng, target_tris, room=(40.0, 12.0, 40.0), arng=None):
    """A hall with a tessellated floor/walls, colonnades, stairs and scattered props.
    Object counts scale so the triangle count lands near `target_tris`.  arng (alpha scenes):
    the generator of the cards' materials, separate so the geometry does not change."""
    B = _Builder()
    X, Y, Z = room
    scale = max(target_tris / 600_000.0, 0.02)
    g = int(np.clip(np.sqrt(target_tris * 0.05 / 2), 8, 900))
    # floor (facing up), ceiling (facing down), walls (facing inward)
    B.grid((-X / 2, 0.0, Z / 2), (X, 0, 0), (0, 0, -Z), g, g)
    B.grid((-X / 2, Y, -Z / 2), (X, 0, 0), (0, 0, Z), g // 2 + 1, g // 2 + 1)
    B.grid((-X / 2, 0.0, -Z / 2), (X, 0, 0), (0, Y, 0), g // 2 + 1, g // 4 + 1)
    B.grid((X / 2, 0.0, Z / 2), (-X, 0, 0), (0, Y, 0), g // 2 + 1, g // 4 + 1)
    B.grid((-X / 2, 0.0, Z / 2), (0, 0, -Z), (0, Y, 0), g // 2 + 1, g // 4 + 1)
    B.grid((X / 2, 0.0, -Z / 2), (0, 0, Z), (0, Y, 0), g // 2 + 1, g // 4 + 1)
    # colonnades along both long sides
    ncol = 10
    segs = int(np.clip(24 * np.sqrt(scale), 8, 96))
    rings = int(np.clip(30 * np.sqrt(scale), 2, 120))
    for side in (-1, 1):
        for k in range(ncol):
            z = -Z / 2 + (k + 0.5) * Z / ncol
            x = side * X * 0.32
            B.box((x, 0.25, z), (0.9, 0.25, 0.9), sub=max(1, segs // 8))
            B.cylinder((x, 0.5, z), 0.55, Y - 1.2, segs, rings)
            B.box((x, Y - 0.35, z), (0.9, 0.35, 0.9), sub=max(1, segs // 8))
    # stairs at the far end
    nsteps = 12
    for k in range(nsteps):
        B.box((0.0, 0.15 + 0.3 * k, -Z / 2 + 1.0 + 0.45 * (nsteps - k)), (5.0, 0.15, 0.45), sub=max(1, segs // 12))
    # scattered props: boxes, spheres, pillars, thin double-sided panels (foliage-like cards)
    total = sum(i.shape[0] for i in B.ind)
    sub_box = int(np.clip(np.sqrt(scale) * 6, 1, 16))
    sph_seg = int(np.clip(np.sqrt(scale) * 24, 8, 64))
    while total < target_tris:
        n0 = len(B.ind)
        kind = rng.integers(0, 4)
        x, z = rng.uniform(-X / 2 + 1.5, X / 2 - 1.5), rng.uniform(-Z / 2 + 1.5, Z / 2 - 1.5)
        if abs(x) < 2.5 + 0.15 * (Z * 0.42 - z) * (z > 0) and z > -Z * 0.2:
            continue  # keep the camera's view corridor clear
        if kind == 0:
            h = rng.uniform(0.1, 0.9, 3)
            B.box((x, h[1], z), h, yaw=rng.uniform(0, np.pi), sub=sub_box)
        elif kind == 1:
            r = rng.uniform(0.15, 0.8)
            B.sphere((x, r, z), r, sph_seg, sph_seg // 2)
        elif kind == 2:
            r = rng.uniform(0.05, 0.3)
            B.cylinder((x, 0.0, z), r, rng.uniform(0.5, 3.0), max(6, sph_seg // 2), max(1, sph_seg // 8))
        else:
            w, hh = rng.uniform(0.3, 1.2), rng.uniform(0.3, 1.5)
            yaw = rng.uniform(0, np.pi)
            ex = (w * np.cos(yaw), 0.0, -w * np.sin(yaw))
            if arng is None:
                B.grid((x, 0.05, z), ex, (0.0, hh, 0.0), max(1, sub_box // 2), max(1, sub_box // 2), FLAG_DOUBLE_SIDED)
            else:
                _card(B, arng, x, 0.05, z, ex, (0.0, hh, 0.0), max(1, sub_box // 2), max(1, sub_box // 2))
        total += sum(i.shape[0] for i in B.ind[n0:])
    if arng is not None:
        # foliage in the view corridor: cards of several sizes, some overlapping
        for k in range(24):
            x, z = arng.uniform(-3.0, 3.0), arng.uniform(-Z * 0.2, Z * 0.35)
            w, hh = arng.uniform(0.4, 2.0), arng.uniform(0.4, 2.5)
            yaw = arng.uniform(0, np.pi)
            _card(B, arng, x, arng.uniform(0.0, 1.5), z, (w * np.cos(yaw), 0.0, -w * np.sin(yaw)), (0.0, hh, 0.0), 2, 2)
    cam = {"pos": [0.0, 1.7, Z * 0.42], "target": [0.0, 1.2, -Z * 0.3], "up": [0.0, 1.0, 0.0]}
    return B, cam


_CONFIGS = {
    # name: (target triangles, seed)
    "arcade_tiny": (20_000, 1),
    "foliage_small": (20_000, 5),  # alpha-masked cards (SURVEY 8(f) row 3 tests)
    "suntemple": (600_000, 2),
    "bistro_exterior": (2_800_000, 3),
    "emerald_square": (10_000_000, 4),
}


def make_scene(name: str = "suntemple", target_tris: int | None = None, seed: int | None = None,
               alpha: bool | None = None) -> Scene:
    """Deterministic synthetic scene.  `name` picks the BASELINE config stand-in; alpha=True
    makes the foliage cards alpha-masked (default: only the "foliage_*" scenes)."""
    if name not in _CONFIGS:
        raise ValueError(f"unknown scene '{name}' (known: {sorted(_CONFIGS)})")
    t, s = _CONFIGS[name]
    target_tris = t if target_tris is None else int(target_tris)
    seed = s if seed is None else int(seed)
    rng = np.random.default_rng(seed)
    if alpha is None:
        alpha = name.startswith("foliage")
    arng = np.random.default_rng(seed + 1000) if alpha else None
    B, cam = _architecture(rng, target_tris, arng=arng)
    if name == "arcade_tiny":
        # the Arcade image tests' cube mesh (data/framework/meshes/cube.obj) as an extra prop
        B.box((0.0, 0.5, 6.0), (0.5, 0.5, 0.5))
    return B.build(name, cam, alpha)
