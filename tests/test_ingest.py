"""CPU tests of scene ingest: OBJ/MTL parsing, SceneBuilder flattening
(world transform, winding unification after mirroring, material flags) and the image readers
used for alpha textures.  The OBJ/PNG inputs are written by the tests themselves."""
import struct
import zlib

import numpy as np
import pytest

F = np.float32

CUBE_OBJ = """# unit cube, quads, counter-clockwise seen from outside
o Box
v -1 -1 -1
v  1 -1 -1
v  1  1 -1
v -1  1 -1
v -1 -1  1
v  1 -1  1
v  1  1  1
v -1  1  1
vt 0 0
vt 1 0
vt 1 1
vt 0 1
f 1/1 4/4 3/3 2/2
f 5/1 6/2 7/3 8/4
f 1/1 2/2 6/3 5/4
f 4/4 8/1 7/2 3/3
f 1/1 5/2 8/3 4/4
f 2/1 3/2 7/3 6/4
"""

AXES = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]


def _front_hits(oracle, scene, center=(0.0, 0.0, 0.0)):
    """For rays from outside along each axis toward `center`: (hit, det > 0) of the nearest hit."""
    out = []
    for a in AXES:
        o = np.array(center) + 5.0 * np.array(a, np.float64) + np.array([0.13, 0.21, 0.17]) * (1 - np.abs(a))
        d = -np.array(a, np.float64)
        best = None
        for tri in scene.indices:
            v = scene.positions[tri]
            hit, t, _, _, det = oracle.intersect(o.tolist(), d.tolist(), v[0].tolist(), v[1].tolist(), v[2].tolist())
            if hit and (best is None or t < best[0]):
                best = (t, det)
        out.append(best)
    return out


def test_obj_cube_faces_outward(oracle, tmp_path):
    from rsd.ingest import load_obj
    (tmp_path / "cube.obj").write_text(CUBE_OBJ)
    s = load_obj(tmp_path / "cube.obj").build("cube")
    assert s.triangle_count == 12 and s.positions.shape[1] == 3
    assert s.alpha is None and (s.flags == 0).all()
    for h in _front_hits(oracle, s):
        assert h is not None and h[1] > 0 and abs(h[0] - 4.0) < 1e-5


@pytest.mark.parametrize("mirror", [(1, 1, 1), (-1, 1, 1), (1, -1, -1), (-1, -1, -1)])
def test_mirrored_instances_keep_front_faces_outward(oracle, tmp_path, mirror):
    """A mirroring transform flips the winding flag, and unifyTriangleWinding then swaps the
    first two indices (SceneBuilder.cpp:1601-1603, 1655-1725): front faces stay outward."""
    from rsd.ingest import load_obj
    (tmp_path / "cube.obj").write_text(CUBE_OBJ)
    T = np.diag([*mirror, 1.0]).astype(F)
    T[:3, 3] = (3.0, -2.0, 0.5)
    s = load_obj(tmp_path / "cube.obj", transform=T).build()
    for h in _front_hits(oracle, s, center=(3.0, -2.0, 0.5)):
        assert h is not None and h[1] > 0


def test_builder_instances_and_flags():
    from rsd.ingest import Material, Mesh, SceneBuilder
    from rsd.scenes import FLAG_ALPHA_MASK, FLAG_DOUBLE_SIDED, NO_TEXTURE
    B = SceneBuilder()
    m0 = B.add_material(Material("opaque"))
    m1 = B.add_material(Material("leaf", double_sided=True, alpha_mode_mask=True, alpha_threshold=0.3,
                                 alpha_texture=np.full((4, 4), 200, np.uint8)))
    m2 = B.add_material(Material("glass", alpha_mode_mask=True, alpha=0.2))
    quad = Mesh(np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]], F), np.array([[0, 1, 2], [0, 2, 3]]),
                np.array([[0, 0], [1, 0], [1, 1], [0, 1]], F))
    ids = []
    for mat in (m0, m1, m2):
        q = Mesh(quad.positions, quad.indices, quad.texcoords, mat)
        ids.append(B.add_mesh(q))
    B.add_instance(ids[0])
    T = np.eye(4, dtype=F)
    T[:3, 3] = (0, 0, -2)
    B.add_instance(ids[1], T)
    B.add_instance(ids[1], np.diag([2, 2, 2, 1]).astype(F))
    B.add_instance(ids[2])
    s = B.build("quads")
    assert s.triangle_count == 8 and len(s.positions) == 16
    assert s.flags.tolist() == [0, 0] + [FLAG_DOUBLE_SIDED | FLAG_ALPHA_MASK] * 4 + [FLAG_ALPHA_MASK] * 2
    assert np.allclose(s.positions[4:8, 2], -2.0) and np.allclose(s.positions[8:12].max(0), [2, 2, 0])
    a = s.alpha
    assert a.tri_material.tolist() == [0, 0, 1, 1, 1, 1, 2, 2]
    assert a.material_textures.tolist() == [NO_TEXTURE, 0, NO_TEXTURE] and len(a.textures) == 1
    assert np.allclose(a.thresholds, [0.5, 0.3, 0.5]) and np.allclose(a.alphas, [1.0, 1.0, 0.2])
    assert a.texcoords.shape == (16, 2)


def _png(img, filters):
    """A minimal PNG encoder (RGBA/grey, 8-bit) using the given per-row filter types."""
    h, w, c = img.shape
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[c]
    rows = []
    prev = np.zeros(w * c, np.int32)
    for y in range(h):
        line = img[y].reshape(-1).astype(np.int32)
        f = filters[y % len(filters)]
        left = np.concatenate([np.zeros(c, np.int32), line[:-c]])
        upleft = np.concatenate([np.zeros(c, np.int32), prev[:-c]])
        if f == 0:
            enc = line
        elif f == 1:
            enc = line - left
        elif f == 2:
            enc = line - prev
        elif f == 3:
            enc = line - ((left + prev) >> 1)
        else:
            p = left + prev - upleft
            pa, pb, pc = np.abs(p - left), np.abs(p - prev), np.abs(p - upleft)
            pr = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, upleft))
            enc = line - pr
        rows.append(bytes([f]) + (enc & 255).astype(np.uint8).tobytes())
        prev = line

    def chunk(k, b):
        return struct.pack(">I", len(b)) + k + b + struct.pack(">I", zlib.crc32(k + b) & 0xffffffff)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(b"".join(rows))) + chunk(b"IEND", b""))


@pytest.mark.parametrize("channels", [1, 2, 3, 4])
def test_png_decoder_all_filters(tmp_path, channels):
    from rsd.ingest import read_image
    img = np.random.default_rng(channels).integers(0, 256, (9, 7, channels)).astype(np.uint8)
    (tmp_path / "t.png").write_bytes(_png(img, [0, 1, 2, 3, 4]))
    assert np.array_equal(read_image(tmp_path / "t.png"), img)


def test_pgm_reader(tmp_path):
    from rsd.ingest import read_image
    img = np.arange(12, dtype=np.uint8).reshape(3, 4) * 20
    (tmp_path / "a.pgm").write_bytes(b"P5\n# comment\n4 3\n255\n" + img.tobytes())
    (tmp_path / "b.pgm").write_text("P2\n4 3\n255\n" + " ".join(map(str, img.ravel())) + "\n")
    assert np.array_equal(read_image(tmp_path / "a.pgm")[..., 0], img)
    assert np.array_equal(read_image(tmp_path / "b.pgm")[..., 0], img)


def _foliage_obj(tmp_path):
    """A ground quad and a leaf card in front of it; the card's map_d is a checkerboard."""
    tex = (np.indices((16, 16)).sum(0) // 4 % 2 * 255).astype(np.uint8)
    (tmp_path / "leaf.pgm").write_bytes(b"P5\n16 16\n255\n" + tex.tobytes())
    (tmp_path / "scene.mtl").write_text("newmtl ground\nKd 0.5 0.5 0.5\n\nnewmtl leaf\nmap_d leaf.pgm\n")
    (tmp_path / "scene.obj").write_text(
        "mtllib scene.mtl\n"
        "v -5 -5 0\nv 5 -5 0\nv 5 5 0\nv -5 5 0\n"
        "v -2 -2 2\nv 2 -2 2\nv 2 2 2\nv -2 2 2\n"
        "vt 0 0\nvt 2 0\nvt 2 2\nvt 0 2\n"
        "g ground\nusemtl ground\nf 1 2 3 4\n"
        "g card\nusemtl leaf\nf 5/1 6/2 7/3 8/4\n")
    return tex


def test_obj_alpha_material_cuts_holes(oracle, tmp_path):
    from rsd.ingest import load_obj
    _foliage_obj(tmp_path)
    B = load_obj(tmp_path / "scene.obj", double_sided={"leaf"})
    B.set_camera((0, 0, 10), (0, 0, 0))
    s = B.build("foliage")
    assert s.alpha is not None and s.alpha.textures[0].shape == (16, 16)
    assert s.flags.tolist() == [0, 0, 5, 5]
    sc = oracle.Scene(s.positions, s.indices, s.flags, s.alpha)
    cam = oracle.camera_look_at(s.camera["pos"], s.camera["target"], s.camera["up"], aspect=1.0)
    z, _ = oracle.gbuffer(sc, cam, 64, 64)
    zo, _ = oracle.gbuffer(oracle.Scene(s.positions, s.indices, s.flags), cam, 64, 64)
    card = np.isclose(zo, 8.0, atol=1e-3)
    assert card.sum() > 500
    holes = card & np.isclose(z, 10.0, atol=1e-3)
    assert 0.3 < holes.sum() / card.sum() < 0.7  # about half of the checkerboard is cut away
