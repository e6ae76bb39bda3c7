"""CPU tests of the binary FBX reader (rsd/fbx.py, SURVEY 8(f) row 3 -- the reference's AssimpImporter path):
the reference's own FBX fixture (data/framework/meshes/sphere.fbx, copied to tests/fixtures as data) and FBX
files written by tests/fbx_writer.py for the container variants, triangulation, node transforms and
materials."""
import numpy as np
import pytest

from conftest import ROOT
import fbx_writer as W

FIX = ROOT / "tests" / "fixtures"


def _load(tmp_path, nodes, name="t.fbx", **kw):
    from rsd.fbx import load_fbx
    (tmp_path / name).write_bytes(W.write(nodes, **kw))
    return load_fbx(tmp_path / name)


def _tri_normals(s):
    p = s.positions.astype(np.float64)[s.indices.astype(np.int64)]
    return np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0]), p


def test_reference_sphere_fixture():
    """The reference's sphere.fbx (Maya, FBX 7500, zlib arrays): 20 x 20 segments -> 360 quads + 40 pole
    triangles = 760 triangles, every vertex on the unit sphere, every face counter-clockwise outward."""
    from rsd.fbx import load_fbx, parse
    raw = (FIX / "sphere.fbx").read_bytes()
    root = parse(raw)
    assert root.props[0] == 7500
    geo = root.first("Objects").first("Geometry")
    pvi = np.asarray(geo.first("PolygonVertexIndex").props[0])
    sizes = np.diff(np.concatenate([[0], np.flatnonzero(pvi < 0) + 1]))
    assert sorted(set(sizes.tolist())) == [3, 4] and (sizes == 4).sum() == 360 and (sizes == 3).sum() == 40
    B = load_fbx(FIX / "sphere.fbx")
    s = B.build("sphere")
    assert s.indices.shape == (760, 3)
    r = np.linalg.norm(s.positions.astype(np.float64), axis=1)
    np.testing.assert_allclose(r, 1.0, atol=1e-6)
    n, p = _tri_normals(s)
    assert (np.einsum("ij,ij->i", n, p.mean(1)) > 0).all()
    # the control points are exactly the file's doubles rounded to float32
    cp = np.asarray(geo.first("Vertices").props[0]).reshape(-1, 3).astype(np.float32)
    assert {tuple(v) for v in s.positions.tolist()} == {tuple(v) for v in cp.tolist()}
    # one Lambert material, opaque, single-sided; UVs flipped (aiProcess_FlipUVs) and split at the seam
    assert len(B.materials) == 1 and B.materials[0].name == "lambert1"
    assert not B.materials[0].alpha_mode_mask and not B.materials[0].double_sided
    assert len(s.positions) > len(cp) and s.flags.max() == 0


@pytest.mark.parametrize("version,compress", [(7400, False), (7500, True), (7300, True)])
def test_container_variants(tmp_path, version, compress):
    pos = [[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]]
    nodes = W.scene([W.mesh_geometry(10, pos, [[0, 1, 2, 3]]), W.model(20, "quad")], [(20, 0), (10, 20)])
    s = _load(tmp_path, nodes, version=version, compress=compress).build()
    assert s.indices.tolist() == [[0, 1, 2], [0, 2, 3]]
    np.testing.assert_array_equal(s.positions, np.asarray(pos, np.float32))


def test_triangulation(tmp_path):
    """aiProcess_Triangulate: a convex quad fans from corner 0, a concave quad from its concave corner, an
    n-gon fans from corner 0; a polygon's winding is kept."""
    from rsd.fbx import _triangulate
    sq = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]], np.float64)
    assert _triangulate(np.arange(4), sq) == [(0, 1, 2), (0, 2, 3)]
    dart = np.array([[0, 0, 0], [2, 1, 0], [4, 0, 0], [2, 3, 0]], np.float64)  # corner 1 is concave
    tris = _triangulate(np.arange(4), dart)
    assert tris == [(1, 2, 3), (1, 3, 0)]
    for t in tris:  # both triangles inside the dart, counter-clockwise like the polygon
        a, b, c = dart[list(t)]
        assert np.cross(b - a, c - a)[2] > 0
    assert _triangulate(np.arange(5), np.random.default_rng(0).random((5, 3))) == [(0, 1, 2), (0, 2, 3), (0, 3, 4)]
    pos = [[0, 0, 0], [1, 0, 0], [1.5, 1, 0], [0.5, 1.5, 0], [-0.5, 1, 0], [2, 2, 0], [3, 2, 0]]
    nodes = W.scene([W.mesh_geometry(10, pos, [[0, 1, 2, 3, 4], [1, 5, 6], [5, 6]]), W.model(20, "m")],
                    [(20, 0), (10, 20)])
    s = _load(tmp_path, nodes).build()
    assert len(s.indices) == 4  # 3 from the pentagon, 1 triangle; the 2-corner "polygon" is dropped


def _xf(tmp_path, point, **props):
    nodes = W.scene([W.mesh_geometry(10, [point, [0, 0, 0], [0, 0, 0]], [[0, 1, 2]]), W.model(20, "m", **props)],
                    [(20, 0), (10, 20)])
    return _load(tmp_path, nodes).build().positions[0].astype(np.float64)


def test_node_transforms(tmp_path):
    # scale, then rotate (+90 about y: x -> -z), then translate
    p = _xf(tmp_path, [1, 0, 0], Lcl_Translation=(1.0, 2.0, 3.0), Lcl_Rotation=(0.0, 90.0, 0.0),
            Lcl_Scaling=(2.0, 2.0, 2.0))
    np.testing.assert_allclose(p, [1, 2, 1], atol=1e-5)
    # RotationOrder: XYZ (x first) vs ZYX (z first, then y, then x)
    np.testing.assert_allclose(_xf(tmp_path, [0, 1, 0], Lcl_Rotation=(90.0, 90.0, 0.0)), [1, 0, 0], atol=1e-6)
    np.testing.assert_allclose(_xf(tmp_path, [0, 1, 0], Lcl_Rotation=(90.0, 90.0, 0.0), RotationOrder=5),
                               [0, 0, 1], atol=1e-6)
    # rotation about a pivot; PreRotation before the Lcl rotation; ScalingPivot
    np.testing.assert_allclose(_xf(tmp_path, [2, 0, 0], Lcl_Rotation=(0.0, 0.0, 90.0), RotationPivot=(1.0, 0.0, 0.0)),
                               [1, 1, 0], atol=1e-6)
    np.testing.assert_allclose(_xf(tmp_path, [1, 0, 0], PreRotation=(90.0, 0.0, 0.0), Lcl_Rotation=(0.0, 0.0, 90.0)),
                               [0, 0, 1], atol=1e-6)
    np.testing.assert_allclose(_xf(tmp_path, [3, 0, 0], Lcl_Scaling=(2.0, 1.0, 1.0), ScalingPivot=(1.0, 0.0, 0.0)),
                               [5, 0, 0], atol=1e-6)
    # PostRotation is inverted: Rpre(z 90) R(0) Rpost^-1(z 90) = identity
    np.testing.assert_allclose(_xf(tmp_path, [1, 2, 3], PreRotation=(0.0, 0.0, 90.0), PostRotation=(0.0, 0.0, 90.0)),
                               [1, 2, 3], atol=1e-6)


def test_hierarchy_and_geometric_transform(tmp_path):
    """World = parent world * local; a parent's geometric transform moves only its own geometry."""
    tri = [[0, 0, 0], [1, 0, 0], [0, 1, 0]]
    objs = [W.mesh_geometry(10, tri, [[0, 1, 2]]), W.mesh_geometry(11, tri, [[0, 1, 2]]),
            W.model(20, "parent", Lcl_Translation=(10.0, 0.0, 0.0), GeometricTranslation=(0.0, 5.0, 0.0)),
            W.model(21, "child", Lcl_Translation=(0.0, 0.0, 1.0), Lcl_Scaling=(3.0, 3.0, 3.0))]
    s = _load(tmp_path, W.scene(objs, [(20, 0), (21, 20), (10, 20), (11, 21)])).build()
    P = s.positions.astype(np.float64)
    np.testing.assert_allclose(P[s.indices[0]], [[10, 5, 0], [11, 5, 0], [10, 6, 0]], atol=1e-6)
    np.testing.assert_allclose(P[s.indices[1]], [[10, 0, 1], [13, 0, 1], [10, 3, 1]], atol=1e-6)


def test_mirrored_model_keeps_front_faces(tmp_path):
    """A negative scale mirrors the mesh; SceneBuilder's unifyTriangleWinding keeps it counter-clockwise."""
    tri = [[0, 0, 0], [1, 0, 0], [0, 1, 0]]  # +z normal
    objs = [W.mesh_geometry(10, tri, [[0, 1, 2]]), W.model(20, "m", Lcl_Scaling=(-1.0, 1.0, 1.0))]
    s = _load(tmp_path, W.scene(objs, [(20, 0), (10, 20)])).build()
    n, _ = _tri_normals(s)
    assert n[0, 2] > 0


def test_materials(tmp_path):
    from rsd.scenes import FLAG_ALPHA_MASK, FLAG_DOUBLE_SIDED
    pos = [[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [2, 0, 0], [2, 1, 0]]
    objs = [W.mesh_geometry(10, pos, [[0, 1, 2], [0, 2, 3], [1, 4, 5]], materials=[1, 0, 2]),
            W.model(20, "m"),
            W.material(30, "glass.doubleSided", Opacity=0.25),
            W.material(31, "leaf", TransparentColor=(1.0, 1.0, 1.0), TransparencyFactor=0.6),
            W.material(32, "stone")]
    # unset properties fall back to the Material template (Assimp's PropertyTable): TransparencyFactor 0 for
    # 'stone', which has no TransparentColor either, so its opacity stays 1
    B = _load(tmp_path, W.scene(objs, [(20, 0), (10, 20), (30, 20), (31, 20), (32, 20)],
                                templates={"Material": {"TransparencyFactor": 0.0}}))
    s = B.build()
    assert len(s.indices) == 3
    names = {m.name: m for m in B.materials}
    g, leaf, stone = names["glass.doubleSided"], names["leaf"], names["stone"]
    assert g.double_sided and g.alpha_mode_mask and g.alpha == pytest.approx(0.25)
    assert leaf.alpha == pytest.approx(0.4) and leaf.alpha_mode_mask and not leaf.double_sided
    assert stone.alpha == 1.0 and not stone.alpha_mode_mask
    # one mesh per (geometry, material): polygon 0 -> leaf, 1 -> glass, 2 -> stone
    fl = {tuple(sorted(map(tuple, s.positions[t].tolist()))): int(f) for t, f in zip(s.indices, s.flags)}
    assert fl[((0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (1.0, 1.0, 0.0))] == FLAG_ALPHA_MASK
    assert fl[((0.0, 0.0, 0.0), (0.0, 1.0, 0.0), (1.0, 1.0, 0.0))] == FLAG_ALPHA_MASK | FLAG_DOUBLE_SIDED
    assert fl[((1.0, 0.0, 0.0), (2.0, 0.0, 0.0), (2.0, 1.0, 0.0))] == 0
    assert s.alpha is not None


def test_template_defaults(tmp_path):
    """An unset Properties70 value falls back to the Definitions template of the object type."""
    objs = [W.mesh_geometry(10, [[1, 0, 0], [0, 0, 0], [0, 0, 0]], [[0, 1, 2]]), W.model(20, "m")]
    s = _load(tmp_path, W.scene(objs, [(20, 0), (10, 20)], templates={"Model": {"Lcl_Translation": (0.0, 7.0, 0.0)}}))
    np.testing.assert_allclose(s.build().positions[0], [1, 7, 0])


def test_uvs_flipped_and_split(tmp_path):
    pos = [[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]]
    uv = [[0, 0], [1, 0], [1, 1], [0, 0], [1, 1], [0, 1]]  # corner 0 appears twice with the same uv
    nodes = W.scene([W.mesh_geometry(10, pos, [[0, 1, 2], [0, 2, 3]], uv=uv), W.model(20, "m")], [(20, 0), (10, 20)])
    B = _load(tmp_path, nodes)
    m = B.meshes[0]
    assert len(m.positions) == 4  # identical (position, uv) polygon vertices joined
    np.testing.assert_allclose(m.texcoords[m.indices[0]], [[0, 1], [1, 1], [1, 0]])  # v -> 1 - v


def test_errors(tmp_path):
    from rsd.fbx import FbxError, load_fbx
    (tmp_path / "a.fbx").write_bytes(b"; FBX 7.4.0 project file\n")
    with pytest.raises(FbxError, match="ASCII"):
        load_fbx(tmp_path / "a.fbx")
    nodes = W.scene([W.mesh_geometry(10, [[0, 0, 0]] * 3, [[0, 1, 7]]), W.model(20, "m")], [(20, 0), (10, 20)])
    with pytest.raises(FbxError, match="out of range"):
        _load(tmp_path, nodes)
    good = W.write(W.scene([W.mesh_geometry(10, [[0, 0, 0]] * 3, [[0, 1, 2]]), W.model(20, "m")], [(20, 0), (10, 20)]))
    (tmp_path / "t.fbx").write_bytes(good[:len(good) // 2])
    with pytest.raises(FbxError):
        load_fbx(tmp_path / "t.fbx")
