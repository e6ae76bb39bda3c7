"""CPU tests of the .pyscene importer (rsd/pyscene.py): Falcor's Transform
and TriangleMesh factories, material alpha-mode rules, the node hierarchy and importScene of an
OBJ, on the repository's own fixture scene (tests/fixtures/courtyard.pyscene); importScene of the
reference's binary FBX fixture (tests/fixtures/sphere.fbx)."""
import numpy as np
import pytest

from conftest import ROOT

FIX = ROOT / "tests" / "fixtures"


def test_transform_euler_and_order():
    from rsd.pyscene import Transform, float3
    # rotationEulerDeg (0, 90, 0): +x -> -z (right-handed rotation about y, QuaternionMath.h:398)
    M = Transform(translation=float3(1, 2, 3), rotationEulerDeg=float3(0, 90, 0)).matrix
    np.testing.assert_allclose(M @ [1, 0, 0, 1], [1, 2, 2, 1], atol=1e-6)
    # default order SRT: scale first, then rotate, then translate (Transform.cpp:89-91)
    M = Transform(translation=float3(0, 0, 5), scaling=2.0, rotationEulerDeg=float3(90, 0, 0)).matrix
    np.testing.assert_allclose(M @ [0, 1, 0, 1], [0, 0, 7, 1], atol=1e-6)
    from rsd.pyscene import CompositionOrder
    T = Transform(translation=float3(0, 0, 5), scaling=2.0, order=CompositionOrder.TRS).matrix  # S * T
    np.testing.assert_allclose(T @ [0, 0, 0, 1], [0, 0, 10, 1], atol=1e-6)


def test_transform_look_at():
    from rsd.pyscene import Transform, float3
    # forward -> -Z (quatFromLookAt, right-handed): looking down -z is the identity rotation
    M = Transform(position=float3(0, 0, 5), target=float3(0, 0, 0), up=float3(0, 1, 0)).matrix
    np.testing.assert_allclose(M[:3, :3], np.eye(3), atol=1e-6)
    np.testing.assert_allclose(M[:3, 3], [0, 0, 5])
    M = Transform(position=float3(0, 0, 0), target=float3(1, 0, 0), up=float3(0, 1, 0)).matrix
    np.testing.assert_allclose(M[:3, :3] @ [0, 0, -1], [1, 0, 0], atol=1e-6)


def test_triangle_mesh_factories():
    from rsd.pyscene import TriangleMesh, float2, float3
    q = TriangleMesh.createQuad(float2(2, 4))
    assert q.indices == [2, 1, 0, 1, 2, 3] and not q.frontFaceCW
    np.testing.assert_array_equal(q.vertices[0]["position"], [-1, 0, -2])
    assert TriangleMesh.createQuad(float2(-1, 1)).frontFaceCW  # TriangleMesh.cpp:61
    c = TriangleMesh.createCube(float3(1, 2, -3))
    assert len(c.vertices) == 24 and len(c.indices) == 36 and c.frontFaceCW
    np.testing.assert_array_equal(c.vertices[0]["position"], [-0.5, -1.0, 1.5])
    s = TriangleMesh.createSphere(2.0, 8, 4)
    assert len(s.vertices) == 9 * 5 and len(s.indices) == 8 * 4 * 6
    r = np.linalg.norm(np.array([v["position"] for v in s.vertices]), axis=1)
    np.testing.assert_allclose(r, 2.0, rtol=1e-6)
    d = TriangleMesh.createDisk(1.0, 6)
    assert len(d.vertices) == 7 and d.indices[-3:] == [0, 6, 1]
    m = TriangleMesh()
    a, b, cc = m.addVertex(float3(0, 0, 0), float3(0, 1, 0), float2(0, 0)), m.addVertex(
        float3(1, 0, 0), float3(0, 1, 0), float2(1, 0)), m.addVertex(float3(0, 0, 1), float3(0, 1, 0), float2(0, 1))
    m.addTriangle(a, b, cc)
    assert m.indices == [0, 1, 2]


def test_material_alpha_mode():
    """BasicMaterial::updateAlphaMode: Mask iff the alpha range minimum < threshold (float16)."""
    from rsd.pyscene import AlphaMode, StandardMaterial, float4
    m = StandardMaterial("m")
    assert m.alphaMode == AlphaMode.Opaque and m.alphaThreshold == 0.5
    m.baseColor = float4(1, 1, 1, 0.25)
    assert m.alphaMode == AlphaMode.Mask
    m.alphaThreshold = 0.2
    assert m.alphaMode == AlphaMode.Opaque
    m.alphaThreshold = 0.3
    assert m.alphaThreshold == float(np.float16(0.3)) and m.alphaMode == AlphaMode.Mask
    m.roughness = 0.4  # kept, not used
    assert m.roughness == 0.4


def test_material_base_color_texture(tmp_path):
    from rsd.pyscene import AlphaMode, MaterialTextureSlot, StandardMaterial
    from test_ingest import _png
    rgba = np.full((4, 4, 4), 255, np.uint8)
    rgba[0, 0, 3] = 10
    (tmp_path / "a.png").write_bytes(_png(rgba, [0, 1, 2, 4]))
    m = StandardMaterial("leaf")
    assert m.loadTexture(MaterialTextureSlot.BaseColor, str(tmp_path / "a.png"))
    assert m.alphaMode == AlphaMode.Mask and m._m.alpha_texture.shape == (4, 4)
    m.clearTexture(MaterialTextureSlot.BaseColor)
    assert m.alphaMode == AlphaMode.Opaque


def test_courtyard_scene():
    from rsd.pyscene import load_pyscene
    from rsd.scenes import FLAG_ALPHA_MASK, FLAG_DOUBLE_SIDED
    B = load_pyscene(FIX / "courtyard.pyscene")
    s = B.build("courtyard")
    # floor 2 + 3 pillars x 12 + sphere 12*8*2 + pane 2 + crate 12
    assert len(s.indices) == 2 + 36 + 192 + 2 + 12
    assert s.camera["pos"] == pytest.approx([0.5, 2.5, 7.0]) and s.camera["target"] == pytest.approx([0, 0.8, 0])
    # the floor: 8 x 8 quad at y = 0
    fl = s.positions[s.indices[:2].reshape(-1)]
    assert fl[:, 1].max() == 0 and fl[:, 0].min() == -4 and fl[:, 2].max() == 4
    # the pillars hang under the 'Pillars' node: x in {-2, 0, 2} +- 0.25, y in [0, 2]
    p = s.positions[s.indices[2:38].reshape(-1)]
    assert p[:, 1].min() == pytest.approx(0.0) and p[:, 1].max() == pytest.approx(2.0)
    assert sorted(set(np.round(p[:, 0], 4))) == [-2.25, -1.75, -0.25, 0.25, 1.75, 2.25]
    # every triangle ends counter-clockwise (unifyTriangleWinding), including the mirrored sphere:
    # outward geometric normals on the sphere
    sph = s.indices[38:38 + 192].astype(np.int64)
    v0, v1, v2 = (s.positions[sph[:, k]].astype(np.float64) for k in range(3))
    n = np.cross(v1 - v0, v2 - v0)
    centre = np.array([2.5, 0.6, 1.5])
    out = np.einsum("ij,ij->i", n, (v0 + v1 + v2) / 3 - centre)
    big = np.linalg.norm(n, axis=1) > 1e-6
    assert (out[big] > 0).all()
    # the glass pane: double-sided and alpha-masked (constant alpha 0.25 < 0.5)
    assert s.flags[230] & FLAG_DOUBLE_SIDED and s.flags[230] & FLAG_ALPHA_MASK
    # the OBJ crate, made double-sided by the script through getMaterial
    assert (s.flags[-12:] & FLAG_DOUBLE_SIDED).all() and not (s.flags[:230] & FLAG_DOUBLE_SIDED).any()
    assert s.alpha is not None and s.alpha.alphas[s.alpha.tri_material[230]] == pytest.approx(0.25)


def test_pyscene_errors(tmp_path):
    from rsd.pyscene import load_pyscene
    from rsd.fbx import FbxError
    (tmp_path / "a.pyscene").write_text("sceneBuilder.importScene('Bistro.fbx')\n")
    (tmp_path / "Bistro.fbx").write_bytes(b"Kaydara FBX Binary  \x00")  # a truncated binary FBX
    with pytest.raises(FbxError, match="malformed"):
        load_pyscene(tmp_path / "a.pyscene")
    (tmp_path / "d.pyscene").write_text("sceneBuilder.importScene('Bistro.gltf')\n")
    (tmp_path / "Bistro.gltf").write_text("{}")
    with pytest.raises(NotImplementedError, match="gltf"):
        load_pyscene(tmp_path / "d.pyscene")
    (tmp_path / "b.pyscene").write_text("sceneBuilder.importScene('missing.obj')\n")
    with pytest.raises(FileNotFoundError):
        load_pyscene(tmp_path / "b.pyscene")
    (tmp_path / "c.pyscene").write_text("sceneBuilder.addMeshInstance(3, 0)\n")
    with pytest.raises(ValueError):
        load_pyscene(tmp_path / "c.pyscene")


def test_pyscene_imports_fbx(tmp_path):
    """sceneBuilder.importScene('*.fbx') routes to rsd.fbx (AssimpImporter's role), and
    TriangleMesh.createFromFile reads it too."""
    import shutil
    from rsd.pyscene import TriangleMesh, load_pyscene
    shutil.copy(FIX / "sphere.fbx", tmp_path / "sphere.fbx")
    (tmp_path / "s.pyscene").write_text(
        "sceneBuilder.importScene('sphere.fbx')\n"
        "m = TriangleMesh.createFromFile('sphere.fbx')\n"
        "mat = StandardMaterial('m')\n"
        "mid = sceneBuilder.addTriangleMesh(m, mat)\n"
        "n = sceneBuilder.addNode('n', Transform(translation=float3(3, 0, 0)))\n"
        "sceneBuilder.addMeshInstance(n, mid)\n")
    s = load_pyscene(tmp_path / "s.pyscene").build("s")
    assert len(s.indices) == 2 * 760
    r0 = np.linalg.norm(s.positions[s.indices[:760].reshape(-1)].astype(np.float64), axis=1)
    r1 = np.linalg.norm(s.positions[s.indices[760:].reshape(-1)].astype(np.float64) - [3, 0, 0], axis=1)
    np.testing.assert_allclose(r0, 1.0, atol=2e-6)
    np.testing.assert_allclose(r1, 1.0, atol=4e-6)
