"""The render-graph host (include/rsd_graph.h, csrc/host/) on the CPU: script loading,
the plugin registry, graph planning (culling, execution order, resource table) and error
behaviour.  No device work: graphs are planned, not compiled (rsd_graph_plan)."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import PKG as PKG_DIR, ROOT

rsdgraph = pytest.importorskip("rsd.graph")
from rsd import abi  # noqa: E402

SCRIPT = ROOT / "tests" / "graphs" / "svao_hotpath.py"
REF_SCRIPTS = Path("/root/reference/scripts")
FB = (192, 128)  # visible 160 x 96 + 2 x 16 guard band


def hotpath():
    return rsdgraph.load_script(SCRIPT)["SVAOHotPath"]


def test_builtin_pass_types():
    assert {"GuardBand", "GBufferRaster", "LinearizeDepth", "CompressNormals", "StochasticDepthMapRT",
            "SVAO"} <= set(rsdgraph.plugin_types())


def test_script_load_and_plan():
    g = hotpath()
    assert g.counts() == (7, 8)
    g.plan(*FB)
    # the ToneMapper stub feeds no output and is culled (RenderGraphCompiler.cpp:121-172)
    assert g.execution_order() == ["GuardBand", "GBufferRaster", "LinearizeDepth", "CompressNormals", "SVAO",
                                   "Blur"]
    res = g.resources()
    assert res["GBufferRaster.depth"] == (FB[0], FB[1], 1, "R32Float")
    assert res["GBufferRaster.faceNormalW"] == (FB[0], FB[1], 1, "RGBA32Float")
    assert res["LinearizeDepth.linearDepth"] == (FB[0], FB[1], 1, "R32Float")
    assert res["CompressNormals.normalOut"] == (FB[0], FB[1], 1, "R16Uint")
    assert res["SVAO.ao"] == (FB[0], FB[1], 1, "R8Unorm")
    assert res["SVAO.stencil"] == (FB[0], FB[1], 1, "R8Uint")
    # SD map = ceil(fb / divisor) + 2 * (64 px guard / divisor)   (SVAO.cpp:700-723)
    sd = ((FB[0] + 1) // 2 + 64, (FB[1] + 1) // 2 + 64)
    assert res["SVAO.internalRayMin"] == (sd[0], sd[1], 1, "R32Uint")
    assert res["SVAO.internalRayMax"] == (sd[0], sd[1], 1, "R32Uint")
    # CrossBilateralBlur is a real pass now: R8Unorm like the reference
    assert res["Blur.colorOut"] == (FB[0], FB[1], 1, "R8Unorm")
    assert "Unused.dst" not in res


def test_script_as_code_through_falcor_module():
    ns = {}
    exec(compile(SCRIPT.read_text(), str(SCRIPT), "exec"), ns)  # our own script
    g = ns["SVAOHotPath"]
    assert g.counts() == (7, 8)
    assert type(g).__module__ == "rsd.graph"


@pytest.mark.skipif(not REF_SCRIPTS.is_dir(), reason="reference scripts not present (GPU box)")
@pytest.mark.parametrize("name", ["SVAO.py", "SVAO_small.py", "SVAO_debugsd.py"])
def test_reference_svao_scripts_plan(name):
    """The reference's SVAO graphs load unchanged (read, not executed) and plan."""
    graphs = rsdgraph.load_script(REF_SCRIPTS / name)
    g = graphs["SVAO"]
    g.plan(1920 + 128, 1080 + 128)
    order = g.execution_order()
    for p in ("GuardBand", "GBufferRaster", "LinearizeDepth", "CompressNormals", "SVAO"):
        assert p in order
    assert order.index("GuardBand") < order.index("GBufferRaster") < order.index("LinearizeDepth") < \
        order.index("SVAO")
    assert order.index("CompressNormals") < order.index("SVAO")
    res = g.resources()
    assert res["SVAO.internalRayMax"][:2] == (768, 558)  # 1080p, divisor 4, 512 px SD guard band
    if name == "SVAO.py":
        # the AO chain to the marked output AmbientRef.out runs real passes:
        # SVAO.ao -> CrossBilateralBlur -> TemporalAO (disabled) -> Switch -> ImageEquation
        for p in ("CrossBilateralBlur0", "TemporalAO", "AOSwitch", "AmbientRef"):
            assert p in order
        assert res["AOSwitch.out"] == (2048, 1208, 1, "R8Unorm")  # shaped like the selected input
        assert res["AmbientRef.out"] == (2048, 1208, 1, "RGBA32Float")


@pytest.mark.skipif(not REF_SCRIPTS.is_dir(), reason="reference scripts not present (GPU box)")
def test_reference_raytraced_svao_script_plans():
    """SAVO_record.py: two SVAO passes in the Raytraced secondary mode."""
    g = next(iter(rsdgraph.load_script(REF_SCRIPTS / "SAVO_record.py").values()))
    g.plan(1920 + 128, 1080 + 128)
    order = g.execution_order()
    assert "SVAO" in order and "SVAO_ref" in order
    # no SD guard band outside the StochasticDepth mode (SVAO.cpp:718-723): divisor 1 -> frame size
    assert g.resources()["SVAO.internalRayMax"][:2] == (2048, 1208)


@pytest.mark.skipif(not REF_SCRIPTS.is_dir(), reason="reference scripts not present (GPU box)")
def test_reference_dual_depth_svao_plans():
    """scripts/SVAO_depth.py: SVAO with primaryDepthMode DualDepth (the second layer from DepthSelect) next
    to the Raytraced reference pass -- both SVAO modes are built since round 4, so the graph plans."""
    g = next(iter(rsdgraph.load_script(REF_SCRIPTS / "SVAO_depth.py").values()))
    g.plan(1920 + 128, 1080 + 128)


def test_graph_errors():
    g = rsdgraph.RenderGraph("errors")
    g.create_pass("A", "LinearizeDepth", {})
    with pytest.raises(abi.RsdError, match="exists"):
        g.create_pass("A", "LinearizeDepth", {})
    with pytest.raises(abi.RsdError, match="unknown pass"):
        g.add_edge("A.linearDepth", "B.depth")
    with pytest.raises(abi.RsdError, match="pass.field"):
        g.mark_output("A")
    # required input not connected
    g.mark_output("A.linearDepth")
    with pytest.raises(abi.RsdError, match="required input 'A.depth'"):
        g.plan(64, 64)
    # edges to a field a built-in pass does not declare
    g.create_pass("B", "LinearizeDepth", {})
    g.add_edge("B.linearDepth", "A.notAField")
    with pytest.raises(abi.RsdError, match="no input 'notAField'"):
        g.plan(64, 64)


def test_graph_cycle():
    g = rsdgraph.RenderGraph("cycle")
    g.create_pass("A", "Foo", {})
    g.create_pass("B", "Foo", {})
    g.add_edge("A.x", "B.y")
    g.add_edge("B.z", "A.w")
    g.mark_output("B.z")
    with pytest.raises(abi.RsdError, match="cycle"):
        g.plan(8, 8)


def test_property_errors():
    g = rsdgraph.RenderGraph("props")
    with pytest.raises(abi.RsdError, match="unknown value 'Sideways'"):
        g.create_pass("G", "GBufferRaster", {"forceCullMode": True, "cull": "Sideways"})
    with pytest.raises(abi.RsdError) as e:
        g.create_pass("S", "StochasticDepthMapRT", {"StoreNormals": True})
    assert e.value.status == 2  # StochasticDepthMapRT.cpp:198-203 throws for StoreNormals
    with pytest.raises(abi.RsdError, match="not a number"):
        g.create_pass("T", "StochasticDepthMapRT", {"SampleCount": "four"})
    with pytest.raises(abi.RsdError) as e:
        g.create_pass("C", "CompressNormals", {"use16Bit": False})
    assert e.value.status == 2


def test_sd_pass_reflection():
    for n, fmt, layers in [(1, "R32Float", 1), (2, "RG32Float", 1), (4, "RGBA32Float", 1), (8, "RGBA32Float", 2),
                           (16, "RGBA32Float", 4)]:
        g = rsdgraph.RenderGraph("sd")
        g.create_pass("SD", "StochasticDepthMapRT", {"SampleCount": n})
        g.create_pass("Z", "Source", {})
        g.add_edge("Z.z", "SD.linearZ")
        g.mark_output("SD.stochasticDepth")
        g.plan(100, 60)
        assert g.resources()["SD.stochasticDepth"] == (100, 60, layers, fmt)
        # the producer of linearZ (a stub) takes the consumer's declared format
        assert g.resources()["Z.z"][3] == "R32Float"


def test_plugin_dlopen(tmp_path):
    """A pass type unknown to librsd is loaded from <plugin dir>/<Type>.so."""
    so = tmp_path / "ConstantDepth.so"
    cmd = ["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           f"-I{PKG_DIR / 'csrc' / 'host'}", str(ROOT / "tests" / "plugins" / "ConstantDepth.cpp"), "-o", str(so)]
    subprocess.run(cmd, check=True, timeout=300)
    assert "ConstantDepth" not in rsdgraph.plugin_types()
    rsdgraph.set_plugin_dir(tmp_path)
    try:
        g = rsdgraph.RenderGraph("plugin")
        g.create_pass("C", "ConstantDepth", {"value": 0.5})
        g.create_pass("L", "LinearizeDepth", {})
        g.add_edge("C.depth", "L.depth")
        g.mark_output("L.linearDepth")
        g.plan(32, 16)
        assert g.execution_order() == ["C", "L"]
        assert g.resources()["C.depth"] == (32, 16, 1, "R32Float")
        assert "ConstantDepth" in rsdgraph.plugin_types()
    finally:
        rsdgraph.set_plugin_dir("")


def test_graph_header_exports():
    """include/rsd_graph.h declares exactly abi.GRAPH_EXPORTS and librsd exports them."""
    import re
    hdr = (ROOT / "include" / "rsd_graph.h").read_text()
    declared = set(re.findall(r"^(?:rsd_status|void)\s+(rsd_\w+)\(", hdr, re.M))
    assert declared == set(abi.GRAPH_EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", str(abi.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (rsd_\w+)$", out, re.M))
    assert set(abi.GRAPH_EXPORTS) <= exported
    assert os.path.getsize(abi.LIB_PATH) > 0


@pytest.mark.parametrize("N,use16,fmt,layers", [(1, False, "R32Float", 1), (4, False, "RGBA32Float", 1),
                                                (8, False, "RGBA32Float", 2), (16, False, "RGBA32Float", 4),
                                                (1, True, "R16Float", 1), (2, True, "RG16Float", 1),
                                                (4, True, "RGBA16Float", 1)])
def test_sd_pass_output_format(N, use16, fmt, layers):
    """StochasticDepthMapRT::reflect (StochasticDepthMapRT.cpp:177-216): 32-bit or, with Use16Bit,
    16-bit float maps; N = 8 is two RGBA layers (16: four, librsd's extension)."""
    g = rsdgraph.RenderGraph("sd")
    g.create_pass("SD", "StochasticDepthMapRT", {"SampleCount": N, "Use16Bit": use16, "HitOrder": "Traversal"})
    g.mark_output("SD.stochasticDepth")
    z = np.zeros((32, 64), np.float32)  # planned only: never read (no device work)
    g.set_input("SD.linearZ", z.ctypes.data, 64, 32, abi.FMT_R32F)
    g.plan(64, 32)
    assert g.resources()["SD.stochasticDepth"] == (64, 32, layers, fmt)
    g.close()


@pytest.mark.parametrize("N,use16", [(8, True), (3, False)])
def test_sd_pass_refuses_like_the_reference(N, use16):
    """StochasticDepthMapRT.cpp:190,199: unsupported sample counts throw."""
    g = rsdgraph.RenderGraph("sd")
    g.create_pass("SD", "StochasticDepthMapRT", {"SampleCount": N, "Use16Bit": use16})
    g.mark_output("SD.stochasticDepth")
    z = np.zeros((32, 64), np.float32)
    g.set_input("SD.linearZ", z.ctypes.data, 64, 32, abi.FMT_R32F)
    with pytest.raises(abi.RsdError):
        g.plan(64, 32)
    g.close()


@pytest.mark.parametrize("fmt,name", [(abi.FMT_R32F, "R32Float"), (abi.FMT_RG32F, "RG32Float"),
                                      (abi.FMT_RGBA32F, "RGBA32Float"), (abi.FMT_R16U, "R16Uint"),
                                      (abi.FMT_R8U, "R8Uint"), (abi.FMT_R8UNORM, "R8Unorm"),
                                      (abi.FMT_R32U, "R32Uint"), (abi.FMT_R16F, "R16Float"),
                                      (abi.FMT_RG16F, "RG16Float"), (abi.FMT_RGBA16F, "RGBA16Float"),
                                      (abi.FMT_RG8UNORM, "RG8Unorm")])
def test_graph_input_format_round_trip(fmt, name):
    """rsd_graph_set_input accepts every real rsd_format (dualAO's RG8Unorm included); a Switch
    output takes the format of its external input (Switch.cpp:95-108)."""
    g = rsdgraph.RenderGraph("fmt")
    g.create_pass("S", "Switch", {"count": 1, "selected": 0})
    g.mark_output("S.out")
    buf = np.zeros(32 * 64 * 16, np.uint8)  # planned only: never read
    g.set_input("S.i0", buf.ctypes.data, 64, 32, fmt)
    g.plan(64, 32)
    assert g.resources()["S.out"] == (64, 32, 1, name)
    g.close()


@pytest.mark.parametrize("fmt", [abi.FMT_UNKNOWN, abi.FMT_RG8UNORM + 1, 255])
def test_graph_input_refuses_unknown_formats(fmt):
    g = rsdgraph.RenderGraph("fmt")
    g.create_pass("S", "Switch", {"count": 1, "selected": 0})
    buf = np.zeros(16, np.uint8)
    with pytest.raises(abi.RsdError):
        g.set_input("S.i0", buf.ctypes.data, 2, 2, fmt)
    g.close()


def test_optional_mvec_allocated_only_when_read():
    """GBuffer.cpp:48: mvec is an optional channel -- a graph that does not read it allocates no
    mvec (and GBufferRaster launches no motion-vector kernels); one that reads it gets RG32Float."""
    g = rsdgraph.RenderGraph("gb")
    g.create_pass("GBufferRaster", "GBufferRaster", {})
    g.mark_output("GBufferRaster.depth")
    g.plan(64, 32)
    assert "GBufferRaster.mvec" not in g.resources() and "GBufferRaster.depth" in g.resources()
    g.close()
    g = rsdgraph.RenderGraph("gb")
    g.create_pass("GBufferRaster", "GBufferRaster", {})
    g.mark_output("GBufferRaster.mvec")
    g.plan(64, 32)
    assert g.resources()["GBufferRaster.mvec"] == (64, 32, 1, "RG32Float")
    g.close()


def test_temporal_ao_enabled_plans():
    """TemporalAO enabled (TemporalAO.cpp:92-103): linearZ and mvec become required inputs;
    GBufferRaster declares mvec (RG32Float)."""
    g = rsdgraph.load_script(ROOT / "tests" / "graphs" / "svao_temporal.py")["SVAOTemporal"]
    g.plan(*FB)
    order = g.execution_order()
    assert order.index("GBufferRaster") < order.index("TemporalAO") and order.index("SVAO") < order.index("TemporalAO")
    res = g.resources()
    assert res["GBufferRaster.mvec"] == (FB[0], FB[1], 1, "RG32Float")
    assert res["TemporalAO.aoOut"] == (FB[0], FB[1], 1, "R8Unorm")
    h = rsdgraph.RenderGraph("tao")
    h.create_pass("GBufferRaster", "GBufferRaster", {})
    h.create_pass("TemporalAO", "TemporalAO", {"enabled": True})
    h.add_edge("GBufferRaster.mvec", "TemporalAO.aoIn")
    h.mark_output("TemporalAO.aoOut")
    with pytest.raises(abi.RsdError, match="required input 'TemporalAO.linearZ'"):
        h.plan(*FB)
    d = rsdgraph.RenderGraph("tao_off")  # disabled: a pass-through needing only aoIn
    d.create_pass("GBufferRaster", "GBufferRaster", {})
    d.create_pass("TemporalAO", "TemporalAO", {"enabled": False})
    d.add_edge("GBufferRaster.mvec", "TemporalAO.aoIn")
    d.mark_output("TemporalAO.aoOut")
    d.plan(*FB)


def test_ray_min_max_length_plan():
    """RayMinMaxLength (RayMinMaxLength.cpp:55-70): R32Float `len` at the interval maps' size."""
    g = hotpath()
    g.create_pass("RayMinMaxLength", "RayMinMaxLength", {})
    g.add_edge("SVAO.internalRayMin", "RayMinMaxLength.kRayMin")
    g.add_edge("SVAO.internalRayMax", "RayMinMaxLength.kRayMax")
    g.mark_output("RayMinMaxLength.len")
    g.plan(*FB)
    res = g.resources()
    sd = ((FB[0] + 1) // 2 + 64, (FB[1] + 1) // 2 + 64)
    assert res["RayMinMaxLength.len"] == (sd[0], sd[1], 1, "R32Float")
    assert g.execution_order()[-1] == "RayMinMaxLength"


def test_deinterleave_shapes_plan():
    """DeinterleaveTexture (DeinterleaveTexture.cpp:80-125): 16 layers of ceil(w/4) x ceil(h/4) in
    the input's format; InterleaveTexture: the input's format at the default size."""
    g = rsdgraph.RenderGraph("dei")
    g.create_pass("GBufferRaster", "GBufferRaster", {})
    g.create_pass("LinearizeDepth", "LinearizeDepth", {})
    g.create_pass("Dei", "DeinterleaveTexture", {})
    g.create_pass("Int", "InterleaveTexture", {})
    g.add_edge("GBufferRaster.depth", "LinearizeDepth.depth")
    g.add_edge("LinearizeDepth.linearDepth", "Dei.texIn")
    g.add_edge("Dei.texOut", "Int.texIn")
    g.mark_output("Int.texOut")
    g.plan(130, 70)
    res = g.resources()
    assert res["Dei.texOut"] == (33, 18, 16, "R32Float")
    assert res["Int.texOut"] == (130, 70, 1, "R32Float")


@pytest.mark.parametrize("n,fmt", [(8, "R8Uint"), (16, "R16Uint"), (32, "R32Uint")])
def test_svao_stencil_format_by_directions(n, fmt):
    """SVAO.cpp:132-134: the stencil holds one bit per direction (sampleCount 8 / 16 / 32)."""
    g = rsdgraph.RenderGraph("svao")
    g.create_pass("Z", "Source", {})
    g.create_pass("N", "Source", {})
    g.create_pass("AO", "SVAO", {"sampleCount": n})
    g.add_edge("Z.z", "AO.depth")
    g.add_edge("N.n", "AO.normals")
    g.mark_output("AO.stencil")
    g.plan(128, 96)
    assert g.resources()["AO.stencil"][3] == fmt


def test_svao_refuses_other_direction_counts():
    g = rsdgraph.RenderGraph("svao")
    g.create_pass("Z", "Source", {})
    g.create_pass("N", "Source", {})
    g.create_pass("AO", "SVAO", {"sampleCount": 12})
    g.add_edge("Z.z", "AO.depth")
    g.add_edge("N.n", "AO.normals")
    g.mark_output("AO.ao")
    with pytest.raises(abi.RsdError, match="sampleCount must be 8, 16 or 32"):
        g.plan(128, 96)


def test_svao_dual_ao_output_format():
    """SVAO.cpp:129-131: dualAO makes the ao output RG8Unorm (bright, dark)."""
    for dual, fmt in ((False, "R8Unorm"), (True, "RG8Unorm")):
        g = rsdgraph.RenderGraph("svao")
        g.create_pass("Z", "Source", {})
        g.create_pass("N", "Source", {})
        g.create_pass("AO", "SVAO", {"dualAO": dual})
        g.add_edge("Z.z", "AO.depth")
        g.add_edge("N.n", "AO.normals")
        g.mark_output("AO.ao")
        g.plan(128, 96)
        assert g.resources()["AO.ao"][3] == fmt
