"""CPU checks of the C ABI boundary: librsd loads, exports exactly what include/rsd.h
declares, its structs have the header's layout, and its host-only helpers (camera,
VAOData) agree bit-for-bit with the oracle's independent restatements.  No compute
calls are made here (there is no GPU in the build container)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from helpers import oracle_vao, to_oracle

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "rsd.h"


@pytest.fixture(scope="module")
def abi():
    from rsd import abi
    if not abi.LIB_PATH.exists():
        subprocess.run(["make", "-C", str(abi.PKG_DIR), "-j8"], check=True, stdout=subprocess.DEVNULL)
    abi.lib()
    return abi


def header_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:rsd_status|void|uint32_t|float|const char\*)\s+(rsd_\w+)\s*\(", text, re.M)))


def test_header_and_binding_agree(abi):
    assert sorted(abi.EXPORTS) == header_functions()


def test_library_exports_every_header_symbol(abi):
    out = subprocess.run(["nm", "-D", "--defined-only", str(abi.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (rsd_\w+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing
    assert abi.lib().rsd_abi_version() == 8


def test_struct_layouts_match_header(abi, tmp_path):
    structs = {"rsd_scene_desc": abi.SceneDesc, "rsd_scene_info": abi.SceneInfo, "rsd_camera": abi.Camera,
               "rsd_sd_params": abi.SDParams, "rsd_vao_data": abi.VAOData, "rsd_svao_params": abi.SVAOParams,
               "rsd_counters": abi.Counters, "rsd_texture": abi.Texture,
               "rsd_alpha_texture": abi.AlphaTexture, "rsd_material": abi.Material, "rsd_alpha_desc": abi.AlphaDesc,
               "rsd_svao_frame_desc": abi.FrameDesc, "rsd_halo_region": abi.HaloRegion,
               "rsd_halo_list": abi.HaloList, "rsd_halo_sd_list": abi.HaloSdList, "rsd_comm_xfer": abi.CommXfer,
               "rsd_band_params": abi.BandParams, "rsd_band_stats": abi.BandStats}
    src = "#include <stdio.h>\n#include \"rsd_graph.h\"\nint main(void){\n"
    for name in structs:
        src += f'printf("%zu\\n", sizeof({name}));\n'
    src += "return 0;}\n"
    (tmp_path / "s.c").write_text(src)
    subprocess.run(["gcc", "-I", str(HEADER.parent), str(tmp_path / "s.c"), "-o", str(tmp_path / "s")], check=True)
    sizes = [int(x) for x in subprocess.run([str(tmp_path / "s")], capture_output=True, text=True).stdout.split()]
    assert sizes == [C.sizeof(s) for s in structs.values()]


def test_device_open_without_gpu_is_an_error_not_a_crash(abi):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = C.c_void_p()
    st = abi.lib().rsd_device_open(0, C.byref(h))
    assert st == 5 and b"no HIP device" in abi.lib().rsd_last_error()


def test_comm_and_band_frame_arguments_are_checked(abi):
    """The band frame's C ABI refuses bad arguments with a status and a message, without a GPU."""
    L = abi.lib()
    hub = C.c_void_p()
    assert L.rsd_comm_hub_create(0, C.byref(hub)) == 1 and b"world" in L.rsd_last_error()
    assert L.rsd_comm_hub_create(2, C.byref(hub)) == 0 and hub.value
    comm = C.c_void_p()
    assert L.rsd_comm_local_create(hub, 2, C.byref(comm)) == 1 and b"rank >= world" in L.rsd_last_error()
    assert L.rsd_comm_rccl_create(None, 1, 0, C.byref(comm)) == 1
    assert L.rsd_comm_all_gather(None, None, None, 0, None) == 1 and b"null communicator" in L.rsd_last_error()
    assert L.rsd_comm_exchange(None, None, 0, None, 0, None) == 1
    assert L.rsd_band_frame_create(None, None, None, C.byref(comm)) == 1
    assert L.rsd_band_frame_front(None, None, None) == 1 and b"null frame" in L.rsd_last_error()
    assert L.rsd_band_frame_back(None, None, None) == 1
    assert L.rsd_band_frame_stats(None, None) == 1
    L.rsd_band_frame_release(None)
    L.rsd_comm_release(None)
    L.rsd_comm_hub_release(hub)


def test_invalid_arguments_are_reported(abi):
    L = abi.lib()
    assert L.rsd_sd_trace(None, None, None, None, 0, 0, None, None, None, 0, 0, None, None) == 1
    assert b"rsd_sd_trace" in L.rsd_last_error()
    assert L.rsd_svao_pass1(None, None, None, None, None, 0, 0, None, None, None, None, 0, 0, None) == 1
    assert L.rsd_svao_pass2(None, None, None, None, None, 0, 0, None, None, 0, 0, None, None) == 1
    assert L.rsd_gbuffer(None, None, 0, 0, 0, None, None, None) == 1
    assert L.rsd_svao_clear_intervals(None, None, 0, None) == 1
    with pytest.raises(abi.RsdError, match="rsd_svao_make_vao_data"):
        abi.check(L.rsd_svao_make_vao_data(0, 0, 0, 0, 0, 0, 0, None, None, None), "rsd_svao_make_vao_data")


@pytest.mark.parametrize("pos,target,aspect", [
    ([0.0, 1.7, 16.8], [0.0, 1.2, -12.0], 2048 / 1208),
    ([3.0, -2.0, 5.0], [0.5, 0.25, -1.0], 1.0),
    ([-10.0, 4.0, 2.0], [10.0, 1.0, 2.5], 3968 / 2288),
])
def test_camera_matches_oracle(abi, oracle, pos, target, aspect):
    cam = abi.Camera()
    f3 = lambda v: (C.c_float * 3)(*v)
    a = float(np.float32(aspect))
    abi.check(abi.lib().rsd_camera_look_at(f3(pos), f3(target), f3([0, 1, 0]), 21.0, 24.0, a, 0.1, 1000.0, 10000.0,
                                           C.byref(cam)), "camera")
    ocam = oracle.camera_look_at(pos, target, [0, 1, 0], aspect=a)
    assert bytes(to_oracle(cam, oracle.Camera)) == bytes(ocam)


@pytest.mark.parametrize("W,H,div", [(2048, 1208, 4), (2048, 1208, 1), (3968, 2288, 4), (256, 256, 1),
                                     (1000, 601, 3), (3968, 2288, 16)])
def test_vao_data_matches_oracle(abi, oracle, W, H, div):
    vao = abi.VAOData()
    w, h = C.c_uint32(), C.c_uint32()
    abi.check(abi.lib().rsd_svao_make_vao_data(W, H, div, 512, 0.2, 2.0, 0.0, C.byref(vao), C.byref(w), C.byref(h)),
              "vao")
    ov, sw, sh = oracle_vao(oracle, W, H, div)
    assert bytes(to_oracle(vao, oracle.VAOData)) == bytes(ov)
    assert (w.value, h.value) == (sw, sh)


def test_sd_map_sizes_of_the_baseline_configs(abi):
    # SD size = ceil(fb / div) + 2 * 512 / div
    from rsd.frame import FrameConfig, make_vao
    for vis, div, want in [((1920, 1080), 4, (768, 558)), ((1920, 1080), 1, (3072, 2232)),
                           ((3840, 2160), 4, (1248, 828)), ((3840, 2160), 1, (4992, 3312))]:
        cfg = FrameConfig(visible_w=vis[0], visible_h=vis[1], divisor=div)
        _, w, h = make_vao(cfg)
        assert (w, h) == want


def test_halo_arguments_are_validated_before_any_gpu_work(abi):
    """The rsd_halo_* entries check their arguments on the host (no HIP call on a bad request)."""
    L, dummy = abi.lib(), C.c_void_p(16)
    one = abi.HaloRegion(0, 8, 16, 10, 1, 16)  # 8 rows x 4 columns = 32 texels > stride 10
    arr = (abi.HaloRegion * 1)(one)
    assert L.rsd_halo_compact(dummy, dummy, 4, 8, arr, 1, None) == abi.ERR_INVALID_ARG  # stride below the texels
    tiled = (abi.HaloRegion * 1)(abi.HaloRegion(3, 8, 16, 1000, 2, 16))
    assert L.rsd_halo_compact(dummy, dummy, 4, 8, tiled, 1, None) == abi.ERR_INVALID_ARG  # tiles off the 8-row grid
    past = (abi.HaloRegion * 1)(abi.HaloRegion(0, 9, 16, 1000, 1, 16))
    assert L.rsd_halo_compact(dummy, dummy, 4, 8, past, 1, None) == abi.ERR_INVALID_ARG  # rows past the map
    many = (abi.HaloRegion * 65)(*[abi.HaloRegion(0, 1, 16, 1000, 1, 16) for _ in range(65)])
    assert L.rsd_halo_compact(dummy, dummy, 4, 8, many, 65, None) == abi.ERR_INVALID_ARG  # > 64 regions
    lists = (abi.HaloList * 1)(abi.HaloList(16, 10, 5))
    assert L.rsd_halo_merge(dummy, dummy, 4, 8, lists, 1, 1, None) == abi.ERR_INVALID_ARG  # stride below n
    sdl = (abi.HaloSdList * 1)(abi.HaloSdList(None, 16, 3, 0))
    assert L.rsd_halo_sd_gather(dummy, 1, 4, 8, 4, sdl, 1, None) == abi.ERR_INVALID_ARG  # null index list
    assert L.rsd_halo_sd_scatter(dummy, 1, 4, 8, 5, sdl, 0, None) == abi.ERR_INVALID_ARG  # 5 channels
    assert L.rsd_halo_merge(dummy, dummy, 4, 8, None, 0, 1, None) == abi.RSD_OK  # nothing to merge
