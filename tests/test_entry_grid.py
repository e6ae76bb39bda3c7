"""The segment entry grid's coverage property on the host (tests/native/check_entry_grid.cpp): librsd's
own BVH and entry-grid builders over random triangle scenes (near the origin and translated far
from it), the SD setup kernel's cell lookup restated with the same float operations, and a double-
precision brute force: every triangle a segment clearly crosses lies under the frontier of the
cell it is given, and a cell reported absent has no such triangle.  The GPU side (same bits with
the grid on and off, and vs the oracle) is tests/test_gpu_entry.py."""
import shutil
import subprocess
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent
CSRC = HERE.parent / "ray-traced-stochastic-depth-map_amd" / "csrc"


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    out = tmp_path_factory.mktemp("entry") / "check_entry_grid"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", f"-I{CSRC}", "-o", str(out),
                    str(HERE / "native" / "check_entry_grid.cpp"), str(CSRC / "entry_grid.cpp"),
                    str(CSRC / "bvh_build.cpp"), "-pthread"], check=True)
    return out


@pytest.mark.parametrize("tris,offset,splits", [(20000, 0.0, 0.0), (20000, 1000.0, 0.0), (5000, -3000.0, 0.0),
                                                (20000, 0.0, 0.5), (5000, -3000.0, 0.5)])
def test_entry_grid_covers_every_crossed_triangle(exe, tris, offset, splits):
    """splits > 0: the spatial-split BVH (bvh_build.h BvhOptions; tools/sbvh_study.cpp): the
    leaves' clipped, padded boxes still contain every crossing point of their triangle."""
    out = subprocess.run([str(exe), str(tris), "3000", str(offset), str(splits)], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    last = out.stdout.strip().splitlines()[-1]
    fields = dict(zip(last.split()[0::2], last.split()[1::2]))
    assert int(fields["violations"]) == 0 and int(fields["hits"]) > 1000, last
    if splits:
        head = out.stdout.strip().splitlines()[0].split()
        info = dict(zip(head[0::2], head[1::2]))
        assert int(info["spatial_splits"]) > 0 and int(info["references"]) > tris, head
