"""bench.py host logic on the CPU: argument defaults (the driver runs `python bench.py` bare)
and the roofline readers over the committed rocprofv3 passes in profiles/round1/."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _bench(monkeypatch, argv=()):
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    import bench
    return bench


def test_bench_defaults(monkeypatch):
    bench = _bench(monkeypatch)
    a = bench.parse()
    assert (a.gpus, a.frames_in_flight, a.shard, a.config) == (1, 4, "frame", "suntemple_1080p_q")
    assert a.steps > 0 and a.warmup >= a.frames_in_flight  # every slot warmed before timing
    a = _bench(monkeypatch, ["--shard", "band", "--frames-in-flight", "1"]).parse()
    assert (a.shard, a.frames_in_flight) == ("band", 1)


def test_committed_pmc_passes_parse(monkeypatch):
    bench = _bench(monkeypatch)
    p = ROOT / "profiles" / "round1"
    v = bench.pmc_valu(p / "pmc_sq_valu.csv", "svao_pass1_kernel")
    assert v is not None and 0.0 < v["frac"] <= 1.0 and v["peak"] == round(bench.VALU_PEAK_LANE_OPS / 1e12, 2)
    t = bench.pmc_traffic([str(p / "pmc_fetch_size.csv"), str(p / "pmc_write_size.csv")], bench.SD_KERNELS)
    assert t is not None and t > 0
