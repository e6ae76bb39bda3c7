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
    assert (a.gpus, a.frames_in_flight, a.shard, a.config) == (1, 4, None, "suntemple_1080p_q")
    assert a.camera_path is None  # the config's own path (static for configs[1])
    assert a.steps > 0 and a.warmup >= a.frames_in_flight  # every slot warmed before timing
    a = _bench(monkeypatch, ["--shard", "band", "--frames-in-flight", "1"]).parse()
    assert (a.shard, a.frames_in_flight) == ("band", 1)


def test_committed_pmc_passes_parse(monkeypatch):
    bench = _bench(monkeypatch)
    p = ROOT / "profiles" / "round1"
    v = bench.pmc_valu(p / "pmc_sq_valu.csv", "svao_pass1_kernel")
    assert v is not None and 0.0 < v["frac"] <= 1.0 and v["peak"] == round(bench.VALU_PEAK_LANE_OPS / 1e12, 2)
    from rsd import abi
    files = [str(p / "pmc_fetch_size.csv"), str(p / "pmc_write_size.csv")]
    split = bench.pmc_traffic(files, abi.WALK_KERNELS[abi.WALK_SPLIT])
    quad = bench.pmc_traffic(files, abi.WALK_KERNELS[abi.WALK_QUAD])
    assert split and quad and split > 0 and quad > 0
    # one trace = the kernels of ONE walk: the walks share only the setup kernel
    both = bench.pmc_traffic(files, abi.WALK_KERNELS[abi.WALK_SPLIT] + ("sd_trace_queue_kernel",))
    setup = bench.pmc_traffic(files, ("sd_setup_kernel",))
    assert abs(both - (split + quad - setup)) <= 2048


def test_host_cpus():
    sys.path.insert(0, str(ROOT))
    import bench as b
    h = b.host_cpus()
    assert h["usable"] >= 1 and h["nproc"] >= h["usable"]
    # the baseline's core count: the affinity mask capped by the cgroup quota
    assert 1 <= h["effective"] <= h["usable"]
    if h["cgroup_cpu_quota"] is not None:
        import math
        assert h["effective"] <= max(1, math.ceil(h["cgroup_cpu_quota"]))


def test_camera_path():
    from rsd.frame import camera_path
    poses = camera_path("orbit120")
    assert len(poses) == 120 and camera_path("static") is None
    assert poses == camera_path("orbit120")  # seeded: deterministic
    import numpy as np
    pos = np.array([p[0] for p in poses])
    # on the 17 m orbit, above the props, never inside a colonnade column (x = +-12.8, r = 0.55)
    assert np.allclose(np.hypot(pos[:, 0], pos[:, 2]), 17.0, atol=1e-4) and (pos[:, 1] >= 5.0).all()
    cols = [(sx * 12.8, -18.0 + 4.0 * k) for sx in (-1, 1) for k in range(10)]
    assert min(np.hypot(pos[:, 0] - cx, pos[:, 2] - cz).min() for cx, cz in cols) > 0.55
