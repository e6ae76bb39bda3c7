"""Multi-process screen-band sharding (rsd/shard.py) over gloo on the CPU.

The GPU backend of BandFrame is librsd (bench.py, tests/test_gpu_parity.py); here the same
orchestration runs with the CPU oracle as backend in world_size 2 and 3 processes, and the
gathered frame must be bit-identical to a single-process oracle frame."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from helpers import oracle_vao, small_frame_config


class OracleBackend:
    """BandFrame backend on the CPU oracle; numpy buffers shared with torch tensors."""

    def __init__(self, O, scene, cfg, ss_max_radius=None):
        self.O, self.cfg = O, cfg
        self.osc = O.Scene(scene.positions, scene.indices, scene.flags)
        W, H = cfg.fb_w, cfg.fb_h
        aspect = float(np.float32(W) / np.float32(H))
        self.cam = O.camera_look_at(scene.camera["pos"], scene.camera["target"], scene.camera["up"], aspect=aspect)
        self.vao, self.sd_w, self.sd_h = oracle_vao(O, W, H, cfg.divisor, cfg.sd_guard_px, cfg.radius)
        if ss_max_radius is not None:  # a small sample reach: halo windows narrower than the map
            self.vao.ssMaxRadius = ss_max_radius
        N = cfg.sd_samples
        self.sdp = O.SDParams(N, cfg.implementation, cfg.max_count, self.vao.sdGuard, 1, 1, 1, cfg.cull_mode, 0,
                              float(np.float32(1.5 / N)))
        self.svp = O.SVAOParams(8, N, 2, 1, 1, cfg.guard_band)
        self.z, self.n = O.gbuffer(self.osc, self.cam, W, H, cfg.cull_mode, threads=2)
        self.np_ao = np.zeros((H, W), np.uint8)
        self.np_st = np.zeros((H, W), np.uint8)
        # rayMin / rayMax in one buffer, like rsd.frame.Renderer (one all-reduce per frame)
        self.np_rminmax = np.zeros((2, self.sd_h, self.sd_w), np.uint32)
        self.np_rmin, self.np_rmax = self.np_rminmax[0], self.np_rminmax[1]
        self.np_sd = np.zeros(((N + 3) // 4, self.sd_h, self.sd_w, min(N, 4)), np.float32)
        self.ao = torch.from_numpy(self.np_ao)
        self.stencil = torch.from_numpy(self.np_st)
        self.ray_minmax = torch.from_numpy(self.np_rminmax.view(np.int32))
        self.ray_min, self.ray_max = self.ray_minmax[0], self.ray_minmax[1]
        self.sd = torch.from_numpy(self.np_sd)

    def clear_intervals(self):
        self.O.svao_clear(self.np_rmin, self.np_rmax)

    def pass1(self, band=(0, 1)):
        self.O.svao_pass1_into(self.cam, self.vao, self.svp, self.z, self.n, self.np_ao, self.np_st, self.np_rmin,
                               self.np_rmax, band)

    def sd_trace(self, band=(0, 1)):
        self.O.sd_trace_into(self.osc, self.cam, self.sdp, self.z, self.np_rmin, self.np_rmax, self.np_sd, band,
                             threads=2)

    def pass2(self, band=(0, 1)):
        self.O.svao_pass2_into(self.cam, self.vao, self.svp, self.z, self.n, self.np_st, self.np_sd, self.np_ao, band,
                               threads=2)

    # contiguous bands (HaloFrame)
    def pass1_rows(self, rows):
        self.O.svao_pass1_rows_into(self.cam, self.vao, self.svp, self.z, self.n, self.np_ao, self.np_st, self.np_rmin,
                                    self.np_rmax, rows)

    def sd_trace_rows(self, rows):
        self.O.sd_trace_rows_into(self.osc, self.cam, self.sdp, self.z, self.np_rmin, self.np_rmax, self.np_sd, rows,
                                  threads=2)

    def pass2_rows(self, rows):
        self.O.svao_pass2_rows_into(self.cam, self.vao, self.svp, self.z, self.n, self.np_st, self.np_sd, self.np_ao,
                                    rows, threads=2)


def _cfg():
    return small_frame_config(visible=(192, 104), guard=16, divisor=2, N=4)


def _worker(rank, world, port, out_dir, mode="band", sd_split="tiles"):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    for p in (str(root), str(root / "ray-traced-stochastic-depth-map_amd"), str(root / "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist

    from oracle import oracle as O
    from rsd.scenes import make_scene
    from rsd.shard import BandFrame, HaloFrame
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    cfg = _cfg() if mode == "band" else _halo_cfg()
    if mode == "halo_lag":
        _lag_frames(O, cfg, rank, world, out_dir)
        dist.barrier()
        dist.destroy_process_group()
        return
    be = OracleBackend(O, make_scene("arcade_tiny"), cfg, None if mode == "band" else HALO_REACH)
    f = BandFrame(be, rank, world) if mode == "band" else HaloFrame(be, rank, world, sd_split=sd_split)
    f.frame()
    if mode == "halo":
        # more frames: intervals cleared again, buffers reused, and the split re-balanced from the
        # measured per-rank times (a skewed first split forces a real move); every frame must still
        # give the 1-process image
        f.gb = [0] + [1 + k for k in range(world - 1)] + [f.G]
        f._plan()
        for _ in range(3):
            be.np_ao[:] = 0
            f.frame()
            np.save(os.path.join(out_dir, f"ao_{rank}_{f.frames}.npy"), be.np_ao)
        np.save(os.path.join(out_dir, f"split_{rank}.npy"), np.array(f.splits))
        np.save(os.path.join(out_dir, f"sdrows_{rank}.npy"), np.array(f.owned_sd_rows()))
        np.save(os.path.join(out_dir, f"bytes_{rank}.npy"), np.array([f.sent["intervals"], f.sent["sd"],
                                                                     f.frames]))
    np.save(os.path.join(out_dir, f"ao_{rank}.npy"), be.np_ao)
    np.save(os.path.join(out_dir, f"sd_{rank}.npy"), be.np_sd)
    dist.barrier()
    dist.destroy_process_group()


def _lag_frames(O, cfg, rank, world, out_dir):
    """bench.py's frames in flight at N > 1: two frame slots (own buffers), back() of each frame issued
    after front() of the next one, so the collectives of different frames interleave -- in the same
    order on every rank.  Every frame must still give the 1-process image."""
    from rsd.scenes import make_scene
    from rsd.shard import HaloFrame
    slots = []
    for _ in range(2):
        be = OracleBackend(O, make_scene("arcade_tiny"), cfg, HALO_REACH)
        slots.append((be, HaloFrame(be, rank, world)))
    pending = []

    def finish(j):
        be, f = slots[j % 2]
        f.back()
        np.save(os.path.join(out_dir, f"lag_{rank}_{j}.npy"), be.np_ao)

    for i in range(5):
        be, f = slots[i % 2]
        be.np_ao[:] = 0
        f.front()
        pending.append(i)
        if len(pending) > 1:
            finish(pending.pop(0))
    finish(pending.pop(0))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_band_sharded_frame_equals_single_process(oracle, tmp_path, world):
    from rsd.scenes import make_scene
    from rsd.shard import BandFrame
    ref = OracleBackend(oracle, make_scene("arcade_tiny"), _cfg())
    BandFrame(ref, 0, 1).frame()
    assert (ref.np_st != 0).any()
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"ao_{r}.npy"), ref.np_ao), f"rank {r} AO"
        assert np.array_equal(np.load(tmp_path / f"sd_{r}.npy").view(np.uint32), ref.np_sd.view(np.uint32)), \
            f"rank {r} SD map"


HALO_REACH = 24.0  # ssMaxRadius of the halo tests: ~40-px windows in a 448-row frame


def _halo_cfg():
    return small_frame_config(visible=(96, 448), guard=16, divisor=2, N=2)


@pytest.mark.parametrize("world,sd_split", [(2, "tiles"), (3, "tiles"), (4, "tiles"), (3, "rows")])
def test_halo_sharded_frame_equals_single_process(oracle, tmp_path, world, sd_split):
    """HaloFrame (contiguous bands, sparse interval + SD halo exchange over point-to-point sends,
    load-balanced re-splits; the SD trace split into round-robin 8-row tiles, or the rows under each
    band): every rank ends every frame with the single-process AO image; the SD rows it traced equal
    the reference; the split moved; the sparse halo moved less than the dense candidate rows would have."""
    from rsd.scenes import make_scene
    from rsd.shard import BandFrame
    ref = OracleBackend(oracle, make_scene("arcade_tiny"), _halo_cfg(), HALO_REACH)
    BandFrame(ref, 0, 1).frame()
    assert (ref.np_st != 0).any()
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), "halo", sd_split), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"ao_{r}.npy"), ref.np_ao), f"rank {r} AO"
        for fr in (2, 3, 4):
            assert np.array_equal(np.load(tmp_path / f"ao_{r}_{fr}.npy"), ref.np_ao), f"rank {r} AO frame {fr}"
        sd = np.load(tmp_path / f"sd_{r}.npy")
        for lo, hi in np.load(tmp_path / f"sdrows_{r}.npy"):
            assert np.array_equal(sd[:, lo:hi].view(np.uint32), ref.np_sd[:, lo:hi].view(np.uint32)), f"rank {r} SD"
    splits = np.load(tmp_path / "split_0.npy")
    assert all(np.array_equal(splits, np.load(tmp_path / f"split_{r}.npy")) for r in range(world))  # same on all
    assert not np.array_equal(splits[1], splits[-1])  # the skewed split was re-balanced
    p = _halo_plan(oracle, world, 0)
    assert p.window[0][1] < p.b.sd_h  # rank 0 did not receive the whole map
    sent = sum(np.load(tmp_path / f"bytes_{r}.npy")[1] / np.load(tmp_path / f"bytes_{r}.npy")[2]
               for r in range(world))
    dense = sum(_halo_plan(oracle, world, r).dense_bytes_per_frame()["sd"] for r in range(world))
    assert 0 < sent < dense  # only the texels the receivers read


def _halo_plan(oracle, world, rank):
    """The HaloFrame partition of _halo_cfg() as seen by `rank` (no process group needed)."""
    from types import SimpleNamespace

    from rsd.shard import HaloFrame
    cfg = _halo_cfg()
    vao, sd_w, sd_h = oracle_vao(oracle, cfg.fb_w, cfg.fb_h, cfg.divisor, cfg.sd_guard_px, cfg.radius)
    vao.ssMaxRadius = HALO_REACH
    N = cfg.sd_samples
    be = SimpleNamespace(cfg=cfg, vao=vao, sd_h=sd_h, sd=torch.zeros((1, sd_h, sd_w, N)),
                         ray_minmax=torch.zeros((2, sd_h, sd_w), dtype=torch.int32),
                         ao=torch.zeros((cfg.fb_h, cfg.fb_w), dtype=torch.uint8))
    import torch.distributed as dist
    orig = dist.get_backend
    dist.get_backend = lambda pg=None: "gloo"
    try:
        return HaloFrame(be, rank, world)
    finally:
        dist.get_backend = orig


def test_halo_plan_partitions_and_bounds(oracle):
    for world in (1, 2, 3, 4):
        plans = [_halo_plan(oracle, world, r) for r in range(world)]
        p0 = plans[0]
        # pixel groups and SD rows partition the frame / map
        assert p0.px_rows[0][0] == 0 and all(p0.px_rows[r][1] == p0.px_rows[r + 1][0] for r in range(world - 1))
        assert p0.sd_rows[0][0] == 0 and p0.sd_rows[-1][1] == plans[0].b.sd_h
        assert all(p0.sd_rows[r][1] == p0.sd_rows[r + 1][0] for r in range(world - 1))
        # the tiled SD split: the ranks' round-robin tiles partition the map's rows
        owned = sorted(y for p in plans for lo, hi in p.owned_sd_rows() for y in range(lo, hi))
        assert owned == list(range(p0.b.sd_h))
        for r, p in enumerate(plans):
            assert p.window[r][0] < p.window[r][1]
            # what r scans for k: every row of r's window in k's tiles, plus at most the rows of the
            # window's first tile below it (whole tiles; r's pass 1 never touches those)
            for k, reg in p.iv_send.items():
                got = set(p._region_rows(reg[0], reg[1], world)) if reg else set()
                lo, hi = p.window[r]
                want = {y for y in range(lo, hi) if (y // 8) % world == k}
                assert want <= got <= {y for y in range(lo // 8 * 8, hi) if (y // 8) % world == k}, (world, r, k)
            if world >= 3:  # the halo is a real restriction: a window leaves rows of the map out
                assert any(q.window[k] != (0, q.b.sd_h) for k, q in enumerate(plans))
            # what r sends to k is what k expects from r (same row ranges on both sides)
            for k, q in enumerate(plans):
                if k != r:
                    assert p.iv_send[k] == q.iv_recv[r] and p.sd_recv[k] == q.sd_send[r]


def test_halo_rebalance_moves_toward_cost():
    """The re-split: an expensive band gives up groups, the same inputs give the same
    split on every rank, and each rank keeps at least one group."""
    import torch.distributed as dist
    from rsd.shard import HaloFrame
    for world in (2, 3, 4, 8):
        from types import SimpleNamespace
        cfg = small_frame_config(visible=(96, 1080), guard=16, divisor=2, N=2)
        sd_h = 600
        be = SimpleNamespace(cfg=cfg, vao=SimpleNamespace(sdGuard=32, ssMaxRadius=24.0), sd_h=sd_h,
                             sd=torch.zeros((1, sd_h, 64, 2)), ray_minmax=torch.zeros((2, sd_h, 64), dtype=torch.int32),
                             ao=torch.zeros((cfg.fb_h, cfg.fb_w), dtype=torch.uint8))
        orig = dist.get_backend
        dist.get_backend = lambda pg=None: "gloo"
        try:
            f = HaloFrame(be, 0, world)
        finally:
            dist.get_backend = orig
        costs = [1.0] * world
        costs[0] = 10.0  # band 0 ten times as expensive per group
        new = f._rebalanced(costs)
        assert new[0] == 0 and new[-1] == f.G and all(new[k] < new[k + 1] for k in range(world))
        assert new[1] < f.gb[1]  # band 0 shrinks
        assert new == f._rebalanced(list(costs))  # deterministic
        assert f._rebalanced([1.0] * world) == f.gb  # balanced costs: no move


def test_band_rows_partition():
    from rsd.shard import band_rows
    for world in (1, 2, 3, 8):
        rows = [band_rows(1144, 32, 64, r, world) for r in range(world)]
        allr = torch.cat(rows).sort().values
        assert torch.equal(allr, torch.arange(64, 64 + 1144))


class _RecordingBackend:
    """Minimal BandFrame backend that records the trace calls (no compute)."""

    def __init__(self, capable):
        from types import SimpleNamespace
        self.cfg = SimpleNamespace(fb_w=64, fb_h=48, guard_band=8, ray_interval=1)
        self.sd_h = 16
        self.sd = torch.zeros((1, 16, 24, 4))
        self.ao = torch.zeros((48, 64), dtype=torch.uint8)
        self.calls = []
        if capable:
            self.can_consume_intervals = True

    def clear_intervals(self):
        self.calls.append(("clear",))

    def pass1(self, band=(0, 1)):
        self.calls.append(("pass1", band))

    def sd_trace(self, band=(0, 1), **kw):
        self.calls.append(("trace", band, tuple(sorted(kw.items()))))

    def pass2(self, band=(0, 1)):
        self.calls.append(("pass2", band))


def test_band_frame_throughput_and_consume_plumbing():
    """bench.py's frames in flight: a librsd-like backend gets consume + throughput on its trace
    (the first frame clears the intervals, later frames rely on the consuming trace); a backend
    without those capabilities (the oracle) gets neither."""
    from rsd.shard import BandFrame
    cap = _RecordingBackend(capable=True)
    bf = BandFrame(cap, throughput=True)
    bf.frame()
    bf.frame()
    assert cap.calls == [("clear",), ("pass1", (0, 1)), ("trace", (0, 1), (("consume", True), ("throughput", True))),
                         ("pass2", (0, 1)),
                         ("pass1", (0, 1)), ("trace", (0, 1), (("consume", True), ("throughput", True))),
                         ("pass2", (0, 1))]
    plain = _RecordingBackend(capable=False)
    bf = BandFrame(plain, throughput=True)
    bf.frame()
    bf.frame()
    assert [c for c in plain.calls if c[0] == "trace"] == [("trace", (0, 1), ())] * 2
    assert plain.calls.count(("clear",)) == 2


@pytest.mark.parametrize("world", [2, 3])
def test_halo_frames_in_flight_interleaved(oracle, tmp_path, world):
    """HaloFrame.front() / back() with frames in flight (the counts of a frame are read on the host one
    frame later): 5 frames over 2 slots, every rank ends every frame with the 1-process AO image."""
    from rsd.scenes import make_scene
    from rsd.shard import BandFrame
    ref = OracleBackend(oracle, make_scene("arcade_tiny"), _halo_cfg(), HALO_REACH)
    BandFrame(ref, 0, 1).frame()
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), "halo_lag"), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        for j in range(5):
            assert np.array_equal(np.load(tmp_path / f"lag_{r}_{j}.npy"), ref.np_ao), f"rank {r} frame {j}"


def _rccl_group_worker(rank, world, port, out_dir, fail):
    """NativeComm.rccl_group over gloo with librsd's RCCL entry points replaced by fakes: a rank that cannot use
    RCCL must make EVERY rank fall back (no rank left blocked in a broadcast or a collective create)."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    for p in (str(root), str(root / "ray-traced-stochastic-depth-map_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist

    from rsd import abi
    from rsd.shard import NativeComm

    class FakeLib:
        def __init__(self, real):
            self.real = real

        def rsd_comm_rccl_available(self):
            return 1 if fail == ("available", rank) else 0

        def rsd_comm_rccl_unique_id(self, uid):
            if fail == ("unique_id", rank):
                return 1
            for i in range(abi.COMM_UNIQUE_ID_BYTES):
                uid[i] = (i * 7 + 3) & 255
            return 0

        def rsd_comm_rccl_create(self, uid, w, r, out):
            return 1 if fail == ("create", rank) else 0

        def rsd_last_error(self):
            return b"fake failure"

        def __getattr__(self, k):
            return getattr(self.real, k)

    real = abi.lib()
    abi._lib = FakeLib(real)
    created = []
    NativeComm.__init__ = lambda self, h: created.append(h)  # no rsd_comm_info on a fake handle
    NativeComm.close = lambda self: None
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comms, why = NativeComm.rccl_group(rank, world, n=3)
    np.save(os.path.join(out_dir, f"rg_{rank}.npy"), np.array([len(comms), why is None]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fail", [None, ("available", 1), ("unique_id", 0), ("create", 1)])
def test_rccl_group_falls_back_together(tmp_path, fail):
    world = 2
    mp.start_processes(_rccl_group_worker, args=(world, _free_port(), str(tmp_path), fail), nprocs=world, join=True,
                       start_method="spawn")
    got = [tuple(np.load(tmp_path / f"rg_{r}.npy")) for r in range(world)]
    want = (3, 1) if fail is None else (0, 0)
    assert got == [want] * world, got


def test_bench_thread_group_reductions():
    """bench.py's ThreadGroup (--local-ranks): barriers and max / sum reductions across rank threads, repeated
    back to back (the slots are reused only after every rank has read them)."""
    import sys
    import threading
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    world = 5
    shared = {"world": world, "barrier": threading.Barrier(world), "slots": [None] * world}
    out = {}

    def run(k):
        g = bench.ThreadGroup(k, shared)
        res = []
        for i in range(20):
            res.append(g.reduce([k + i, 2.0 * k], "max"))
            res.append(g.reduce([1.0, k * i], "sum"))
            g.barrier()
        out[k] = res

    ts = [threading.Thread(target=run, args=(k,)) for k in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    for k in range(world):
        for i in range(20):
            assert out[k][2 * i] == [world - 1 + i, 2.0 * (world - 1)]
            assert out[k][2 * i + 1] == [float(world), float(i * sum(range(world)))]
