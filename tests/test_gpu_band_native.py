"""The native band frame (include/rsd.h rsd_band_frame_*, csrc/band_frame.cpp) and its communicators
(rsd_comm_*: RCCL, in-process) on the GPU.

SURVEY 8(e) / north_star: frames shard by screen band across the GPUs of a node, the AO image is
all-gathered over RCCL.  The reference renders on one GPU, so the bar is the 1-GPU frame of librsd
itself (rsd_svao_frame, which the parity tests pin to the oracle): every rank's gathered AO image and
its own SD share must equal it bit for bit, whatever the split and its re-balancing.

  * 8 rank threads sharing this GPU through the in-process communicator, two frame slots each with
    back() of a frame after front() of the next (bench.py's frames in flight), at configs[1], [3] and
    [4] (the 8-GPU configs of BASELINE.json);
  * the RCCL communicator at world 1 -- ncclCommInitRank with one rank, an all-gather and a self
    send / receive, then the band frame over it (RCCL needs one GPU per rank: the N > 1 RCCL run is the
    driver's 8-GPU bench)."""
import ctypes as C
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _renderer(config):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS[config]
    r = Renderer(make_scene(name), FrameConfig(**kw))
    r.gbuffer()
    r.frame()
    ref = r.numpy()
    assert (ref["ray_max"] != 0).any()
    return r, ref


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config,world", [("suntemple_1080p_q", 8), ("suntemple_1080p_q", 3),
                                          ("emerald_4k_q", 8), ("bistro_4k_full_n16", 8)])
def test_native_band_frame_local_ranks_equal_one_gpu(config, world):
    import torch
    from rsd.shard import NativeComm, NativeHaloFrame, NativeHub
    r, ref = _renderer(config)
    hub = NativeHub(world)
    comms = [NativeComm.local(hub, k) for k in range(world)]
    ranks = []
    for k in range(world):  # two frame slots per rank over the shared scene and G-buffer
        slots = []
        for _ in range(2):
            rr = r.frame_slot()
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            slots.append((rr, st, NativeHaloFrame(rr, comms[k], throughput=True)))
        ranks.append(slots)
    torch.cuda.synchronize()
    frames = 4
    out, errors = {}, []

    def run(k):
        try:
            slots = ranks[k]
            pending = []

            def finish(j):
                rr, st, f = slots[j % 2]
                with torch.cuda.stream(st):
                    f.back()
                    out[(k, j)] = rr.ao.clone()

            for i in range(frames):
                rr, st, f = slots[i % 2]
                with torch.cuda.stream(st):
                    rr.ao.zero_()
                    f.front()
                pending.append(i)
                if len(pending) > 1:
                    finish(pending.pop(0))
            finish(pending.pop(0))
        except Exception:  # noqa: BLE001 -- reported by the main thread
            import traceback
            errors.append((k, traceback.format_exc()))

    threads = [threading.Thread(target=run, args=(k,)) for k in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=500)
    torch.cuda.synchronize()
    assert not errors, errors
    assert not any(t.is_alive() for t in threads)
    splits = set()
    for k in range(world):
        for j in range(frames):
            assert np.array_equal(out[(k, j)].cpu().numpy(), ref["ao"]), f"rank {k} frame {j} AO"
        for rr, _, f in ranks[k]:
            g = rr.numpy()
            for lo, hi in f.owned_sd_rows():
                assert bits_equal(g["sd"][:, lo:hi], ref["sd"][:, lo:hi]), f"rank {k} SD rows {lo}-{hi}"
            s = f.stats()
            assert s.frames == frames // 2 and s.world == world and s.rank == k
            splits.add(tuple(f.gb))
            b = f.bytes_per_frame()
            d = f.dense_bytes_per_frame()
            assert b["ao"] > 0 and b["intervals"] + b["sd"] <= d["intervals"] + d["sd"]
    assert len(splits) >= 1
    for slots in ranks:
        for _, _, f in slots:
            f.close()
    for c in comms:
        c.close()
    hub.close()
    r.close()


@pytest.mark.timeout(300)
def test_native_band_frame_camera_path_and_rebalance():
    """Every front() takes the renderer's current camera (an animated camera path: each rank renders the
    pose's G-buffer itself); the frames stay equal to the 1-GPU frame of each pose while the split
    re-balances from the measured times, and every rank computes the same split."""
    import torch
    from rsd.frame import camera_path
    from rsd.shard import NativeComm, NativeHaloFrame, NativeHub
    r, _ = _renderer("suntemple_1080p_q")
    poses = camera_path("orbit120")[:6]
    world = 4
    refs = []
    for p in poses:  # 1-GPU frames of the poses (the orbit of configs[4] around the hall)
        r.set_pose(*p)
        r.gbuffer()
        r.frame()
        refs.append(r.numpy()["ao"])
    hub = NativeHub(world)
    comms = [NativeComm.local(hub, k) for k in range(world)]
    slots = []
    for k in range(world):
        rr = r.frame_slot(own_gbuffer=True)
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        slots.append((rr, st, NativeHaloFrame(rr, comms[k])))
    torch.cuda.synchronize()
    out, errors = {}, []

    def run(k):
        try:
            rr, st, f = slots[k]
            with torch.cuda.stream(st):
                for i, p in enumerate(poses):
                    rr.set_pose(*p)
                    rr.gbuffer()
                    f.frame()
                    out[(k, i)] = rr.ao.clone()
        except Exception:  # noqa: BLE001
            import traceback
            errors.append((k, traceback.format_exc()))

    threads = [threading.Thread(target=run, args=(k,)) for k in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=250)
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(world):
        for i in range(len(poses)):
            assert np.array_equal(out[(k, i)].cpu().numpy(), refs[i]), f"rank {k} pose {i}"
    gbs = {tuple(s[2].gb) for s in slots}
    assert len(gbs) == 1  # every rank computed the same split
    for _, _, f in slots:
        f.close()
    for c in comms:
        c.close()
    hub.close()
    r.close()


def _rank_threads(world, run):
    threads = [threading.Thread(target=run, args=(k,)) for k in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=250)
    assert not any(t.is_alive() for t in threads)


@pytest.mark.timeout(300)
def test_native_band_frame_skewed_split_rebalances():
    """A deliberately skewed first split (rsd_band_frame_set_split: three ranks with one 32-row group each) is
    re-balanced from the measured per-rank times -- the re-split path on a live stream (tile-state voiding, region
    and buffer re-sizing) -- while every frame stays equal to the 1-GPU frame and every rank holds the same split
    (resplits > 0 asserted)."""
    import torch
    from rsd.shard import NativeComm, NativeHaloFrame, NativeHub
    r, ref = _renderer("suntemple_1080p_q")
    r.keep_clean_tiles()
    world, frames = 4, 13
    hub = NativeHub(world)
    comms = [NativeComm.local(hub, k) for k in range(world)]
    slots = []
    for k in range(world):
        rr = r.frame_slot()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        slots.append((rr, st, NativeHaloFrame(rr, comms[k])))
    G = slots[0][2].stats().groups
    skew = [0, 1, 2, 3, G]
    for _, _, f in slots:
        f.set_split(skew)
    torch.cuda.synchronize()
    out, errors, splits = {}, [], {}

    def run(k):
        try:
            rr, st, f = slots[k]
            with torch.cuda.stream(st):
                for i in range(frames):
                    rr.ao.zero_()
                    f.frame()
                    out[(k, i)] = rr.ao.clone()
                    splits[(k, i)] = tuple(f.gb)
        except Exception:  # noqa: BLE001
            import traceback
            errors.append((k, traceback.format_exc()))

    _rank_threads(world, run)
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(world):
        for i in range(frames):
            assert np.array_equal(out[(k, i)].cpu().numpy(), ref["ao"]), f"rank {k} frame {i}"
        g = slots[k][0].numpy()
        for lo, hi in slots[k][2].owned_sd_rows():
            assert bits_equal(g["sd"][:, lo:hi], ref["sd"][:, lo:hi]), f"rank {k} SD rows {lo}-{hi}"
    for i in range(frames):
        assert len({splits[(k, i)] for k in range(world)}) == 1, f"frame {i}: ranks disagree on the split"
    assert splits[(0, 0)] == tuple(skew)
    st = [f.stats() for _, _, f in slots]
    assert all(x.resplits >= 1 for x in st), [x.resplits for x in st]
    # the last rank held 3/4 of the rows: the re-balancing moved boundaries towards it
    assert splits[(0, frames - 1)][3] > 3
    for _, _, f in slots:
        f.close()
    for c in comms:
        c.close()
    hub.close()
    r.close()


@pytest.mark.timeout(300)
def test_native_band_frame_zoom_replans_halo():
    """A camera whose focal length changes between frames (a zoom) changes how far a sample reaches on screen:
    the band frame re-plans its windows and exchange regions, and every rank's frame of every pose
    stays equal to the 1-GPU frame."""
    import dataclasses

    import torch
    from rsd.frame import look_at
    from rsd.shard import NativeComm, NativeHaloFrame, NativeHub
    r, _ = _renderer("suntemple_1080p_q")
    sc = r.scene.camera
    poses = [dataclasses.replace(r.cfg, focal_length=f) for f in (21.0, 9.0, 35.0, 9.0, 14.0)]
    cams = [look_at(sc["pos"], sc["target"], sc["up"], c) for c in poses]
    refs = []
    for cam in cams:
        r.cam = cam
        r.gbuffer()
        r.frame()
        refs.append(r.numpy()["ao"])
    world = 4
    hub = NativeHub(world)
    comms = [NativeComm.local(hub, k) for k in range(world)]
    slots = []
    for k in range(world):
        rr = r.frame_slot(own_gbuffer=True)
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        slots.append((rr, st, NativeHaloFrame(rr, comms[k])))
    torch.cuda.synchronize()
    out, errors, halo = {}, [], {}

    def run(k):
        try:
            rr, st, f = slots[k]
            with torch.cuda.stream(st):
                for i, cam in enumerate(cams):
                    rr.cam = cam
                    rr.gbuffer()
                    rr.ao.zero_()
                    f.frame()
                    out[(k, i)] = rr.ao.clone()
                    halo[(k, i)] = int(f.stats().halo_px)
        except Exception:  # noqa: BLE001
            import traceback
            errors.append((k, traceback.format_exc()))

    _rank_threads(world, run)
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(world):
        for i in range(len(cams)):
            assert np.array_equal(out[(k, i)].cpu().numpy(), refs[i]), f"rank {k} pose {i}"
    assert halo[(0, 1)] > halo[(0, 0)] > halo[(0, 2)] and halo[(0, 3)] == halo[(0, 1)]
    for _, _, f in slots:
        f.close()
    for c in comms:
        c.close()
    hub.close()
    r.close()


@pytest.mark.timeout(300)
def test_rccl_world1_collectives_and_band_frame():
    """RCCL executes: a one-rank communicator (ncclCommInitRank, nranks = 1), an all-gather and a
    self send / receive on a torch stream, then the band frame over it, bit-identical to the 1-GPU frame."""
    import torch
    from rsd import abi
    from rsd.shard import NativeComm, NativeHaloFrame
    comm = NativeComm.rccl(0, 1)
    assert (comm.kind, comm.rank, comm.world) == (abi.COMM_RCCL, 0, 1)
    x = torch.arange(1000, dtype=torch.int32, device="cuda")
    y = torch.zeros(1000, dtype=torch.int32, device="cuda")
    comm.all_gather(y.view(1, -1), x)
    z = torch.zeros(1000, dtype=torch.int32, device="cuda")
    comm.exchange({0: x * 3}, {0: z})
    torch.cuda.synchronize()
    assert torch.equal(y, x) and torch.equal(z, x * 3)
    r, ref = _renderer("suntemple_1080p_q")
    f = NativeHaloFrame(r, comm)
    for _ in range(3):  # frame 2 relies on frame 1's consumed intervals
        r.ao.zero_()
        f.frame()
        torch.cuda.synchronize()
        g = r.numpy()
        assert np.array_equal(g["ao"], ref["ao"])
        assert bits_equal(g["sd"], ref["sd"])
    st = f.stats()
    assert st.frames == 3 and st.world == 1 and st.bytes_ao == 0  # one rank: nothing to send
    f.close()
    comm.close()
    r.close()


@pytest.mark.timeout(120)
def test_local_comm_exchange_checks_sizes():
    """The in-process communicator refuses a receive whose size the sender does not match (instead of
    copying past a buffer), with a message naming both ranks."""
    import torch
    from rsd import abi
    from rsd.shard import NativeComm, NativeHub
    hub = NativeHub(1)
    c = NativeComm.local(hub, 0)
    x = torch.ones(16, dtype=torch.int32, device="cuda")
    y = torch.zeros(32, dtype=torch.int32, device="cuda")
    with pytest.raises(abi.RsdError, match="expects 128 bytes from rank 0"):
        c.exchange({0: x}, {0: y})
    c.exchange({0: x}, {0: y[:16]})
    torch.cuda.synchronize()
    assert int(y[:16].sum()) == 16
    c.close()
    hub.close()
