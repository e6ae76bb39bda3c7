"""Contiguous screen bands on the GPU (rsd/shard.py HaloFrame, the multi-GPU split of SURVEY 8(e)):

  * the row-range entry points (rsd_svao_pass1_rows, rsd_sd_trace_rows, rsd_svao_pass2_rows)
    over a partition of the frame give the full-frame call bit for bit;
  * HaloFrame with 3 ranks (gloo, sharing this GPU -- RCCL needs one GPU per rank; the 8-GPU
    run is the driver's) gives every rank the 1-GPU AO image, and each rank's own SD rows equal
    the 1-GPU SD map."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CONFIG = "suntemple_1080p_q"


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _plan(r, world):
    """HaloFrame's partition without a process group (its constructor only reads dist for world > 1)."""
    import torch.distributed as dist

    from rsd.shard import HaloFrame
    orig = dist.get_backend
    dist.get_backend = lambda pg=None: "gloo"
    try:
        return [HaloFrame(r, k, world) for k in range(world)]
    finally:
        dist.get_backend = orig


@pytest.mark.timeout(300)
def test_row_ranges_union_equals_full_frame():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS[CONFIG]
    r = Renderer(make_scene(name), FrameConfig(**kw))
    r.gbuffer()
    r.frame()
    ref = r.numpy()
    plans = _plan(r, 5)
    r.ao.zero_()
    r.stencil.zero_()
    r.sd.zero_()
    r.clear_intervals()
    for p in plans:
        r.pass1_rows(p.px_rows[p.rank])
    g = r.numpy()
    assert np.array_equal(g["ray_min"], ref["ray_min"]) and np.array_equal(g["ray_max"], ref["ray_max"])
    assert np.array_equal(g["stencil"], ref["stencil"])
    for p in plans:
        r.sd_trace_rows(p.sd_rows[p.rank])
    for p in plans:
        r.pass2_rows(p.px_rows[p.rank])
    g = r.numpy()
    assert bits_equal(g["sd"], ref["sd"])
    assert np.array_equal(g["ao"], ref["ao"])
    # the tiled split (HaloFrame's default): every rank's round-robin 8-row tiles, traced as bands
    r.sd.zero_()
    for p in plans:
        assert p.sd_split == "tiles"
        p.trace()
    assert bits_equal(r.numpy()["sd"], ref["sd"])
    # consume: a band trace resets the WHOLE interval map
    r.sd_trace_rows(plans[2].sd_rows[2], consume=True)
    g = r.numpy()
    assert (g["ray_max"] == 0).all() and (g["ray_min"] == np.uint32(0x7F7FFFFF)).all()
    r.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    for p in (str(root), str(root / "ray-traced-stochastic-depth-map_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    from rsd.shard import HaloFrame
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    kw, name = CONFIGS[CONFIG]
    r = Renderer(make_scene(name), FrameConfig(**kw))
    r.gbuffer()
    f = HaloFrame(r, rank, world)
    for i in range(4):  # frame 2 relies on frame 1's consume; frames 3-4 run re-balanced splits
        r.ao.zero_()
        f.frame()
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, f"ao_{rank}_{i}.npy"), r.ao.cpu().numpy())
    g = r.numpy()
    np.save(os.path.join(out_dir, f"sdrows_{rank}.npy"), np.array(f.owned_sd_rows()))
    np.save(os.path.join(out_dir, f"ao_{rank}.npy"), g["ao"])
    np.save(os.path.join(out_dir, f"sd_{rank}.npy"), g["sd"])
    np.save(os.path.join(out_dir, f"bytes_{rank}.npy"), np.array(list(f.bytes_per_frame().values())))
    dist.barrier()
    dist.destroy_process_group()
    r.close()


@pytest.mark.timeout(600)
def test_halo_frame_three_ranks_equals_one_gpu(tmp_path):
    import torch
    import torch.multiprocessing as mp
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    kw, name = CONFIGS[CONFIG]
    r = Renderer(make_scene(name), FrameConfig(**kw))
    r.gbuffer()
    r.frame()
    ref = r.numpy()
    plans = _plan(r, 3)
    full = r.ray_minmax.numel() * 4 + r.sd.numel() * 4
    r.close()
    torch.cuda.synchronize()
    mp.start_processes(_worker, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True, start_method="spawn")
    for k in range(3):
        assert np.array_equal(np.load(tmp_path / f"ao_{k}.npy"), ref["ao"]), f"rank {k} AO"
        for i in range(4):
            assert np.array_equal(np.load(tmp_path / f"ao_{k}_{i}.npy"), ref["ao"]), f"rank {k} AO frame {i}"
        sd = np.load(tmp_path / f"sd_{k}.npy")
        for lo, hi in np.load(tmp_path / f"sdrows_{k}.npy"):  # the SD rows (tiles) rank k traced
            assert bits_equal(sd[:, lo:hi], ref["sd"][:, lo:hi]), f"rank {k} SD rows {lo}-{hi}"
        iv, sd, _ = np.load(tmp_path / f"bytes_{k}.npy")
        assert iv + sd < full  # less than the whole interval + SD maps


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_halo_frame_sync_free_threads(world):
    """The N > 1 frame without host synchronisation: HaloFrame over LocalComm -- `world`
    host threads on this GPU, one HIP stream and one librsd device each, exchanges as device-to-device
    copies ordered by events (the stream semantics of RCCL) -- runs 4 frames per rank, two frame slots
    interleaved like bench.py's frames in flight (back() of a frame after front() of the next), under
    torch.cuda.set_sync_debug_mode("error"): no torch op of front() / back() waits for the GPU (the
    only host wait is the event of a frame's counts, one frame later).  Every frame of every rank
    equals the 1-GPU AO image; each rank's own SD rows equal the 1-GPU SD map."""
    import threading

    import torch
    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene
    from rsd.shard import HaloFrame, LocalComm, LocalHub
    kw, name = CONFIGS[CONFIG]
    scene = make_scene(name)
    r = Renderer(scene, FrameConfig(**kw))
    r.gbuffer()
    r.frame()
    ref = r.numpy()
    r.close()
    hub = LocalHub(world)
    ranks = []
    for k in range(world):  # setup (allocations, uploads, G-buffers) before the sync check
        slots = []
        comm = LocalComm(hub, k)  # one communicator per rank, shared by its frame slots
        for _ in range(2):
            rr = Renderer(scene, FrameConfig(**kw))
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                rr.gbuffer()
            slots.append((rr, st, HaloFrame(rr, k, world, comm=comm)))
        ranks.append(slots)
    torch.cuda.synchronize()
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

            for i in range(4):
                rr, st, f = slots[i % 2]
                with torch.cuda.stream(st):
                    rr.ao.zero_()
                    f.front()
                pending.append(i)
                if len(pending) > 1:
                    finish(pending.pop(0))
            finish(pending.pop(0))
        except Exception:  # noqa: BLE001 -- reported by the main thread, with the line that synchronised
            import traceback
            errors.append((k, traceback.format_exc()))

    torch.cuda.set_sync_debug_mode("error")
    try:
        threads = [threading.Thread(target=run, args=(k,)) for k in range(world)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=240)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(world):
        for j in range(4):
            assert np.array_equal(out[(k, j)].cpu().numpy(), ref["ao"]), f"rank {k} frame {j}"
        f = ranks[k][1][2]
        g = ranks[k][1][0].numpy()
        for lo, hi in f.owned_sd_rows():
            assert bits_equal(g["sd"][:, lo:hi], ref["sd"][:, lo:hi]), f"rank {k} SD rows {lo}-{hi}"
        assert f.frames == 2 and sum(f.bytes_per_frame().values()) > 0
    for slots in ranks:
        for rr, _, _ in slots:
            rr.close()
