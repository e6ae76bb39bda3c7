#!/usr/bin/env python3
"""Where the host time of an N > 1 band frame goes (diagnostics): HaloFrame.front() + back() of one rank
with the collectives stubbed out (as tools/scaling_model.py's host measurement), under cProfile, and
the per-call host time of each librsd entry / torch op it issues.

usage: python tools/halo_host_profile.py [config] [--world 8] [--rank 3] [--frames 100]

The last section times the native band frame (rsd_band_frame) of the same rank over the null communicator."""
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ray-traced-stochastic-depth-map_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from rsd.frame import CONFIGS, FrameConfig, Renderer  # noqa: E402
from rsd.scenes import make_scene  # noqa: E402
from rsd.shard import HaloFrame  # noqa: E402


def arg(flag, default):
    return sys.argv[sys.argv.index(flag) + 1] if flag in sys.argv else default


name = next((a for a in sys.argv[1:] if not a.startswith("--") and a in CONFIGS), "suntemple_1080p_q")
world, rank, frames = int(arg("--world", "8")), int(arg("--rank", "3")), int(arg("--frames", "100"))
kw, sc = CONFIGS[name]
r = Renderer(make_scene(sc), FrameConfig(**kw))
r.gbuffer()
dist.get_backend = lambda pg=None: "gloo"  # plans only: no process group


class NoComm:
    nccl = False

    def all_gather(self, out, inp):
        out[0].copy_(inp.view(out[0].shape))

    def exchange(self, sends, recvs):
        pass


for rebalance in (False, True):
    f = HaloFrame(r, rank, world, rebalance=rebalance, comm=NoComm())
    for _ in range(5):
        f.front()
        f.back()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(frames):
        f.front()
        f.back()
    host = (time.perf_counter() - t0) / frames * 1e6
    torch.cuda.synchronize()
    print(f"rebalance={rebalance}: host {host:.1f} us per frame (front + back, collectives stubbed)")
    if rebalance:
        continue
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(frames):
        f.front()
        f.back()
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())

# ---- the native band frame (rsd_band_frame): front() + back() are one librsd call each; the null communicator
#      (rsd_comm_null_create) stands in for RCCL, so this is librsd's host issue of one rank's frame.  Four frame
#      slots in flight (back() of frame i after front() of frames i+1..i+3, as bench.py), so the count matrix a
#      back() reads is normally complete; the stats split the host time into front, back and the count wait.
from rsd.shard import NativeComm, NativeHaloFrame  # noqa: E402

F = 4
for rebalance in (False, True):
    comm = NativeComm.null(rank, world)
    rends = [r] + [r.frame_slot() for _ in range(F - 1)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(F - 1)]
    fs = [NativeHaloFrame(x, comm, rebalance=rebalance, throughput=True) for x in rends]

    def run(n):
        pending = []
        for i in range(n):
            with torch.cuda.stream(streams[i % F]):
                fs[i % F].front()
            pending.append(i)
            if len(pending) > F - 1:
                j = pending.pop(0)
                with torch.cuda.stream(streams[j % F]):
                    fs[j % F].back()
        while pending:
            j = pending.pop(0)
            with torch.cuda.stream(streams[j % F]):
                fs[j % F].back()

    run(8)
    torch.cuda.synchronize()
    s0 = [f.stats() for f in fs]
    t0 = time.perf_counter()
    run(frames)
    host = (time.perf_counter() - t0) / frames * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / frames * 1e6
    s1 = [f.stats() for f in fs]
    d = lambda k: sum(getattr(b, k) - getattr(a, k) for a, b in zip(s0, s1)) / frames / 1e3  # noqa: E731
    blocked = sum(b.blocked_waits - a.blocked_waits for a, b in zip(s0, s1))
    print(f"native rebalance={rebalance}: host {host:.1f} us per frame (Python loop), librsd front {d('host_front_ns'):.1f}"
          f" + back {d('host_back_ns'):.1f} us (of which count wait {d('host_wait_ns'):.1f} us, {blocked} of {frames} "
          f"back() calls blocked), wall {wall:.1f} us per frame; collectives stubbed, world {world} rank {rank}")
    for f in fs:
        f.close()
    comm.close()
