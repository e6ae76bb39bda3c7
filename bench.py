#!/usr/bin/env python3
"""Headline benchmark: Ray-SD + SVAO on MI355X (BASELINE.json metric "Mrays/s + AO frames/s,
1080p 1/4-res Ray-SD, 1/2/4/8 MI355X"; definitions BASELINE.md section 4).

A step = one AO frame of the reference's SVAO::execute span (SVAO.cpp:327-455: clear ray
intervals, "AO 1", StochasticDepthMapRT, "AO 2") over the configs[1] workload by default:
Sun Temple stand-in (~0.6 M triangles, seed 2), 1920x1080 visible + 64-px guard band
(2048x1208 frame buffer), 1/4-res SD map (768x558 texels incl. the 128-texel SD guard),
N = 4, MAX_COUNT = 8.  Inputs (BVH, G-buffer) are resident in HBM before timing.

Two timed regions, each K frames between a barrier + torch.cuda.synchronize() pair:

  latency    one frame in flight (the reference's own schedule: one frame after the other).
             HIP events around every SD trace and around every AO span (clear -> pass 1 ->
             trace -> pass 2) give BASELINE.md's two numbers:
               value (Mrays/s)     = dispatched SD rays / SD-kernel time   (whole job)
               active_mrays_per_s  = active SD rays (TMin <= TMax) / SD-kernel time
               ao_frames_per_s     = 1 / AO-span time
  throughput F frames in flight (--frames-in-flight, default 4): frame i runs on HIP stream
             i % F with its own frame buffers, frames of different slots overlap (the latency-
             bound SD trace of one frame shares the machine with the VALU-bound passes of
             others; traces are flagged RSD_SD_THROUGHPUT, which librsd may use to pick a walk).
               ms_per_step, throughput.ao_frames_per_s, throughput.frame_mrays_per_s

--camera-path orbit120 (default for configs[4], bistro_4k_full_n16): every frame renders the
next pose of a 120-pose orbit (rsd.frame.camera_path): camera update + G-buffer + AO frame.
The G-buffer is inside the frame's wall time but outside the AO span (AO frames/s
excludes the G-buffer).

Multi-GPU (torchrun, one rank per GPU), sharding modes (--shard):
  band (the default for every config): the north_star's screen split (rsd/shard.py HaloFrame) --
    each frame is split into contiguous screen bands re-balanced from the previous frame's
    per-band time; pass 1 of the rank's rows, a SPARSE interval halo (only the SD texels its
    samples touched, as (index, rayMin, rayMax) triples; point-to-point send / recv = ncclSend /
    ncclRecv under RCCL), trace of the rank's SD rows, a sparse SD halo (the depths of exactly
    those texels), pass 2 of the rank's rows, AO all-gather.  Strong scaling.
  frame: frames are the independent units -- every rank renders whole frames (its own frame
    stream, BVH + G-buffer replicated), no data-path collective.  Weak scaling.
  gather: round-1 v1 of band -- interleaved bands, whole-map interval all-reduce and SD all-gather.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "ray-traced-stochastic-depth-map_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
DEFAULT_CONFIG = "suntemple_1080p_q"
# committed rocprofv3 passes of the default bench (newest round first)
PROFILE_DIRS = [ROOT / "profiles" / "round6", ROOT / "profiles" / "round5", ROOT / "profiles" / "round4", ROOT / "profiles" / "round3",
                ROOT / "profiles" / "round2", ROOT / "profiles" / "round1"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default=DEFAULT_CONFIG)
    ap.add_argument("--camera-path", default=None,
                    help="static | orbitN (default: the config's own, orbit120 for bistro_4k_full_n16)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0,
                    help="target wall time of the bounded CPU-oracle sample (0 disables)")
    ap.add_argument("--frames-in-flight", type=int, default=4,
                    help="throughput region: frame i runs on stream i %% F with its own frame buffers")
    ap.add_argument("--shard", choices=("frame", "band", "gather"), default=None,
                    help="N > 1: band (default) = each frame split into contiguous, re-balanced screen bands "
                         "with sparse interval / SD halo exchanges (point-to-point RCCL) + AO all-gather (strong "
                         "scaling, the north_star split); frame = every rank renders whole frames (weak scaling, "
                         "no per-frame collective); gather = interleaved bands with whole-map all-reduce / "
                         "all-gather (round-1 v1)")
    ap.add_argument("--clean-tiles", choices=("on", "off"), default="on",
                    help="SD traces skip rewriting 8x8 tiles they left at DEFAULT_DEPTH without a live ray "
                         "(rsd_sd_params.d_tile_state; same bits; off: every texel every frame)")
    ap.add_argument("--frame-impl", choices=("native", "python"), default="native",
                    help="N > 1 band frames: native = rsd_band_frame (the frame's passes and exchanges issued from C++, "
                         "RCCL communicators driven by librsd: one per frame slot); python = rsd/shard.py HaloFrame "
                         "(torch.distributed collectives; also the gloo rehearsal's path)")
    ap.add_argument("--scene-file", default=None,
                    help="a .pyscene or .obj scene (rsd.pyscene / rsd.ingest) instead of the config's stand-in "
                         "scene; the config still sets the frame, SD map and N")
    ap.add_argument("--pmc-csv", nargs="*", default=None,
                    help="rocprofv3 --pmc counter_collection.csv file(s) with FETCH_SIZE / WRITE_SIZE for "
                         "roofline.traffic (default: the committed passes of the default config)")
    ap.add_argument("--hit-order-record", type=int, default=1,
                    help="1: add the hit_order_traversal sub-record (the latency region again with the DXR-like "
                         "traversal-order any-hit stream, rsd_hit_order TRAVERSAL); 0: skip it")
    ap.add_argument("--local-ranks", type=int, default=1,
                    help="pre-flight of the N > 1 path on ONE GPU: run this many ranks as threads of this process over "
                         "librsd's in-process communicator, through the same band-frame code as a torchrun launch "
                         "(native frames, per-rank counter reductions, summed value / roofline, lag = F - 1 schedule); "
                         "a rehearsal of the driver's multi-GPU run, not a measurement of N GPUs")
    ap.add_argument("--timing-events", choices=("hip", "torch", "off"), default="hip",
                    help="per-kernel timing events: hip = fence-free timing events (rsd.timing, default); "
                         "torch = torch.cuda.Event (a system-scope fence per record); off = none in the "
                         "throughput region (the latency region still needs them for value)")
    return ap.parse_args()


def host_cpus():
    """The CPUs the baseline may use and what they are (cores + model)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:  # cgroup v2 CPU quota ("max 100000" = none)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    # the CPU time the process may actually use: the affinity mask capped by the cgroup quota
    # (a 256-CPU mask under a 16-CPU quota runs at most 16 CPUs' worth of threads at once)
    effective = usable if quota is None else max(1, min(usable, math.ceil(quota)))
    return {"usable": usable, "nproc": os.cpu_count(), "cgroup_cpu_quota": quota, "effective": effective,
            "model": model}


class SoloGroup:
    """One rank (N = 1)."""
    rank, world, native_ok, kind = 0, 1, False, "solo"

    def barrier(self):
        pass

    def reduce(self, values, op):
        return [float(v) for v in values]

    def comms(self, n, device):
        return [], "one rank"

    def close(self):
        pass


class TorchGroup:
    """One process per GPU under torchrun: torch.distributed (nccl = RCCL, or gloo for rehearsals); the band
    frame's own communicators are librsd's RCCL ones, created collectively (NativeComm.rccl_group)."""
    kind = "torch.distributed"

    def __init__(self, rank, world, backend, device):
        import torch.distributed as dist
        self.dist, self.rank, self.world, self.backend, self.device = dist, rank, world, backend, device
        self.native_ok = backend == "nccl"

    def barrier(self):
        self.dist.barrier()

    def reduce(self, values, op):
        import torch
        t = torch.tensor([float(v) for v in values], dtype=torch.float64,
                         device=self.device if self.backend == "nccl" else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return [float(x) for x in t.tolist()]

    def comms(self, n, device):
        from rsd.shard import NativeComm
        return NativeComm.rccl_group(self.rank, self.world, n, device=device)

    def close(self):
        self.dist.destroy_process_group()


class ThreadGroup:
    """--local-ranks N: rank k of N threads of this process sharing one GPU (the pre-flight of the N > 1 path):
    barriers and reductions through host memory, the band frame's exchanges through librsd's in-process
    communicator (one hub per frame slot, like one RCCL communicator per slot under torchrun)."""
    kind = "threads (in-process communicator, one GPU)"
    native_ok = True

    def __init__(self, rank, shared):
        self.rank, self.world, self.sh = rank, shared["world"], shared

    def barrier(self):
        self.sh["barrier"].wait()

    def reduce(self, values, op):
        sh = self.sh
        sh["slots"][self.rank] = [float(v) for v in values]
        sh["barrier"].wait()
        cols = list(zip(*sh["slots"]))
        out = [max(c) if op == "max" else math.fsum(c) for c in cols]
        sh["barrier"].wait()  # every rank read the slots before the next reduction writes them
        return out

    def comms(self, n, device):
        from rsd.shard import NativeComm
        return [NativeComm.local(self.sh["hubs"][j], self.rank) for j in range(n)], None

    def close(self):
        pass


def main():
    args = parse()
    if args.local_ranks > 1:
        return run_threads(args)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    grp = SoloGroup()
    if world > 1:
        import torch.distributed as dist
        # RSD_BENCH_BACKEND=gloo: rehearsal of the N > 1 code paths with several ranks on one GPU
        # (RCCL needs one GPU per rank); production runs use nccl = RCCL with LOCAL_RANK = GPU
        backend = os.environ.get("RSD_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group(backend)
        grp = TorchGroup(rank, world, backend, torch.device("cuda", local))
    run_rank(args, grp, local)


def run_threads(args):
    """--local-ranks N: N rank threads over one GPU through run_rank (the same N > 1 code as torchrun's ranks).
    The scene, its BVH and the device handle are shared (one GPU); every rank has its own renderer, frame
    buffers, G-buffer, streams and band frames."""
    import threading

    import torch

    from rsd.frame import CONFIGS, Device, GpuScene
    from rsd.scenes import make_scene
    from rsd.shard import NativeHub
    world = args.local_ranks
    F = max(1, args.frames_in_flight)
    torch.cuda.set_device(0)
    _, scene_name = CONFIGS[args.config]
    if args.scene_file:
        from rsd.pyscene import load_scene_file
        scene = load_scene_file(args.scene_file).build(os.path.basename(args.scene_file))
    else:
        scene = make_scene(scene_name)
    dev = Device(0)
    gs = GpuScene(dev, scene)
    shared = {"world": world, "barrier": threading.Barrier(world), "slots": [None] * world,
              "hubs": [NativeHub(world) for _ in range(F)], "scene": scene, "gscene": gs, "dev": dev}
    errors = []

    def rank_main(k):
        try:
            with torch.cuda.stream(torch.cuda.Stream()):  # this rank's own default stream (torch's is per thread)
                run_rank(args, ThreadGroup(k, shared), 0, shared)
        except BaseException:  # noqa: BLE001 -- reported below; the other ranks may then wait at a barrier
            import traceback
            errors.append((k, traceback.format_exc()))
            shared["barrier"].abort()

    threads = [threading.Thread(target=rank_main, args=(k,)) for k in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    torch.cuda.synchronize()
    for h in shared["hubs"]:
        h.close()
    gs.release()
    dev.close()
    if errors:
        for k, tb in errors:
            print(f"bench.py: rank thread {k} failed:\n{tb}", file=sys.stderr)
        raise SystemExit(1)


def run_rank(args, grp, local, shared=None):
    """One rank's bench (rank 0 prints the line): grp = SoloGroup (N = 1), TorchGroup (torchrun, one GPU per
    rank) or ThreadGroup (--local-ranks: rank threads sharing one GPU)."""
    import numpy as np
    import torch

    from rsd import abi
    from rsd.frame import CONFIGS, DEFAULT_CAMERA_PATH, FrameConfig, Renderer, camera_path
    from rsd.scenes import make_scene
    from rsd.shard import BandFrame, HaloFrame, NativeHaloFrame

    rank, world = grp.rank, grp.world
    dist = grp if world > 1 else None
    kw, scene_name = CONFIGS[args.config]
    cfg = FrameConfig(**kw)
    shard = args.shard or "band"
    path_name = args.camera_path or DEFAULT_CAMERA_PATH.get(args.config, "static")
    poses = camera_path(path_name)
    if shared is not None:
        scene = shared["scene"]
        scene_name = scene.name
        r = Renderer(scene, cfg, device=local, gpu_scene=shared["gscene"], dev=shared["dev"])
    else:
        if args.scene_file:
            from rsd.pyscene import load_scene_file
            scene_name = os.path.basename(args.scene_file)
            scene = load_scene_file(args.scene_file).build(scene_name)
        else:
            scene = make_scene(scene_name)
        r = Renderer(scene, cfg, device=local)
    # clean tiles: band frames void the stamps on a re-split; the gather split all-reduces whole maps
    r.keep_clean_tiles(args.clean_tiles == "on" and shard != "gather")
    bvh_build_s = r.gscene.info.build_ms * 1e-3
    bw = (rank, world) if shard == "gather" else (0, 1)
    F = max(1, args.frames_in_flight)
    # N > 1 band frames issued from C++ (rsd_band_frame) over librsd's own communicators -- one per frame slot,
    # so every communicator's operations stay on one stream: RCCL under torchrun (created collectively: the ranks
    # fall back to rsd/shard.py HaloFrame together when any rank cannot), in-process for rank threads; the gloo
    # rehearsal keeps HaloFrame
    native = shard == "band" and world > 1 and grp.native_ok and args.frame_impl == "native"
    comms = []
    if native:
        comms, why = grp.comms(F, torch.device("cuda", local))
        if not comms:
            if rank == 0:
                print(f"bench.py: librsd's RCCL communicators are not usable ({why}); every rank falls back to "
                      "rsd/shard.py HaloFrame", file=sys.stderr)
            native = False

    def make_frame(rend, throughput=False, slot=0):
        if shard == "band":
            if native:
                return NativeHaloFrame(rend, comms[slot], throughput=throughput)
            return HaloFrame(rend, rank, world, throughput=throughput)
        return BandFrame(rend, *bw, throughput=throughput)

    seq = make_frame(r)  # latency region: one frame in flight, the latency-optimised trace walk
    n_poses = len(poses) if poses else 1

    def pose(rend, i):
        if poses:
            rend.set_pose(*poses[i % n_poses])
            rend.gbuffer()

    # ---- instrumented traces (untimed): traversal counters for the roofline bytes, for both
    #      walks, averaged over the poses the timed frames render
    if not poses:
        r.gbuffer()
    cnt_seq, cnt_thr = [], []
    for i in range(min(args.steps, n_poses)):
        pose(r, i)
        for acc, thr in ((cnt_seq, False), (cnt_thr, True)):
            # pass 1 over the whole frame = the exact interval union a band frame all-reduces
            r.clear_intervals()
            r.pass1()
            if shard == "band" and seq.sd_band is not None:  # N > 1: this rank's round-robin SD tiles
                acc.append(r.sd_trace(counters=True, band=seq.sd_band, throughput=thr))
            elif shard == "band":  # the SD rows under this rank's band
                acc.append(r.sd_trace_rows(seq.owned_sd_rows()[0], counters=True, throughput=thr))
            else:
                acc.append(r.sd_trace(counters=True, throughput=thr, band=bw))
    torch.cuda.synchronize()
    walk_seq, walk_thr = int(cnt_seq[0].walk), int(cnt_thr[0].walk)
    walk_seq_inst = int(cnt_seq[0].walk_instrumented)
    mean_cnt = lambda cs, f: float(np.mean([getattr(c, f) for c in cs]))  # noqa: E731
    if dist:
        dist.barrier()

    def timed(fn, n):
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(n)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if dist:
            wall = dist.reduce([wall], "max")[0]
        return wall

    # ---- latency region: one frame in flight, the latency-optimised trace walk
    # per-kernel timing: fence-free HIP events by default -- a torch.cuda.Event record carries a
    # system-scope release fence that left ~5 us bubbles in the stream it sat in (rsd/timing.py)
    if args.timing_events == "torch":
        new_ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    else:
        from rsd.timing import TimingEvent as new_ev
    mk_ev = lambda n: [(new_ev(), new_ev()) for _ in range(n)]  # noqa: E731
    ev_sd, ev_ao = mk_ev(args.steps), mk_ev(args.steps)

    def run_seq(n, timed_ev=True):
        for i in range(n):
            pose(r, i)
            if timed_ev:
                ev_ao[i][0].record()
            seq.frame(sd_events=ev_sd[i] if timed_ev else None)
            if timed_ev:
                ev_ao[i][1].record()

    run_seq(args.warmup, timed_ev=False)
    wall_seq = timed(run_seq, args.steps)
    seq_sd_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_sd]))
    seq_ao_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_ao]))

    # ---- throughput region: F frames in flight on F streams
    slots = [make_frame(r, throughput=F > 1)] + \
        [make_frame(r.frame_slot(own_gbuffer=bool(poses)), throughput=True, slot=j) for j in range(1, F)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(F - 1)]
    for st in streams[1:]:
        st.wait_stream(streams[0])
    thr_ev = args.timing_events != "off"
    ev_thr = mk_ev(args.steps) if thr_ev else None

    # N > 1 band frames: back() of frame i is issued after front() of the next F - 1 frames, so the
    # host reads frame i's exchange counts once they are long complete (HaloFrame: no host wait
    # drains the frames in flight); 1 rank: one rsd_svao_frame call per frame
    lag = F - 1 if shard == "band" and world > 1 else 0

    # native band frames without a camera path: librsd's calls take each slot's stream explicitly, without a torch
    # stream context per call (~6 us of host time each; at N >= 4 a rank's frame is host-bound)
    raw = [st.cuda_stream for st in streams]
    direct = native and lag and not poses

    def run_thr(n, timed_ev=thr_ev):
        pending = []

        def finish(j):
            if direct:
                slots[j % F].back(sd_events=ev_thr[j] if timed_ev else None, stream=raw[j % F])
                return
            with torch.cuda.stream(streams[j % F]):
                slots[j % F].back(sd_events=ev_thr[j] if timed_ev else None)

        for i in range(n):
            if direct:
                slots[i % F].front(stream=raw[i % F])
            else:
                with torch.cuda.stream(streams[i % F]):
                    pose(slots[i % F].b, i)
                    if lag:
                        slots[i % F].front()
                    else:
                        slots[i % F].frame(sd_events=ev_thr[i] if timed_ev else None)
            if lag:
                pending.append(i)
                if len(pending) > lag:
                    finish(pending.pop(0))
        while pending:
            finish(pending.pop(0))

    run_thr(args.warmup, timed_ev=False)
    wall_thr = timed(run_thr, args.steps)
    thr_sd_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_thr])) if thr_ev else float("nan")

    if dist:  # per-kernel times: the slowest rank
        seq_sd_ms, seq_ao_ms, thr_sd_ms = dist.reduce([seq_sd_ms, seq_ao_ms, thr_sd_ms], "max")

    # N > 1 band frames (untimed): one more frame of the split, checked on rank 0 against the 1-GPU frame of the same
    # pose (rsd_svao_frame on a frame slot of its own) -- every rank's gathered AO image must be those bits
    band_check = None
    if world > 1 and shard == "band":
        pose(r, 0)
        r.ao.zero_()
        seq.frame()
        torch.cuda.synchronize()
        if rank == 0:
            one = r.frame_slot(own_gbuffer=True)
            one.gbuffer()
            one.frame()
            torch.cuda.synchronize()
            band_check = {"ao_equals_one_gpu": bool(torch.equal(one.ao, r.ao)),
                          "note": "rank 0's gathered AO image of one band frame vs rsd_svao_frame of the same pose"}
        if dist:
            dist.barrier()

    rays = r.sd_rays
    N = cfg.sd_samples
    # frame mode: every rank renders whole frames; band mode: the ranks share each frame
    units = world if shard == "frame" else 1
    rays_active = mean_cnt(cnt_seq, "rays_active")
    # the segment entry grid's lookups: one 16-B hash slot + 32 B per frontier item tested
    entry_bytes = 16 * mean_cnt(cnt_seq, "entry_lookups") + 32 * mean_cnt(cnt_seq, "entry_items")
    if dist and shard != "frame":  # counters are per band: the frame's totals
        rays_active, nodes_seq, tris_seq, entry_bytes = dist.reduce(
            [rays_active, mean_cnt(cnt_seq, "nodes_visited"), mean_cnt(cnt_seq, "tris_tested"), entry_bytes], "sum")
    else:
        nodes_seq, tris_seq = mean_cnt(cnt_seq, "nodes_visited"), mean_cnt(cnt_seq, "tris_tested")
    value = units * rays / (seq_sd_ms * 1e-3) / 1e6
    # B_ray = 16 (linearZ bilinear) + 8 (rayMin+rayMax) + 4N (store) + node bytes + 48 n_tri
    # (+ the entry grid's lookups, which replace the top of the walk);
    # librsd's nodes are 4-wide (128 B per visit = two of SURVEY's 64-B BVH2 nodes).  Per launch =
    # per frame (band mode: the whole frame's bytes over the slowest rank's trace time).
    # (the store term counts only the texels written: clean tiles, --clean-tiles, are not rewritten)
    texels_clean = mean_cnt(cnt_seq, "texels_clean")
    if dist and shard != "frame":
        texels_clean = dist.reduce([texels_clean], "sum")[0]
    alg_bytes = rays * (16 + 8) + (rays - texels_clean) * 4 * N + 128 * nodes_seq + 48 * tris_seq + entry_bytes
    achieved = alg_bytes / (seq_sd_ms * 1e-3) / 1e9
    kernels_seq = abi.WALK_KERNELS[walk_seq]
    if r.sd_w * r.sd_h > 2_000_000 and walk_seq != abi.WALK_RASTER:
        # the full-resolution maps' two-pass setup (sd_trace.hip: sd_classify_kernel + sd_live_kernel above 2 M
        # texels) in place of the one-pass setup kernel
        kernels_seq = ("sd_classify_kernel", "sd_live_kernel") + tuple(k for k in kernels_seq if k != "sd_setup_kernel")
    lat = latency_floor(cnt_seq, seq_sd_ms)
    if lat.get("latency_floor_us") is not None:
        # the step clocks come from the instrumented launch, which walks the row or quad walk alone -- for the hybrid
        # launch (walk 6), the row walk its first blocks run over the longest-first rays
        lat["latency_walk"] = abi.WALK_NAMES[walk_seq_inst]
    pmc = args.pmc_csv
    if pmc is None and not args.scene_file:
        # the committed passes of this config (tools/config_measure.sh -> profiles/roundN/configs/<config>/),
        # or of the default config (tools/round_measure.sh -> profiles/roundN/)
        for d in PROFILE_DIRS:
            dd = d / "configs" / args.config
            cands = [[dd / "pmc_fetch_size.csv", dd / "pmc_write_size.csv"]]
            if args.config == DEFAULT_CONFIG and not poses:
                cands.append([d / "pmc_fetch_size.csv", d / "pmc_write_size.csv"])
            cand = next((c for c in cands if all(p.exists() for p in c)), None)
            if cand:
                pmc = [str(p) for p in cand]
                break
    pmc = [p for p in (pmc or []) if Path(p).exists()]
    traffic = pmc_traffic(pmc, kernels_seq)
    valu_csv = next((d / "pmc_sq_valu.csv" for d in PROFILE_DIRS if (d / "pmc_sq_valu.csv").exists()), None)

    # DXR-like any-hit order (rsd_hit_order TRAVERSAL): the same latency region with
    # the traversal-order hit stream -- the mode closest to the reference's DXR semantics
    # (Common.slangh:137-151: the reservoir samples among the hits in traversal order)
    hit_trav = hit_wave = None
    if world == 1 and args.hit_order_record:
        hit_trav = hit_order_record(r, HaloFrame, new_ev, min(args.steps, 50), min(args.warmup, 5), pose,
                                    rays, rays_active)
        # the wavefront order (round 5): the same stochastic semantics on the row walk's traversal
        hit_wave = hit_order_record(r, HaloFrame, new_ev, min(args.steps, 50), min(args.warmup, 5), pose,
                                    rays, rays_active, order=abi.HIT_ORDER_WAVEFRONT)

    if rank != 0:
        close_frames([seq] + slots, comms)
        grp.close()
        return

    cpu = None
    if args.cpu_baseline_seconds > 0 and world == 1:
        cpu = cpu_baseline(r, scene, args.cpu_baseline_seconds, poses)

    frames_thr = args.steps * units
    rel = lambda p: str(Path(p).relative_to(ROOT)) if Path(p).is_relative_to(ROOT) else str(p)  # noqa: E731
    line = {
        "metric": "Mrays/s + AO frames/s, 1080p 1/4-res Ray-SD, 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_thr / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if shard != "frame" and world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded procedural stand-in scene; no reference assets in the container)",
        "config": {"workload": args.config, "scene": scene_name, "triangles": scene.triangle_count,
                   "frame_buffer": [cfg.fb_w, cfg.fb_h], "visible": [cfg.visible_w, cfg.visible_h],
                   "sd_map": [r.sd_w, r.sd_h], "sd_samples": N, "max_count": cfg.max_count,
                   "stoch_map_divisor": cfg.divisor, "camera_path": path_name,
                   "parallelism": {"band": f"screen-band+halo x{world}", "gather": f"screen-band+allgather x{world}",
                                   "frame": f"frame-parallel x{world}"}[shard],
                   "frame_impl": (("native (rsd_band_frame, librsd in-process communicator)" if args.local_ranks > 1
                                   else "native (rsd_band_frame, librsd RCCL communicators)") if native else
                                  "python (rsd/shard.py)") if shard == "band" and world > 1 else "rsd_svao_frame",
                   "frames_in_flight": F},
        "value_definition": "dispatched SD rays / SD-kernel time (HIP events around every rsd_sd_trace of the "
                            "latency region; BASELINE.md section 4), summed over ranks",
        "sd_kernel_ms": round(seq_sd_ms, 4),
        "rays_dispatched": rays * units,
        "active_rays": int(round(rays_active)) * units,
        "active_mrays_per_s": round(units * rays_active / (seq_sd_ms * 1e-3) / 1e6, 2),
        "ao_frames_per_s": round(units * 1e3 / seq_ao_ms, 2),
        "ao_span_ms": round(seq_ao_ms, 4),
        "latency": {"ms_per_frame": round(wall_seq / args.steps * 1e3, 4), "frames": args.steps,
                    "walk": abi.WALK_NAMES[walk_seq],
                    "note": "one frame in flight; ms_per_frame includes the G-buffer of a camera path, "
                            "ao_span_ms does not"},
        "throughput": {"frames_in_flight": F, "frames": frames_thr, "ms_per_frame": round(wall_thr / args.steps * 1e3, 4),
                       "ao_frames_per_s": round(frames_thr / wall_thr, 2),
                       "frame_mrays_per_s": round(rays * frames_thr / wall_thr / 1e6, 2),
                       "sd_kernel_ms_overlapped": round(thr_sd_ms, 4) if thr_ev else None,
                       "timing_events": args.timing_events,
                       "walk": abi.WALK_NAMES[walk_thr]},
        "traversal": {"nodes_per_ray": round(nodes_seq / rays / units, 3),
                      "tris_per_ray": round(tris_seq / rays / units, 3),
                      "nodes_per_active_ray": round(nodes_seq / max(rays_active, 1), 2),
                      "tris_per_active_ray": round(tris_seq / max(rays_active, 1), 2),
                      "max_steps_per_ray": int(max(c.max_steps_per_ray for c in cnt_seq))},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "rsd_sd_trace = " + " + ".join(kernels_seq),
                     "alg_bytes_per_launch": int(alg_bytes),
                     "duration_us": round(seq_sd_ms * 1e3, 2),
                     "note": "achieved = SURVEY 8(d) algorithmic bytes of one trace / its HIP-event duration in "
                             "the latency region; traffic = FETCH_SIZE + WRITE_SIZE of the same kernels "
                             "(per launch, committed rocprofv3 --pmc passes)",
                     "traffic_source": ", ".join(rel(p) for p in pmc) or None,
                     **lat},
        # the frame's largest kernel is pass 1, bound by VALU issue rather than HBM
        "pass1_roofline": pmc_valu(valu_csv, "svao_pass1_kernel") if valu_csv and args.config == DEFAULT_CONFIG and not args.scene_file
        else None,
        "exchange_bytes_per_frame": dict(seq.bytes_per_frame(), dense_halo_equivalent=seq.dense_bytes_per_frame(),
                                         final_split_groups=list(seq.gb))
        if shard == "band" and world > 1 else None,
        "band_check": band_check,
        "hit_order_traversal": hit_trav,
        "hit_order_wavefront": hit_wave,
        "bvh_build_s": round(bvh_build_s, 3),
        "bvh_build_threads": int(r.gscene.info.build_threads),
        "cpu_baseline": cpu,
    }
    if isinstance(grp, ThreadGroup):
        line["n_gpus"] = 1
        line["preflight"] = {"ranks": world, "group": grp.kind,
                             "note": "--local-ranks: the N > 1 band-frame path run by N rank threads sharing ONE GPU "
                                     "over librsd's in-process communicator -- the same bench.py code as a torchrun "
                                     "launch, a rehearsal of the driver's multi-GPU run; its times are not those of "
                                     "N GPUs (the ranks share one GPU and one Python interpreter)"}
    print(json.dumps(line))
    close_frames([seq] + slots, comms)
    grp.close()


def close_frames(frames, comms):
    """Release the native band frames before their communicators (each waits for its stream)."""
    for f in frames:
        if hasattr(f, "close"):
            f.close()
    for c in comms:
        c.close()


def hit_order_record(r, frame_cls, new_ev, steps, warmup, pose, rays, rays_active, order=None):
    """The latency region with a DXR-like hit stream (rsd.h RSD_HIT_ORDER_TRAVERSAL: a depth-first walk of the
    4-wide BVH delivering each triangle once in leaf order, a commit shrinking TMax -- DXR's any-hit semantics,
    StochasticDepthMapRT.rt.slang:83-88; or RSD_HIT_ORDER_WAVEFRONT: the same semantics over the 8-wide
    wavefront traversal of the row walk): SD-trace time, dispatched / active Mrays/s and the AO span over
    `steps` frames, one in flight."""
    import numpy as np
    import torch

    from rsd import abi
    order = abi.HIT_ORDER_TRAVERSAL if order is None else order
    keep = r.sdp
    sdp = abi.SDParams.from_buffer_copy(keep)
    sdp.hit_order = order
    r.sdp = sdp
    try:
        fr = frame_cls(r)
        ev_sd = [(new_ev(), new_ev()) for _ in range(steps)]
        ev_ao = [(new_ev(), new_ev()) for _ in range(steps)]
        for i in range(warmup):
            pose(r, i)
            fr.frame()
        for i in range(steps):
            pose(r, i)
            ev_ao[i][0].record()
            fr.frame(sd_events=ev_sd[i])
            ev_ao[i][1].record()
        torch.cuda.synchronize()
        sd_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_sd]))
        ao_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_ao]))
    finally:
        r.sdp = keep
    name = {abi.HIT_ORDER_TRAVERSAL: ("ordered", "RSD_HIT_ORDER_TRAVERSAL", "sd_trace_ordered_kernel"),
            abi.HIT_ORDER_WAVEFRONT: ("wavefront", "RSD_HIT_ORDER_WAVEFRONT", "sd_trace_wavefront_kernel")}[order]
    return {"frames": steps, "walk": name[0], "sd_kernel_ms": round(sd_ms, 4),
            "mrays_per_s": round(rays / (sd_ms * 1e-3) / 1e6, 1),
            "active_mrays_per_s": round(rays_active / (sd_ms * 1e-3) / 1e6, 2),
            "ao_span_ms": round(ao_ms, 4), "ao_frames_per_s": round(1e3 / ao_ms, 1),
            "note": f"latency region with rsd_sd_params.hit_order = {name[1]} (DXR-like any-hit order, {name[2]}); "
                    "the headline value keeps the canonical order"}


def latency_floor(cnts, trace_ms):
    """Latency roofline of the SD walk: the slowest ray is a chain of
    max_steps_per_ray dependent steps (row walk: LDS pop -> node / leaf fetch -> box or triangle tests
    -> row merge -> push; quad walk: one iteration of the ray's quad, fetch -> tests -> stack); its
    floor is max_steps x the mean step time measured by the instrumented walk under the same load
    (rsd_counters.step_*_clocks over row_steps, s_memtime converted with the launch's measured clock).  latency_frac = floor / the trace's HIP-event duration (setup +
    walk): near 1 means the trace lasts as long as its slowest ray's dependency chain."""
    import numpy as np
    c = [x for x in cnts if x.row_steps and x.shader_clock_mhz > 0]
    if not c:
        return {"latency_floor_us": None}
    mhz = float(np.mean([x.shader_clock_mhz for x in c]))
    steps = sum(x.row_steps for x in c)
    fetch = sum(x.step_fetch_clocks for x in c) / steps / mhz
    comp = sum(x.step_compute_clocks for x in c) / steps / mhz
    pool = sum(x.step_pool_clocks for x in c) / steps / mhz
    ms = max(x.max_steps_per_ray for x in c)
    floor = ms * (fetch + comp + pool)
    # latency-bound: the floor explains most of the trace.  Below 0.6 the launch outlasts its longest chain (the
    # summed work sets it); above 1.05 the floor model fails the other way -- the mean step of a fully loaded launch
    # overstates the longest rays' late steps, which run on a draining machine -- again a throughput-bound walk
    lf = floor / (trace_ms * 1e3)
    return {"latency_floor_us": round(floor, 2), "latency_frac": round(lf, 3),
            "latency_floor_fetch_only_us": round(ms * fetch, 2),
            "walk_bound": "latency" if 0.6 <= lf <= 1.05 else "throughput",
            "step_us": {"fetch": round(fetch, 3), "tests_merge": round(comp, 3), "pool": round(pool, 3)},
            "max_steps_per_ray": int(ms), "shader_clock_mhz": round(mhz, 1),
            "latency_note": "floor = max_steps_per_ray x mean step time of the instrumented walk (row walk: one row "
                            "step = fetch wait + tests/merge + LDS pool; quad walk, maps above 0.6 M texels: one quad "
                            "iteration = own fetch wait + own tests and the wave's other branch + stack); "
                            "latency_frac = floor / trace duration; walk_bound = latency for 0.6 <= latency_frac <= 1.05 (the "
                            "longest chain sets the launch), else throughput (below: the summed work outlasts it; "
                            "above: the loaded mean step overstates the longest rays' late steps)"}


def pmc_traffic(csv_paths, kernel_substrs):
    """HBM bytes of one SD trace from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (KB units;
    FETCH_SIZE doubled on gfx950 per MI355X_MICROARCH.md section HBM): per kernel, the median over
    its launches (the instrumented counter launches of the row walk -- CNT = true in its name --
    excluded; the quad walk's instrumented launches are a minority the median ignores); summed over
    the kernels of ONE trace of the given walk."""
    import csv
    import re
    import statistics
    if not csv_paths:
        return None
    per = {}  # (kernel, counter) -> values
    for path in csv_paths:
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                k = next((s for s in kernel_substrs if s in name), None)
                if k is None:
                    continue
                m = re.search(r"sd_trace_row_kernel<([^>]*)>", name)
                if m and [x.strip() for x in m.group(1).split(",")][4:5] == ["true"]:
                    continue  # the instrumented row walk (template parameter CNT)
                per.setdefault((k, row.get("Counter_Name")), []).append(float(row.get("Counter_Value", 0)))
    if not per:
        return None
    med = lambda k, c: statistics.median(per[(k, c)]) if (k, c) in per else 0.0  # noqa: E731
    return int(sum(2 * med(k, "FETCH_SIZE") + med(k, "WRITE_SIZE") for k in kernel_substrs) * 1024)


# VALU issue peak of MI355X (MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles,
# 32 lanes/cycle; 157.3 TFLOPS FP32 vector = 2 x this FMA rate): 256 CUs x 4 SIMDs x 32 lanes x
# 2.4 GHz.  Nominal: f64, transcendental and v_div_* instructions take more than 2 cycles.
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9


def pmc_valu(csv_path, kernel_substr):
    """VALU issue roofline of one kernel from a rocprofv3 --pmc SQ_INSTS_VALU pass (one frame in
    flight): lane-instructions per launch / that launch's duration, against VALU_PEAK_LANE_OPS."""
    import csv
    if not Path(csv_path).exists():
        return None
    insts, durs = [], []
    with open(csv_path) as f:
        for row in csv.DictReader(f):
            if kernel_substr in row.get("Kernel_Name", "") and row.get("Counter_Name") == "SQ_INSTS_VALU":
                insts.append(float(row["Counter_Value"]))
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    if not insts:
        return None
    lane_ops = sum(insts) / len(insts) * 64
    dur = sum(durs) / len(durs)
    return {"kernel": kernel_substr, "bound": "valu", "achieved": round(lane_ops / dur / 1e12, 2),
            "peak": round(VALU_PEAK_LANE_OPS / 1e12, 2), "unit": "T lane-instr/s",
            "frac": round(lane_ops / dur / VALU_PEAK_LANE_OPS, 3), "duration_us": round(dur * 1e6, 1),
            "source": str(Path(csv_path).relative_to(ROOT)) if Path(csv_path).is_relative_to(ROOT) else csv_path}


def cpu_baseline(r, scene, target_s, poses=None):
    """The CPU oracle (kind "port") timed on the same frame's SD trace, on every CPU this process
    may use.  The whole SD map when one trace takes < target_s / 4, else a band of rows sized to
    ~target_s; the traced rows are checked bit-for-bit against the GPU frame."""
    import numpy as np

    from oracle import oracle as O
    sys.path.insert(0, str(ROOT / "tests"))
    from helpers import to_oracle

    # one full frame with explicit interval maps (the timed frames consume them): the baseline
    # traces exactly this frame's SD map (pose 0 of a camera path)
    if poses:
        r.set_pose(*poses[0])
        r.gbuffer()
    r.frame()
    g = r.numpy()
    assert (g["ray_max"] != 0).any(), "the baseline frame has no live SD rays"
    cpus = host_cpus()
    cores = cpus["effective"]
    osc = O.Scene(scene.positions, scene.indices, scene.flags)
    cam, sdp = to_oracle(r.cam, O.Camera), to_oracle(r.sdp, O.SDParams)

    def trace(rows):
        return O.sd_trace(osc, cam, sdp, g["depth"], g["ray_min"], g["ray_max"], r.sd_w, r.sd_h, rows=rows,
                          threads=cores)

    # probe: 8 rows through the middle, then the whole map if it is cheap enough
    mid = r.sd_h // 2 // 8 * 8
    t0 = time.perf_counter()
    trace((mid, mid + 8))
    per_row = (time.perf_counter() - t0) / 8
    if per_row * r.sd_h < target_s / 4:
        y0, y1 = 0, r.sd_h
    else:
        n = max(8, min(r.sd_h, int(target_s / 4 / max(per_row, 1e-9)) // 8 * 8))
        y0 = max(0, min(r.sd_h - n, mid - n // 2)) // 8 * 8
        y1 = min(r.sd_h, y0 + n)
    t0 = time.perf_counter()
    sd, stats = trace((y0, y1))
    dt = time.perf_counter() - t0
    reps = max(1, int(target_s / max(dt, 1e-4)))
    t0 = time.perf_counter()
    for _ in range(reps):
        sd, stats = trace((y0, y1))
    dt = (time.perf_counter() - t0) / reps
    n = (y1 - y0) * r.sd_w
    same = bool(np.array_equal(sd[:, y0:y1].view(np.uint32), g["sd"][:, y0:y1].view(np.uint32)))
    what = "the frame's full SD trace" if (y0, y1) == (0, r.sd_h) else f"SD rows [{y0}, {y1}) of the frame"
    return {"value": round(n / dt / 1e6, 4), "unit": "Mrays/s", "cores": cores, "kind": "port",
            "sample": f"{what} ({n} rays, {int(stats[0])} live) x {reps} repetitions, oracle pthreads on "
                      f"{cores} host threads (= min(affinity mask {cpus['usable']} CPUs, ceil(cgroup quota "
                      f"{cpus['cgroup_cpu_quota']})): the effective core count)",
            "active_mrays_per_s": round(float(stats[0]) / dt / 1e6, 4),
            "host": cpus, "seconds": round(dt * reps, 2), "bit_identical_to_gpu": same}


if __name__ == "__main__":
    main()
