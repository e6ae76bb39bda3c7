#!/usr/bin/env python3
"""Headline benchmark: Ray-SD + SVAO AO frames on MI355X (BASELINE.json metric
"Mrays/s + AO frames/s, 1080p 1/4-res Ray-SD").

A step = one AO frame of the reference's SVAO::execute span (SVAO.cpp:327-455: clear
ray intervals, "AO 1", StochasticDepthMapRT, "AO 2") over the configs[1] workload:
Sun Temple stand-in (~0.6 M triangles, seed 2), 1920x1080 visible + 64-px guard band
(2048x1208 frame buffer), 1/4-res SD map (768x558 texels incl. the 128-texel SD guard),
N = 4, MAX_COUNT = 8.  Inputs (BVH, G-buffer) are resident in HBM before timing.

  value            = SD rays dispatched per frame * frames / timed wall  (Mrays/s, whole job)
  ao_frames_per_s  = frames / timed wall
  sd_kernel_mrays  = SD rays / SD-kernel time (HIP events around the trace launch)

Frames in flight (--frames-in-flight F, default 4, the measured optimum of F = 1..6):
frame i runs on HIP stream i % F with its own frame buffers (ao, stencil, interval maps, SD
map; BVH and G-buffer shared).  Every frame still runs the whole clear -> "AO 1" -> SD trace ->
"AO 2" chain in order on its stream; frames of different slots overlap, so the latency-bound
SD trace of one frame (~22 K live rays on 256 CUs) shares the machine with the VALU-bound
passes of the others.  Overlapping frames trace with librsd's work-efficient walk
(RSD_SD_THROUGHPUT: 4 lanes per ray) instead of the latency-optimised row walk (8 lanes per ray):
the row walk's idle lanes would be VALU time taken from the other frames.  `sequential` reports the
one-frame-in-flight latency of the same frame (row walk).

Multi-GPU (torchrun, one rank per GPU), two sharding modes (--shard):
  frame (default): frames are the independent units -- every rank renders whole frames of the
    configs[1] size (its own frame stream, BVH + G-buffer replicated), no data-path
    collective; the barrier and max-over-ranks wall bracket the timed region.  Weak scaling:
    value = world * K frames * rays / wall.
  band: one frame sharded by screen band (rsd/shard.py, the north_star's tile split).  Every
    rank runs pass 1 on its band of rows, all-reduces the ray-interval maps (MIN/MAX),
    traces its band of SD tile rows, all-gathers the SD map, runs pass 2 on its band and
    all-gathers the AO image (RCCL over xGMI).  Strong scaling: the whole job renders the
    same frame whatever N is; at 1080p/4 the three collectives per frame outweigh the
    per-rank compute, so this is the mode for large frames (4K, full-res SD).
"""
from __future__ import annotations

import argparse
import json
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
SD_KERNELS = ("sd_setup_kernel", "sd_trace_row_kernel", "sd_resolve_row_kernel", "sd_trace_queue_kernel")  # launches of one rsd_sd_trace


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="suntemple_1080p_q")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0,
                    help="target wall time of the bounded CPU-oracle sample (0 disables)")
    ap.add_argument("--frames-in-flight", type=int, default=4,
                    help="frames in flight: frame i runs on stream i %% F with its own frame buffers "
                         "(1 = strictly sequential frames)")
    ap.add_argument("--shard", choices=("frame", "band"), default="frame",
                    help="N > 1: frame = every rank renders whole frames (weak scaling, no per-frame "
                         "collective); band = each frame split by screen band + RCCL exchanges (strong)")
    ap.add_argument("--pmc-csv", nargs="*", default=None,
                    help="rocprofv3 --pmc counter_collection.csv file(s) with FETCH_SIZE / WRITE_SIZE for "
                         "roofline.traffic (default: the committed profiles/round1 passes)")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch

    from rsd.frame import CONFIGS, FrameConfig, Renderer
    from rsd.scenes import make_scene

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
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

    kw, scene_name = CONFIGS[args.config]
    cfg = FrameConfig(**kw)
    scene = make_scene(scene_name)
    r = Renderer(scene, cfg, device=local)
    r.gbuffer()
    torch.cuda.synchronize()

    # instrumented full-frame trace (not timed): traversal counters for the roofline bytes
    r.clear_intervals()
    r.pass1()
    # counters of the walk the timed frames use (frames in flight: RSD_SD_THROUGHPUT)
    cnt = r.sd_trace(counters=True, throughput=args.frames_in_flight > 1)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()

    from rsd.shard import BandFrame
    # frames in flight: F buffer sets (slots) on F streams; frame i runs on slot i % F.  Every
    # frame does the whole pass 1 -> SD trace -> pass 2 chain; frames of different slots overlap
    # (the latency-bound SD trace of one frame shares the CUs with another frame's passes)
    F = max(1, args.frames_in_flight)
    # band: this rank's screen band of every frame; frame: whole frames on every rank
    bw = (rank, world) if args.shard == "band" else (0, 1)
    # with frames overlapping, the trace uses librsd's work-efficient walk (RSD_SD_THROUGHPUT)
    slots = [BandFrame(r, *bw, throughput=F > 1)] + [BandFrame(r.frame_slot(), *bw, throughput=True)
                                                     for _ in range(F - 1)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(F - 1)]
    for st in streams[1:]:
        st.wait_stream(streams[0])
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def frame(i, timed=False):
        with torch.cuda.stream(streams[i % F]):
            slots[i % F].frame(sd_events=ev[i] if timed else None)

    for i in range(args.warmup):
        frame(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        frame(i, timed=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if dist:
        t = torch.tensor([wall], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())

    sd_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # untimed for `value`: the single-frame latency (one frame in flight, slot 0 only)
    n_seq = min(args.steps, 20)
    seq = BandFrame(r, *bw)  # latency-optimised trace walk (no frames overlap)
    ev_seq = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_seq)]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(n_seq):
        seq.frame(sd_events=ev_seq[i])
    torch.cuda.synchronize()
    seq_ms = (time.perf_counter() - t0) / n_seq * 1e3
    seq_sd_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_seq]))
    rays = r.sd_rays
    N = cfg.sd_samples
    # B_ray = 16 (linearZ bilinear) + 8 (rayMin+rayMax) + 4N (store) + node bytes + 48 n_tri;
    # librsd's nodes are 4-wide (128 B per visit = two of SURVEY's 64-B BVH2 nodes)
    alg_bytes = rays * (16 + 8 + 4 * N) + 128 * cnt.nodes_visited + 48 * cnt.tris_tested
    achieved = alg_bytes / (sd_ms * 1e-3) / 1e9
    pmc = args.pmc_csv if args.pmc_csv is not None else [str(ROOT / "profiles" / "round1" / f)
                                                          for f in ("pmc_fetch_size.csv", "pmc_write_size.csv")]
    traffic = pmc_traffic([p for p in pmc if Path(p).exists()], SD_KERNELS)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    cpu = None
    if args.cpu_baseline_seconds > 0 and world == 1:
        cpu = cpu_baseline(r, scene, args.cpu_baseline_seconds)

    # whole job: frame mode renders `steps` whole frames on every rank, band mode `steps` frames in all
    frames_total = args.steps * (world if args.shard == "frame" else 1)
    frames_per_s = frames_total / wall
    value = rays * frames_per_s / 1e6 * 1.0
    line = {
        "metric": "Mrays/s + AO frames/s, 1080p 1/4-res Ray-SD, 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.shard == "band" and world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded procedural stand-in scene; no reference assets in the container)",
        "config": {"workload": args.config, "scene": scene_name, "triangles": scene.triangle_count,
                   "frame_buffer": [cfg.fb_w, cfg.fb_h], "visible": [cfg.visible_w, cfg.visible_h],
                   "sd_map": [r.sd_w, r.sd_h], "sd_samples": N, "max_count": cfg.max_count,
                   "stoch_map_divisor": cfg.divisor,
                   "parallelism": f"screen-band x{world}" if args.shard == "band" else f"frame-parallel x{world}",
                   "frames_in_flight": F},
        "ao_frames_per_s": round(frames_per_s, 2),
        "frames_total": frames_total,
        "sd_kernel_ms": round(sd_ms, 4),
        "sequential": {"ms_per_frame": round(seq_ms, 4), "ao_frames_per_s": round(1e3 / seq_ms, 2),
                       "sd_kernel_ms": round(seq_sd_ms, 4), "frames": n_seq,
                       "note": "one frame in flight: the frame latency (value counts frames in flight)"},
        "sd_kernel_mrays_per_s": round(rays / (sd_ms * 1e-3) / 1e6, 2),
        "active_rays": int(cnt.rays_active),
        "traversal": {"nodes_per_ray": round(cnt.nodes_visited / rays, 3),
                      "tris_per_ray": round(cnt.tris_tested / rays, 3),
                      "nodes_per_active_ray": round(cnt.nodes_visited / max(cnt.rays_active, 1), 2),
                      "tris_per_active_ray": round(cnt.tris_tested / max(cnt.rays_active, 1), 2)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": ("rsd_sd_trace = sd_setup_kernel + sd_trace_queue_kernel (frames in flight: RSD_SD_THROUGHPUT)"
                                if F > 1 else "rsd_sd_trace = sd_setup_kernel + sd_trace_row_kernel + sd_resolve_row_kernel"),
                     "alg_bytes_per_launch": int(alg_bytes),
                     "achieved_sequential": round(alg_bytes / (seq_sd_ms * 1e-3) / 1e9, 1),
                     "note": "achieved uses the trace's duration with frames in flight (it shares the CUs); "
                             "achieved_sequential the one-frame-in-flight duration",
                     "traffic_source": ", ".join(str(Path(p).relative_to(ROOT)) if Path(p).is_relative_to(ROOT)
                                                 else p for p in pmc if Path(p).exists()) or None},
        # the frame's largest kernel is pass 1, bound by VALU issue rather than HBM
        "pass1_roofline": pmc_valu(ROOT / "profiles" / "round1" / "pmc_sq_valu.csv", "svao_pass1_kernel"),
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


def pmc_traffic(csv_paths, kernel_substrs):
    """HBM bytes of one SD pass from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (KB units;
    FETCH_SIZE doubled on gfx950 per MI355X_MICROARCH.md §HBM): per kernel, the mean over its
    launches; summed over the kernels of the pass."""
    import csv
    import re
    if not csv_paths:
        return None
    per = {}  # (kernel, counter) -> values
    for path in csv_paths:
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                k = next((s for s in kernel_substrs if s in name), None)
                if k is None or re.search(r", (true|false), true>", name):  # skip the instrumented launch
                    continue
                per.setdefault((k, row.get("Counter_Name")), []).append(float(row.get("Counter_Value", 0)))
    if not per:
        return None
    mean = lambda k, c: (sum(per[(k, c)]) / len(per[(k, c)])) if (k, c) in per else 0.0  # noqa: E731
    return int(sum(2 * mean(k, "FETCH_SIZE") + mean(k, "WRITE_SIZE") for k in kernel_substrs) * 1024)


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


def cpu_baseline(r, scene, target_s):
    """The CPU oracle (kind "port") timed on the same frame's SD trace, repeated to ~target_s."""
    import numpy as np

    from oracle import oracle as O
    sys.path.insert(0, str(ROOT / "tests"))
    from helpers import to_oracle

    # one full frame with explicit interval maps (the timed frames consume them, so the maps are
    # cleared by now): the baseline traces exactly this frame's SD map
    r.frame()
    g = r.numpy()
    assert (g["ray_max"] != 0).any(), "the baseline frame has no live SD rays"
    cores = min(os.cpu_count() or 1, 16)
    osc = O.Scene(scene.positions, scene.indices, scene.flags)
    cam, sdp = to_oracle(r.cam, O.Camera), to_oracle(r.sdp, O.SDParams)
    # the whole SD map of the frame, repeated until ~target_s of CPU work
    t0 = time.perf_counter()
    sd, stats = O.sd_trace(osc, cam, sdp, g["depth"], g["ray_min"], g["ray_max"], r.sd_w, r.sd_h, threads=cores)
    dt = time.perf_counter() - t0
    reps = max(1, int(target_s / max(dt, 1e-4)))
    t0 = time.perf_counter()
    for _ in range(reps):
        sd, stats = O.sd_trace(osc, cam, sdp, g["depth"], g["ray_min"], g["ray_max"], r.sd_w, r.sd_h,
                               threads=cores)
    dt = (time.perf_counter() - t0) / reps
    y0, y1 = 0, r.sd_h
    n = (y1 - y0) * r.sd_w
    # the sample's share of the GPU result must be bit-identical (the baseline computes the same thing)
    same = bool(np.array_equal(sd[:, y0:y1].view(np.uint32), g["sd"][:, y0:y1].view(np.uint32)))
    return {"value": round(n / dt / 1e6, 4), "unit": "Mrays/s", "cores": cores, "kind": "port",
            "sample": f"the frame's full SD trace ({n} rays, {int(stats[0])} live) x {reps} repetitions, "
                      f"oracle pthreads on {cores} host threads",
            "seconds": round(dt * reps, 2), "bit_identical_to_gpu": same}


if __name__ == "__main__":
    main()
