"""Screen-band sharding of one AO frame across ranks.

One process per GPU, torch.distributed over RCCL (backend "nccl") on the node; the same
code runs over gloo on CPU tensors for the multi-process tests.  Every rank holds the
replicated BVH and G-buffer.  Per frame, rank r of B:

  1. clears the ray-interval maps and runs pass 1 ("AO 1") on its band of rows;
  2. all-reduces the interval maps in one collective (MIN on rayMin and on -rayMax: int32
     bit patterns of non-negative floats order like the floats) -- now every rank has the
     exact union the single-GPU pass 1 would have produced;
  3. traces its band of SD-map tile rows;
  4. all-gathers the SD map (pass 2 reads SD texels up to ssMaxRadius away);
  5. runs pass 2 ("AO 2") on its band and all-gathers the AO image.

Bands interleave 32-row groups (passes 1/2) and 8-row SD tiles, so sky and geometry spread
evenly over ranks.  Each SD texel and each AO pixel is produced by exactly one rank with
the same deterministic kernels, so the gathered frame is bit-identical to the 1-GPU frame.
"""
from __future__ import annotations

import time

import torch


def band_rows(n_rows: int, group: int, offset: int, rank: int, world: int) -> torch.Tensor:
    """Rows y in [offset, offset + n_rows) whose group ((y - offset) // group) % world == rank."""
    y = torch.arange(n_rows, dtype=torch.int64)
    return (y[(y // group) % world == rank] + offset)


class BandFrame:
    """Runs the frame of `backend` as band `rank` of `world` and exchanges the results.

    `backend` provides clear_intervals(), pass1(band), sd_trace(band), pass2(band) and the
    tensors ray_min, ray_max (int32 [sdH, sdW]), sd (float32 [layers, sdH, sdW, ch]),
    ao and stencil (uint8 [H, W]), plus cfg (fb_w, fb_h, guard_band) and sd_h."""

    def __init__(self, backend, rank: int = 0, world: int = 1, pg=None, throughput: bool = False):
        """throughput=True: this frame overlaps other frames in flight; a backend that supports it
        (librsd: RSD_SD_THROUGHPUT) then traces with its work-efficient walk."""
        import torch.distributed as dist
        self.b, self.rank, self.world, self.pg = backend, rank, world, pg
        self.trace_kw = {"throughput": True} if throughput and getattr(backend, "can_consume_intervals", False) else {}
        self._intervals_clear = False  # set after a trace that consumed (reset) the intervals
        self.dist = dist if world > 1 else None
        self.nccl = world > 1 and dist.get_backend(pg) == "nccl"
        cfg = backend.cfg
        dev = backend.sd.device
        g, H = cfg.guard_band, cfg.fb_h
        ny = (H - 2 * g + 31) // 32 * 32
        # pass-1 rows (padded dispatch, SVAO.cpp:347-349) -- includes the pass-2 rows of the band
        ao_rows = [band_rows(min(ny, H - g), 32, g, r, world) for r in range(world)]
        sd_rows = [band_rows(backend.sd_h, 8, 0, r, world) for r in range(world)]
        self.ao_rows = [r.to(dev) for r in ao_rows]
        self.sd_rows = [r.to(dev) for r in sd_rows]
        self.ao_max = max(len(r) for r in ao_rows)
        self.sd_max = max(len(r) for r in sd_rows)
        b = backend
        self.sd_send = torch.zeros((b.sd.shape[0], self.sd_max) + tuple(b.sd.shape[2:]), dtype=b.sd.dtype, device=dev)
        self.sd_recv = torch.zeros((world,) + tuple(self.sd_send.shape), dtype=b.sd.dtype, device=dev)
        self.ao_send = torch.zeros((self.ao_max, b.ao.shape[1]), dtype=b.ao.dtype, device=dev)
        self.ao_recv = torch.zeros((world, self.ao_max, b.ao.shape[1]), dtype=b.ao.dtype, device=dev)
        # unpack maps: the valid rows of recv (flattened over ranks) and where they go -- one
        # index_select + one index_copy per exchange instead of one copy per rank
        self.sd_unpack = self._unpack_map(self.sd_rows, self.sd_max, dev)
        self.ao_unpack = self._unpack_map(self.ao_rows, self.ao_max, dev)

    @staticmethod
    def _unpack_map(rows, cap, dev):
        src = torch.cat([k * cap + torch.arange(len(r), device=dev) for k, r in enumerate(rows)])
        dst = torch.cat(list(rows))
        return src, dst

    def _all_gather(self, recv, send):
        if self.nccl:
            self.dist.all_gather_into_tensor(recv.view(-1), send.view(-1), group=self.pg)
        else:
            self.dist.all_gather(list(recv.unbind(0)), send, group=self.pg)

    def _gather_rows(self, t, rows, send, recv, dim, unpack):
        mine = rows[self.rank]
        torch.index_select(t, dim, mine, out=send.narrow(dim, 0, len(mine)))
        self._all_gather(recv, send)
        # recv [world, ..., cap, ...] -> rows (ranks x cap) along dim, then scatter the valid ones
        # (the own band is written back unchanged)
        src, dst = unpack
        flat = recv.movedim(0, dim).flatten(dim, dim + 1) if dim > 0 else recv.flatten(0, 1)
        t.index_copy_(dim, dst, flat.index_select(dim, src))

    def frame(self, sd_events=None):
        """One AO frame.  sd_events: optional (start, end) torch.cuda.Event pair recorded
        around this rank's SD trace (per-kernel timing in bench.py)."""
        if self.world == 1 and _one_call_frame(self, sd_events):
            return
        self.front()
        self.back(sd_events)

    def front(self):
        """The frame up to pass 1 ("AO 1"): the interval clear when the previous trace did not
        consume the maps, then pass 1 of this band."""
        b, band = self.b, (self.rank, self.world)
        # the previous frame's trace reset the intervals if the backend can fold the clear in
        consume = getattr(b, "can_consume_intervals", False) and bool(b.cfg.ray_interval)
        if not (consume and self._intervals_clear):
            b.clear_intervals()
        b.pass1(band=band)

    def back(self, sd_events=None):
        """The rest of the frame after front(): interval exchange, SD trace, SD exchange, pass 2,
        AO exchange (a host may run it on another stream than front(), ordered by an event)."""
        b, band = self.b, (self.rank, self.world)
        consume = getattr(b, "can_consume_intervals", False) and bool(b.cfg.ray_interval)
        if self.world > 1:
            both = getattr(b, "ray_minmax", None)
            if both is not None:
                # one collective: MIN over [rayMin, -rayMax] (non-negative float bit patterns
                # as int32: negation reverses their order exactly)
                b.ray_max.neg_()
                self.dist.all_reduce(both, op=self.dist.ReduceOp.MIN, group=self.pg)
                b.ray_max.neg_()
            else:
                self.dist.all_reduce(b.ray_min, op=self.dist.ReduceOp.MIN, group=self.pg)
                self.dist.all_reduce(b.ray_max, op=self.dist.ReduceOp.MAX, group=self.pg)
        if sd_events:
            sd_events[0].record()
        if consume:
            b.sd_trace(band=band, consume=True, **self.trace_kw)
        else:
            b.sd_trace(band=band, **self.trace_kw)
        self._intervals_clear = consume
        if sd_events:
            sd_events[1].record()
        if self.world > 1:
            self._gather_rows(b.sd, self.sd_rows, self.sd_send, self.sd_recv, 1, self.sd_unpack)
        b.pass2(band=band)
        if self.world > 1:
            self._gather_rows(b.ao, self.ao_rows, self.ao_send, self.ao_recv, 0, self.ao_unpack)


def _one_call_frame(fr, sd_events) -> bool:
    """The 1-rank frame of a BandFrame / HaloFrame as ONE librsd call (rsd_svao_frame: the same
    kernels and bits as the per-pass calls, issued from C++).  False when the backend has no such
    entry (the CPU oracle backend of the tests) or the SD events are not HIP timing events."""
    b = fr.b
    if not hasattr(b, "svao_frame") or (sd_events and not all(hasattr(e, "h") for e in sd_events)):
        return False
    consume = getattr(b, "can_consume_intervals", False) and bool(b.cfg.ray_interval)
    ev = [None, sd_events[0], sd_events[1], None] if sd_events else None
    b.svao_frame(intervals_clear=consume and fr._intervals_clear, keep_intervals=not consume,
                 throughput=bool(fr.trace_kw), events=ev)
    fr._intervals_clear = consume
    return True


def halo_px(cfg, max_radius_px: float = 512.0) -> int:
    """Bound (frame-buffer pixels, vertical) on how far from its pixel an SVAO sample lands: the
    AO disk (world radius R with R * f / z <= ssMaxRadius, VAOData.slang:44; Common.slang:285-300)
    lies in the plane perpendicular to the view ray, so off-axis it projects larger than
    ssMaxRadius (perspective stretch, ~1/cos of the ray angle and more at the frame corners).
    Evaluated numerically over the frame border (where the stretch is largest) for the config's
    pinhole camera (focal length / frame height, Camera.cpp:99-185), plus 4 px of slack."""
    import numpy as np
    W, H = cfg.fb_w, cfg.fb_h
    f = cfg.focal_length / cfg.frame_height * H  # focal length in pixels (preserveHeight)
    # border pixels (x, y) relative to the principal point, and 64 disk directions
    t = np.linspace(0.0, 1.0, 257)
    xs = np.concatenate([(t - 0.5) * W, np.full_like(t, -0.5 * W), np.full_like(t, 0.5 * W), (t - 0.5) * W])
    ys = np.concatenate([np.full_like(t, -0.5 * H), (t - 0.5) * H, (t - 0.5) * H, np.full_like(t, 0.5 * H)])
    worst = 0.0
    for x, y in zip(xs, ys):
        d = np.array([x, y, f]) / np.linalg.norm([x, y, f])  # view ray (z = 1 at the image plane)
        P = d / d[2]  # the point at linear depth z = 1
        R = max_radius_px / f  # world radius at z = 1 whose screen radius is max_radius_px
        a = np.cross(d, [0.0, 1.0, 0.0]) if abs(d[1]) < 0.99 else np.cross(d, [1.0, 0.0, 0.0])
        a /= np.linalg.norm(a)
        b = np.cross(d, a)
        ang = np.linspace(0.0, 2.0 * np.pi, 64, endpoint=False)
        S = P[None, :] + R * (np.cos(ang)[:, None] * a[None, :] + np.sin(ang)[:, None] * b[None, :])
        worst = max(worst, float(np.abs(f * S[:, 1] / S[:, 2] - y).max()))
    return int(np.ceil(worst)) + 4


FLT_MAX_BITS = 0x7F7FFFFF  # asuint(FLT_MAX): a cleared rayMin (SVAO.cpp:339)


class DistComm:
    """HaloFrame's collectives over torch.distributed: RCCL under backend "nccl" (one GPU per rank;
    point-to-point send / recv = ncclSend / ncclRecv, stream-ordered, no host wait), gloo for the CPU
    rehearsals (and several ranks sharing one GPU, staged through host copies)."""

    def __init__(self, pg=None):
        import torch.distributed as dist
        self.dist, self.pg = dist, pg
        self.nccl = dist.get_backend(pg) == "nccl"

    def all_gather(self, out, inp):
        """out [world, *inp.shape] <- every rank's inp."""
        if self.nccl:
            self.dist.all_gather_into_tensor(out.view(-1), inp.reshape(-1), group=self.pg)
        else:
            self.dist.all_gather(list(out.unbind(0)), inp.contiguous(), group=self.pg)

    def exchange(self, sends, recvs):
        """Point-to-point: sends {peer: tensor}, recvs {peer: tensor} (sizes agreed beforehand)."""
        sends = {k: t for k, t in sends.items() if t.numel()}
        recvs = {k: t for k, t in recvs.items() if t.numel()}
        staged = not self.nccl and any(t.is_cuda for t in list(sends.values()) + list(recvs.values()))
        if staged:  # gloo rehearsal with device tensors (several ranks on one GPU): via host copies
            sends = {k: t.cpu() for k, t in sends.items()}
            recvs_dev, recvs = recvs, {k: torch.empty(t.shape, dtype=t.dtype) for k, t in recvs.items()}
        ops = [self.dist.P2POp(self.dist.isend, t.contiguous(), k, group=self.pg) for k, t in sends.items()]
        ops += [self.dist.P2POp(self.dist.irecv, t, k, group=self.pg) for k, t in recvs.items()]
        if ops:
            for w in self.dist.batch_isend_irecv(ops):
                w.wait()  # NCCL: the current stream waits for the transfer (no host wait)
        if staged:
            for k, t in recvs.items():
                recvs_dev[k].copy_(t)


class LocalHub:
    """Rendezvous of LocalComm ranks: `world` host threads of one process, one HIP stream each."""

    def __init__(self, world: int):
        import threading
        self.world = world
        self.cv = threading.Condition()
        self.posts = {}


class LocalComm:
    """HaloFrame's collectives between host threads of one process on one GPU, with the semantics of
    stream-ordered RCCL and no host synchronisation: a rank posts its tensors with an event recorded
    on its stream; every reader makes ITS stream wait for that event and copies (device to device),
    then posts a done event that the writer's stream waits for before it may touch the tensors
    again.  The threads only rendezvous on Python conditions; the GPU work stays asynchronous.  A
    rehearsal device for the sync-free N > 1 frame (tests/test_gpu_sharding.py)."""

    def __init__(self, hub: LocalHub, rank: int):
        self.hub, self.rank, self.seq = hub, rank, 0

    def _post(self, key, value):
        with self.hub.cv:
            self.hub.posts.setdefault(key, {})[self.rank] = value
            self.hub.cv.notify_all()

    def _wait(self, key, ranks):
        with self.hub.cv:
            self.hub.cv.wait_for(lambda: all(r in self.hub.posts.get(key, {}) for r in ranks), timeout=120)
            got = dict(self.hub.posts.get(key, {}))
        if not all(r in got for r in ranks):
            raise RuntimeError(f"LocalComm: rank {self.rank} timed out in {key}")
        return got

    def _event(self):
        e = torch.cuda.Event()
        e.record(torch.cuda.current_stream())
        return e

    def _finish(self, key, readers):
        """After reading: post my done event, then wait (on my stream) for the readers of my tensors."""
        self._post(("done",) + key, self._event())
        done = self._wait(("done",) + key, readers)
        st = torch.cuda.current_stream()
        for r in readers:
            if r != self.rank:
                st.wait_event(done[r])

    def all_gather(self, out, inp):
        key = ("ag", self.seq)
        self.seq += 1
        world = range(self.hub.world)
        self._post(key, (inp, self._event()))
        got = self._wait(key, world)
        st = torch.cuda.current_stream()
        for k in world:
            t, e = got[k]
            if k != self.rank:
                st.wait_event(e)
            out[k].copy_(t.view(out[k].shape))
        self._finish(key, world)

    def exchange(self, sends, recvs):
        key = ("x", self.seq)
        self.seq += 1
        world = range(self.hub.world)
        self._post(key, ({k: t for k, t in sends.items()}, self._event()))
        got = self._wait(key, world)
        st = torch.cuda.current_stream()
        for k, t in recvs.items():
            src, e = got[k]
            if t.numel():
                st.wait_event(e)
                t.copy_(src[self.rank].view(t.shape))
        self._finish(key, world)


class HaloFrame:
    """One AO frame split into CONTIGUOUS screen bands with SPARSE halo exchanges.

    Rank r of B owns the visible rows of its 32-row groups [g_r, g_{r+1}) and the SD rows under
    them (8-row aligned).  A frame is front() then back():

      front  1. pass 1 of its own rows (rsd_svao_pass1_rows).  Its interval atomics land on SD texels
                within `halo` rows of its band (the window W_r): exactly the texels its pass 2 will
                read (pass 1 and pass 2 place a refined direction's sample on the same SD texel,
                Common.slang:164-168; an atomic always lowers rayMin below asuint(FLT_MAX) or sets
                rayMax);
             2. ON THE DEVICE: the TOUCHED texels of W_r inside each band k (rayMin != asuint(FLT_MAX)
                or rayMax != 0) are compacted into a fixed-capacity buffer of (texel index, rayMin,
                rayMax) int32 triples (cumulative-sum positions, one scatter; the capacity is the
                candidate region, so it never overflows), and their counts -- with the compute time
                of this rank's previous frame -- are all-gathered as a device tensor, then copied to
                pinned host memory without waiting (one event marks the copy).
      back   3. the host reads the counts once that event has completed -- with frames in flight
                (bench.py issues back() of frame i after front() of the next frames) it completed
                long before, so the GPU never drains -- and sizes the point-to-point transfers of the
                triples' prefixes; rank k merges them with scatter MIN / MAX (exact on the
                non-negative float bit patterns) and holds the exact 1-GPU union for its SD rows;
             4. SD trace of its own SD rows (rsd_sd_trace_rows; consume resets the whole map);
             5. sparse SD halo: rank k returns the N depths of exactly the texels r sent it in step 3
                (k holds r's index list, so the reply carries values only);
             6. pass 2 of its own rows (rsd_svao_pass2_rows) and an all-gather of the AO bands.

    No step synchronises the host with the GPU except the event wait of step 3 (no
    nonzero(), no .cpu(), no .item(); tests/test_gpu_sharding.py runs it under
    torch.cuda.set_sync_debug_mode("error")).

    Load balance ("re-split from the previous frame's per-band time"): every rank
    times its own pass 1 + trace + pass 2 (HIP events, read only once complete); the times travel
    with the step-2 counts, and every rank computes the same new split of the 32-row groups (cost
    spread uniformly over each band's groups, equal predicted cost per rank, moved half-way from the
    current split), applied from this object's next frame.  Every SD texel and AO pixel is still
    produced by exactly one rank with the same kernels, so the frame is bit-identical to the 1-GPU
    frame whatever the split.

    `backend` provides pass1_rows(rows), sd_trace_rows(rows, consume=...), pass2_rows(rows),
    clear_intervals(), tensors ray_minmax (int32 [2, sdH, sdW]), sd, ao, and cfg / vao / sd_h.
    `comm`: DistComm (default; torch.distributed) or LocalComm (threads on one GPU)."""

    def __init__(self, backend, rank: int = 0, world: int = 1, pg=None, throughput: bool = False,
                 rebalance: bool = True, comm=None, sd_split: str = "auto"):
        b = self.b = backend
        self.rank, self.world, self.pg = rank, world, pg
        if sd_split not in ("tiles", "rows", "auto"):
            raise ValueError("HaloFrame sd_split must be 'tiles', 'rows' or 'auto'")
        # who traces which SD texel: "tiles" deals the 8-row SD tiles round-robin to the ranks (tile t to
        # rank t % world), so every rank traces a share of the frame's long rays -- the trace is
        # latency-bound by its slowest rays, which cluster on the screen; "rows": the SD rows under each
        # rank's pass-1 band (HaloFrame v4), which sends only the texels beyond a band's edge.  "auto":
        # tiles for reduced-resolution SD maps (few touched texels per pixel row: the extra exchange is
        # small), rows for full-resolution maps, whose touched sets are dense (configs[4]: 14.9 vs 2.9 MB
        # per rank and frame at N = 8) -- DESIGN.md section 6, profiles/round4/multigpu/
        if sd_split == "auto":
            sd_split = "tiles" if backend.cfg.divisor > 1 else "rows"
        self.sd_split = sd_split if world > 1 else "rows"
        self.comm = comm if comm is not None else (DistComm(pg) if world > 1 else None)
        self.nccl = bool(getattr(self.comm, "nccl", False))
        self.trace_kw = {"throughput": True} if throughput and getattr(b, "can_consume_intervals", False) else {}
        self._intervals_clear = False
        cfg = b.cfg
        self.V = cfg.fb_h - 2 * cfg.guard_band
        self.G = (self.V + 31) // 32
        self.gb = [self.G * r // world for r in range(world + 1)]  # first split: equal group counts
        self.rebalance = rebalance and world > 1
        self.halo_px = halo_px(cfg, float(b.vao.ssMaxRadius))
        self.cuda = b.sd.is_cuda
        # the halo's device steps through librsd (rsd_halo_*: one call each instead of a dozen torch ops
        # per peer); the CPU rehearsal backends (gloo tests) keep the torch formulation of the same steps
        self.native = self.cuda and hasattr(b, "stream")
        self._ao_cap = 0
        self._next_gb = None
        self._prev = None  # timing events of this object's previous frame
        self._open = None  # state of the frame between front() and back()
        self.sent = {"intervals": 0, "sd": 0, "ao": 0}
        self.frames = 0
        self.blocked_waits = 0  # back() calls whose counts were not yet on the host (frames in flight: ~0)
        self.splits = []  # the group split of every frame (diagnostics)
        self._plan()

    # ---- the partition implied by self.gb
    def _plan(self):
        b, world, me = self.b, self.world, self.rank
        # a new split changes which SD texels this rank's traces write (and the SD replies it scatters): the
        # renderer's clean-tile stamps are void (Renderer.keep_clean_tiles)
        if hasattr(b, "invalidate_sd_tiles"):
            b.invalidate_sd_tiles()
        cfg = b.cfg
        g, div, sdg, sdh = cfg.guard_band, cfg.divisor, int(b.vao.sdGuard), b.sd_h
        gb, V = self.gb, self.V
        self.px_rows = [(32 * gb[r], 32 * gb[r + 1]) for r in range(world)]  # visible rows, API ranges
        # SD rows under each band: SD row of frame-buffer row y = y / div + sdGuard (SVAO.cpp:700-716)
        S = [0] + [min(sdh, ((g + 32 * gb[r]) // div + sdg) // 8 * 8) for r in range(1, world)] + [sdh]
        for r in range(1, world + 1):
            S[r] = max(S[r], S[r - 1])
        self.sd_rows = [(S[r], S[r + 1]) for r in range(world)]
        self.sd_band = (me, world) if self.sd_split == "tiles" else None  # rsd_sd_trace_band_ex's tiles
        self.window = []
        for r in range(world):
            a_px = g + self.px_rows[r][0] - self.halo_px
            b_px = g + min(self.px_rows[r][1], V) + self.halo_px
            self.window.append((max(0, a_px // div + sdg - 1), min(sdh, b_px // div + sdg + 2)))

        def overlap(a, c):
            lo, hi = max(a[0], c[0]), min(a[1], c[1])
            return (lo, hi) if lo < hi else None
        # candidate rows: my window inside band k (my intervals -> k, k's depths -> me), and k's
        # window inside my band (k's intervals -> me, my depths -> k); tiles: my window's tiles of rank k
        # (from the first tile of k at or after the window's first tile, every world-th tile, rows below
        # the window's end) -- a region (row0, row1, period = world) of rsd_halo_compact
        if self.sd_split == "tiles":
            def tiles_of(k, win):
                lo, hi = win
                t = lo // 8
                t += (k - t) % world
                return (8 * t, hi) if 8 * t < hi else None
            self.iv_send = {k: tiles_of(k, self.window[me]) for k in range(world) if k != me}
            self.iv_recv = {k: tiles_of(me, self.window[k]) for k in range(world) if k != me}
        else:
            self.iv_send = {k: overlap(self.window[me], self.sd_rows[k]) for k in range(world) if k != me}
            self.iv_recv = {k: overlap(self.window[k], self.sd_rows[me]) for k in range(world) if k != me}
        self.sd_send = dict(self.iv_recv)
        self.sd_recv = dict(self.iv_send)
        # AO bands (frame-buffer rows), padded to the largest for one all-gather.  Pass 1 dispatches
        # roundup32 of the visible rows (SVAO.cpp:347-349), so the last band also writes the AO of up
        # to 31 guard-band rows below the visible region.
        self.ao_rows = [(g + self.px_rows[r][0], min(cfg.fb_h, g + self.px_rows[r][1])) for r in range(world)]
        self.ao_max = max(hi - lo for lo, hi in self.ao_rows)
        row = b.ao[0].numel()  # elements per AO row (2 with dualAO)
        if self.ao_max > self._ao_cap:
            self._ao_send_buf = torch.zeros(self.ao_max * row, dtype=b.ao.dtype, device=b.ao.device)
            self._ao_recv_buf = torch.zeros(world * self.ao_max * row, dtype=b.ao.dtype, device=b.ao.device)
            self._ao_cap = self.ao_max
        # exact-size contiguous views of the grow-only buffers (one all-gather of ao_max rows each)
        shape = (self.ao_max,) + tuple(b.ao.shape[1:])
        self.ao_send = self._ao_send_buf[:self.ao_max * row].view(shape)
        self.ao_recv = self._ao_recv_buf[:world * self.ao_max * row].view((world,) + shape)
        # the other bands' rows of the gathered AO: one index_select + one index_copy per frame
        # (built by device arange kernels: a host list copied to the device would be a synchronous copy)
        aod = b.ao.device
        others = [(k, lo, hi) for k, (lo, hi) in enumerate(self.ao_rows) if k != me and hi > lo]
        self._ao_dst = torch.cat([torch.arange(lo, hi, dtype=torch.int64, device=aod) for _, lo, hi in others]) \
            if others else torch.zeros(0, dtype=torch.int64, device=aod)
        self._ao_src = torch.cat([torch.arange(k * self.ao_max, k * self.ao_max + hi - lo, dtype=torch.int64, device=aod)
                                  for k, lo, hi in others]) if others else torch.zeros(0, dtype=torch.int64, device=aod)
        if not hasattr(self, "_bufs"):
            self._bufs = {}  # grow-only per-peer exchange buffers (_buf)
        # device compaction of the touched texels: per peer, the candidate region's texel indices and a
        # [3, cap + 1] int32 buffer (column cap collects the untouched texels' scatter writes)
        if world > 1:
            dev = b.ray_minmax.device
            sdw = b.ray_minmax.shape[2]
            self._cand = {}
            period = world if self.sd_split == "tiles" else 1
            for k, rows in self.iv_send.items():
                if rows:
                    lo, hi = rows
                    rl = self._region_rows(lo, hi, period)
                    n = (((hi - lo + 7) // 8 + period - 1) // period) * 8 * sdw if period > 1 else (hi - lo) * sdw
                    # the device path (librsd rsd_halo_compact) needs no index list; the torch path gathers
                    # the region's rows and their texel indices
                    idx = rsel = None
                    if not self.native:
                        rsel = torch.tensor(rl, dtype=torch.int64, device=dev)
                        idx = (rsel[:, None] * sdw + torch.arange(sdw, device=dev)).reshape(-1).to(torch.int32)
                    self._cand[k] = (lo, hi, idx, self._buf("cand", k, (3, n + 1), torch.int32, dev), rsel)
            if not hasattr(self, "_row"):  # shapes fixed by world: allocated once (a re-plan allocates nothing)
                self._row = torch.zeros(world + 1, dtype=torch.int64, device=dev)
                self._M_dev = torch.zeros((world, world + 1), dtype=torch.int64, device=dev)
                self._M_host = torch.zeros((world, world + 1), dtype=torch.int64,
                                           pin_memory=self.cuda and torch.cuda.is_available())
            else:
                self._row.zero_()  # the peers of the new plan write their counts; the others stay 0
            if self.native:
                from . import abi
                regs = [abi.HaloRegion(lo, hi, buf.data_ptr(), buf.shape[1], period, self._row.data_ptr() + 8 * k)
                        for k, (lo, hi, _, buf, _) in self._cand.items()]
                self._regions = (abi.HaloRegion * max(1, len(regs)))(*regs)
                self._n_regions = len(regs)

    @staticmethod
    def _region_rows(lo, hi, period):
        """The SD rows of a compaction region: [lo, hi), or every period-th 8-row tile from lo."""
        if period <= 1:
            return list(range(lo, hi))
        return [y for t0 in range(lo, hi, 8 * period) for y in range(t0, min(t0 + 8, hi))]

    def owned_sd_rows(self, rank=None):
        """The SD row ranges `rank` traces (default: this rank): its contiguous rows, or its tiles."""
        rank = self.rank if rank is None else rank
        if self.sd_split != "tiles":
            return [self.sd_rows[rank]]
        sdh = self.b.sd_h
        return [(y, min(y + 8, sdh)) for y in range(8 * rank, sdh, 8 * self.world)]

    def trace(self, consume=False, counters=False):
        """The SD trace of this rank's texels (rsd_sd_trace_band_ex over its tiles, or rsd_sd_trace_rows)."""
        b, kw = self.b, dict(self.trace_kw)
        if consume:
            kw["consume"] = True
        if counters:
            kw["counters"] = True
        if self.sd_band is not None:
            return b.sd_trace(band=self.sd_band, **kw)
        return b.sd_trace_rows(self.sd_rows[self.rank], **kw)

    def dense_bytes_per_frame(self):
        """What the round-2 dense halo (whole candidate rows) would send per frame from this rank."""
        b = self.b
        period = self.world if self.sd_split == "tiles" else 1
        nrows = lambda r: len(self._region_rows(r[0], r[1], period)) if r else 0  # noqa: E731
        iv = sum(2 * 4 * nrows(r) * b.sd.shape[2] for r in self.iv_send.values())
        sd_row = b.sd[:, 0].numel() * b.sd.element_size()
        sd = sum(nrows(r) * sd_row for r in self.sd_send.values())
        return {"intervals": iv, "sd": sd, "ao": self.ao_send.numel() * self.ao_send.element_size()}

    def bytes_per_frame(self):
        """Mean bytes this rank sent per frame so far: sparse interval halo, sparse SD halo, AO band."""
        n = max(1, self.frames)
        return {k: int(v // n) for k, v in self.sent.items()}

    def _buf(self, kind, k, shape, dtype, device):
        """A contiguous tensor of `shape` carved from a grow-only flat buffer per (kind, peer): the exchange
        buffers of a frame are the previous frame's memory (stream-ordered reuse; the comm's handshakes
        order the peers' reads), so steady state allocates nothing."""
        n = 1
        for x in shape:
            n *= x
        cur = self._bufs.get((kind, k))
        if cur is None or cur.numel() < n or cur.dtype != dtype:
            cur = torch.empty(max(n, 1) * 3 // 2 + 64, dtype=dtype, device=device)
            self._bufs[(kind, k)] = cur
        return cur[:n].view(shape)

    # ---- timing of this rank's compute (load balance)
    def _mark(self):
        """A timestamp for the re-balancing cost (None when nothing re-balances: world 1).  Device: the next
        event of this frame's set of six fence-free timing events (rsd/timing.py); two sets alternate, so the
        previous frame's events stay readable while this frame records (no event is created per frame)."""
        if not self.rebalance:
            return None
        if self.cuda:
            if not hasattr(self, "_evsets"):
                from .timing import TimingEvent
                self._evsets = [[TimingEvent() for _ in range(6)] for _ in range(2)]
                self._evn = 0
            e = self._evsets[(self._evn // 6) % 2][self._evn % 6]
            self._evn += 1
            e.record()
            return e
        return time.perf_counter()

    def _prev_cost_us(self):
        """This object's previous frame's compute time (us), or -1 while its events are incomplete
        (never waits: every rank then sees the -1 and nobody re-balances this frame)."""
        if self._prev is None:
            return -1
        if self.cuda:
            if not all(c.query() for _, c in self._prev):
                return -1
            return int(sum(a.elapsed_time(c) * 1e3 for a, c in self._prev))
        return int(sum((c - a) * 1e6 for a, c in self._prev))

    def _rebalanced(self, costs):
        """The next split of the 32-row groups from every rank's measured cost of the current one:
        cost spread uniformly over each band's groups, boundaries where the cumulative cost crosses
        k / world of the total, moved half-way (damping), at least one group per rank."""
        import numpy as np
        G, world, gb = self.G, self.world, self.gb
        n = np.diff(np.asarray(gb))
        dens = np.repeat(np.maximum(np.asarray(costs, dtype=np.float64), 1e-3) / np.maximum(n, 1), n)
        cum = np.concatenate(([0.0], np.cumsum(dens)))  # left-to-right float64 sums, as a Python loop adds
        total = cum[-1]
        new = [0]
        for k in range(1, world):
            target = total * k / world
            j = min(int(np.searchsorted(cum[1:], target, side="left")) + 1, G)  # first i >= 1 with cum[i] >= target
            # the nearer of the two group boundaries around the crossing
            if j > 0 and target - cum[j - 1] < cum[j] - target:
                j -= 1
            new.append(int(round(0.5 * gb[k] + 0.5 * j)))
        new.append(G)
        if G >= world:  # monotone, one group per rank at least
            for k in range(1, world):
                new[k] = min(max(new[k], new[k - 1] + 1), G - (world - k))
        # hysteresis: keep the split unless the cost model predicts the slowest band at least 3 % faster (a
        # re-split re-plans the exchange regions: host work every frame for a split that only oscillates)
        pred = max(cum[new[k + 1]] - cum[new[k]] for k in range(world))
        if pred > 0.97 * max(cum[gb[k + 1]] - cum[gb[k]] for k in range(world)):
            return list(gb)
        return new

    def frame(self, sd_events=None):
        b, me, world = self.b, self.rank, self.world
        if world == 1 and _one_call_frame(self, sd_events):
            self.splits.append(tuple(self.gb))
            self.frames += 1
            return
        self.front()
        self.back(sd_events)

    def front(self):
        """Steps 1-2: pass 1 of this rank's rows, the device compaction of the touched texels per
        peer and the all-gather of the counts (device tensors; the copy to the host is not waited for)."""
        assert self._open is None, "HaloFrame: front() twice without back()"
        b, me, world = self.b, self.rank, self.world
        if self._next_gb is not None and self._next_gb != self.gb:
            self.gb = self._next_gb
            self._plan()
        self._next_gb = None
        self.splits.append(tuple(self.gb))
        consume = getattr(b, "can_consume_intervals", False) and bool(b.cfg.ray_interval)
        if not (consume and self._intervals_clear):
            b.clear_intervals()
        st = {"consume": consume, "t": [self._mark()]}
        prev_us = self._prev_cost_us() if self.rebalance else -1
        b.pass1_rows(self.px_rows[me])
        st["t"].append(self._mark())
        if world > 1:
            row = self._row
            if self.native:
                # rsd_halo_compact: every peer's touched texels as triples and their counts in row[k] (the other
                # entries of row stay 0); triple order unspecified -- the receiver's min / max merge is exact
                from . import abi
                _, sdh, sdw = b.ray_minmax.shape
                abi.check(abi.lib().rsd_halo_compact(b.ray_minmax[0].data_ptr(), b.ray_minmax[1].data_ptr(), sdw, sdh,
                                                     self._regions, self._n_regions, b.stream), "rsd_halo_compact")
            else:
                row.zero_()
                for k, (lo, hi, idx, buf, rsel) in self._cand.items():
                    reg = b.ray_minmax.index_select(1, rsel).reshape(2, -1)
                    touched = (reg[0] != FLT_MAX_BITS) | (reg[1] != 0)
                    pos = torch.cumsum(touched, 0)  # int64: 1-based position of each touched texel
                    dst = torch.where(touched, pos - 1, torch.full_like(pos, buf.shape[1] - 1))
                    buf.scatter_(1, dst.expand(3, -1), torch.stack((idx, reg[0], reg[1])))
                    row[k:k + 1].copy_(pos[-1:])
            row[world:].fill_(prev_us)  # a kernel argument (row[world] = x is a synchronous host-to-device copy)
            self.comm.all_gather(self._M_dev, row)
            self._M_host.copy_(self._M_dev, non_blocking=True)
            if self.cuda:
                if not hasattr(self, "_cnt_ev"):  # one event per object: front() / back() strictly alternate
                    from .timing import TimingEvent
                    self._cnt_ev = TimingEvent()
                self._cnt_ev.record()
                st["ev"] = self._cnt_ev
        self._open = st

    def back(self, sd_events=None):
        """Steps 3-6 of the frame opened by front()."""
        assert self._open is not None, "HaloFrame: back() without front()"
        st, self._open = self._open, None
        b, me, world = self.b, self.rank, self.world
        t = st["t"]
        mine, theirs = {}, {}
        if world > 1:
            if self.cuda:
                if not st["ev"].query():
                    self.blocked_waits += 1
                st["ev"].synchronize()  # the counts of THIS frame on the host (lagged: already there)
            M = self._M_host.numpy().copy()
            # re-split on every second frame (each rank sees the same counts, so all skip or all re-split)
            if self.rebalance and self.frames % 2 == 0 and int(M[:, world].min()) >= 0:
                self._next_gb = self._rebalanced([float(x) for x in M[:, world]])
            dev = b.ray_minmax.device
            iv_send = {k: self._cand[k][3][:, :int(M[me, k])] for k in self._cand if M[me, k] > 0}
            iv_recv = {k: self._buf("iv", k, (3, int(M[k, me])), torch.int32, dev)
                       for k in range(world) if k != me and M[k, me] > 0}
            self.comm.exchange(iv_send, iv_recv)
            self.sent["intervals"] += sum(x.numel() * 4 for x in iv_send.values())
            if self.native:
                from . import abi
                L_ = abi.lib()
                _, sdh, sdw = b.ray_minmax.shape
                for k, x in iv_send.items():
                    mine[k] = x[0]  # int32 texel indices (row 0 of the persistent triple buffer)
                for k, x in iv_recv.items():
                    theirs[k] = x[0]
                if iv_recv:  # every peer's triples in one launch
                    lists = (abi.HaloList * len(iv_recv))(*[abi.HaloList(x.data_ptr(), x.shape[1], x.shape[1])
                                                            for x in iv_recv.values()])
                    abi.check(L_.rsd_halo_merge(b.ray_minmax[0].data_ptr(), b.ray_minmax[1].data_ptr(), sdw, sdh,
                                                lists, len(iv_recv), int(bool(b.cfg.ray_interval)), b.stream),
                              "rsd_halo_merge")
            else:
                for k, x in iv_send.items():
                    mine[k] = x[0].long()
                for k, x in iv_recv.items():
                    idx = x[0].long()
                    theirs[k] = idx
                    if b.cfg.ray_interval:
                        b.ray_minmax[0].view(-1).scatter_reduce_(0, idx, x[1], reduce="amin")
                    b.ray_minmax[1].view(-1).scatter_reduce_(0, idx, x[2], reduce="amax")
        if sd_events:
            sd_events[0].record()
        t.append(self._mark())
        self.trace(consume=st["consume"])
        self._intervals_clear = st["consume"]
        t.append(self._mark())
        if sd_events:
            sd_events[1].record()
        if world > 1:
            L, sdh, sdw, ch = b.sd.shape
            flat_sd = b.sd.view(L, sdh * sdw, ch)
            if self.native:
                from . import abi
                L_ = abi.lib()
                sd_send = {k: self._buf("sds", k, (L, idx.numel(), ch), b.sd.dtype, b.sd.device)
                           for k, idx in theirs.items()}
                if sd_send:  # every peer's reply in one launch
                    lists = (abi.HaloSdList * len(sd_send))(*[abi.HaloSdList(theirs[k].data_ptr(), x.data_ptr(),
                                                                             x.shape[1], 0) for k, x in sd_send.items()])
                    abi.check(L_.rsd_halo_sd_gather(b.sd.data_ptr(), L, sdw, sdh, ch, lists, len(sd_send), b.stream),
                              "rsd_halo_sd_gather")
            else:
                sd_send = {k: flat_sd.index_select(1, idx) for k, idx in theirs.items()}
            sd_recv = {k: self._buf("sdr", k, (L, idx.numel(), ch), b.sd.dtype, b.sd.device)
                       for k, idx in mine.items() if idx.numel()}
            self.comm.exchange(sd_send, sd_recv)
            self.sent["sd"] += sum(x.numel() * x.element_size() for x in sd_send.values())
            if self.native:
                if sd_recv:
                    lists = (abi.HaloSdList * len(sd_recv))(*[abi.HaloSdList(mine[k].data_ptr(), x.data_ptr(),
                                                                             x.shape[1], 0) for k, x in sd_recv.items()])
                    abi.check(L_.rsd_halo_sd_scatter(b.sd.data_ptr(), L, sdw, sdh, ch, lists, len(sd_recv), b.stream),
                              "rsd_halo_sd_scatter")
            else:
                for k, x in sd_recv.items():
                    flat_sd.index_copy_(1, mine[k], x)
        t.append(self._mark())
        b.pass2_rows(self.px_rows[me])
        t.append(self._mark())
        self._prev = [(t[0], t[1]), (t[2], t[3]), (t[4], t[5])] if self.rebalance else None
        if world > 1:
            lo, hi = self.ao_rows[me]
            send, recv = self.ao_send, self.ao_recv
            send[:hi - lo].copy_(b.ao[lo:hi])
            self.comm.all_gather(recv, send)
            self.sent["ao"] += send.numel() * send.element_size()
            if self._ao_dst.numel():
                b.ao.index_copy_(0, self._ao_dst, recv.view((-1,) + tuple(b.ao.shape[1:])).index_select(0, self._ao_src))
        self.frames += 1


# ---- the native band frame (include/rsd.h rsd_comm_* / rsd_band_frame_*; csrc/band_frame.cpp) --------------

class NativeHub:
    """rsd_comm_hub: the rendezvous of in-process communicators (`world` host threads sharing one GPU)."""

    def __init__(self, world: int):
        import ctypes as C

        from . import abi
        self.h = C.c_void_p()
        abi.check(abi.lib().rsd_comm_hub_create(world, C.byref(self.h)), "rsd_comm_hub_create")
        self.world = world

    def close(self):
        from . import abi
        if self.h:
            abi.lib().rsd_comm_hub_release(self.h)
            self.h = None


class NativeComm:
    """rsd_comm: the band frame's collectives in librsd -- RCCL (one process per GPU; ncclAllGather,
    ncclSend / ncclRecv on the caller's stream) or in-process (threads of one process sharing a GPU)."""

    def __init__(self, h):
        import ctypes as C

        from . import abi
        self.h = h
        k, r, w = C.c_uint32(), C.c_uint32(), C.c_uint32()
        abi.check(abi.lib().rsd_comm_info(h, C.byref(k), C.byref(r), C.byref(w)), "rsd_comm_info")
        self.kind, self.rank, self.world = k.value, r.value, w.value

    @classmethod
    def rccl(cls, rank: int, world: int, pg=None, device=None):
        """An RCCL communicator over the ranks of torch.distributed's group: rank 0's id travels over the
        group (a broadcast), then every rank joins (ncclCommInitRank on its current GPU)."""
        import ctypes as C

        import torch
        import torch.distributed as dist

        from . import abi
        L = abi.lib()
        uid = (C.c_uint8 * abi.COMM_UNIQUE_ID_BYTES)()
        if rank == 0:
            abi.check(L.rsd_comm_rccl_unique_id(uid), "rsd_comm_rccl_unique_id")
        if world > 1:
            on_gpu = dist.get_backend(pg) == "nccl"
            t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=device if on_gpu else "cpu")
            dist.broadcast(t, src=0, group=pg)
            uid = (C.c_uint8 * abi.COMM_UNIQUE_ID_BYTES)(*t.cpu().tolist())
        h = C.c_void_p()
        abi.check(L.rsd_comm_rccl_create(uid, world, rank, C.byref(h)), "rsd_comm_rccl_create")
        return cls(h)

    @classmethod
    def rccl_group(cls, rank: int, world: int, n: int = 1, pg=None, device=None):
        """`n` RCCL communicators over torch.distributed's group, created COLLECTIVELY so that the ranks fall back
        together: every rank first checks that librccl loads (rsd_comm_rccl_available) and the ranks
        agree on it (all-reduce MIN); rank 0 then draws the n ids and broadcasts them with a success flag (a
        failing rank 0 sends the flag, it does not raise before the broadcast); every rank creates its
        communicators and the ranks agree again.  Returns (communicators, None), or ([], reason) on every rank
        when any rank failed -- the caller takes the torch.distributed path.  (A rank failing INSIDE
        ncclCommInitRank after its peers entered it cannot be recovered from here: RCCL's own init is the
        collective.)"""
        import ctypes as C

        import torch
        import torch.distributed as dist

        from . import abi
        L = abi.lib()
        on_gpu = world > 1 and dist.get_backend(pg) == "nccl"
        dev = device if on_gpu else "cpu"

        def agree(ok: bool) -> bool:
            if world == 1:
                return ok
            t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=pg)
            return bool(int(t.item()))

        if not agree(L.rsd_comm_rccl_available() == 0):
            return [], "librccl.so.1 is not usable on every rank: " + abi.last_error()
        B = abi.COMM_UNIQUE_ID_BYTES
        buf = bytearray(1 + n * B)
        if rank == 0:
            ok, uid = True, (C.c_uint8 * B)()
            for j in range(n):
                if L.rsd_comm_rccl_unique_id(uid) != 0:
                    ok = False
                    break
                buf[1 + j * B:1 + (j + 1) * B] = bytes(uid)
            buf[0] = 1 if ok else 0
        if world > 1:
            t = torch.tensor(list(buf), dtype=torch.uint8, device=dev)
            dist.broadcast(t, src=0, group=pg)
            buf = bytearray(t.cpu().tolist())
        if not buf[0]:
            return [], "rank 0 could not draw the RCCL unique ids"
        comms, err = [], None
        for j in range(n):
            uid = (C.c_uint8 * B)(*buf[1 + j * B:1 + (j + 1) * B])
            h = C.c_void_p()
            if L.rsd_comm_rccl_create(uid, world, rank, C.byref(h)) != 0:
                err = abi.last_error()
                break
            comms.append(cls(h))
        if not agree(err is None):
            for c in comms:
                c.close()
            return [], f"rsd_comm_rccl_create failed on some rank ({err or 'peer'})"
        return comms, None

    @classmethod
    def local(cls, hub: NativeHub, rank: int):
        import ctypes as C

        from . import abi
        h = C.c_void_p()
        abi.check(abi.lib().rsd_comm_local_create(hub.h, rank, C.byref(h)), "rsd_comm_local_create")
        return cls(h)

    @classmethod
    def null(cls, rank: int, world: int):
        """A communicator that moves nothing (rsd_comm_null_create): host-cost probes of one rank's frame."""
        import ctypes as C

        from . import abi
        h = C.c_void_p()
        abi.check(abi.lib().rsd_comm_null_create(world, rank, C.byref(h)), "rsd_comm_null_create")
        return cls(h)

    def all_gather(self, out, inp, stream=None):
        """out [world, *inp.shape] <- every rank's inp (device tensors), on torch's current stream."""
        from . import abi
        import torch
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        abi.check(abi.lib().rsd_comm_all_gather(self.h, inp.data_ptr(), out.data_ptr(),
                                                inp.numel() * inp.element_size(), s), "rsd_comm_all_gather")

    def exchange(self, sends, recvs, stream=None):
        """Point-to-point: sends {peer: tensor}, recvs {peer: tensor} (sizes agreed beforehand)."""
        from . import abi
        import torch
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        xs = [abi.CommXfer(t.data_ptr(), t.numel() * t.element_size(), k, 0) for k, t in sends.items()]
        xr = [abi.CommXfer(t.data_ptr(), t.numel() * t.element_size(), k, 0) for k, t in recvs.items()]
        S = (abi.CommXfer * max(1, len(xs)))(*xs)
        R = (abi.CommXfer * max(1, len(xr)))(*xr)
        abi.check(abi.lib().rsd_comm_exchange(self.h, S, len(xs), R, len(xr), s), "rsd_comm_exchange")

    def close(self):
        from . import abi
        if self.h:
            abi.lib().rsd_comm_release(self.h)
            self.h = None


class NativeHaloFrame:
    """HaloFrame's band split issued from C++ (rsd_band_frame): front() / back() are ONE librsd call each --
    pass 1 of the rank's rows, the device compaction of the touched texels, the count all-gather and its
    copy to the host (front); the count read, the interval triples' point-to-point transfer and merge, the
    trace of the rank's SD share, the SD replies, pass 2 of its rows and the AO all-gather (back) -- with the
    exchanges on `comm` (NativeComm: RCCL, or in-process threads).  Same kernels, same bits as HaloFrame
    and as the 1-GPU frame; the re-balancing rule is HaloFrame._rebalanced's, its cadence is not: HaloFrame
    re-splits every second frame from the previous frame's time, the native frame every fourth frame (frame
    4j + 1 timed, decided at 4j + 3, applied at 4j + 4: the time is read without waiting, rsd.h).  A camera
    whose focal length or frame height changes re-plans the halo windows.  `backend` is a Renderer (or a frame
    slot of one): its buffers are used in place, its current camera is passed on every front()."""

    def __init__(self, backend, comm: NativeComm, throughput: bool = False, rebalance: bool = True,
                 sd_split: str = "auto"):
        import ctypes as C

        from . import abi
        self.b, self.comm = backend, comm
        self.rank, self.world = comm.rank, comm.world
        desc = abi.FrameDesc.from_buffer_copy(backend._frame_desc())
        bp = abi.BandParams(int(backend.cfg.divisor), abi.SD_SPLITS[sd_split], int(bool(rebalance)),
                            int(bool(throughput)))
        self.h = C.c_void_p()
        abi.check(abi.lib().rsd_band_frame_create(C.byref(desc), C.byref(bp), comm.h, C.byref(self.h)),
                  "rsd_band_frame_create")
        self.throughput = bool(throughput)
        self._ev = (C.c_void_p * 2)()
        self._L = abi.lib()

    def front(self, stream=None):
        """stream: a raw HIP stream handle (default: torch's current stream of the renderer's device) -- a caller that
        keeps one stream per frame slot passes it and saves the torch stream context per call (~6 us of host time)."""
        import ctypes as C
        b = self.b
        st = self._L.rsd_band_frame_front(self.h, C.byref(b.cam), b.stream if stream is None else stream)
        if st:
            from . import abi
            abi.check(st, "rsd_band_frame_front")

    def back(self, sd_events=None, stream=None):
        ev = None
        if sd_events:
            ev = self._ev
            ev[0] = sd_events[0].h.value if sd_events[0] is not None else None
            ev[1] = sd_events[1].h.value if sd_events[1] is not None else None
        st = self._L.rsd_band_frame_back(self.h, ev, self.b.stream if stream is None else stream)
        if st:
            from . import abi
            abi.check(st, "rsd_band_frame_back")

    def frame(self, sd_events=None):
        self.front()
        self.back(sd_events)

    def set_split(self, groups):
        """A split of the 32-row groups applied by the next front() (every rank the same; rsd_band_frame_set_split)."""
        import ctypes as C

        from . import abi
        a = (C.c_uint32 * len(groups))(*[int(g) for g in groups])
        abi.check(self._L.rsd_band_frame_set_split(self.h, a, len(groups)), "rsd_band_frame_set_split")

    def stats(self):
        import ctypes as C

        from . import abi
        s = abi.BandStats()
        abi.check(self._L.rsd_band_frame_stats(self.h, C.byref(s)), "rsd_band_frame_stats")
        return s

    # ---- HaloFrame's descriptive surface (bench.py, tests)
    @property
    def sd_split(self):
        return "tiles" if self.stats().sd_split == 1 else "rows"

    @property
    def sd_band(self):
        return (self.rank, self.world) if self.sd_split == "tiles" else None

    @property
    def gb(self):
        s = self.stats()
        return [int(x) for x in s.split[:s.world + 1]]

    @property
    def frames(self):
        return int(self.stats().frames)

    @property
    def blocked_waits(self):
        return int(self.stats().blocked_waits)

    def owned_sd_rows(self):
        s = self.stats()
        if s.sd_split != 1:
            return [(int(s.sd_row0), int(s.sd_row1))]
        sdh = self.b.sd_h
        return [(y, min(y + 8, sdh)) for y in range(8 * self.rank, sdh, 8 * self.world)]

    def trace(self, consume=False, counters=False):
        """The SD trace of this rank's share alone (rsd_sd_trace_band_ex / _rows): the instrumented traces
        of bench.py's roofline."""
        kw = {"throughput": True} if self.throughput else {}
        if consume:
            kw["consume"] = True
        if counters:
            kw["counters"] = True
        if self.sd_band is not None:
            return self.b.sd_trace(band=self.sd_band, **kw)
        s = self.stats()
        return self.b.sd_trace_rows((int(s.sd_row0), int(s.sd_row1)), **kw)

    def bytes_per_frame(self):
        s = self.stats()
        n = max(1, int(s.frames))
        return {"intervals": int(s.bytes_intervals) // n, "sd": int(s.bytes_sd) // n, "ao": int(s.bytes_ao) // n}

    def dense_bytes_per_frame(self):
        s = self.stats()
        n = max(1, int(s.frames))
        return {"intervals": int(s.dense_intervals), "sd": int(s.dense_sd), "ao": int(s.bytes_ao) // n}

    def close(self):
        if self.h:
            self._L.rsd_band_frame_release(self.h)
            self.h = None
