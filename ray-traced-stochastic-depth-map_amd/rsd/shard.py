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
