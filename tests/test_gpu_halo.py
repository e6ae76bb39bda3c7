"""GPU checks of the band split's device steps (include/rsd.h rsd_halo_*, csrc/halo.hip) against numpy on
random maps, edge cases included: row and round-robin-tile regions (partial last tile, a window not
starting on a tile, regions sharing one output and count), empty regions and lists, several lists per
launch.  The triples' order is unspecified (the merge is min / max), so sets are compared."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FLT_MAX_BITS = 0x7F7FFFFF


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from rsd import abi
    abi.lib()
    return torch, abi


def _stream(torch):
    return torch.cuda.current_stream().cuda_stream


def _maps(rng, sdh, sdw, frac):
    rmin = np.full((sdh, sdw), FLT_MAX_BITS, np.uint32)
    rmax = np.zeros((sdh, sdw), np.uint32)
    t = rng.random((sdh, sdw)) < frac
    vals = rng.random((2, sdh, sdw), dtype=np.float32) * 100
    rmin[t] = vals[0][t].view(np.uint32)
    rmax[t] = np.maximum(vals[0][t], vals[1][t]).view(np.uint32)
    only_max = rng.random((sdh, sdw)) < frac / 4  # rayMax set without RayInterval's rayMin
    rmax[only_max & ~t] = 1
    return rmin, rmax


def _region_rows(row0, row1, period):
    if period <= 1:
        return list(range(row0, row1))
    return [y for t0 in range(row0, row1, 8 * period) for y in range(t0, min(t0 + 8, row1))]


@pytest.mark.parametrize("sdh,sdw", [(53, 37), (64, 64), (9, 130)])
def test_compact_regions_match_numpy(dev, sdh, sdw):
    torch, abi = dev
    rng = np.random.default_rng(sdh * 1000 + sdw)
    rmin, rmax = _maps(rng, sdh, sdw, 0.15)
    mm = torch.from_numpy(np.stack([rmin, rmax]).view(np.int32)).cuda()
    specs = [(0, sdh, 1), (5, min(20, sdh), 1), (0, sdh, 3), (8, sdh, 2), (16, 16, 1), (8 * (sdh // 8), sdh, 4)]
    specs = [(a, b, p) for a, b, p in specs if a <= b <= sdh and (p <= 1 or a % 8 == 0)]
    outs, regs = [], []
    counts = torch.zeros(len(specs) + 1, dtype=torch.int64, device="cuda")
    for i, (a, b, p) in enumerate(specs):
        tiles = ((b - a + 7) // 8 + p - 1) // p if p > 1 and b > a else 0
        n = tiles * 8 * sdw if p > 1 else (b - a) * sdw
        out = torch.full((3, n + 1), -7, dtype=torch.int32, device="cuda")
        outs.append(out)
        regs.append(abi.HaloRegion(a, b, out.data_ptr(), n + 1, p, counts.data_ptr() + 8 * i))
    # two regions sharing the last output and count: each region's texels once
    shared = torch.full((3, 2 * sdw * sdh + 1), -7, dtype=torch.int32, device="cuda")
    half = sdh // 2
    regs.append(abi.HaloRegion(0, half, shared.data_ptr(), shared.shape[1], 1, counts.data_ptr() + 8 * len(specs)))
    regs.append(abi.HaloRegion(half, sdh, shared.data_ptr(), shared.shape[1], 1, counts.data_ptr() + 8 * len(specs)))
    arr = (abi.HaloRegion * len(regs))(*regs)
    abi.check(abi.lib().rsd_halo_compact(mm[0].data_ptr(), mm[1].data_ptr(), sdw, sdh, arr, len(regs), _stream(torch)),
              "rsd_halo_compact")
    torch.cuda.synchronize()
    cnt = counts.cpu().numpy()
    touched = (rmin != FLT_MAX_BITS) | (rmax != 0)
    for i, ((a, b, p), out) in enumerate(zip(specs + [(0, sdh, 1)], outs + [shared])):
        rows = _region_rows(a, b, p)
        want = {(y * sdw + x, int(rmin[y, x].view(np.int32)), int(rmax[y, x].view(np.int32)))
                for y in rows for x in range(sdw) if touched[y, x]}
        o = out.cpu().numpy()[:, :cnt[i]]
        got = set(zip(o[0].tolist(), o[1].tolist(), o[2].tolist()))
        assert cnt[i] == len(want) and got == want, (a, b, p)


def test_merge_is_the_exact_union(dev):
    torch, abi = dev
    rng = np.random.default_rng(7)
    sdh, sdw = 40, 50
    base_min, base_max = _maps(rng, sdh, sdw, 0.2)
    lists, want_min, want_max = [], base_min.copy(), base_max.copy()
    for k in range(3):
        n = int(rng.integers(0, 300)) if k != 1 else 0  # an empty list among them
        idx = rng.integers(0, sdh * sdw, n).astype(np.int32)
        mn = (rng.random(n, dtype=np.float32) * 100).view(np.uint32)
        mx = (rng.random(n, dtype=np.float32) * 100).view(np.uint32)
        stride = n + int(rng.integers(0, 5))
        tr = np.zeros((3, max(stride, 1)), np.int32)
        tr[0, :n], tr[1, :n], tr[2, :n] = idx, mn.view(np.int32), mx.view(np.int32)
        lists.append((torch.from_numpy(tr).cuda(), n, max(stride, 1)))
        np.minimum.at(want_min.reshape(-1), idx, mn)
        np.maximum.at(want_max.reshape(-1), idx, mx)
    for interval in (1, 0):
        mm = torch.from_numpy(np.stack([base_min, base_max]).view(np.int32)).cuda()
        arr = (abi.HaloList * len(lists))(*[abi.HaloList(t.data_ptr(), n, s) for t, n, s in lists])
        abi.check(abi.lib().rsd_halo_merge(mm[0].data_ptr(), mm[1].data_ptr(), sdw, sdh, arr, len(lists), interval,
                                           _stream(torch)), "rsd_halo_merge")
        got = mm.cpu().numpy().view(np.uint32)
        assert np.array_equal(got[0], want_min if interval else base_min)  # no RayInterval: rayMin untouched
        assert np.array_equal(got[1], want_max)


@pytest.mark.parametrize("layers,ch", [(1, 1), (1, 2), (1, 4), (2, 4), (4, 4)])
def test_sd_gather_scatter(dev, layers, ch):
    torch, abi = dev
    rng = np.random.default_rng(layers * 10 + ch)
    sdh, sdw = 23, 31
    sd = rng.random((layers, sdh, sdw, ch), dtype=np.float32)
    sd_t = torch.from_numpy(sd).cuda()
    idx_lists = [rng.permutation(sdh * sdw)[:int(n)].astype(np.int32) for n in (0, 17, 300)]
    idx_t = [torch.from_numpy(i).cuda() for i in idx_lists]
    outs = [torch.zeros((layers, len(i), ch), dtype=torch.float32, device="cuda") for i in idx_lists]
    arr = (abi.HaloSdList * 3)(*[abi.HaloSdList(i.data_ptr() if i.numel() else None, o.data_ptr() if o.numel() else None,
                                                len(il), 0) for i, o, il in zip(idx_t, outs, idx_lists)])
    abi.check(abi.lib().rsd_halo_sd_gather(sd_t.data_ptr(), layers, sdw, sdh, ch, arr, 3, _stream(torch)),
              "rsd_halo_sd_gather")
    flat = sd.reshape(layers, sdh * sdw, ch)
    for il, o in zip(idx_lists, outs):
        assert np.array_equal(o.cpu().numpy(), flat[:, il, :])
    # scatter the gathered values, doubled, into a zero map: exactly those texels change
    dst = torch.zeros_like(sd_t)
    for o in outs:
        o.mul_(2.0)
    abi.check(abi.lib().rsd_halo_sd_scatter(dst.data_ptr(), layers, sdw, sdh, ch, arr, 3, _stream(torch)),
              "rsd_halo_sd_scatter")
    want = np.zeros_like(flat)
    for il in idx_lists:
        want[:, il, :] = 2.0 * flat[:, il, :]
    assert np.array_equal(dst.cpu().numpy().reshape(layers, sdh * sdw, ch), want)
