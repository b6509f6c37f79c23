"""CPU check of k_scan_g's carried-window arithmetic (sydelta_kernels.hip, k_scan_g and
window_at): a run's first window summed lane by lane, then per wave tile of 4096
positions every lane's first window from the tile's (A0, B0) and exclusive wave scans
of the out/in rows' sums, and the next tile's (A0, B0) from lane 63's 64 rolls
(rolling.rs:66-79) -- restated with the kernel's integer widths (u32 dot products and
wave scans, u64 products, the mod-M reductions, asserted to stay in range) -- equal
zlib's Adler-32 of the window (rolling.rs:35-45 / zlib.adler32), for windows with every
n mod 64 class that matters, shorter and longer than a tile, over several tiles.
Pure numpy + zlib; no GPU."""
import zlib

import numpy as np
import pytest

M = 65521
WT = 4096  # positions per wave tile (kWTR)
U32 = 2 ** 32


def _rows(data: np.ndarray, at: int):
    """The 64 lanes' 64-byte rows at byte offset at: (S, V) per lane, S = sum x,
    V = sum i x_i (udot4 with offw weights)."""
    r = data[at:at + 64 * 64].astype(np.uint64).reshape(64, 64)
    S = r.sum(1)
    V = (r * np.arange(64, dtype=np.uint64)).sum(1)
    assert S.max() < U32 and V.max() < U32
    return S, V


def _excl(v: np.ndarray):
    e = np.concatenate([[0], np.cumsum(v)[:-1]]).astype(np.uint64)
    assert e.max() < U32 and int(v.sum()) < U32  # wave_scan_excl's u32 total
    return e


def window_at(data: np.ndarray, P: int, n: int):
    """window_at: (1 + s) mod M, (n + n s - t) mod M with t = sum i x_i."""
    x = data[P:P + n].astype(np.uint64)
    s = int(x.sum())
    t = int((x * np.arange(n, dtype=np.uint64)).sum())
    return (1 + s) % M, (n + n * s - t) % M


def tile_windows(data: np.ndarray, P: int, n: int, A0: int, B0: int):
    """The window block of one wave tile: lane l's window at P + 64 l."""
    so, vo = _rows(data, P)
    si, vi = _rows(data, P + n)
    lane = np.arange(64, dtype=np.uint64)
    Ox, Ix = _excl(so), _excl(si)
    ROx, RIx = _excl(lane * so), _excl(lane * si)
    VOx, VIx = _excl(vo), _excl(vi)
    nm = n % M
    out = []
    for l in range(64):
        d = 64 * l
        pin = 64 * (l * int(Ix[l]) - int(RIx[l])) - int(VIx[l])
        pout = 64 * (l * int(Ox[l]) - int(ROx[l])) - int(VOx[l])
        assert pin >= 0 and pout >= 0
        assert int(Ox[l]) <= 16 * M
        am = (A0 + int(Ix[l]) + 16 * M - int(Ox[l])) % M
        bpos = B0 + d * (A0 + M - 1) + pin
        bneg = (pout + nm * int(Ox[l])) % M
        assert bpos < 2 ** 64 and pout + nm * int(Ox[l]) < 2 ** 64
        out.append((am, (bpos % M + M - bneg) % M))
    return out


def roll(a: int, b: int, xo: int, xi: int, n: int):
    """rolling.rs:66-79: one byte out, one in."""
    a = (a + M - xo + xi) % M
    b = (b + M * 256 - (n * xo) % M + a + M - 1) % M
    return a, b


@pytest.mark.parametrize("n", [64, 100, 1007, 4095, 4096, 4097, 8193, 9999, 31622, 65536, 131071])
def test_carried_windows_equal_adler(n):
    rng = np.random.default_rng(n)
    ntiles = 3
    data = rng.integers(0, 256, ntiles * WT + n + 64 * 64 + 64, dtype=np.uint8)
    if n % 3 == 0:
        data[: n // 2 + 4096] = 255  # large sums: the u32 scans and u64 products at their widest
    A0, B0 = window_at(data, 0, n)
    for k in range(ntiles):
        P = k * WT
        res = tile_windows(data, P, n, A0, B0)
        for l in list(range(0, 64, 9)) + [63]:
            p = P + 64 * l
            ad = zlib.adler32(data[p:p + n].tobytes())
            assert res[l] == (ad & 0xFFFF, ad >> 16), (n, k, l)
        # lane 63 rolls its 64 positions: the next tile's start window
        a, b = res[63]
        for j in range(64):
            q = P + 64 * 63 + j
            a, b = roll(a, b, int(data[q]), int(data[q + n]), n)
        assert (a, b) == window_at(data, P + WT, n), (n, k)
        A0, B0 = a, b
