"""CPU check of k_scan_w's carried-window arithmetic (sydelta_kernels.hip, k_scan_w):
the first window of every thread of a tile, and the next tile's carried window, from
the two staged regions' 64-byte row sums -- restated here with the kernel's integer
widths (u32 sums, u64 products, the mod-M reductions) -- equal zlib's Adler-32 of the
window (rolling.rs:35-45 / zlib.adler32), for window sizes with every n mod 16 and
several tiles in a row (the carry).  Pure numpy + zlib; no GPU."""
import zlib

import numpy as np
import pytest

M = 65521
TILE = 32768
ROWS = TILE // 64


def _row_sums(b: np.ndarray):
    """Per 64-byte row h of b (len 64*k): byte sum s_h and sum_i i*x_{64h+i}."""
    h = b.reshape(-1, 64).astype(np.uint64)
    return h.sum(1), (h * np.arange(64, dtype=np.uint64)).sum(1)


def _partial(b32: np.ndarray, on: int):
    """Sums of the first `on` bytes of a row: (sum x, sum i*x)."""
    x = b32[:on].astype(np.uint64)
    return int(x.sum()), int((x * np.arange(on, dtype=np.uint64)).sum())


def _tile_windows(data: np.ndarray, T0: int, n: int, S0: int, B0: int):
    """k_scan_w's window phase for the tile at T0 given (S0, B0) of the window at T0:
    -> (A, B) Adler halves of the window of every thread (64 t), and the carry (S0', B0')."""
    on = n & 15
    nal = n - on
    out_reg = data[T0:T0 + TILE]
    in_reg = data[T0 + nal:T0 + nal + TILE + 16]  # rows 512..1023 + row 1024's 16 bytes
    so, uo = _row_sums(out_reg)
    si, ui = _row_sums(in_reg[:TILE])
    t = np.arange(ROWS, dtype=np.uint64)
    assert int((64 * t * so + uo).max()) < 2 ** 32  # the kernel's u32 before the reduction
    wo = (64 * t * so + uo) % M
    wi = (64 * t * si + ui) % M
    Eso = np.concatenate([[0], np.cumsum(so)[:-1]])
    Ewo = np.concatenate([[0], np.cumsum(wo)[:-1]])
    Esi = np.concatenate([[0], np.cumsum(si)[:-1]])
    Ewi = np.concatenate([[0], np.cumsum(wi)[:-1]])
    ps0, pu0 = _partial(in_reg[0:64], on)
    psT, puT = _partial(in_reg[TILE:TILE + 16], on)

    def window(d, Os, Ow, Is, Iw, p_s, p_u):
        Rs = Is + p_s
        Rw = (Iw + d * p_s + p_u) % M
        InS = Rs - ps0
        Rw_d = (Rw + M - pu0 % M) % M
        InW = ((on + d) * InS + M - Rw_d) % M
        OutW = (d * Os + M - Ow % M) % M
        S = S0 + InS - Os
        b = B0 + d * (S0 % M) + InW + M - OutW
        b += M * M - (n % M) * (Os % M)
        return S, b % M

    res = []
    for th in range(ROWS):
        p_s, p_u = _partial(in_reg[64 * th:64 * th + 64], on)
        S, B = window(64 * th, int(Eso[th]), int(Ewo[th]) % M, int(Esi[th]), int(Ewi[th]) % M, p_s, p_u)
        res.append(((1 + S) % M, (n + B) % M))
    Sn, Bn = window(TILE, int(so.sum()), int(wo.sum()) % M, int(si.sum()), int(wi.sum()) % M, psT, puT)
    return res, (Sn, Bn)


def _fresh(data, T0, n):
    x = data[T0:T0 + n].astype(np.uint64)
    return int(x.sum()), int((x * (n - np.arange(n, dtype=np.uint64))).sum() % M)


@pytest.mark.parametrize("n", [8193, 8208, 9999, 10007, 16384, 31622, 65536, 65551, 131071, 131072])
def test_carried_windows_equal_adler(n):
    rng = np.random.default_rng(n)
    ntiles = 3
    data = rng.integers(0, 256, ntiles * TILE + n + 64, dtype=np.uint8)
    if n % 3 == 0:
        data[: n // 2] = 255  # large sums: the exact u32 byte sums and u64 products
    S0, B0 = _fresh(data, 0, n)
    for k in range(ntiles):
        T0 = k * TILE
        res, (S0n, B0n) = _tile_windows(data, T0, n, S0, B0)
        for th in list(range(0, ROWS, 37)) + [ROWS - 1]:
            p = T0 + 64 * th
            ad = zlib.adler32(data[p:p + n].tobytes())
            assert res[th] == (ad & 0xFFFF, ad >> 16), (n, k, th)
        assert (S0n, B0n) == _fresh(data, T0 + TILE, n), (n, k)
        S0, B0 = S0n, B0n
