"""Level-2 filter false-pass rates on Adler-32 values of random data.

Keys: the Adler halves (A, B) of 2^20 random 4 KiB blocks (the C3 basis).  Queries:
every window of a 32 MiB random source (prefix sums).  The probe hashes q, r are
sydelta_kernels.hip's probe_hash (two 24-bit multiplies each); the level-2 word comes
from r's top bits, its bits from q's low fields; the level-1 Bloom is k_scan_r's (38400
words, word floor(q*38400/2^32) from q >> 8, bit q[0..4]).  Prints each layout's pass
rate over all positions and over the positions the level-1 filter passes (those are the
ones that send a level-2 request and, on a pass, an exact-table lookup).

    python tools/l2_filter_sim.py      (about a minute, ~6 GB of memory)
"""
import numpy as np

M, N = 65521, 4096
rng = np.random.default_rng(1)


def keys(nk=1 << 20, ch=1 << 14):
    A = np.empty(nk, np.uint64)
    B = np.empty(nk, np.uint64)
    w = N - np.arange(N, dtype=np.int64)
    for c in range(0, nk, ch):
        x = rng.integers(0, 256, (ch, N), dtype=np.uint8).astype(np.int64)
        A[c:c + ch] = (1 + x.sum(1)) % M
        B[c:c + ch] = (N + x @ w) % M
    return A, B


def windows(L=32 << 20):
    src = rng.integers(0, 256, L + N, dtype=np.uint8).astype(np.int64)
    S = np.concatenate([[0], np.cumsum(src)])
    T = np.concatenate([[0], np.cumsum(src * np.arange(L + N, dtype=np.int64))])
    p = np.arange(L, dtype=np.int64)
    s = S[p + N] - S[p]
    t = T[p + N] - T[p] - p * s
    return ((1 + s) % M).astype(np.uint64), ((N + N * s - t) % M).astype(np.uint64)


def probe_hash(A, B):
    q = (A * 0x9E3779 + B * 0x85EBCB) & 0xFFFFFFFF
    r = (A * 0xC2B2AF + B * 0x27D4EB) & 0xFFFFFFFF
    return q, r


def mask(q, bits, fieldw):
    m = np.zeros(q.shape, np.uint64)
    for i in range(bits):
        m |= np.uint64(1) << ((q >> np.uint64(fieldw * i)) & np.uint64((1 << fieldw) - 1))
    return m


def main():
    Ak, Bk = keys()
    Aq, Bq = windows()
    qk, rk = probe_hash(Ak, Bk)
    qq, rq = probe_hash(Aq, Bq)
    kw = np.unique((Bk << np.uint64(16)) | Ak)
    true = np.isin((Bq << np.uint64(16)) | Aq, kw)
    l1w = 38400
    wk = ((qk >> np.uint64(8)) * np.uint64(l1w << 8)) >> np.uint64(32)
    wq = ((qq >> np.uint64(8)) * np.uint64(l1w << 8)) >> np.uint64(32)
    F1 = np.zeros(l1w, np.uint64)
    np.bitwise_or.at(F1, wk.astype(np.int64), np.uint64(1) << (qk & np.uint64(31)))
    l1 = ((F1[wq.astype(np.int64)] >> (qq & np.uint64(31))) & np.uint64(1)).astype(bool)
    print(f"true weak hits {true.mean():.5f} of positions; Bloom level-1 passes {l1.mean():.4f}")
    for name, wbits, bits in (("32-bit words, 3 bits (rounds 1-3)", 32, 3), ("32-bit words, 5 bits (round 4)", 32, 5),
                              ("64-bit words, 5 bits", 64, 5), ("64-bit words, 6 bits", 64, 6)):
        nwords = (1 << 24) // wbits  # 2 MiB: 16 bits per key at 2^20 keys
        sh = np.uint64(32 - int(np.log2(nwords)))
        fieldw = 5 if wbits == 32 else 6
        F = np.zeros(nwords, np.uint64)
        np.bitwise_or.at(F, (rk >> sh).astype(np.int64), mask(qk, bits, fieldw))
        mq = mask(qq, bits, fieldw)
        p = (F[(rq >> sh).astype(np.int64)] & mq) == mq
        print(f"{name:36s} pass {p.mean():.5f}, false {(p & ~true).mean():.5f}, "
              f"after level-1 {(p & l1).mean() / l1.mean():.5f}")


if __name__ == "__main__":
    main()
