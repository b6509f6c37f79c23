"""GPU parity for large single-file indexes (> 16 Ki basis blocks) at bs 4096: the
register-fed level-1-filter scan k_scan_r against the oracle (round 4 removed the
superseded large-index kernels), with both level-1 layouts forced on the smaller cases
(SYDELTA_L1=bloom|ribbon); the 4 GiB C3 case runs with the default (the ribbon),
started at each of its three points (SYDELTA_EARLY_RIBBON).

* 96 MiB basis, mixed edits (an all-literal stretch, sparse substitutions, a shift,
  planted unaligned copies, duplicated blocks): bit-exact op list against the C
  restatement of generator.rs, with the aligned probe forced off (every window
  start through the scan) and on.
* BASELINE C3 at its configured size (4 GiB basis, 4 GiB source with Bernoulli(5 %)
  byte substitutions, bs 4096) with 64 basis blocks planted at seeded unaligned
  offsets and the basis's partial last block at the end of the source: the op list
  equals the analytic one (Data runs between the planted Copies, then the tail
  Copy, generator.rs:116-221), each planted neighbourhood (+-2 blocks) re-derived by
  the C oracle, and the identical source is all Copy.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["bloom", "ribbon"])
def level1(request, monkeypatch):
    """k_scan_r's level-1 filter layout (SYDELTA_L1, read when the index is built): the
    one-hash Bloom or the ribbon (the default from 852 K keys, so C3 uses it)."""
    monkeypatch.setenv("SYDELTA_L1", request.param)
    return request.param


def _ops_device(gpu, basis_t, src_t, bs, src_len=None, probe=None):
    import torch

    w, s = gpu.signature(basis_t, bs)
    nb = w.numel()
    last = basis_t.numel() - (nb - 1) * bs
    idx = gpu.Index(w, s, bs, last)
    old = os.environ.get("SYDELTA_PROBE")
    try:
        if probe is not None:
            os.environ["SYDELTA_PROBE"] = probe
        d = gpu.match(idx, src_t, length=src_len)
    finally:
        if old is None:
            os.environ.pop("SYDELTA_PROBE", None)
        else:
            os.environ["SYDELTA_PROBE"] = old
    idx.close()
    torch.cuda.synchronize()
    return d, w, s


def _mixed_source(basis: np.ndarray, bs: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    n = basis.size
    q = n // 6
    parts = []
    # an all-literal stretch: Bernoulli(5%) byte substitutions
    a = basis[:q].copy()
    m = rng.random(q) < 0.05
    a[m] ^= rng.integers(1, 256, int(m.sum()), dtype=np.uint8)
    parts.append(a)
    # sparse: one substituted byte in 2% of blocks
    b = basis[q:3 * q].copy()
    for k in rng.choice(b.size // bs, b.size // bs // 50, replace=False):
        b[k * bs + rng.integers(0, bs)] ^= 0x5A
    parts.append(b)
    # a 17-byte insertion shifts the rest of this stretch off the block grid
    c = basis[3 * q:4 * q]
    parts.append(np.concatenate([c[:1000], rng.integers(0, 256, 17, dtype=np.uint8), c[1000:]]))
    # planted copies of random basis blocks at random gaps, some duplicated
    out = []
    for _ in range(400):
        out.append(rng.integers(0, 256, int(rng.integers(1, 3 * bs)), dtype=np.uint8))
        k = int(rng.integers(0, n // bs))
        blk = basis[k * bs:(k + 1) * bs]
        out.append(blk)
        if rng.random() < 0.3:
            out.append(blk)
    parts.append(np.concatenate(out))
    parts.append(basis[4 * q:5 * q])  # untouched
    return np.concatenate(parts)


@pytest.mark.parametrize("probe", ["0", "1"])
def test_large_index_mixed_edits(gpu, oracle_c, level1, probe):
    import torch

    bs = 4096
    n = 96 << 20  # 24576 blocks: level-1 filter path
    basis_t = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(basis_t[:n], 0x5E1D0101)
    basis = basis_t[:n].cpu().numpy()
    src = _mixed_source(basis, bs, 0x5E1D0102)
    src_t = torch.zeros(src.size + 16, dtype=torch.uint8, device="cuda")
    src_t[:src.size] = torch.from_numpy(src).cuda()
    d, w, s = _ops_device(gpu, basis_t[:n], src_t, bs, src_len=src.size, probe=probe)
    ew, es, ez = oracle_c.compute_checksums(basis, bs, threads=8)
    assert np.array_equal(w.cpu().numpy().view(np.uint32), ew)
    expect = O.ops_from_arrays(*oracle_c.generate_delta(src, ew, es, ez, bs))
    assert d.tuples() == expect
    assert d.stats["copy_ops"] > 10000


def test_large_index_dense_passes(gpu, oracle_c, level1):
    """All-zero and period-3 stretches against a random basis that holds a zero block
    and the three phases of the period-3 block: every window start there is a weak
    hit, so the per-wave pass queue overflows inside one batch (the one position at
    a time path) and the walk copies a block at every jump (generator.rs:116-155)."""
    import torch

    bs = 4096
    n = 80 << 20
    basis_t = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(basis_t[:n], 0x5E1D0111)
    basis = basis_t[:n].cpu().numpy()
    abc = np.frombuffer(b"ABC" * ((1 << 20) // 3 + 2), np.uint8)
    basis[5 * bs:6 * bs] = 0
    for ph in range(3):
        basis[(6 + ph) * bs:(7 + ph) * bs] = abc[ph:ph + bs]
    basis_t[:n] = torch.from_numpy(basis).cuda()
    rng = np.random.default_rng(7)
    src = np.concatenate([np.zeros(1 << 20, np.uint8), rng.integers(0, 256, 999, dtype=np.uint8),
                          abc[:1 << 20], basis[:4 << 20]])
    src_t = torch.zeros(src.size + 16, dtype=torch.uint8, device="cuda")
    src_t[:src.size] = torch.from_numpy(src).cuda()
    d, _, _ = _ops_device(gpu, basis_t[:n], src_t, bs, src_len=src.size, probe="0")
    ew, es, ez = oracle_c.compute_checksums(basis, bs, threads=8)
    assert d.tuples() == O.ops_from_arrays(*oracle_c.generate_delta(src, ew, es, ez, bs))


@pytest.mark.parametrize("early", ["0", "1", "2"])
def test_config3_full_size_planted(gpu, oracle_c, monkeypatch, early):
    """C3 at 4 GiB with a non-trivial expected op list; the ribbon
    level-1 started at index creation (SYDELTA_EARLY_RIBBON=2, the default), at the match
    call (1) or by the first scan (0)."""
    import torch

    monkeypatch.setenv("SYDELTA_EARLY_RIBBON", early)

    bs = 4096
    n = (4 << 30) - 1000  # partial last basis block of 3096 bytes
    last = n % bs
    nblk = n // bs + 1
    basis_t = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(basis_t[:n], 0x5E1D0002)
    src_t = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    gpu.synth_mutate(src_t[:n], basis_t[:n], 0x5E1D0003, 50000)
    rng = np.random.default_rng(0x5E1D0103)
    # 64 planted blocks at unaligned offsets, at least 3 blocks apart
    slots = np.sort(rng.choice((n - 4 * bs) // (4 * bs), 64, replace=False))
    pos = [int(sl * 4 * bs + bs + rng.integers(1, bs)) for sl in slots]
    blks = [int(k) for k in rng.integers(0, nblk - 1, 64)]
    for p, k in zip(pos, blks):
        src_t[p:p + bs] = basis_t[k * bs:(k + 1) * bs]
    tail = n - last  # the partial last block ends the source (tail rule)
    src_t[tail:n] = basis_t[tail:n]
    d, w, s = _ops_device(gpu, basis_t[:n], src_t, bs, src_len=n)
    expect = []
    lit = 0
    for p, k in zip(pos, blks):
        expect += [("D", lit, p - lit), ("C", k * bs, bs)]
        lit = p + bs
    expect += [("D", lit, tail - lit), ("C", (nblk - 1) * bs, last)]
    assert d.tuples() == expect
    assert d.stats["verified_hits"] == 64
    # the oracle on each planted neighbourhood (+-2 blocks) against the full signature
    hw = w.cpu().numpy().view(np.uint32)
    hs = s.cpu().numpy().view(np.uint64)
    hz = np.full(nblk, bs, np.uint64)
    hz[-1] = last
    for p, k in zip(pos[:16], blks[:16]):
        lo, hi = p - 2 * bs, p + 3 * bs
        win = src_t[lo:hi].cpu().numpy()
        got = O.ops_from_arrays(*oracle_c.generate_delta(win, hw, hs, hz, bs))
        assert got == [("D", 0, 2 * bs), ("C", k * bs, bs), ("D", 3 * bs, 2 * bs)], (p, k)
    # identical source: every block copied, in order
    d2, _, _ = _ops_device(gpu, basis_t[:n], basis_t, bs, src_len=n)
    kind = np.asarray(d2.kind)
    a = np.asarray(d2.a, dtype=np.uint64)
    assert kind.size == nblk and not kind.any()
    assert np.array_equal(a, np.arange(nblk, dtype=np.uint64) * bs)
