"""GPU checks of round 5's stream contracts: an index over device arrays is returned before
it is built (the build runs on a library stream, and every use orders its own stream after
it), and a chunk launches its probe and walk at classify time (sydelta_chunk_walk waits for
them, sydelta_chunk_free waits for a chunk never walked).  Results against the C oracle."""
import random

import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _dev(data: bytes, pad: int = 16):
    import torch

    t = torch.zeros(len(data) + pad, dtype=torch.uint8, device="cuda")
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    return t


def _pair(rng, nblk, bs):
    basis = rng.randbytes(nblk * bs + rng.randint(1, bs - 1))
    s = bytearray(basis)
    for _ in range(max(1, nblk // 50)):
        s[rng.randrange(len(s))] ^= rng.randrange(1, 256)
    s[7 * bs + 3:7 * bs + 3] = b"inserted"
    return bytes(s), basis


def _oracle(oracle_c, src, basis, bs):
    w, s, z = oracle_c.compute_checksums(basis, bs)
    return O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs))


@pytest.mark.parametrize("bs", [512, 4096])
def test_index_used_on_other_streams(gpu, oracle_c, bs):
    """Signature and index on stream A; the match on stream B and a chunk walk on stream C,
    queued at once with no host synchronisation: both wait for the build."""
    import torch

    rng = random.Random(bs)
    src, basis = _pair(rng, 600, bs)
    exp = _oracle(oracle_c, src, basis, bs)
    b, sd = _dev(basis), _dev(src)
    torch.cuda.synchronize()
    sa, sb, sc = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        w, s = gpu.signature(b[:len(basis)], bs, stream=sa)
        nb = w.numel()
        idx = gpu.Index(w, s, bs, len(basis) - (nb - 1) * bs, stream=sa)
        d = gpu.match(idx, sd, stream=sb, length=len(src))
        L = len(src)
        ch = gpu.Chunk(idx, sd, 0, L, 0, L, stream=sc)
        dc, ex = ch.walk(0)
        ch.close()
        idx.close()
        assert d.tuples() == exp
        assert dc.tuples() == exp and ex == L


def test_index_freed_unused(gpu):
    """Indexes over device arrays created and freed at once, many times (the build may still
    run when the free comes): no fault, and a later index still matches."""
    import torch

    bs = 1024
    b = _dev(bytes(range(256)) * 4096)
    s = torch.cuda.Stream()
    w, st = gpu.signature(b[:1 << 20], bs, stream=s)
    for _ in range(50):
        gpu.Index(w, st, bs, bs, stream=s).close()
    torch.cuda.synchronize()


def test_chunk_freed_unwalked(gpu, oracle_c):
    """Chunks classified (probe and walk launched) and freed without a walk; then one walked."""
    rng = random.Random(5)
    bs = 4096
    src, basis = _pair(rng, 900, bs)
    b, sd = _dev(basis), _dev(src)
    w, s = gpu.signature(b[:len(basis)], bs)
    nb = w.numel()
    idx = gpu.Index(w, s, bs, len(basis) - (nb - 1) * bs)
    L = len(src)
    for _ in range(5):
        gpu.Chunk(idx, sd, 0, L, 0, L).close()
    ch = gpu.Chunk(idx, sd, 0, L, 0, L)
    d, ex = ch.walk(0)
    ch.close()
    idx.close()
    assert d.tuples() == _oracle(oracle_c, src, basis, bs) and ex == L


def test_chunk_walked_twice_from_other_entries(gpu, oracle_c, monkeypatch):
    """A chunk walked from its start and then from later entries (segments re-walked from
    them): the first equals the oracle, the others the classifier + host walk of a chunk
    walked from the same entry (SYDELTA_CHUNK_WALK=0)."""
    rng = random.Random(9)
    bs = 512
    src, basis = _pair(rng, 800, bs)
    b, sd = _dev(basis), _dev(src)
    w, s = gpu.signature(b[:len(basis)], bs)
    nb = w.numel()
    idx = gpu.Index(w, s, bs, len(basis) - (nb - 1) * bs)
    L = len(src)
    monkeypatch.delenv("SYDELTA_CHUNK_WALK", raising=False)
    ch = gpu.Chunk(idx, sd, 0, L, 0, L)
    d0, ex0 = ch.walk(0)
    assert d0.tuples() == _oracle(oracle_c, src, basis, bs) and ex0 == L
    monkeypatch.setenv("SYDELTA_CHUNK_WALK", "0")
    ref = gpu.Chunk(idx, sd, 0, L, 0, L)
    for e in (1, 129 * bs + 77, 300 * bs, L - bs - 5):
        d1, ex1 = ch.walk(e)
        d2, ex2 = ref.walk(e)
        assert d1.tuples() == d2.tuples() and ex1 == ex2 == L, e
    ch.close()
    ref.close()
    idx.close()
