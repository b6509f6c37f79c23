"""GPU parity for the device-resolved walk (K5b, sydelta_chain.hpp; SYDELTA_DEVICE_WALK=1).

The walk of generator.rs:116-221 is resolved on the device (merge of the aligned and
scan hit lists, successors, pointer-jumping path marking, op emission) instead of on host
threads.  Every op list must equal the C oracle's, and the library's walk counters must
show the device walk ran (a path that reaches a position only an on-demand scan
classifies is handed back to the host walk, which the counters show too).

Marked late (green on hardware since round 3; the per-thread bodies are also run by
the CPU suite's emulated device, tests/test_host_emulated.py)."""
import ctypes
import os
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.late]


@pytest.fixture
def device_walk():
    keys = ("SYDELTA_DEVICE_WALK", "SYDELTA_DEVICE_WALK_MIN", "SYDELTA_PROBE", "SYDELTA_PHASE_PROBE",
            "SYDELTA_CHUNK_WALK", "SYDELTA_FILE_WALK")
    old = {k: os.environ.get(k) for k in keys}
    os.environ["SYDELTA_DEVICE_WALK"] = "1"
    os.environ["SYDELTA_DEVICE_WALK_MIN"] = "1"
    # K5b resolves the classifier's walks: chunks and batches go through the classifier, not K10
    os.environ["SYDELTA_CHUNK_WALK"] = "0"
    os.environ["SYDELTA_FILE_WALK"] = "0"
    # phase-probed sources are walked on the host (walk_device hands them back); the
    # phase probe is on by default since round 4
    os.environ["SYDELTA_PHASE_PROBE"] = "0"
    yield
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _counters():
    from sy_amd._lib import lib

    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    lib.sydelta_walk_counters(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def _to_dev(data: bytes):
    import torch

    t = torch.zeros(len(data) + 16, dtype=torch.uint8, device="cuda")
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    return t


def _match(gpu, basis: bytes, src: bytes, bs: int):
    b = _to_dev(basis)
    w, s = gpu.signature(b[:len(basis)], bs)
    nb = w.numel()
    idx = gpu.Index(w, s, bs, (len(basis) - (nb - 1) * bs) if nb else 0)
    d = gpu.match(idx, _to_dev(src), length=len(src))
    idx.close()
    return d


def _oracle(oracle_c, src, basis, bs):
    w, s, z = oracle_c.compute_checksums(basis, bs)
    return O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs))


@pytest.mark.parametrize("probe", ["0", "1"])
@pytest.mark.parametrize("bs", [64, 512, 4096, 8192])
def test_device_walk_edits(bs, probe, device_walk, gpu, oracle_c):
    """Block edits (the C5 shape: aligned Copy runs), insertions and deletions (unaligned
    hits, on-demand scans), a duplicated block and a partial tail block."""
    os.environ["SYDELTA_PROBE"] = probe
    rng = random.Random(bs * 7 + int(probe))
    basis = rng.randbytes(bs * 600 + 123)
    src = bytearray(basis)
    for _ in range(30):
        src[rng.randrange(len(src))] ^= 0x5A
    for _ in range(4):
        p = rng.randrange(len(src))
        src[p:p] = rng.randbytes(rng.randint(1, 9))
        q = rng.randrange(len(src))
        del src[q:q + rng.randint(1, 9)]
    k = rng.randrange(500)
    src += basis[k * bs:(k + 1) * bs] + basis[-123:]
    src = bytes(src)
    w0, f0 = _counters()
    d = _match(gpu, basis, src, bs)
    assert d.tuples() == _oracle(oracle_c, src, basis, bs)
    w1, f1 = _counters()
    assert w1 > w0 or (probe == "1" and f1 > f0), "the device walk did not run"


@pytest.mark.parametrize("probe", ["0", "1"])
def test_device_walk_c5_shape(probe, device_walk, gpu, oracle_c):
    """64 MiB, bs 8192, 1 % of blocks with one substituted byte (BASELINE C5's edit
    model): 8 Ki hits, one walk."""
    import torch

    import sy_amd.device as dev

    os.environ["SYDELTA_PROBE"] = probe
    n, bs = 64 << 20, 8192
    basis = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    dev.synth_fill(basis[:n], 0xD1CE)
    src = basis.clone()
    g = np.random.default_rng(3)
    for k in g.choice(n // bs, (n // bs) // 100, replace=False):
        p = int(k) * bs + int(g.integers(0, bs))
        src[p] = (src[p] + 1) % 256
    w, s = dev.signature(basis[:n], bs)
    idx = dev.Index(w, s, bs, bs)
    w0, _ = _counters()
    d = dev.match(idx, src, length=n)
    idx.close()
    assert _counters()[0] > w0
    hb, hs = basis[:n].cpu().numpy(), src[:n].cpu().numpy()
    assert d.tuples() == _oracle(oracle_c, hs, hb, bs)


def test_device_walk_dense(device_walk, gpu, oracle_c):
    """Hits at every position (periodic and low-alphabet data): walks from neighbouring
    entries never merge; paths into unscanned blocks go back to the host walk."""
    rng = np.random.default_rng(9)
    per = np.tile(rng.integers(0, 256, 100, dtype=np.uint8), 3000)
    A = rng.integers(0, 256, 64, dtype=np.uint8)
    rot = np.concatenate([A[5:], A[:5]])
    Z = np.concatenate([rng.integers(0, 256, 5, dtype=np.uint8), A[5:]])
    parts = []
    for k in range(60):
        r = lambda m: rng.integers(0, 256, 64 * m, dtype=np.uint8)
        parts += [r(1), A, A, A] if k % 3 else [r(2), Z, A, A, A, r(1), A]
    cases = [
        (per, np.concatenate([per[:777], per[5:20000], per[3:]])),
        (np.concatenate([A, rot, rng.integers(0, 256, 64 * 40, dtype=np.uint8)]), np.concatenate(parts)),
    ]
    for probe in ("0", "1"):
        os.environ["SYDELTA_PROBE"] = probe
        for basis, src in cases:
            d = _match(gpu, basis.tobytes(), src.tobytes(), 64)
            assert d.tuples() == _oracle(oracle_c, src, basis, 64), probe


def test_device_walk_chunks(device_walk, gpu, oracle_c):
    """The chained chunk walks of the C5 path (entries inside blocks after a Copy that
    crosses a chunk boundary), 1/2/3/8 chunks, against the whole-file oracle result."""
    import sy_amd.device as dev

    bs = 4096
    rng = np.random.default_rng(21)
    basis = rng.integers(0, 256, 300 * bs + 77, dtype=np.uint8)
    s2 = np.concatenate([basis[:10 * bs], np.frombuffer(b"Q", np.uint8), basis[10 * bs:150 * bs], basis[200 * bs:]])
    for q in rng.integers(0, s2.size, 20):
        s2[q] ^= 0x22
    L = s2.size
    sb = _to_dev(s2.tobytes())
    bd = _to_dev(basis.tobytes())
    w, st = dev.signature(bd[:basis.size], bs)
    nb = w.numel()
    idx = dev.Index(w, st, bs, basis.size - (nb - 1) * bs)
    exp = _oracle(oracle_c, s2, basis, bs)
    npos = L - bs + 1
    nbp = -(-npos // bs)
    for nch in (1, 2, 3, 8):
        for probe in ("0", "1"):
            os.environ["SYDELTA_PROBE"] = probe
            cuts = sorted(int(c) for c in rng.choice(np.arange(1, nbp), nch - 1, replace=False)) if nch > 1 else []
            bounds = [0] + [c * bs for c in cuts] + [npos]
            parts, entry = [], 0
            for g in range(len(bounds) - 1):
                p0, p1 = bounds[g], bounds[g + 1]
                final = g == len(bounds) - 2
                bpos = p0 & ~15
                end = L if final else min(L, p1 + bs - 1)
                ch = dev.Chunk(idx, sb[bpos:end], bpos, L, p0, max(p1, L) if final else p1)
                part, entry = ch.walk(entry)
                ch.close()
                parts.append(part)
            assert dev.join_deltas(parts, L, bs).tuples() == exp, (nch, probe)
    idx.close()
