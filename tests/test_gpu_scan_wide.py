"""GPU parity of the register-fed scan k_scan_g on windows above 8 KiB (sy's own block
size calculate_block_size = sqrt(file size) for every file over 64 MiB, mod.rs:20-23)
against the C restatement of generator.rs, and against the per-thread k_scan
(SYDELTA_SCAN_WIDE=0, which also turns the aligned probe off).  The deferred weak-hit
list of k_verify_w also runs with a cap of 64 entries (SYDELTA_WDEF_CAP), so that hits
past it are verified inline beside the deferred ones.  (Round 3's k_scan_w, which this
file tested before, was replaced by k_scan_g in round 4.)

* every n mod 16 class that matters (8193, 9999, 16384, 31622, 65536, 131071, 131072):
  random edits (substitutions, insertions, deletions, block moves) over several tiles,
  probe forced on and off (on: the scan covers only the blocks whose aligned window
  missed, several segments per launch, on-demand rescans);
* a source shifted by an insertion at its start (a hit per block at an unaligned
  phase: dense verifications from global memory);
* a source shorter than a tile, one window long, and empty of full windows;
* periodic data (every window a weak and strong hit, lowest index wins);
* the streamed path API at bs 65536 (chunk machinery + k_scan_g).
"""
import os
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


WIDE = [8193, 9999, 16384, 31622, 65536, 131071, 131072]


def _to_dev(data: bytes):
    import torch

    t = torch.zeros(len(data) + 16, dtype=torch.uint8, device="cuda")
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    return t


def _device(gpu, src: bytes, basis: bytes, bs: int, env=None):
    import torch

    old = {k: os.environ.get(k) for k in (env or {})}
    try:
        for k, v in (env or {}).items():
            os.environ[k] = v
        b = _to_dev(basis)
        w, s = gpu.signature(b[:len(basis)], bs)
        nb = w.numel()
        last = (len(basis) - (nb - 1) * bs) if nb else 0
        idx = gpu.Index(w, s, bs, last)
        d = gpu.match(idx, _to_dev(src), length=len(src))
        idx.close()
        torch.cuda.synchronize()
        return d
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _oracle(oracle_c, src, basis, bs):
    w, s, z = oracle_c.compute_checksums(basis, bs)
    return O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs))


def _edit(basis: bytes, rng, bs, nops=30):
    src = bytearray(basis)
    for _ in range(nops):
        op, p = rng.randint(0, 3), rng.randrange(len(src))
        if op == 0:
            src[p] ^= 1 + rng.randrange(255)
        elif op == 1:
            src[p:p] = rng.randbytes(rng.randint(1, 300))
        elif op == 2:
            del src[p:p + rng.randint(1, 300)]
        else:
            q = rng.randrange(len(src))
            src[p:p] = src[q:q + rng.randint(1, 3 * bs)]
    return bytes(src)


@pytest.mark.parametrize("bs", WIDE)
def test_wide_random_edits(bs, gpu, oracle_c):
    rng = random.Random(bs)
    # 12 MiB: ~770 tiles, so every workgroup carries its windows over several tiles
    basis = rng.randbytes((12 << 20) + rng.randrange(bs))
    src = _edit(basis, rng, bs)
    exp = _oracle(oracle_c, src, basis, bs)
    for probe in ("0", "1"):
        d = _device(gpu, src, basis, bs, {"SYDELTA_PROBE": probe})
        assert d.tuples() == exp, (bs, probe)
    assert O.py_apply_delta(basis, src, exp) == src
    # the kernel it replaces gives the same ops
    assert _device(gpu, src, basis, bs, {"SYDELTA_SCAN_WIDE": "0"}).tuples() == exp


@pytest.mark.parametrize("bs", [9999, 65536, 131072])
def test_wide_shifted_source(bs, gpu, oracle_c):
    """An insertion at the start: every block matches at an unaligned phase, so the
    scan verifies one weak hit per block from global memory."""
    rng = random.Random(bs + 1)
    basis = rng.randbytes(24 * bs + 777)
    src = rng.randbytes(5) + basis[: 12 * bs] + rng.randbytes(3) + basis[12 * bs:]
    exp = _oracle(oracle_c, src, basis, bs)
    assert sum(1 for k, _, _ in exp if k == "C") >= 22
    for probe in ("0", "1"):
        assert _device(gpu, src, basis, bs, {"SYDELTA_PROBE": probe}).tuples() == exp, probe


@pytest.mark.parametrize("bs", [8193, 65536])
def test_wide_short_sources(bs, gpu, oracle_c):
    rng = random.Random(bs + 2)
    basis = rng.randbytes(5 * bs + 123)
    for src in (basis[:bs], basis[bs:2 * bs + 1], basis[:bs - 1], rng.randbytes(bs + 17) + basis[3 * bs:4 * bs],
                basis[2 * bs:] + basis[:bs // 2], b""):
        for probe in ("0", "1"):
            assert _device(gpu, src, basis, bs, {"SYDELTA_PROBE": probe}).tuples() == _oracle(oracle_c, src, basis, bs)


def test_wide_deferred_list_overflow(gpu, oracle_c):
    """More weak hits than the deferred list holds: a child process with
    SYDELTA_WDEF_CAP=64 (read once per process) runs shifted and periodic sources whose
    hits overflow it, so k_verify_w verifies the first 64 and drain_w the rest inline."""
    import subprocess
    import sys

    code = r"""
import random, sys
sys.path.insert(0, %r)
import numpy as np, torch
import sy_amd.device as gpu
from oracle import oracle as O
C = O.C()
def run(src, basis, bs):
    def dev(b):
        t = torch.zeros(len(b) + 16, dtype=torch.uint8, device="cuda")
        if b: t[:len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()
        return t
    bt = dev(basis)
    w, s = gpu.signature(bt[:len(basis)], bs)
    nb = w.numel()
    idx = gpu.Index(w, s, bs, len(basis) - (nb - 1) * bs)
    d = gpu.match(idx, dev(src), length=len(src))
    idx.close()
    ew, es, ez = C.compute_checksums(basis, bs)
    assert d.tuples() == O.ops_from_arrays(*C.generate_delta(src, ew, es, ez, bs)), (len(src), bs)
    return d.stats["verified_hits"]
rng = random.Random(11)
bs = 9999
basis = rng.randbytes(300 * bs + 77)
nv = run(rng.randbytes(3) + basis, basis, bs)
assert nv >= 290, nv
pat = (b"ABC" * 70000)[:200000]
run(pat[:150000], pat, 9000)
print("ok", nv)
""" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),)
    env = dict(os.environ, SYDELTA_WDEF_CAP="64", SYDELTA_PROBE="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok")


@pytest.mark.parametrize("pattern", [b"\x00", b"ABC", b"0123456789" * 7])
def test_wide_periodic_data(pattern, gpu, oracle_c):
    """Every window start a weak and strong hit (duplicate keys: lowest index wins)."""
    bs = 9000
    basis = (pattern * (200000 // len(pattern) + 1))[:200000]
    for src in (basis[:120000], basis[5:90000] + b"xyz", b"q" + basis[:60000]):
        for probe in ("0", "1"):
            got = _device(gpu, src, basis, bs, {"SYDELTA_PROBE": probe}).tuples()
            assert got == _oracle(oracle_c, src, basis, bs), (pattern[:3], len(src), probe)


def test_wide_streamed_path_api(tmp_path, monkeypatch, oracle_c, gpu):
    import sy_amd.delta as D

    monkeypatch.setenv("SYDELTA_STREAM_CHUNK", str(3 << 20))
    bs = 65536
    rng = random.Random(7)
    basis = rng.randbytes((20 << 20) + 4321)
    src = _edit(basis, rng, bs, nops=60)
    pb, ps, po = tmp_path / "dest", tmp_path / "src", tmp_path / "out"
    pb.write_bytes(basis)
    ps.write_bytes(src)
    sigs = D.compute_checksums(pb, bs)
    delta = D.generate_delta_streaming(ps, sigs, bs)
    exp = _oracle(oracle_c, src, basis, bs)
    got = [("C", op.offset, op.size) if isinstance(op, D.Copy) else ("D", len(op.data)) for op in delta.ops]
    assert got == [("C", a, b) if k == "C" else ("D", b) for k, a, b in exp]
    D.apply_delta(pb, delta, po)
    assert po.read_bytes() == src
