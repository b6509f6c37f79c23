"""GPU parity: signature kernels (K1) vs the oracle — bit-exact u32/u64."""
import os
import random

import numpy as np
import pytest

from golden_io import dec, load_cases

pytestmark = pytest.mark.gpu


def _dev_sig(gpu, data: bytes, bs: int, offset: int = 0):
    import torch

    raw = torch.zeros(len(data) + offset + 16, dtype=torch.uint8, device="cuda")
    if data:
        raw[offset:offset + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    view = raw[offset:offset + len(data)]
    w, s = gpu.signature(view, bs)
    torch.cuda.synchronize()
    return (w.cpu().numpy().view(np.uint32).astype(np.uint64).tolist(), s.cpu().numpy().view(np.uint64).tolist())


@pytest.mark.parametrize("case", load_cases("signature"), ids=lambda c: c["name"])
def test_golden_signature_device(case, gpu):
    data, bs = dec(case["data"]), case["block_size"]
    w, s = _dev_sig(gpu, data, bs)
    assert [[e[3], e[4]] for e in case["expect"]] == [[a, b] for a, b in zip(w, s)]


@pytest.mark.parametrize("case", load_cases("signature"), ids=lambda c: c["name"])
def test_golden_signature_path_api(case, gpu, tmp_path):
    import sy_amd.delta as d

    p = tmp_path / "f"
    p.write_bytes(dec(case["data"]))
    got = [[c.index, c.offset, c.size, c.weak, c.strong] for c in d.compute_checksums(p, case["block_size"])]
    assert got == case["expect"]


BLOCK_SIZES = [1, 3, 16, 64, 100, 240, 241, 255, 256, 320, 512, 1000, 1024, 1536, 4096, 5000, 8192, 10000,
               65536, 131072]


@pytest.mark.parametrize("bs", BLOCK_SIZES)
def test_signature_sizes_vs_oracle(bs, gpu, oracle_c):
    rng = random.Random(bs)
    for n in sorted({0, 1, bs - 1, bs, bs + 1, 3 * bs + 17, 5 * bs, min(1 << 20, 40 * bs + 7)}):
        if n < 0:
            continue
        data = rng.randbytes(n)
        w, s = _dev_sig(gpu, data, bs)
        ew, es, _ = oracle_c.compute_checksums(data, bs)
        assert w == ew.astype(np.uint64).tolist() and s == es.tolist(), (bs, n)


@pytest.mark.parametrize("offset", [1, 3, 5, 8, 13])
def test_signature_unaligned_buffer(offset, gpu, oracle_c):
    data = random.Random(offset).randbytes(4096 * 5 + 77)
    for bs in (512, 4096, 1000):
        w, s = _dev_sig(gpu, data, bs, offset=offset)
        ew, es, _ = oracle_c.compute_checksums(data, bs)
        assert w == ew.astype(np.uint64).tolist() and s == es.tolist()


@pytest.mark.parametrize("fill", [0x00, 0xFF, 0xAB])
def test_signature_constant_data(fill, gpu, oracle_c):
    data = bytes([fill]) * (8192 * 3 + 100)
    for bs in (4096, 8192, 1000, 17):
        w, s = _dev_sig(gpu, data, bs)
        ew, es, _ = oracle_c.compute_checksums(data, bs)
        assert w == ew.astype(np.uint64).tolist() and s == es.tolist()


def test_signature_64mib_vs_oracle(gpu, oracle_c):
    import torch

    from oracle.oracle import synth_bytes

    n = 64 << 20
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(buf, 0x5E1D0002)
    host = buf.cpu().numpy()
    assert np.array_equal(host[:4096], synth_bytes(4096, 0x5E1D0002))  # device generator == numpy generator
    for bs in (4096, 8192):
        w, s = gpu.signature(buf, bs)
        ew, es, _ = oracle_c.compute_checksums(host, bs, threads=os.cpu_count() or 8)
        assert np.array_equal(w.cpu().numpy().view(np.uint32), ew)
        assert np.array_equal(s.cpu().numpy().view(np.uint64), es)


def test_signature_4gib_sampled(gpu, oracle_c):
    """BASELINE config 2 size: a seeded sample of 2048 blocks is checked against the
    oracle, and the full weak/strong arrays against a second device run (idempotence)."""
    import torch

    n = 4 << 30
    bs = 4096
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(buf, 0x5E1D0002)
    w, s = gpu.signature(buf, bs)
    w2, s2 = gpu.signature(buf, bs)
    assert torch.equal(w, w2) and torch.equal(s, s2)
    rng = np.random.default_rng(3)
    idx = np.unique(rng.integers(0, n // bs, 2048))
    wc = w.cpu().numpy().view(np.uint32)
    sc = s.cpu().numpy().view(np.uint64)
    for i in idx[:2048]:
        blk = buf[i * bs:(i + 1) * bs].cpu().numpy()
        assert oracle_c.adler32(blk) == int(wc[i]) and oracle_c.xxh3(blk) == int(sc[i])
    del buf
    torch.cuda.empty_cache()


@pytest.mark.parametrize("nfiles,align", [(40, 16), (40, 1), (3000, 16)])
def test_signature_batch_matches_per_file(nfiles, align, gpu, oracle_c):
    """Row kernel (bs % 64 == 0, 16-byte aligned files: k_sig_fast_batch + k_sig_list
    for partial blocks), the generic wave kernel otherwise; runs of empty and short
    files between long ones; 3000 files exercise the 64-way file search."""
    import torch

    rng = random.Random(11 + nfiles + align)
    sizes = [0, 0, 0, 1, 100, 255, 4095, 4096, 4097, 8192, 20000, 1 << 17]
    files = [rng.randbytes(rng.choice(sizes if nfiles < 100 else sizes[:9])) for _ in range(nfiles)]
    offs, pos = [], 0
    for f in files:
        offs.append(pos)
        pos += (len(f) + align - 1) // align * align
    packed = bytearray(pos + 16)
    for o, f in zip(offs, files):
        packed[o:o + len(f)] = f
    buf = torch.frombuffer(packed, dtype=torch.uint8).cuda()
    for bs in (4096, 1000, 256, 8192):
        w, s = gpu.signature_batch(buf, offs, [len(f) for f in files], bs)
        w = w.cpu().numpy().view(np.uint32).tolist()
        s = s.cpu().numpy().view(np.uint64).tolist()
        k = 0
        for f in files:
            ew, es, _ = oracle_c.compute_checksums(f, bs)
            m = len(ew)
            assert w[k:k + m] == ew.tolist() and s[k:k + m] == es.tolist(), (bs, k)
            k += m
        assert k == len(w)
