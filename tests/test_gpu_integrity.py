"""Whole-file XXH3-64 on the device (k_xxh_pieces + k_xxh_chain) against the oracle's
hash_file (integrity/xxhash3.rs:17-33): every XXH3 length class, block/stripe edges,
unaligned file starts, batches whose chains are ragged within a wave, and one 1 GiB
file (a 1 Mi-step scramble chain)."""
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 3, 4, 8, 9, 16, 17, 100, 128, 129, 200, 240, 241, 255, 256, 1023, 1024, 1025, 1087, 1088, 1089,
         1100, 2047, 2048, 2049, 4096, 33 * 1024 + 5, 64 * 1024, 65 * 1024 + 63, (1 << 20) + 1, (3 << 20) + 777]


def _dev(b: bytes, shift: int = 0):
    import torch

    t = torch.zeros(len(b) + shift + 64, dtype=torch.uint8, device="cuda")
    if b:
        t[shift:shift + len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()
    return t[shift:shift + len(b)]


@pytest.mark.parametrize("shift", [0, 1, 5, 16])
@pytest.mark.parametrize("n", SIZES)
def test_single_file(n, shift, gpu):
    data = random.Random(n * 7 + shift).randbytes(n)
    assert gpu.xxh3(_dev(data, shift)) == O.py_hash_file(data)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_batch_ragged(seed, gpu):
    import torch

    rng = random.Random(seed)
    lens = [rng.choice([0, 5, 17, 200, 241, 1500, 70000, 130 * 1024 + 3, 300000, 1 << 20]) + rng.randrange(0, 64)
            for _ in range(37)]
    offs, pos = [], 0
    for ln in lens:
        pos += rng.randrange(0, 19)  # arbitrary (unaligned) file starts
        offs.append(pos)
        pos += ln
    blob = rng.randbytes(pos + 64)
    buf = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    got = gpu.xxh3_batch(buf, offs, lens)
    exp = [O.py_hash_file(blob[o:o + ln]) for o, ln in zip(offs, lens)]
    assert [int(x) for x in got] == exp


def test_batch_rejects_out_of_range(gpu):
    import torch

    buf = torch.zeros(1000, dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        gpu.xxh3_batch(buf, [990], [20])

    from sy_amd._lib import lib

    offs = np.array([990], dtype=np.uint64)
    lens = np.array([20], dtype=np.uint64)
    out = np.zeros(1, dtype=np.uint64)
    rc = lib.sydelta_xxh3_batch_device(0, buf.data_ptr(), 1000, offs.ctypes.data, lens.ctypes.data, 1, None,
                                       out.ctypes.data)
    assert rc != 0 and b"outside" in lib.sydelta_last_error()


def test_one_gib(gpu):
    import torch

    n = (1 << 30) + 12345
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(buf, seed=21)
    host = buf.cpu().numpy().tobytes()
    assert gpu.xxh3(buf) == O.py_xxh3(host)
