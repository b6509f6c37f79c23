"""GPU parity for the device zstd encoder (k_zstd_block + k_zstd_frame, sydelta_zstd.hpp):
the frame of every text must equal the sequential host form's byte for byte
(tests/csrc/zstd_ref.cpp, the same code builder and header writers) and the system
libzstd must decode it to the text.  The texts: Delta JSON written on the device
(copy-heavy ones take literals + sequences blocks), block-size edges, RLE / Raw blocks,
skewed symbol counts (codes folded to 11 bits), runs, batches of 1 and 3 blocks, and a
192 MiB text (three batches of 512 blocks, and one batch of the default 4096).

Marked late (runs after the kernel parity tests); green on hardware since round 3."""
import os
import random

import numpy as np
import pytest

import test_zstd as Z

pytestmark = [pytest.mark.gpu, pytest.mark.late, pytest.mark.firstrun]


def _device(data: bytes):
    import torch

    t = torch.zeros(len(data) + 16, dtype=torch.uint8, device="cuda")
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    return t[:len(data)]


@pytest.mark.parametrize("case", list(Z._cases()), ids=lambda c: c[0])
def test_device_frame_equals_host(case, gpu):
    from sy_amd import wire

    name, data = case
    frame = bytes(wire.zstd_compress_device(_device(data)).cpu().numpy())
    assert frame == Z.ref_compress(data), name
    assert Z.zstd_decode(frame, len(data)) == data


@pytest.mark.parametrize("batch", ["1", "3"])
def test_device_frame_batches(batch, gpu):
    from sy_amd import wire

    old = os.environ.get("SYDELTA_ZSTD_BATCH")
    os.environ["SYDELTA_ZSTD_BATCH"] = batch
    try:
        data = Z.delta_json(random.Random(7), 40000, 0.4)
        frame = bytes(wire.zstd_compress_device(_device(data)).cpu().numpy())
    finally:
        if old is None:
            os.environ.pop("SYDELTA_ZSTD_BATCH", None)
        else:
            os.environ["SYDELTA_ZSTD_BATCH"] = old
    assert frame == Z.ref_compress(data)
    assert Z.zstd_decode(frame, len(data)) == data


def test_device_json_then_zstd(gpu):
    """The sender's path: Delta JSON written on the device (K7), then compressed (K7z)."""
    import torch

    from sy_amd import wire

    rng = random.Random(11)
    src = rng.randbytes(4 << 20)
    kind, a, b, pos = [], [], [], 0
    while pos < len(src) - 70000:
        if rng.random() < 0.7:
            kind.append(0); a.append(rng.randrange(1 << 30) * 4096); b.append(4096)
        else:
            n = rng.randint(1, 60000)
            kind.append(1); a.append(pos); b.append(n)
            pos += n
    d = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
    text = wire.delta_to_json_device(kind, a, b, len(src), 4096, d)
    frame = bytes(wire.zstd_compress_device(text).cpu().numpy())
    host_text = wire.delta_to_json(kind, a, b, len(src), 4096, src)
    assert Z.zstd_decode(frame, len(host_text)) == host_text
    assert len(frame) < 0.5 * len(host_text)


@pytest.mark.parametrize("batch", ["512", None])
def test_device_frame_large(batch, gpu):
    """192 MiB of decimal-list text (3 batches of 512 blocks: first, middle and last batch
    placement; then one batch at the default size): the frame against the host form
    (compared on the device) and decoded by libzstd.  The host form encodes ~5 MiB/s on
    one core, so the size is kept to what checks the batching."""
    import torch

    from sy_amd import wire

    old = os.environ.get("SYDELTA_ZSTD_BATCH")
    if batch is None:
        os.environ.pop("SYDELTA_ZSTD_BATCH", None)
    else:
        os.environ["SYDELTA_ZSTD_BATCH"] = batch
    try:
        _large_frame(wire, torch)
    finally:
        if old is None:
            os.environ.pop("SYDELTA_ZSTD_BATCH", None)
        else:
            os.environ["SYDELTA_ZSTD_BATCH"] = old


_LARGE = {}


def _large_frame(wire, torch):
    L = 3 << 26
    if not _LARGE:  # the text and its host form, made once for both batch sizes
        rng = np.random.default_rng(5)
        period = (",".join(str(int(x)) for x in rng.integers(0, 256, 50000)) + ",").encode()
        reps = L // len(period) + 1
        per = torch.frombuffer(bytearray(period), dtype=torch.uint8).cuda()
        _LARGE["text"] = per.repeat(reps)[:L].contiguous()
        _LARGE["host"] = Z.ref_compress(bytes(_LARGE["text"].cpu().numpy()))
        assert Z.zstd_decode(_LARGE["host"], L) == bytes(_LARGE["text"].cpu().numpy())
    text, host = _LARGE["text"], _LARGE["host"]
    frame = wire.zstd_compress_device(text)
    assert frame.numel() == len(host)
    assert bool((frame == torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()).all())
