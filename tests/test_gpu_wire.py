"""Device Delta JSON writer (K7) against the host writer (itself checked against
json.dumps in test_wire.py): bit-identical text for copy-heavy, literal-heavy
(multi-chunk Data runs) and mixed deltas, including empty Data ops."""
import random

import numpy as np
import pytest

from sy_amd import wire

pytestmark = pytest.mark.gpu


def _cases():
    rng = random.Random(9)
    src = rng.randbytes(3 << 20)
    yield "one-literal", [1], [0], [len(src)], src
    yield "empty", [], [], [], src
    yield "empty-data", [1, 0, 1], [0, 4096, 5], [0, 4096, 0], src
    kind, a, b = [], [], []
    pos = 0
    while pos < len(src) - 20000:
        if rng.random() < 0.5:
            kind.append(0); a.append(rng.randrange(1 << 40)); b.append(rng.choice([4096, 8192, 17]))
        else:
            n = rng.choice([1, 2, 99, 4095, 4096, 4097, 16383, 16384, 16385, 40000])
            kind.append(1); a.append(pos); b.append(n)
            pos += n
    yield "mixed", kind, a, b, src
    yield "copies", [0] * 5000, [i * 8192 for i in range(5000)], [8192] * 5000, src


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_device_json_equals_host(case, gpu):
    import torch

    name, kind, a, b, src = case
    host = wire.delta_to_json(kind, a, b, len(src), 4096, src)
    d = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
    dev = wire.delta_to_json_device(kind, a, b, len(src), 4096, d)
    torch.cuda.synchronize()
    got = bytes(dev.cpu().numpy())
    assert len(got) == len(host)
    assert got == host


def test_device_json_text_past_4gib(gpu):
    """A 1.25 GiB literal run: ~3.75 GiB of Data text plus a second run pushes the text
    offsets past 2^32 (a 32-bit scan would wrap)."""
    import torch

    L = 5 << 28  # 1.25 GiB
    lit = torch.full((L + 16,), 200, dtype=torch.uint8, device="cuda")  # "200," per byte
    lit[L - 1] = 7
    kind, a, b = [1, 0, 1], [0, 12345, L - 5], [L, 4096, 5]
    text = wire.delta_to_json_device(kind, a, b, L + 4096, 4096, lit[:L])
    torch.cuda.synchronize()
    body0 = 9 + 4 * (L - 1) + 1 + 2              # {"Data":[200,...,200,7]}
    copy = 1 + len('{"Copy":{"offset":12345,"size":4096}}')
    tail_data = 1 + len('{"Data":[200,200,200,200,7]}')
    tail = len('],"source_size":%d,"block_size":4096}' % (L + 4096))
    assert text.numel() == 8 + body0 + copy + tail_data + tail
    assert text.numel() > (1 << 32)
    head = bytes(text[:24].cpu().numpy())
    assert head == b'{"ops":[{"Data":[200,200'
    end = bytes(text[-(copy + tail_data + tail + 7):].cpu().numpy())
    assert end == (b'200,7]},{"Copy":{"offset":12345,"size":4096}},{"Data":[200,200,200,200,7]}'
                   + b'],"source_size":%d,"block_size":4096}' % (L + 4096))
