"""Device Delta JSON writer (K7) against the host writer and against an independent
writer -- Python's json.dumps with serde's compact separators and the field order of
generator.rs:10-25 (ssh.rs:1003 serde_json::to_string(&delta)): bit-identical text for
copy-heavy, literal-heavy (multi-chunk Data runs) and mixed deltas, including empty
Data ops, and for a text past 2^32 bytes."""
import json
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


def _dumps(kind, a, b, source_size, bs, src) -> bytes:
    """serde_json::to_string(&Delta) restated with json.dumps (generator.rs:10-25:
    DeltaOp::Copy{offset,size} / DeltaOp::Data(Vec<u8>), then source_size, block_size)."""
    ops = [{"Copy": {"offset": x, "size": y}} if k == 0 else {"Data": list(src[x:x + y])}
           for k, x, y in zip(kind, a, b)]
    return json.dumps({"ops": ops, "source_size": source_size, "block_size": bs}, separators=(",", ":")).encode()


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
    assert got == _dumps(kind, a, b, len(src), 4096, src)


def test_device_json_past_4gib_against_dumps(gpu):
    """A 1.25 GiB literal run of a 256-byte period (a permutation of 0..255), then a
    Copy and a short Data run: > 4 GiB of text.  json.dumps writes one period's text and
    the ops around the run; the device text is compared with them on the device, the
    run as a [periods x period-text] view."""
    import torch

    P, L = 256, 5 << 28
    perm = np.random.default_rng(17).permutation(P).astype(np.uint8)
    lit = torch.from_numpy(perm).cuda().repeat(L // P + 1)[:L + 16].contiguous()
    kind, a, b = [1, 0, 1], [0, 12345, 100], [L, 4096, 5]
    text = wire.delta_to_json_device(kind, a, b, L + 4096, 4096, lit[:L])
    torch.cuda.synchronize()
    period = json.dumps(perm.tolist(), separators=(",", ":"))[1:-1].encode() + b","  # "v0,v1,...,v255,"
    T = len(period)
    head = b'{"ops":[{"Data":['
    rest = json.dumps({"ops": [{"Data": []}, {"Copy": {"offset": 12345, "size": 4096}},
                               {"Data": perm[100:105].tolist()}], "source_size": L + 4096, "block_size": 4096},
                      separators=(",", ":")).encode()
    rest = rest[rest.index(b"]},"):]  # from the first (empty) Data op's "]"
    nrep = L // P
    assert text.numel() == len(head) + nrep * T - 1 + len(rest)
    assert text.numel() > (1 << 32)
    assert bytes(text[:len(head)].cpu().numpy()) == head
    body = text[len(head):len(head) + nrep * T].view(nrep, T)
    row = torch.frombuffer(bytearray(period), dtype=torch.uint8).cuda()
    assert bool((body[:-1] == row).all())
    assert bool((body[-1, :T - 1] == row[:T - 1]).all())
    assert bytes(text[len(head) + nrep * T - 1:].cpu().numpy()) == rest


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
