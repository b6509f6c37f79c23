"""Delta JSON parsed on the device (K7d, sydelta_delta_from_json_device): the receiver's
serde_json::from_str::<Delta> (sy-remote.rs:175) for the compact text the sender writes.

* The text json.dumps writes for mixed, literal-heavy and copy-only deltas (empty Data
  ops, every byte value, multi-chunk literal runs) parses to the host parser's ops and
  literal bytes.
* The receiver's path end to end on the device: the match of a source against a basis
  (K1-K5), its JSON written on the device (K7), parsed back on the device (K7d), and
  applied on the device (K6) rebuilds the source.
* Spellings outside the compact form are refused with their byte.

Marked late (green on hardware since round 3). The CPU suite also runs the
same chunk bodies on the emulated device and under ASan/UBSan
(tests/csrc/emulated_checks.py, kernel_bodies_fuzz.cpp)."""
import ctypes
import json
import random

import numpy as np
import pytest

from sy_amd import wire

pytestmark = [pytest.mark.gpu, pytest.mark.late, pytest.mark.firstrun]


def _compact(ops, ss, bs) -> bytes:
    return json.dumps({"ops": [{"Copy": {"offset": o[1], "size": o[2]}} if o[0] == "C" else {"Data": list(o[1])}
                               for o in ops], "source_size": ss, "block_size": bs}, separators=(",", ":")).encode()


def _cases():
    rng = random.Random(31)
    yield "empty", [], 0, 4096
    yield "bytes", [("D", bytes(range(256)) * 40), ("D", b""), ("C", 2**64 - 1, 0)], 10240, 4096
    ops = []
    for _ in range(3000):
        if rng.random() < 0.5:
            ops.append(("C", rng.randrange(1 << 40), 4096))
        else:
            ops.append(("D", rng.randbytes(rng.choice([0, 1, 63, 64, 65, 700, 20000]))))
    yield "mixed", ops, 123456789, 4096
    yield "copies", [("C", 8192 * k, 8192) for k in range(20000)], 20000 * 8192, 8192


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_delta_json_parse_on_device(case, gpu):
    import torch

    name, ops, ss, bs = case
    text = _compact(ops, ss, bs)
    d = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
    dops, lit, dss, dbs = wire.delta_from_json_device(d)
    lit_h = lit.cpu().numpy().tobytes()
    got = [("C", a, b) if k == 0 else ("D", lit_h[a:a + b]) for k, a, b in dops]
    assert (got, dss, dbs) == (ops, ss, bs)
    assert wire.delta_from_json(text) == (ops, ss, bs)


def test_receiver_path_on_device(gpu):
    """match -> JSON (device) -> parse (device) -> apply (device) == source."""
    import torch

    from sy_amd import _lib
    from sy_amd._lib import check, lib

    n, bs = 32 << 20, 4096
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(basis, 0x5E1D0720)
    src = basis.clone()
    idx = torch.from_numpy(np.random.default_rng(3).integers(0, n, 3000).astype(np.int64)).cuda()
    src[idx] = src[idx] ^ 0x5A
    w, s = gpu.signature(basis, bs)
    ix = gpu.Index(w, s, bs, bs)
    delta = gpu.match(ix, src)
    ix.close()
    text = wire.delta_to_json_device(delta.kind, delta.a, delta.b, n, bs, src)
    lit_len = ctypes.c_uint64()
    check(lib.sydelta_delta_from_json_device(text.data_ptr(), text.numel(), None, 0, ctypes.byref(lit_len), None, None))
    lit = torch.empty(max(1, lit_len.value), dtype=torch.uint8, device="cuda")
    h = ctypes.c_void_p()
    check(lib.sydelta_delta_from_json_device(text.data_ptr(), text.numel(), lit.data_ptr(), lit.numel(),
                                             ctypes.byref(lit_len), ctypes.byref(h), None))
    try:
        assert lib.sydelta_delta_num_ops(h) == len(delta.kind)
        out = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
        st = _lib.DeltaStatsC()
        check(lib.sydelta_apply_delta_device(0, basis.data_ptr(), n, h, lit.data_ptr(), lit.numel(), out.data_ptr(),
                                             out.numel(), None, ctypes.byref(st)))
        torch.cuda.synchronize()
    finally:
        lib.sydelta_delta_free(h)
    assert bool((out[:n] == src).all())


def test_delta_json_refused_spellings(gpu):
    import torch

    from sy_amd._lib import SyDeltaError

    good = _compact([("C", 4096, 4096), ("D", b"\x01\xff"), ("D", b"")], 8192, 4096)
    for bad in (good.replace(b",", b", ", 1), good[:-1], good.replace(b"[1,255]", b"[01,255]"),
                good.replace(b"[1,255]", b"[1,256]"), good.replace(b'"Copy"', b'"copy"'),
                b'{"ops":[xyz},{"Data":[5]}],"source_size":1,"block_size":1}'):
        with pytest.raises(SyDeltaError, match="compact form at byte"):
            wire.delta_from_json_device(torch.frombuffer(bytearray(bad), dtype=torch.uint8).cuda())
