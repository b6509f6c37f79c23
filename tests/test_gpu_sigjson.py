"""Device signature JSON writer (K7s, sydelta_checksums_to_json_device) and parser (K7p,
sydelta_checksums_from_json_device). The writer is checked against an
independent writer: json.dumps, with serde's compact separators and checksum.rs:9-21's
field order, of the C oracle's signature of the same bytes. This is the text
`sy-remote checksums` prints (sy-remote.rs:146-147) and ssh.rs:967-973 parses. The
cases cover block sizes with a partial and a full last block, and tile edges (255, 256
and 257 entries). The destination views start at every alignment, with guard bytes
checked around them. A C2-sized signature (4 GiB basis, 1 Mi entries) is parsed back
with json.loads and compared field by field. The parser is checked on json.dumps's text
of the oracle's signature (against the oracle and the host parser), on spellings outside
the compact form (refused), and on the writer's C2 text (round trip on the device).

Marked late (green on hardware since round 3). The CPU suite also runs the same per-thread bodies on the emulated device and under
ASan/UBSan (tests/csrc/emulated_checks.py, kernel_bodies_fuzz.cpp)."""
import json

import numpy as np
import pytest

from sy_amd import wire

pytestmark = [pytest.mark.gpu, pytest.mark.late]


def _dumps(w, s, z, bs) -> bytes:
    return json.dumps([{"index": i, "offset": i * bs, "size": int(z[i]), "weak": int(w[i]), "strong": int(s[i])}
                       for i in range(len(w))], separators=(",", ":")).encode()


@pytest.mark.parametrize("bs,length", [(4096, 4096 * 255), (4096, 4096 * 256), (4096, 4096 * 257 - 5),
                                       (8192, (64 << 20) + 77), (1007, 3 << 20), (131072, (5 << 20) + 1),
                                       (64, 1)])
def test_signature_json_equals_json_dumps(bs, length, gpu, oracle_c):
    import torch

    from oracle import oracle as O

    host = O.synth_bytes(length, 0x5E1D0700 + bs)
    buf = torch.from_numpy(host).cuda()
    w, s = gpu.signature(buf, bs)
    ew, es, ez = oracle_c.compute_checksums(host, bs)
    assert np.array_equal(w.cpu().numpy().view(np.uint32), ew)
    last = length - (len(ew) - 1) * bs
    ref = _dumps(ew, es, ez, bs)
    text = wire.checksums_to_json_device(w, s, bs, last)
    torch.cuda.synchronize()
    assert text.cpu().numpy().tobytes() == ref
    # every destination alignment, guard bytes around the text untouched
    from sy_amd._lib import check, lib
    import ctypes

    got = ctypes.c_uint64()
    for shift in (1, 3, 8, 15):
        out = torch.full((len(ref) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
        check(lib.sydelta_checksums_to_json_device(w.data_ptr(), s.data_ptr(), w.numel(), bs, last,
                                                   out.data_ptr() + 16 + shift, len(ref), ctypes.byref(got), None))
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        assert got.value == len(ref)
        assert o[16 + shift:16 + shift + len(ref)].tobytes() == ref, shift
        assert (o[:16 + shift] == 0xEE).all() and (o[16 + shift + len(ref):] == 0xEE).all(), shift


def test_signature_json_empty(gpu):
    import torch

    w = torch.empty(0, dtype=torch.int32, device="cuda")
    s = torch.empty(0, dtype=torch.int64, device="cuda")
    assert wire.checksums_to_json_device(w, s, 4096, 0).cpu().numpy().tobytes() == b"[]"


@pytest.mark.slow
def test_signature_json_c2_size(gpu):
    """C2's signature (4 GiB basis, bs 4096, 1 Mi entries): the device text, parsed by
    json.loads, holds the device signature's values with index/offset/size implied."""
    import torch

    n, bs = 4 << 30, 4096
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(basis, 0x5E1D0002)
    w, s = gpu.signature(basis, bs)
    del basis
    text = wire.checksums_to_json_device(w, s, bs, bs)
    torch.cuda.synchronize()
    sigs = json.loads(text.cpu().numpy().tobytes())
    hw = w.cpu().numpy().view(np.uint32)
    hs = s.cpu().numpy().view(np.uint64)
    assert len(sigs) == hw.size == 1 << 20
    assert [e["weak"] for e in sigs] == hw.tolist()
    assert [e["strong"] for e in sigs] == hs.tolist()
    assert all(e["index"] == i and e["offset"] == i * bs and e["size"] == bs for i, e in enumerate(sigs))
    assert list(sigs[0]) == ["index", "offset", "size", "weak", "strong"]


@pytest.mark.parametrize("bs,length", [(4096, 4096 * 257 - 5), (1007, 3 << 20), (64, 1)])
def test_signature_json_parse_on_device(bs, length, gpu, oracle_c):
    """K7p: the compact text (as json.dumps writes it) parsed on the device gives the
    oracle's signature; the host parser agrees; a spelling outside the compact form is
    refused with its position."""
    import torch

    from oracle import oracle as O
    from sy_amd._lib import SyDeltaError

    host = O.synth_bytes(length, 0x5E1D0710 + bs)
    ew, es, ez = oracle_c.compute_checksums(host, bs)
    ref = _dumps(ew, es, ez, bs)
    d = torch.frombuffer(bytearray(ref), dtype=torch.uint8).cuda()
    recs, n = wire.checksums_from_json_device(d)
    got = recs.cpu().numpy().view(wire._SIG_DTYPE)
    assert n == len(ew)
    assert np.array_equal(got["weak"], ew) and np.array_equal(got["strong"], es)
    assert np.array_equal(got["size"], ez)
    assert np.array_equal(got["offset"], np.arange(n, dtype=np.uint64) * np.uint64(bs))
    assert np.array_equal(got, wire.checksums_from_json(ref))
    for bad in (ref.replace(b",", b", ", 1), ref[:-1], ref.replace(b'"weak"', b'"Weak"', 1)):
        with pytest.raises(SyDeltaError, match="compact form at byte"):
            wire.checksums_from_json_device(torch.frombuffer(bytearray(bad), dtype=torch.uint8).cuda())


@pytest.mark.slow
def test_signature_json_round_trip_on_device_c2(gpu):
    """C2's signature written on the device (K7s) and parsed back on the device (K7p):
    every entry equals the signature, with index/offset/size as implied."""
    import torch

    n, bs = 4 << 30, 4096
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(basis, 0x5E1D0002)
    w, s = gpu.signature(basis, bs)
    del basis
    text = wire.checksums_to_json_device(w, s, bs, bs)
    recs, m = wire.checksums_from_json_device(text)
    assert m == w.numel() == 1 << 20
    r = recs.view(torch.int64).view(-1, 5)  # index, offset, size, weak | reserved << 32, strong
    idx = torch.arange(m, device="cuda", dtype=torch.int64)
    assert bool((r[:, 0] == idx).all()) and bool((r[:, 1] == idx * bs).all()) and bool((r[:, 2] == bs).all())
    assert bool(((r[:, 3] & 0xFFFFFFFF) == (w.to(torch.int64) & 0xFFFFFFFF)).all())
    assert bool((r[:, 4] == s.view(torch.int64)).all())
