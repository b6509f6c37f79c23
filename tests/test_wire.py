"""Wire formats on the host: libsydelta's serde_json text of
Vec<BlockChecksum> and Delta against Python's json.dumps with serde's compact
separators and the field order of checksum.rs:10-21 / generator.rs:10-25 (parity
pinned by the struct declarations, not by a reference fixture: the reference's tests
never print these types), and the parsers against the writers."""
import json
import random

import numpy as np
import pytest

from oracle import oracle as O
from sy_amd import wire


def _sig_json(basis: bytes, bs: int) -> str:
    sigs = O.py_compute_checksums(basis, bs)
    return json.dumps([{"index": s.index, "offset": s.offset, "size": s.size, "weak": s.weak, "strong": s.strong}
                       for s in sigs], separators=(",", ":")), sigs


@pytest.mark.parametrize("n,bs", [(0, 16), (51, 16), (5000, 64), (100000, 4096)])
def test_checksums_json_matches_serde_layout(n, bs):
    data = O.synth_bytes(n, 77).tobytes()
    expect, sigs = _sig_json(data, bs)
    arr = wire.sig_array([s.index for s in sigs], [s.offset for s in sigs], [s.size for s in sigs],
                         [s.weak for s in sigs], [s.strong for s in sigs])
    text = wire.checksums_to_json(arr)
    assert text.decode() == expect
    back = wire.checksums_from_json(text)
    assert np.array_equal(back, arr)


def test_checksums_json_parser_accepts_whitespace_and_field_order():
    text = b' [ { "strong" : 18446744073709551615 , "weak":1, "size":3,"offset":2,"index":0 , "extra": [1, {"a": "}"}] } ] '
    a = wire.checksums_from_json(text)
    assert len(a) == 1 and int(a["strong"][0]) == 2**64 - 1 and int(a["weak"][0]) == 1 and int(a["offset"][0]) == 2


@pytest.mark.parametrize("bad", [b"", b"[", b"[{}]", b'[{"index":0,"offset":0,"size":1,"weak":4294967296,"strong":0}]',
                                 b'[{"index":-1,"offset":0,"size":1,"weak":1,"strong":0}]', b"[] x",
                                 # serde_json: "invalid number" (no leading zeros)
                                 b'[{"index":0,"offset":0,"size":01,"weak":1,"strong":0}]',
                                 b'[{"index":00,"offset":0,"size":1,"weak":1,"strong":0}]'])
def test_checksums_json_rejects(bad):
    import sy_amd._lib as L

    with pytest.raises(L.SyDeltaError):
        wire.checksums_from_json(bad)


def _delta_json(ops, source_size, bs):
    out = []
    for op in ops:
        if op[0] == "C":
            out.append({"Copy": {"offset": op[1], "size": op[2]}})
        else:
            out.append({"Data": list(op[1])})
    return json.dumps({"ops": out, "source_size": source_size, "block_size": bs}, separators=(",", ":"))


def test_delta_json_round_trip_random():
    rng = random.Random(5)
    for it in range(60):
        bs = rng.choice([4, 64, 4096])
        basis = rng.randbytes(rng.randint(0, 20 * bs))
        src = bytearray(basis)
        for _ in range(rng.randint(0, 5)):
            p = rng.randint(0, len(src))
            src[p:p] = rng.randbytes(rng.randint(1, 2 * bs))
        src = bytes(src)
        ops = O.py_generate_delta(src, O.py_compute_checksums(basis, bs), bs)
        # device-style table: Data ops index the source (generator.rs Data(Vec<u8>) = src[off, +len))
        kind, a, b = [], [], []
        expect_ops = []
        for k, x, y in ops:
            kind.append(0 if k == "C" else 1)
            a.append(x)
            b.append(y)
            expect_ops.append(("C", x, y) if k == "C" else ("D", src[x:x + y]))
        text = wire.delta_to_json(kind, a, b, len(src), bs, src)
        assert text.decode() == _delta_json(expect_ops, len(src), bs)
        back, ss, bb = wire.delta_from_json(text)
        assert back == expect_ops and ss == len(src) and bb == bs


def test_delta_json_edge_cases():
    for kind, a, b, lit in [([], [], [], b""), ([1], [0], [0], b""), ([0, 0], [0, 8], [8, 3], b""),
                            ([1, 0, 1], [0, 99, 3], [3, 4, 2], bytes([0, 9, 255, 10, 100]))]:
        text = wire.delta_to_json(kind, a, b, 17, 8, lit)
        exp = []
        for k, x, y in zip(kind, a, b):
            exp.append({"Copy": {"offset": x, "size": y}} if k == 0 else {"Data": list(lit[x:x + y])})
        assert text.decode() == json.dumps({"ops": exp, "source_size": 17, "block_size": 8}, separators=(",", ":"))


_SIG = '"index":0,"offset":0,"size":1,"weak":1,"strong":0'


@pytest.mark.parametrize("bad", [
    '[{' + _SIG + ',"index":0}]',                   # duplicate field (serde: "duplicate field `index`")
    '[{' + _SIG + ',"weak":2}]',
    '[{' + _SIG + ',"x":tru}]',                     # unknown key with an invalid value
    '[{' + _SIG + ',"x":01}]',
    '[{' + _SIG + ',"x":1.}]',
    '[{' + _SIG + ',"x":"a\\q"}]',
    '[{' + _SIG + ',"x":[1,]}]',
    '[{' + _SIG + ',"x":{"a"}}]',
    '[{' + _SIG + ',"x":' + '[' * 200 + ']' * 200 + '}]',  # past serde_json's recursion limit
    '[{' + _SIG + ',"x":"\x01"}]',
])
def test_checksums_json_rejects_malformed(bad):
    import sy_amd._lib as L

    with pytest.raises(L.SyDeltaError):
        wire.checksums_from_json(bad.encode())


@pytest.mark.parametrize("good", [
    '[{' + _SIG + ',"x":-1.5e+3}]', '[{' + _SIG + ',"x":null,"y":true,"z":[false,{"k":"v\\u00e9"}]}]',
    '[{' + _SIG + ',"x":0,"x":1}]',  # repeated unknown keys are ignored, as serde does
])
def test_checksums_json_accepts_valid_unknown_values(good):
    assert len(wire.checksums_from_json(good.encode())) == 1


@pytest.mark.parametrize("bad", [
    '{"ops":[],"ops":[],"source_size":0,"block_size":4}',
    '{"ops":[],"source_size":0,"source_size":1,"block_size":4}',
    '{"ops":[{"Copy":{"offset":0,"size":1,"size":2}}],"source_size":1,"block_size":4}',
    '{"ops":[{"Copy":{"offset":0,"offset":0,"size":1}}],"source_size":1,"block_size":4}',
    '{"ops":[],"source_size":0,"block_size":4,"x":[}',
    '{"ops":[{"Data":[256]}],"source_size":1,"block_size":4}',
    # serde_json: "invalid number" (no leading zeros)
    '{"ops":[{"Data":[01]}],"source_size":1,"block_size":4}',
    '{"ops":[{"Copy":{"offset":00,"size":1}}],"source_size":1,"block_size":4}',
    '{"ops":[],"source_size":01,"block_size":4}',
])
def test_delta_json_rejects_malformed(bad):
    import sy_amd._lib as L

    with pytest.raises(L.SyDeltaError):
        wire.delta_from_json(bad.encode())
