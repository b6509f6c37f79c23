"""TEST INFRASTRUCTURE: the library's host logic run on the CPU against the host
emulation of the device layer (tests/csrc/fake_device.cpp), checked against the C
oracle.  Run by tests/test_host_emulated.py as `python emulated_checks.py <repo> <lib>`;
loads sy_amd/_lib.py's bindings onto <lib> instead of libsydelta.so (the product
module is not modified and never loads this library).

Covers what the GPU tests cover for the host side: the streamed path API over many
chunks (compute_checksums, generate_delta_streaming, bs up to 128 KiB), the in-memory
generator, tiny and empty files, the probe + on-demand scan walk (SYDELTA_PROBE=1),
the split walk (SYDELTA_WALK_PAR_MIN=1), the path-level change ratio on ratio.rs's
cases, 10 threads calling the path API at once, the batched device-pointer path (80
files incl. empty and sub-block ones, threaded walks) and a file matched in 1/2/3/8
chained chunks, the device zstd and signature-JSON writers' host sides.
"""
import os
import subprocess
import sys
import tempfile
import types
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT, LIB = sys.argv[1], sys.argv[2]
sys.path.insert(0, ROOT)

# sy_amd._lib with LIB_PATH pointing at the emulation build (exec'd from the source)
import sy_amd  # noqa: E402

src = open(os.path.join(ROOT, "sy_amd", "_lib.py")).read()
anchor = 'LIB_PATH = os.path.join(HERE, "libsydelta.so")'
assert anchor in src
mod = types.ModuleType("sy_amd._lib")
mod.__file__ = os.path.join(ROOT, "sy_amd", "_lib.py")
exec(compile(src.replace(anchor, f"LIB_PATH = {LIB!r}"), mod.__file__, "exec"), mod.__dict__)
sys.modules["sy_amd._lib"] = mod
sy_amd._lib = mod

import sy_amd.delta as D  # noqa: E402
from oracle import oracle as O  # noqa: E402

C = O.C()


def tuples(delta):
    return [("C", op.offset, op.size) if isinstance(op, D.Copy) else ("D", len(op.data)) for op in delta.ops]


def expect(src_b, basis_b, bs):
    w, s, z = C.compute_checksums(basis_b, bs)
    return [("C", a, b) if k == "C" else ("D", b) for k, a, b in O.ops_from_arrays(*C.generate_delta(src_b, w, s, z, bs))]


def case(seed, n, bs):
    rng = np.random.default_rng(seed)
    basis = O.synth_bytes(n, 0x5E1D0300 + seed)
    s = basis.copy()
    for p in rng.integers(0, n, 25):
        s[p] ^= 0x33
    ins = int(rng.integers(n // 3, n // 2))
    s = np.concatenate([s[:ins], rng.integers(0, 256, 7, dtype=np.uint8), s[ins:]])
    k = int(rng.integers(0, max(1, n // bs - 1)))
    s = np.concatenate([s, basis[k * bs:(k + 1) * bs], basis[(n // bs) * bs:]])
    return basis, s


def check_pair(tmp, basis, s, bs, tag):
    pb, ps, po = os.path.join(tmp, "dest"), os.path.join(tmp, "src"), os.path.join(tmp, "out")
    basis.tofile(pb)
    s.tofile(ps)
    sigs = D.compute_checksums(pb, bs)
    w, st, z = C.compute_checksums(basis, bs)
    assert [x.weak for x in sigs] == w.tolist() and [x.strong for x in sigs] == st.tolist(), tag
    assert [x.size for x in sigs] == z.tolist(), tag
    exp = expect(s, basis, bs)
    d = D.generate_delta_streaming(ps, sigs, bs)
    assert tuples(d) == exp, (tag, "streaming")
    D.apply_delta(pb, d, po)
    assert open(po, "rb").read() == s.tobytes(), (tag, "apply")
    d2 = D.generate_delta(ps, sigs, bs)
    assert d2 == d, (tag, "in-memory")


PIECES_CHILD = """
import sys, tempfile
sys.path.insert(0, sys.argv[3])
import emulated_checks as E
n = 0
with tempfile.TemporaryDirectory() as tmp:
    for bs, size in [(4096, (3 << 20) + 1234), (1007, (2 << 20) + 99), (131072, (3 << 20) + 17)]:
        basis, s = E.case(bs % 89, size, bs)
        E.check_pair(tmp, basis, s, bs, ("pieces", bs))
        n += 1
print(n)
"""


def main():
    n_checks = 0
    with tempfile.TemporaryDirectory() as tmp:
        for chunk in (1 << 16, 1 << 20):
            os.environ["SYDELTA_STREAM_CHUNK"] = str(chunk)
            for bs, n in [(4096, (1 << 20) + 1234), (1007, (1 << 20) + 99), (64, (1 << 18) + 5),
                          (16384, (1 << 20) + 4321), (131072, (3 << 20) + 17), (512, 300000)]:
                for probe in ("0", "1", "auto"):
                    if probe == "auto":
                        os.environ.pop("SYDELTA_PROBE", None)
                    else:
                        os.environ["SYDELTA_PROBE"] = probe
                    basis, s = case(bs % 97, n, bs)
                    check_pair(tmp, basis, s, bs, (chunk, bs, n, probe))
                    n_checks += 1
        os.environ.pop("SYDELTA_PROBE", None)
        # chunks read in parallel pieces (the path API's reader splits a chunk over the
        # host pool; SYDELTA_READ_PIECE is read once per process, so a child runs them)
        r = subprocess.run([sys.executable, "-c", PIECES_CHILD, ROOT, LIB, os.path.dirname(os.path.abspath(__file__))], env=dict(os.environ, SYDELTA_READ_PIECE="65536",
                           SYDELTA_STREAM_CHUNK=str(1 << 20)), capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout + r.stderr
        n_checks += int(r.stdout.split()[-1])
        # tiny and empty files
        os.environ["SYDELTA_STREAM_CHUNK"] = "65536"
        for size in (0, 1, 63, 64, 65, 4095, 4096, 4097):
            b = O.synth_bytes(size, 5)
            check_pair(tmp, b, b.copy(), 64, ("tiny", size))
            n_checks += 1
        # the split walk on every source with hits (probe on: the aligned-run fast path)
        os.environ["SYDELTA_WALK_PAR_MIN"] = "1"
        for t in ("2", "3", "8"):
            os.environ["SYDELTA_WALK_THREADS"] = t
            os.environ["SYDELTA_PROBE"] = "1"
            basis, s = case(11, (2 << 20) + 77, 4096)
            check_pair(tmp, basis, s, 4096, ("split", t))
            n_checks += 1
        for k in ("SYDELTA_WALK_PAR_MIN", "SYDELTA_WALK_THREADS", "SYDELTA_PROBE"):
            os.environ.pop(k, None)
        # probe results split into 64 Ki-block pieces: 160 000 blocks, the miss run after
        # the insertion crosses piece boundaries
        os.environ["SYDELTA_STREAM_CHUNK"] = str(16 << 20)
        os.environ["SYDELTA_PROBE"] = "1"
        basis, s = case(31, 64 * 160000 + 5, 64)
        check_pair(tmp, basis, s, 64, ("pieces",))
        n_checks += 1
        os.environ.pop("SYDELTA_PROBE", None)
        # change ratio on paths: ratio.rs's cases against the oracle
        MiB = 1 << 20
        for name in ("same", "all", "partial", "threshold", "size"):
            a = bytearray(b"\x2a" * MiB)
            b = bytes(b"\x2a" * MiB)
            if name == "all":
                b = b"\x63" * MiB
            elif name == "partial":
                a[:256 * 1024] = b"\x63" * (256 * 1024)
            elif name == "threshold":
                a[:800 * 1024] = b"\x63" * (800 * 1024)
            elif name == "size":
                a = bytearray(b"\x2a" * (2 * MiB))
            ps, pd = os.path.join(tmp, "rs"), os.path.join(tmp, "rd")
            open(ps, "wb").write(bytes(a))
            open(pd, "wb").write(b)
            for sc, thr in ((None, None), (5, None), (1, 0.5), (0, None), (64, 0.9)):
                r = D.estimate_change_ratio(ps, pd, 64 * 1024, sc, thr)
                e = O.py_estimate_change_ratio(bytes(a), b, 64 * 1024, sc, thr)
                assert (r.change_ratio, r.blocks_sampled, r.blocks_changed, r.use_delta, r.threshold) == e, (name, sc)
                n_checks += 1
        # 10 threads through the path API at once
        os.environ["SYDELTA_STREAM_CHUNK"] = str(1 << 18)
        pairs = [case(200 + k, (1 << 20) + 977 * k, 4096) for k in range(10)]

        def one(k):
            d = os.path.join(tmp, f"t{k}")
            os.makedirs(d, exist_ok=True)
            check_pair(d, pairs[k][0], pairs[k][1], 4096, ("thread", k))
            return True

        with ThreadPoolExecutor(10) as ex:
            assert all(ex.map(one, range(10)))
        n_checks += 10
        n_checks += batch_and_chunk_checks()
        n_checks += error_checks(tmp)
        n_checks += device_walk_checks(tmp)
        n_checks += zstd_checks()
        n_checks += sigjson_checks()
    print(f"emulated host checks ok: {n_checks}")


def zstd_checks():
    """sydelta_zstd_compress_device's batching and frame assembly (the emulated blocks are
    sydelta_zstd.hpp's sequential form): frames equal to the test reference encoder's and
    decoded by the system libzstd, with batches of 1, 3 and 512 blocks, and the default
    batch halved on a device that refuses its scratch."""
    import ctypes
    import json
    import random

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_zstd as Z
    from sy_amd._lib import SYDELTA_E_OOM, check, lib

    if Z._libzstd() is None:
        return 0
    rng = random.Random(4)
    texts = [b"", b"x", b"ab" * 70000, Z.delta_json(rng, 30000, 0.3), bytes(rng.randrange(256) for _ in range(300000))]
    n = 0
    for batch in ("1", "3", "512"):
        os.environ["SYDELTA_ZSTD_BATCH"] = batch
        for t in texts:
            src = np.zeros(len(t) + 16, np.uint8)
            src[:len(t)] = np.frombuffer(t, np.uint8)
            cap = int(lib.sydelta_zstd_bound(len(t)))
            out = np.zeros(cap, np.uint8)
            got = ctypes.c_uint64()
            check(lib.sydelta_zstd_compress_device(0, ctypes.c_void_p(src.ctypes.data), len(t),
                                                   ctypes.c_void_p(out.ctypes.data), cap, ctypes.byref(got), None))
            frame = out[:got.value].tobytes()
            assert frame == Z.ref_compress(t), ("zstd", batch, len(t))
            assert Z.zstd_decode(frame, len(t)) == t
            n += 1
    os.environ.pop("SYDELTA_ZSTD_BATCH", None)
    # a device short of memory: the default batch's scratch is refused, the call halves the
    # batch until it fits (here 128 of the 201 blocks) and writes the same frame
    t = (Z.delta_json(rng, 30000, 0.3) * 5)[: 200 * 131072 + 777]
    src = np.zeros(len(t) + 16, np.uint8)
    src[:len(t)] = np.frombuffer(t, np.uint8)
    cap = int(lib.sydelta_zstd_bound(len(t)))
    out = np.zeros(cap, np.uint8)
    got = ctypes.c_uint64()
    os.environ["SYDELTA_EMU_POOL_CAP"] = str(200 << 20)  # < 201 blocks' scratch (~1.5 MiB each), > 128 blocks'
    try:
        check(lib.sydelta_zstd_compress_device(0, ctypes.c_void_p(src.ctypes.data), len(t),
                                               ctypes.c_void_p(out.ctypes.data), cap, ctypes.byref(got), None))
    finally:
        os.environ.pop("SYDELTA_EMU_POOL_CAP", None)
    frame = out[:got.value].tobytes()
    assert frame == Z.ref_compress(t), ("zstd", "oom fallback", len(t))
    assert Z.zstd_decode(frame, len(t)) == t
    # the cap is real: below 64 blocks' scratch the call reports the device as full
    os.environ["SYDELTA_EMU_POOL_CAP"] = str(50 << 20)
    try:
        rc = lib.sydelta_zstd_compress_device(0, ctypes.c_void_p(src.ctypes.data), len(t),
                                              ctypes.c_void_p(out.ctypes.data), cap, ctypes.byref(got), None)
    finally:
        os.environ.pop("SYDELTA_EMU_POOL_CAP", None)
    assert rc == SYDELTA_E_OOM, rc
    n += 2
    return n


def sigjson_checks():
    """sydelta_checksums_to_json_device (K7s; the emulated launches run sydelta_sigjson.hpp's
    per-thread bodies tile by tile): the text equals json.dumps of the same list of dicts
    with serde's separators and the host writer's, written at every destination alignment
    without touching a byte outside it; the length query, a too-small buffer (nothing
    written), the empty signature and the argument checks."""
    import ctypes
    import json

    from sy_amd import wire
    from sy_amd._lib import check, lib

    rng = np.random.default_rng(7)
    n_checks = 0
    cases = [(1, 4096, 1), (1, 4096, 4096), (255, 512, 100), (256, 4096, 4096), (257, 8192, 17),
             (1000, 131072, 65536), (3 * 256 + 5, 1 << 32, 1 << 32), (20000, 4096, 3000)]
    for n, bs, last in cases:
        for dist in ("uniform", "extremes"):
            if dist == "uniform":
                weak = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
                strong = rng.integers(0, 1 << 64, n, dtype=np.uint64)
            else:  # 0, 9, 10, max and every digit count
                wv = np.array([0, 9, 10, 99, 100, 65535, 0xFFFFFFFF], np.uint32)
                sv = np.array([0, 9, 10, 10**10, 10**19 - 1, 10**19, 0xFFFFFFFFFFFFFFFF], np.uint64)
                weak, strong = wv[rng.integers(0, wv.size, n)], sv[rng.integers(0, sv.size, n)]
            sizes = np.full(n, bs, np.uint64)
            sizes[-1] = last
            idx = np.arange(n, dtype=np.uint64)
            ref = json.dumps([{"index": int(i), "offset": int(i) * bs, "size": int(z), "weak": int(w), "strong": int(t)}
                              for i, z, w, t in zip(idx, sizes, weak, strong)], separators=(",", ":")).encode()
            assert wire.checksums_to_json(wire.sig_array(idx, idx * np.uint64(bs), sizes, weak, strong)) == ref
            got = ctypes.c_uint64()
            check(lib.sydelta_checksums_to_json_device(ctypes.c_void_p(weak.ctypes.data),
                                                       ctypes.c_void_p(strong.ctypes.data), n, bs, last, None, 0,
                                                       ctypes.byref(got), None))
            assert got.value == len(ref), (n, bs, dist, got.value, len(ref))
            for shift in (0, 1, 7, 15) if n < 5000 else (3,):
                buf = np.full(len(ref) + 64, 0xEE, np.uint8)
                # too small by one: nothing written
                check(lib.sydelta_checksums_to_json_device(ctypes.c_void_p(weak.ctypes.data),
                                                           ctypes.c_void_p(strong.ctypes.data), n, bs, last,
                                                           ctypes.c_void_p(buf.ctypes.data + 16 + shift),
                                                           len(ref) - 1, ctypes.byref(got), None))
                assert got.value == len(ref) and (buf == 0xEE).all()
                check(lib.sydelta_checksums_to_json_device(ctypes.c_void_p(weak.ctypes.data),
                                                           ctypes.c_void_p(strong.ctypes.data), n, bs, last,
                                                           ctypes.c_void_p(buf.ctypes.data + 16 + shift), len(ref),
                                                           ctypes.byref(got), None))
                o = 16 + shift
                assert buf[o:o + len(ref)].tobytes() == ref, (n, bs, dist, shift)
                assert (buf[:o] == 0xEE).all() and (buf[o + len(ref):] == 0xEE).all(), (n, bs, dist, shift)
                n_checks += 1
    buf = np.zeros(8, np.uint8)
    got = ctypes.c_uint64()
    check(lib.sydelta_checksums_to_json_device(None, None, 0, 4096, 0, ctypes.c_void_p(buf.ctypes.data), 8,
                                               ctypes.byref(got), None))
    assert got.value == 2 and buf[:2].tobytes() == b"[]"
    w1, s1 = np.zeros(4, np.uint32), np.zeros(4, np.uint64)
    for bs, last in ((0, 1), (4096, 0), (4096, 4097), ((1 << 32) + 1, 1)):
        rc = lib.sydelta_checksums_to_json_device(ctypes.c_void_p(w1.ctypes.data), ctypes.c_void_p(s1.ctypes.data), 4,
                                                  bs, last, None, 0, ctypes.byref(got), None)
        assert rc != 0, (bs, last)
    assert lib.sydelta_checksums_to_json_device(None, None, 4, 4096, 4096, None, 0, ctypes.byref(got), None) != 0
    return n_checks + 6 + sigparse_checks() + dparse_checks()


def dparse_checks():
    """sydelta_delta_from_json_device (K7d; the emulated launches run sydelta_dparse.hpp's
    chunk bodies): the compact Delta JSON of random deltas (copy-heavy, literal-heavy,
    empty Data ops, no ops, literal runs across many chunks) parses to the host parser's
    ops and literal bytes; the length query and a short literal buffer; and every
    non-compact or malformed spelling is refused while the host parser keeps its own
    verdict; random mutations are refused or re-serialize to themselves."""
    import ctypes
    import json
    import random

    from sy_amd import wire
    from sy_amd._lib import SyDeltaError, check, lib

    rng = random.Random(21)

    def dev_parse(text: bytes):
        buf = np.frombuffer(text, np.uint8).copy() if text else np.zeros(1, np.uint8)
        n = ctypes.c_uint64()
        if lib.sydelta_delta_from_json_device(ctypes.c_void_p(buf.ctypes.data), len(text), None, 0, ctypes.byref(n),
                                              None, None):
            return None
        lit = np.zeros(max(1, n.value), np.uint8)
        if n.value:
            short = ctypes.c_uint64()
            assert lib.sydelta_delta_from_json_device(ctypes.c_void_p(buf.ctypes.data), len(text),
                                                      ctypes.c_void_p(lit.ctypes.data), n.value - 1,
                                                      ctypes.byref(short), None, None) != 0
        h = ctypes.c_void_p()
        check(lib.sydelta_delta_from_json_device(ctypes.c_void_p(buf.ctypes.data), len(text),
                                                 ctypes.c_void_p(lit.ctypes.data), lit.size, ctypes.byref(n),
                                                 ctypes.byref(h), None))
        try:
            cnt = lib.sydelta_delta_num_ops(h)
            p = lib.sydelta_delta_ops(h)
            ops = []
            for i in range(cnt):
                if p[i].kind == 0:
                    ops.append(("C", int(p[i].a), int(p[i].b)))
                else:
                    ops.append(("D", lit[p[i].a:p[i].a + p[i].b].tobytes()))
            return ops, int(lib.sydelta_delta_source_size(h)), int(lib.sydelta_delta_block_size(h))
        finally:
            lib.sydelta_delta_free(h)

    def compact(ops, ss, bs):
        return json.dumps({"ops": [{"Copy": {"offset": o[1], "size": o[2]}} if o[0] == "C" else {"Data": list(o[1])}
                                   for o in ops], "source_size": ss, "block_size": bs}, separators=(",", ":")).encode()

    def expect(text):
        d = json.loads(text)
        ops = [("C", o["Copy"]["offset"], o["Copy"]["size"]) if "Copy" in o else ("D", bytes(o["Data"]))
               for o in d["ops"]]
        return ops, d["source_size"], d["block_size"]

    n_checks = 0
    cases = [([], 0, 4096), ([("D", b"")], 0, 1), ([("C", 0, 4096)], 4096, 4096),
             ([("D", bytes(range(256)) * 3)], 768, 4096), ([("D", b""), ("C", 2**64 - 1, 2**64 - 1), ("D", b"\x00")], 7, 9)]
    for it in range(12):
        ops = []
        for _ in range(rng.randint(1, 400)):
            if rng.random() < 0.6:
                ops.append(("C", rng.randrange(1 << 40), rng.choice([4096, 17, 0])))
            else:
                ops.append(("D", bytes(rng.randrange(256) for _ in range(rng.choice([0, 1, 2, 63, 64, 65, 300, 5000])))))
        cases.append((ops, rng.randrange(1 << 50), rng.choice([512, 4096, 131072])))
    for ops, ss, bs in cases:
        text = compact(ops, ss, bs)
        got = dev_parse(text)
        assert got == (ops, ss, bs), (len(ops), got if got is None else len(got[0]))
        assert wire.delta_from_json(text) == got  # the host parser reads the same delta
        n_checks += 1
    good = compact([("C", 4096, 4096), ("D", b"\x01\xff"), ("D", b"")], 8192, 4096)
    assert dev_parse(good) is not None
    bad = [b"", b"{}", b'{"ops":[]}', good[:-1], good + b" ", b" " + good, good.replace(b",", b", ", 1),
           good.replace(b'"Copy"', b'"copy"'), good.replace(b'"offset":4096,"size":4096', b'"size":4096,"offset":4096'),
           good.replace(b"[1,255]", b"[1,256]"), good.replace(b"[1,255]", b"[01,255]"), good.replace(b"[1,255]", b"[1,,255]"),
           good.replace(b"[1,255]", b"[1,255,]"), good.replace(b"[1,255]", b"[-1,255]"), good.replace(b"},{", b"}{", 1),
           good.replace(b'"source_size":8192', b'"source_size":08192'), good.replace(b'"block_size":4096}', b'"block_size":4096,"x":1}'),
           good.replace(b'{"Data":[]}', b'{"Data":[],"x":0}'), good.replace(b'{"ops":[', b'{"ops" :['),
           good.replace(b"]}]", b"]}}]"), good.replace(b'{"Copy":{"offset":4096,"size":4096}}', b'{"Copy":{"offset":4096,"size":4096},"x":1}'),
           # junk before the first op (the chain must start at byte 8: ADVICE r02)
           b'{"ops":[xyz},{"Data":[5]}],"source_size":1,"block_size":1}',
           b'{"ops":[1},{"Copy":{"offset":0,"size":1}}],"source_size":1,"block_size":1}',
           good.replace(b'{"ops":[{', b'{"ops":[ {', 1)]
    for t in bad:
        assert dev_parse(t) is None, t
        n_checks += 1
    for it in range(300):
        b = bytearray(good)
        for _ in range(rng.randint(1, 3)):
            b[rng.randrange(len(b))] = rng.choice(b'0123456789{}[],:"aDC ')
        t = bytes(b)
        got = dev_parse(t)
        if got is not None:
            assert compact(*got) == t, t
            assert got == expect(t) == wire.delta_from_json(t), t
        n_checks += 1
    return n_checks


def sigparse_checks():
    """sydelta_checksums_from_json_device (K7p; the emulated launches run
    sydelta_sigjson.hpp's chunk bodies): serde's compact text of random signatures (tile
    and chunk edges, extreme values) parses to the entries the host parser gives; the
    count-only call; a buffer shorter than the count; and the device parser refuses every
    text outside the compact form -- whitespace, another key order, an unknown key, a
    missing or duplicated field, leading zeros, out-of-range values, a trailing comma or
    byte, a truncated text -- while the host parser's verdict on it stays its own."""
    import ctypes
    import json

    from sy_amd import wire
    from sy_amd._lib import SyDeltaError, check, lib

    rng = np.random.default_rng(11)
    n_checks = 0

    def dev_parse(text: bytes, cap=None):
        buf = np.frombuffer(text, np.uint8).copy() if text else np.zeros(1, np.uint8)
        got = ctypes.c_uint64()
        rc = lib.sydelta_checksums_from_json_device(ctypes.c_void_p(buf.ctypes.data), len(text), None, 0,
                                                    ctypes.byref(got), None)
        if rc:
            return None
        n = got.value
        k = n if cap is None else cap
        out = np.zeros(max(k, 1), wire._SIG_DTYPE)
        check(lib.sydelta_checksums_from_json_device(ctypes.c_void_p(buf.ctypes.data), len(text),
                                                     ctypes.c_void_p(out.ctypes.data), k, ctypes.byref(got), None))
        assert got.value == n
        return out[:min(k, n)]

    for n in (0, 1, 2, 3, 255, 256, 257, 1000, 5000):
        idx = np.arange(n, dtype=np.uint64)
        if n and rng.random() < 0.5:
            w = np.array([0, 9, 0xFFFFFFFF], np.uint32)[rng.integers(0, 3, n)]
            st = np.array([0, 10, 0xFFFFFFFFFFFFFFFF], np.uint64)[rng.integers(0, 3, n)]
        else:
            w = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
            st = rng.integers(0, 1 << 64, n, dtype=np.uint64)
        sizes = np.full(n, 4096, np.uint64)
        if n:
            sizes[-1] = 17
        text = wire.checksums_to_json(wire.sig_array(idx, idx * np.uint64(4096), sizes, w, st))
        host = wire.checksums_from_json(text)
        dev = dev_parse(text)
        assert dev is not None and np.array_equal(dev, host), n
        if n > 3:
            part = dev_parse(text, cap=3)
            assert np.array_equal(part, host[:3])
        n_checks += 1
    good = b'[{"index":0,"offset":0,"size":4096,"weak":1,"strong":2},{"index":1,"offset":4096,"size":5,"weak":3,"strong":4}]'
    assert dev_parse(good) is not None
    bad = [
        b"", b"[", b"]", b"[}", b"[{]", b"[ ]", b" []", b"[] ", b"[,]",
        good.replace(b",{", b", {"), good.replace(b'"index":0', b'"index": 0'),
        good.replace(b'"offset":0,"size":4096', b'"size":4096,"offset":0'),
        good.replace(b'"strong":2}', b'"strong":2,"x":1}'),
        good.replace(b',"weak":1', b''), good.replace(b'"weak":1', b'"weak":1,"weak":1'),
        good.replace(b'"size":5', b'"size":05'), good.replace(b'"weak":3', b'"weak":4294967296'),
        good.replace(b'"strong":4', b'"strong":18446744073709551616'), good.replace(b'"index":1', b'"index":-1'),
        good.replace(b'"weak":3', b'"weak":3.0'), good[:-1] + b",]", good + b"\n", good[:-1], good[:-2] + b"]",
        good.replace(b"},{", b"}{"), good.replace(b"},{", b"},,{"), b"[" + good[1:-1] + b",{}]",
    ]
    for t in bad:
        assert dev_parse(t) is None, t
        try:
            host = wire.checksums_from_json(t)
        except SyDeltaError:
            host = None
        ok_json = True
        try:
            json.loads(t)
        except ValueError:
            ok_json = False
        if host is not None:  # a spelling serde accepts that is not the compact form
            assert ok_json, t
        n_checks += 1
    # random byte mutations of a valid text: the device accepts only what equals the
    # host parser's result on a text that re-serializes to itself
    for it in range(300):
        b = bytearray(good)
        for _ in range(int(rng.integers(1, 4))):
            b[int(rng.integers(0, len(b)))] = int(rng.choice(list(b'0123456789{}[],:"ax ')))
        t = bytes(b)
        dev = dev_parse(t)
        if dev is not None:
            host = wire.checksums_from_json(t)
            assert np.array_equal(dev, host), t
            assert wire.checksums_to_json(host) == t, t
        n_checks += 1
    return n_checks


def _walk_counters():
    import ctypes

    from sy_amd._lib import lib

    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    lib.sydelta_walk_counters(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def device_walk_checks(tmp):
    """K5b (sydelta_chain.hpp, SYDELTA_DEVICE_WALK=1, every source with a hit): the
    kernels' per-thread bodies run by the emulated launch_chain, through the path API,
    the chunked walks and dense/periodic data where walks from different entries never
    merge; each op list against the oracle.  Also counts that the device walk ran and
    that a path into an unscanned block was handed back to the host walk."""
    os.environ["SYDELTA_DEVICE_WALK"] = "1"
    os.environ["SYDELTA_DEVICE_WALK_MIN"] = "1"
    n = 0
    w0, f0 = _walk_counters()
    try:
        os.environ["SYDELTA_STREAM_CHUNK"] = str(1 << 20)
        for bs, size in [(4096, (1 << 20) + 1234), (1007, (1 << 20) + 99), (64, (1 << 18) + 5),
                         (16384, (2 << 20) + 4321), (512, 300000)]:
            for probe in ("0", "1", "auto"):
                if probe == "auto":
                    os.environ.pop("SYDELTA_PROBE", None)
                else:
                    os.environ["SYDELTA_PROBE"] = probe
                basis, s = case(bs % 89 + 3, size, bs)
                check_pair(tmp, basis, s, bs, ("device walk", bs, probe))
                n += 1
        # dense hits: low-alphabet and periodic data (every window hits; chains from
        # neighbouring entries stay apart), a zero file, duplicated blocks
        rng = np.random.default_rng(5)
        for probe in ("0", "1"):
            os.environ["SYDELTA_PROBE"] = probe
            for name, basis, s in _dense_cases(rng):
                check_pair(tmp, basis, s, 64, ("device walk dense", name, probe))
                n += 1
        os.environ.pop("SYDELTA_PROBE", None)
        # the chunked walks (entries inside blocks) and the batched path
        n += batch_and_chunk_checks()
        # shifted data with the probe on: walks that jump into blocks classified only by
        # their aligned window (on-demand scans through the host walk)
        os.environ["SYDELTA_PROBE"] = "1"
        for seed in range(4):
            basis = O.synth_bytes(400 * 256 + 3, 0x900 + seed)
            s = basis.copy()
            r = np.random.default_rng(seed)
            for p in sorted(r.integers(0, s.size - 300, 6))[::-1]:
                k = int(r.integers(1, 255))
                s = np.concatenate([s[:p], basis[p + 40:p + 40 + k], s[p:]])  # copies of nearby unaligned bytes
            check_pair(tmp, basis, s, 256, ("device walk shifted", seed))
            n += 1
    finally:
        for k in ("SYDELTA_DEVICE_WALK", "SYDELTA_DEVICE_WALK_MIN", "SYDELTA_PROBE"):
            os.environ.pop(k, None)
    w1, f1 = _walk_counters()
    assert w1 - w0 >= 40, ("device walks ran", w1 - w0)
    print(f"device walks: {w1 - w0}, handed back to the host walk: {f1 - f0}")
    return n


def _dense_cases(rng):
    period = rng.integers(0, 256, 100, dtype=np.uint8)
    per = np.tile(period, 3000)
    yield "periodic", per, np.concatenate([per[:777], per[5:20000], per[3:]])
    low = rng.integers(0, 2, 120000, dtype=np.uint8)
    low2 = low.copy()
    low2[rng.integers(0, low2.size, 50)] ^= 1
    yield "binary", low, low2
    z = np.zeros(90000, np.uint8)
    yield "zeros", z, np.concatenate([z[:5000], np.ones(3, np.uint8), z[:70001]])
    blk = rng.integers(0, 256, 64, dtype=np.uint8)
    dup = np.tile(blk, 500)
    yield "duplicated", dup, np.concatenate([dup[:1000], rng.integers(0, 256, 33, dtype=np.uint8), dup[7:]])
    # basis blocks A and rot5(A): a run of A's hits at every aligned position and at every
    # aligned position + 5, so scanned blocks whose aligned window hit hold unaligned hits
    # too (the merge's ranks); Z = 5 other bytes + A[5:] enters the +5 phase, so paths run
    # through those unaligned hits
    A = rng.integers(0, 256, 64, dtype=np.uint8)
    rot = np.concatenate([A[5:], A[:5]])
    rnd = lambda k: rng.integers(0, 256, 64 * k, dtype=np.uint8)
    Z = np.concatenate([rng.integers(0, 256, 5, dtype=np.uint8), A[5:]])
    basis = np.concatenate([A, rot, rnd(40)])
    parts = []
    for k in range(60):
        parts += [rnd(1), A, A, A] if k % 3 else [rnd(2), Z, A, A, A, rnd(1), A]
    yield "rotated", basis, np.concatenate(parts + [A[:17]])


def error_checks(tmp):
    """I/O errors surface as SYDELTA_E_IO with the path in the message, as io::Error
    would: missing files, a directory, a checksum list not in compute_checksums layout."""
    from sy_amd._lib import SyDeltaError, SYDELTA_E_IO, SYDELTA_E_INVAL

    n = 0
    missing = os.path.join(tmp, "no_such_file")
    for fn in (lambda: D.compute_checksums(missing, 4096),
               lambda: D.generate_delta_streaming(missing, [], 4096),
               lambda: D.generate_delta(missing, [], 4096),
               lambda: D.compute_checksums(tmp, 4096),
               lambda: D.generate_delta_streaming(tmp, [], 4096)):
        try:
            fn()
        except SyDeltaError as e:
            assert e.code == SYDELTA_E_IO, e
            n += 1
        else:
            raise AssertionError("no error")
    p = os.path.join(tmp, "small")
    O.synth_bytes(10000, 3).tofile(p)
    sigs = D.compute_checksums(p, 4096)
    bad = [D.BlockChecksum(s.index, s.offset + 1, s.size, s.weak, s.strong) for s in sigs]
    try:
        D.generate_delta_streaming(p, bad, 4096)
    except SyDeltaError as e:
        assert e.code == SYDELTA_E_INVAL, e
        n += 1
    else:
        raise AssertionError("layout not checked")
    return n


def _ops(lib, h):
    import ctypes

    n = lib.sydelta_delta_num_ops(h)
    if not n:
        return []
    p = lib.sydelta_delta_ops(h)
    raw = np.frombuffer((ctypes.c_uint8 * (24 * n)).from_address(ctypes.addressof(p.contents)),
                        dtype=np.dtype([("kind", "<u4"), ("r", "<u4"), ("a", "<u8"), ("b", "<u8")]))
    return [("C" if int(k) == 0 else "D", int(x), int(y)) for k, x, y in zip(raw["kind"], raw["a"], raw["b"])]


def batch_and_chunk_checks():
    """The device-pointer entry points on host memory: batched signature + index + match
    (the C4 path, threaded walks at >= 64 files) and a file matched in 1/2/3/8 chained
    chunks (the C5 path), each against the oracle."""
    import ctypes

    from sy_amd._lib import check, lib

    vp = lambda a: ctypes.c_void_p(a.ctypes.data)
    rng = np.random.default_rng(77)
    n_checks = 0
    for bs in (1024, 4096):
        # "0" / "1" / "auto": the classifier path (SYDELTA_FILE_WALK=0); "walk": the file
        # walk (K10), which a batch of >= 64 small files takes by default
        # walk8: segments of >= 8 blocks (SYDELTA_FILE_SEGS=8); *dx: the op lists expanded on the
        # device (SYDELTA_DEVICE_EXPAND=1, k_walk_expand), else on the host
        for probe in ("0", "1", "auto", "walk", "walk8", "walkdx", "walk8dx"):
            os.environ["SYDELTA_FILE_WALK"] = "0"
            os.environ["SYDELTA_FILE_SEGS"] = "8" if probe.startswith("walk8") else ""
            os.environ["SYDELTA_DEVICE_EXPAND"] = "1" if probe.endswith("dx") else "0"
            if probe in ("auto", "walk", "walk8", "walkdx", "walk8dx"):
                os.environ.pop("SYDELTA_PROBE", None)
            else:
                os.environ["SYDELTA_PROBE"] = probe
            if probe.startswith("walk"):
                os.environ.pop("SYDELTA_FILE_WALK")
            nf = 80
            bases, srcs = [], []
            for k in range(nf):
                size = [0, 100, bs - 1, bs, int(rng.integers(bs, 40 * bs))][k % 5]
                b = O.synth_bytes(size, 0x600 + k)
                s2 = b.copy()
                if size > 10:
                    p = int(rng.integers(0, size))
                    s2 = np.concatenate([s2[:p], np.frombuffer(b"Z", np.uint8), s2[p:]])
                    for q in rng.integers(0, s2.size, 3):
                        s2[q] ^= 0x11
                bases.append(b)
                srcs.append(s2)

            def pack(parts):
                offs, cur = [], 0
                for x in parts:
                    offs.append(cur)
                    cur += (x.size + 15) // 16 * 16 + 16
                buf = np.zeros(cur + 16, np.uint8)
                for o, x in zip(offs, parts):
                    buf[o:o + x.size] = x
                return buf, np.array(offs, np.uint64), np.array([x.size for x in parts], np.uint64)

            bbuf, boff, blen = pack(bases)
            sbuf, soff, slen = pack(srcs)
            nblk = (blen + bs - 1) // bs
            tot = int(nblk.sum())
            w = np.zeros(max(tot, 1), np.uint32)
            st = np.zeros(max(tot, 1), np.uint64)
            check(lib.sydelta_signature_batch_device(0, vp(bbuf), vp(boff), vp(blen), nf, bs, vp(w), vp(st), None))
            fb = np.concatenate([[0], np.cumsum(nblk)]).astype(np.int64)
            last = np.where(nblk > 0, blen - (nblk - 1) * bs, 0).astype(np.uint64)
            ix = ctypes.c_void_p()
            check(lib.sydelta_index_create_batch(0, vp(w), vp(st), vp(nblk.astype(np.uint64)), vp(last), nf, bs, 1,
                                                 None, ctypes.byref(ix)))
            bt = ctypes.c_void_p()
            lib.emu_expand_files.restype = ctypes.c_uint64
            ex0 = lib.emu_expand_files()
            check(lib.sydelta_match_batch_device(ix, vp(sbuf), vp(soff), vp(slen), nf, None, ctypes.byref(bt)))
            assert (lib.emu_expand_files() > ex0) == probe.endswith("dx"), (bs, probe)  # the expansion's path
            for k in range(nf):
                ew, es, ez = C.compute_checksums(bases[k], bs)
                assert np.array_equal(w[fb[k]:fb[k + 1]], ew) and np.array_equal(st[fb[k]:fb[k + 1]], es), (bs, k)
                exp = O.ops_from_arrays(*C.generate_delta(srcs[k], ew, es, ez, bs))
                got = _ops(lib, lib.sydelta_delta_batch_get(bt, k))
                assert got == exp, ("batch", bs, probe, k)
                n_checks += 1
            lib.sydelta_delta_batch_free(bt)
            lib.sydelta_index_free(ix)
            if probe.startswith("walk"):  # the same pairs through the one-call form (two groups from 128 files)
                for reps in (1, 2):
                    pb, pbo, pbl = pack(bases * reps)
                    ps_, pso, psl = pack(srcs * reps)
                    bt = ctypes.c_void_p()
                    check(lib.sydelta_delta_pairs_device(0, vp(pb), vp(pbo), vp(pbl), vp(ps_), vp(pso), vp(psl),
                                                         nf * reps, bs, None, ctypes.byref(bt)))
                    for k in range(nf * reps):
                        ew, es, ez = C.compute_checksums(bases[k % nf], bs)
                        exp = O.ops_from_arrays(*C.generate_delta(srcs[k % nf], ew, es, ez, bs))
                        assert _ops(lib, lib.sydelta_delta_batch_get(bt, k)) == exp, ("pairs", bs, probe, reps, k)
                        n_checks += 1
                    lib.sydelta_delta_batch_free(bt)
    os.environ.pop("SYDELTA_PROBE", None)
    os.environ.pop("SYDELTA_FILE_WALK", None)
    os.environ.pop("SYDELTA_FILE_SEGS", None)
    os.environ.pop("SYDELTA_DEVICE_EXPAND", None)
    # chunked: one file in 1/2/3/8 chunks, walks chained in order, parts appended
    for bs in (512, 4096):
        basis = O.synth_bytes(300 * bs + 77, 0x700)
        s2 = np.concatenate([basis[:10 * bs], np.frombuffer(b"Q", np.uint8), basis[10 * bs:150 * bs],
                             basis[200 * bs:]])
        for q in rng.integers(0, s2.size, 20):
            s2[q] ^= 0x22
        L = s2.size
        sb = np.zeros(L + 32, np.uint8)
        sb[:L] = s2
        nb = -(-basis.size // bs)
        w = np.zeros(nb, np.uint32)
        st = np.zeros(nb, np.uint64)
        bb = np.zeros(basis.size + 16, np.uint8)
        bb[:basis.size] = basis
        check(lib.sydelta_signature_device(0, vp(bb), basis.size, bs, vp(w), vp(st), None))
        ix = ctypes.c_void_p()
        check(lib.sydelta_index_create(0, vp(w), vp(st), nb, bs, basis.size - (nb - 1) * bs, 1, None,
                                       ctypes.byref(ix)))
        ew, es, ez = C.compute_checksums(basis, bs)
        exp = O.ops_from_arrays(*C.generate_delta(s2, ew, es, ez, bs))
        npos = L - bs + 1
        nbp = -(-npos // bs)
        lib.emu_chunk_units.restype = ctypes.c_uint64
        for nch in (1, 2, 3, 8):
            # 1p: the device walk's launches in one sub-range per segment; ...dx: the ops written
            # by the emulated k_chunk_write (SYDELTA_DEVICE_EXPAND=1); 1pa: the default with this
            # host's threads (> 4): the last part's ops written by it, the others' on the host
            for probe in ("0", "1", "1p", "1dx", "1pdx", "1pa"):
                os.environ["SYDELTA_PROBE"] = probe[0]
                os.environ["SYDELTA_CHUNK_PIPE"] = "3" if probe.startswith("1p") else ""
                os.environ["SYDELTA_DEVICE_EXPAND"] = "" if probe == "1pa" else "1" if probe.endswith("dx") else "0"
                cu0 = lib.emu_chunk_units()
                cuts = sorted(set(int(c) for c in rng.choice(np.arange(1, nbp), nch - 1, replace=False))) if nch > 1 \
                    else []
                bounds = [0] + [c * bs for c in cuts] + [npos]
                acc = lib.sydelta_delta_new(L, bs)
                entry = 0
                for g in range(len(bounds) - 1):
                    p0, p1 = bounds[g], bounds[g + 1]
                    final = g == len(bounds) - 2
                    bpos = p0 & ~15
                    end = L if final else min(L, p1 + bs - 1)
                    ch = ctypes.c_void_p()
                    check(lib.sydelta_chunk_classify(ix, ctypes.c_void_p(sb.ctypes.data + bpos), bpos, end - bpos, L,
                                                     p0, max(p1, L) if final else p1, None, ctypes.byref(ch)))
                    d = ctypes.c_void_p()
                    ex = ctypes.c_uint64()
                    check(lib.sydelta_chunk_walk(ch, entry, ctypes.byref(ex), ctypes.byref(d)))
                    check(lib.sydelta_delta_append(acc, d))
                    lib.sydelta_delta_free(d)
                    lib.sydelta_chunk_free(ch)
                    entry = ex.value
                assert _ops(lib, acc) == exp, ("chunks", bs, nch, probe)
                if probe not in ("0", "1pa"):  # the path the ops took (1pa: as the re-walks leave it)
                    assert (lib.emu_chunk_units() > cu0) == probe.endswith("dx"), ("chunk writes", bs, nch, probe)
                lib.sydelta_delta_free(acc)
                n_checks += 1
        lib.sydelta_index_free(ix)
    os.environ.pop("SYDELTA_PROBE", None)
    os.environ.pop("SYDELTA_CHUNK_PIPE", None)
    os.environ.pop("SYDELTA_DEVICE_EXPAND", None)
    return n_checks


def multi_device_checks():
    """EMU_DEVICES=4: the path API's per-thread device binding (10 concurrent callers
    spread over the devices, explicit binding, a restricted device set) and
    sydelta_delta_multi_device (one file chunk-sharded over devices, the signature
    gathered by peer copies, the walks chained inside the library) against the oracle."""
    import ctypes
    import threading

    from sy_amd._lib import check, lib

    n_checks = 0
    ndev = ctypes.c_int()
    check(lib.sydelta_device_count(ctypes.byref(ndev)))
    assert ndev.value == 4, ndev.value
    lib.emu_device_sets.restype = ctypes.c_uint64
    lib.emu_device_sets.argtypes = [ctypes.c_int]
    sets0 = [lib.emu_device_sets(d) for d in range(4)]
    # 10 concurrent callers: bound to the least-loaded device, sticky, spread evenly
    bar = threading.Barrier(10)
    got = [None] * 10

    def bind(k, out):
        d = ctypes.c_int(-1)
        check(lib.sydelta_thread_device(ctypes.byref(d)))
        d2 = ctypes.c_int(-1)
        check(lib.sydelta_thread_device(ctypes.byref(d2)))
        assert d.value == d2.value, "binding is sticky"
        out[k] = d.value
        bar.wait()  # every thread stays bound until all have bound

    th = [threading.Thread(target=bind, args=(k, got)) for k in range(10)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    cnt = [got.count(d) for d in range(4)]
    assert sorted(cnt) == [2, 2, 3, 3], cnt
    n_checks += 1
    # explicit binding and a restricted set
    check(lib.sydelta_set_thread_device(2))
    d = ctypes.c_int(-1)
    check(lib.sydelta_thread_device(ctypes.byref(d)))
    assert d.value == 2
    assert lib.sydelta_set_thread_device(7) != 0  # not visible
    check(lib.sydelta_set_thread_device(-1))
    allowed = (ctypes.c_int * 2)(1, 3)
    check(lib.sydelta_set_devices(allowed, 2))
    got2 = [None] * 6
    bar = threading.Barrier(6)
    th = [threading.Thread(target=bind, args=(k, got2)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert sorted(got2) == [1, 1, 1, 3, 3, 3], got2
    check(lib.sydelta_set_devices(None, 0))
    n_checks += 1
    # the path API from 10 threads, each on its bound device, against the oracle
    os.environ["SYDELTA_STREAM_CHUNK"] = str(1 << 18)
    pairs = [case(300 + k, (1 << 20) + 1231 * k, 4096) for k in range(10)]
    with tempfile.TemporaryDirectory() as tmp:
        def one(k):
            dd = os.path.join(tmp, f"m{k}")
            os.makedirs(dd, exist_ok=True)
            check_pair(dd, pairs[k][0], pairs[k][1], 4096, ("multi thread", k))
            return True

        with ThreadPoolExecutor(10) as ex:
            assert all(ex.map(one, range(10)))
    n_checks += 10
    sets1 = [lib.emu_device_sets(d) for d in range(4)]
    assert all(b > a for a, b in zip(sets0, sets1)), (sets0, sets1)
    # one file over several devices inside the library
    rng = np.random.default_rng(91)
    vpa = lambda arrs: (ctypes.c_void_p * len(arrs))(*[ctypes.c_void_p(x) for x in arrs])
    u64a = lambda xs: (ctypes.c_uint64 * len(xs))(*[int(x) for x in xs])
    for bs in (512, 4096):
        basis = O.synth_bytes(301 * bs + 77, 0x800 + bs)
        s2 = np.concatenate([basis[:40 * bs + 3], np.frombuffer(b"QQ", np.uint8), basis[40 * bs + 3:170 * bs],
                             basis[210 * bs:], basis[5 * bs:9 * bs]])
        for q in rng.integers(0, s2.size, 30):
            s2[q] ^= 0x44
        L = s2.size
        sb = np.zeros(L + 64, np.uint8)
        sb[:L] = s2
        bb = np.zeros(basis.size + 64, np.uint8)
        bb[:basis.size] = basis
        ew, es, ez = C.compute_checksums(basis, bs)
        exp = O.ops_from_arrays(*C.generate_delta(s2, ew, es, ez, bs))
        nbb = -(-basis.size // bs)
        npos = L - bs + 1
        for devs in ([0], [0, 1], [0, 1, 2, 3], [3, 3, 1], [2, 0, 1, 3, 2, 0, 1, 3]):
            k = len(devs)
            bcut = sorted(int(c) for c in rng.choice(np.arange(1, nbb), k - 1, replace=False)) if k > 1 else []
            bb_pos = [0] + [c * bs for c in bcut]
            blen = [(bb_pos[g + 1] if g + 1 < k else basis.size) - bb_pos[g] for g in range(k)]
            scut = sorted(int(c) for c in rng.choice(np.arange(1, -(-npos // bs)), k - 1, replace=False)) if k > 1 \
                else []
            sp = [0] + [c * bs for c in scut]
            slen = [(min(L, sp[g + 1] + bs - 1) if g + 1 < k else L) - sp[g] for g in range(k)]
            out = ctypes.c_void_p()
            for probe in ("0", "1"):
                os.environ["SYDELTA_PROBE"] = probe
                check(lib.sydelta_delta_multi_device(
                    (ctypes.c_int * k)(*devs), k, vpa([bb.ctypes.data + x for x in bb_pos]), u64a(blen),
                    vpa([sb.ctypes.data + x for x in sp]), u64a(sp), u64a(slen), L, bs, ctypes.byref(out)))
                assert _ops(lib, out) == exp, ("multi", bs, devs, probe)
                lib.sydelta_delta_free(out)
                n_checks += 1
    os.environ.pop("SYDELTA_PROBE", None)
    # argument checks: a basis chunk that is not whole blocks, a misaligned source start
    out = ctypes.c_void_p()
    basis = O.synth_bytes(10 * 512, 1)
    rc = lib.sydelta_delta_multi_device((ctypes.c_int * 2)(0, 1), 2, vpa([basis.ctypes.data, basis.ctypes.data + 500]),
                                        u64a([500, 4620]), vpa([basis.ctypes.data, basis.ctypes.data]), u64a([0, 512]),
                                        u64a([1023, 4608]), 5120, 512, ctypes.byref(out))
    assert rc == -3, rc
    rc = lib.sydelta_delta_multi_device((ctypes.c_int * 2)(0, 1), 2, vpa([basis.ctypes.data, basis.ctypes.data + 512]),
                                        u64a([512, 4608]), vpa([basis.ctypes.data, basis.ctypes.data]), u64a([0, 100]),
                                        u64a([1023, 4608]), 5120, 512, ctypes.byref(out))
    assert rc == -3, rc
    n_checks += 2
    n_checks += device_restore_checks(lib)
    print(f"emulated multi-device checks ok: {n_checks}")


def device_restore_checks(lib):
    """Every entry point leaves the calling thread's current device as it found it
    (sydelta.h, "Devices"): from each starting device, calls that work on other devices --
    a device-pointer signature, an index built and freed on another device, the path API on
    a bound device, sydelta_trim, sydelta_delta_multi_device (success and argument errors)."""
    import ctypes

    from sy_amd._lib import check

    vpa = lambda arrs: (ctypes.c_void_p * len(arrs))(*[ctypes.c_void_p(x) for x in arrs])
    u64a = lambda xs: (ctypes.c_uint64 * len(xs))(*[int(x) for x in xs])
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)

    def cur():
        d = ctypes.c_int(-1)
        assert lib.hipGetDevice(ctypes.byref(d)) == 0
        return d.value

    n = 0
    bs = 512
    basis = O.synth_bytes(20 * bs + 7, 0x901)
    src = basis.copy()
    src[3000] ^= 1
    L = src.size
    with tempfile.TemporaryDirectory() as tmp:
        pb, ps = os.path.join(tmp, "b"), os.path.join(tmp, "s")
        basis.tofile(pb)
        src.tofile(ps)
        for start in range(4):
            assert lib.hipSetDevice(start) == 0
            other = (start + 1) % 4
            nb = -(-basis.size // bs)
            w = np.zeros(nb, np.uint32)
            st = np.zeros(nb, np.uint64)
            check(lib.sydelta_signature_device(other, vp(basis), basis.size, bs, vp(w), vp(st), None))
            assert cur() == start, ("signature", start)
            ix = ctypes.c_void_p()
            check(lib.sydelta_index_create(other, vp(w), vp(st), nb, bs, basis.size - (nb - 1) * bs, 1, None,
                                           ctypes.byref(ix)))
            assert cur() == start, ("index_create", start)
            out = ctypes.c_void_p()
            check(lib.sydelta_match_device(ix, vp(src), L, None, ctypes.byref(out)))
            assert cur() == start, ("match", start)
            lib.sydelta_delta_free(out)
            lib.sydelta_index_free(ix)
            assert cur() == start, ("index_free", start)
            check(lib.sydelta_set_thread_device(other))
            from sy_amd._lib import BlockChecksumC

            ck = ctypes.POINTER(BlockChecksumC)()
            nck = ctypes.c_uint64()
            check(lib.sydelta_compute_checksums(pb.encode(), bs, ctypes.byref(ck), ctypes.byref(nck)))
            assert cur() == start, ("compute_checksums", start)
            h = ctypes.c_void_p()
            check(lib.sydelta_generate_delta_streaming(ps.encode(), ck, nck.value, bs, ctypes.byref(h)))
            assert cur() == start, ("generate_delta_streaming", start)
            lib.sydelta_delta_free(h)
            lib.sydelta_checksums_free(ctypes.cast(ck, ctypes.c_void_p))
            check(lib.sydelta_set_thread_device(-1))
            lib.sydelta_trim()
            assert cur() == start, ("trim", start)
            bb = np.zeros(basis.size + 64, np.uint8)
            bb[:basis.size] = basis
            sb = np.zeros(L + 64, np.uint8)
            sb[:L] = src
            devs = [3, 1, 0, 2]
            bpos = [0, 5 * bs, 10 * bs, 15 * bs]
            blen = [5 * bs, 5 * bs, 5 * bs, basis.size - 15 * bs]
            sp = [0, 4 * bs, 9 * bs, 14 * bs]
            slen = [min(L, sp[g + 1] + bs - 1) - sp[g] if g < 3 else L - sp[g] for g in range(4)]
            out = ctypes.c_void_p()
            check(lib.sydelta_delta_multi_device((ctypes.c_int * 4)(*devs), 4, vpa([bb.ctypes.data + x for x in bpos]),
                                                 u64a(blen), vpa([sb.ctypes.data + x for x in sp]), u64a(sp),
                                                 u64a(slen), L, bs, ctypes.byref(out)))
            assert cur() == start, ("multi_device", start)
            lib.sydelta_delta_free(out)
            # an argument error after validation of the devices
            rc = lib.sydelta_delta_multi_device((ctypes.c_int * 2)(other, start), 2,
                                                vpa([bb.ctypes.data, bb.ctypes.data + 500]), u64a([500, 4620]),
                                                vpa([sb.ctypes.data, sb.ctypes.data]), u64a([0, 512]),
                                                u64a([1023, 4608]), 5120, bs, ctypes.byref(out))
            assert rc == -3 and cur() == start, ("multi_device error", start)
            n += 1
    assert lib.hipSetDevice(0) == 0
    return n


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[3] == "multi":
        multi_device_checks()
    else:
        main()
