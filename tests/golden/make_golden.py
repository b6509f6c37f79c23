"""Generate tests/golden/cases.json — golden vectors for the delta hot path.

Run in the build container:  python tests/golden/make_golden.py

Expected outputs come from the pure-Python restatement in oracle/oracle.py
(line-by-line after src/delta), whose primitives are pinned by zlib.adler32 and
python-xxhash 3.8.1 (libxxhash 0.8.2 — the frozen XXH3 algorithm that crate
xxhash-rust 0.8.15 implements).  The reference (Rust) cannot be run here, so
these vectors restate (a) every input/expectation of the reference's own unit
tests in src/delta (rolling.rs:95-266, checksum.rs:88-146,
generator.rs:388-604, applier.rs:87-234, mod.rs:29-35) and (b) the worked
examples of SURVEY.md Appendix B, plus seeded random edit cases.
"""
import json
import os
import random
import sys
import zlib

import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402


def enc(data: bytes):
    """Inputs: hex, or run-length [[hex_chunk, repeat], ...] for large regular ones."""
    if len(data) <= 16384:
        return {"hex": data.hex()}
    runs = []
    i = 0
    while i < len(data):
        j = i
        while j < len(data) and data[j] == data[i]:
            j += 1
        runs.append([data[i:i + 1].hex(), j - i])
        i = j
    assert len(runs) <= 1024, "large fixture inputs must be run-length regular"
    return {"rle": runs}


def sig_case(name, data: bytes, bs: int, ref):
    sigs = O.py_compute_checksums(data, bs)
    for c in sigs:  # primitive pins
        blk = data[c.offset:c.offset + c.size]
        assert c.weak == zlib.adler32(blk) and c.strong == xxhash.xxh3_64_intdigest(blk)
    return {"kind": "signature", "name": name, "ref": ref, "data": enc(data), "block_size": bs,
            "expect": [[c.index, c.offset, c.size, c.weak, c.strong] for c in sigs]}


def delta_case(name, src: bytes, basis: bytes, bs: int, ref, chunk=256 * 1024):
    sigs = O.py_compute_checksums(basis, bs)
    ops = O.py_generate_delta(src, sigs, bs)
    ops_s = O.py_generate_delta_streaming(src, sigs, bs, chunk)
    assert ops == ops_s, name
    assert O.py_apply_delta(basis, src, ops) == src
    return {"kind": "delta", "name": name, "ref": ref, "src": enc(src), "basis": enc(basis),
            "block_size": bs, "expect_ops": [list(o) for o in ops],
            "compression_ratio": O.compression_ratio(ops)}


def mutate(b: bytes, rng: random.Random) -> bytes:
    b = bytearray(b)
    for _ in range(rng.randint(0, 6)):
        op = rng.randint(0, 3)
        p = rng.randint(0, max(0, len(b) - 1))
        if op == 0 and b:
            b[p] = rng.randint(0, 255)
        elif op == 1:
            b[p:p] = bytes(rng.randint(0, 255) for _ in range(rng.randint(1, 20)))
        elif op == 2:
            del b[p:p + rng.randint(1, 20)]
        else:
            q = rng.randint(0, max(0, len(b) - 1))
            b[p:p] = b[q:q + rng.randint(1, 40)]
    return bytes(b)


def main():
    cases = []
    # ---- rolling.rs tests (values are Adler-32 of windows; recorded as signature cases
    # with block size = window so the device path is exercised on the same bytes)
    cases.append({"kind": "adler", "name": "adler_hello_world", "ref": "rolling.rs:99-104",
                  "data": enc(b"hello world"), "expect": zlib.adler32(b"hello world")})
    cases.append({"kind": "adler", "name": "adler_empty_is_1", "ref": "rolling.rs:165-168",
                  "data": enc(b""), "expect": 1})
    # ---- checksum.rs tests
    cases.append(sig_case("checksums_51B_bs16", b"Hello, World! This is a test file for checksumming.", 16,
                          "checksum.rs:88-113; SURVEY App.B"))
    cases.append(sig_case("checksums_empty", b"", 1024, "checksum.rs:115-120"))
    cases.append(sig_case("checksums_test_data_bs4", b"test data", 4, "checksum.rs:122-132"))
    cases.append(sig_case("checksums_a100_bs10", b"a" * 100, 10, "checksum.rs:134-146"))
    cases.append(sig_case("checksums_a100_bs50", b"a" * 100, 50, "checksum.rs:134-146"))
    cases.append(sig_case("checksums_range256x16_bs4096", bytes(range(256)) * 16, 4096, "SURVEY App.B"))
    # ---- generator.rs tests
    cases.append(delta_case("delta_identical_bs8", b"Hello, World! This is a test.", b"Hello, World! This is a test.",
                            8, "generator.rs:388-411, 492-511"))
    cases.append(delta_case("delta_completely_different", b"AAAAAAAA", b"BBBBBBBB", 4, "generator.rs:413-432"))
    cases.append(delta_case("delta_partial_match", b"AAAABBBBCCCC", b"AAAADDDDCCCC", 4,
                            "generator.rs:434-461; SURVEY App.B"))
    cases.append(delta_case("delta_empty_source", b"", b"some data", 4, "generator.rs:463-475, 592-604"))
    cases.append(delta_case("delta_empty_dest", b"some data", b"", 4, "generator.rs:477-489"))
    cases.append(delta_case("delta_streaming_vs_nonstreaming_40B", b"AAAABBBBCCCCDDDDEEEEFFFFGGGGHHHHIIIIJJJJ",
                            b"AAAABBBBXXXXDDDDEEEEYYYYGGGGHHHHZZZZJJJJ", 4, "generator.rs:537-561; SURVEY App.B"))
    cases.append(delta_case("delta_streaming_large_0xAB", b"\xab" * (256 * 1024), b"\xab" * (256 * 1024), 4096,
                            "generator.rs:513-535"))
    refill = b"".join(bytes([i % 256]) * 1024 for i in range(512))
    cases.append(delta_case("delta_streaming_window_refill", refill, refill, 8192, "generator.rs:563-590"))
    # ---- applier.rs round trips (same generator inputs as its tests)
    d = b"Hello, World! This is a test of delta sync."
    cases.append(delta_case("apply_identical_bs8", d, d, 8, "applier.rs:87-113"))
    cases.append(delta_case("apply_modified_bs4", b"AAAAXXXXYYYYDDDD", b"AAAABBBBCCCCDDDD", 4, "applier.rs:115-145"))
    cases.append(delta_case("apply_all_different_bs4", b"completely new content!", b"old data here", 4,
                            "applier.rs:147-173"))
    cases.append(delta_case("apply_no_base_bs4", b"new file content", b"", 4, "applier.rs:175-193"))
    orig = bytes(i % 256 for i in range(10000))
    mod = bytearray(orig)
    mod[2000:3000] = b"\xff" * 1000
    cases.append(delta_case("apply_large_bs512", bytes(mod), orig, 512, "applier.rs:195-234"))
    # ---- seeded random edit cases (alphabets 2/4/256, tiny block sizes, quirks)
    rng = random.Random(0x5E1D0000)
    for i in range(60):
        alpha = rng.choice([2, 4, 256])
        n = rng.randint(0, 700)
        basis = bytes(rng.randrange(alpha) for _ in range(n))
        src = mutate(basis, rng)
        bs = rng.choice(list(range(1, 49)) + [64, 100, 241, 256, 300])
        cases.append(delta_case(f"random_{i}_a{alpha}_bs{bs}", src, basis, bs, "SURVEY §4 item 3", chunk=2 * bs + 7))
    # ---- signature of odd lengths across the XXH3 length classes
    for ln in [1, 3, 4, 8, 9, 16, 17, 128, 129, 240, 241, 1023, 1024, 1025, 4095, 4096, 4097]:
        data = bytes(rng.randrange(256) for _ in range(ln))
        cases.append(sig_case(f"sig_len{ln}", data, ln, "xxh3 length classes"))
    meta = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/oracle.py (py_*)",
            "pins": {"adler32": "zlib.adler32", "xxh3_64": f"python-xxhash {xxhash.VERSION} (libxxhash {xxhash.XXHASH_VERSION})"},
            "ops_format": "[kind, a, b]: C = Copy{offset=a,size=b}; D = Data(src[a:a+b])"}
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump({"meta": meta, "cases": cases}, f, indent=0)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
