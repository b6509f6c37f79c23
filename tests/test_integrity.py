"""Whole-file XXH3-64, CPU side: the oracle's streamed
hash_file (integrity/xxhash3.rs:17-33, 1 MiB updates) equals the one-shot hash_data
(:36-38) at every length class of XXH3 (0, 1-3, 4-8, 9-16, 17-128, 129-240, and the
long path around stripe/block/chunk edges), the spec KAT for the empty input, and the
reference's own tests (:50-108: non-zero, deterministic, different inputs differ)."""
import random

import pytest

from oracle import oracle as O

SIZES = [0, 1, 3, 4, 8, 9, 16, 17, 128, 129, 240, 241, 255, 256, 1023, 1024, 1025, 1087, 1088, 1089, 2048, 4096,
         (1 << 20) - 1, 1 << 20, (1 << 20) + 1, (3 << 20) + 777]


@pytest.mark.parametrize("n", SIZES)
def test_streamed_equals_one_shot(n):
    data = random.Random(n).randbytes(n)
    assert O.py_hash_file(data) == O.py_xxh3(data)


def test_kat_empty():
    assert O.py_hash_file(b"") == 0x2D06800538D394C2


def test_reference_unit_tests():
    assert O.py_xxh3(b"Hello, xxHash3!") != 0  # xxhash3.rs:50-55
    assert O.py_xxh3(b"Test data") == O.py_xxh3(b"Test data")  # :58-63
    assert O.py_xxh3(b"Data 1") != O.py_xxh3(b"Data 2")  # :66-71
    c = b"File content for xxHash3"  # :74-85: file hash == data hash
    assert O.py_hash_file(c) == O.py_xxh3(c)
