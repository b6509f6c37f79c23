"""CPU tests of the drop-in boundary: libsydelta.so loads, exports every symbol
include/sydelta.h declares, and fails loudly (no CPU fallback) without a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sydelta.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sydelta_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_api():
    syms = header_symbols()
    for s in ["sydelta_compute_checksums", "sydelta_generate_delta_streaming", "sydelta_generate_delta",
              "sydelta_apply_delta", "sydelta_calculate_block_size", "sydelta_signature_device",
              "sydelta_index_create", "sydelta_match_device", "sydelta_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from sy_amd import _lib

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (sydelta_[a-z0-9_]+)", out.stdout))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    # and the ctypes table covers them all
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == header_symbols()


def test_library_is_built_for_gfx950():
    from sy_amd import _lib

    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", _lib.LIB_PATH], capture_output=True, text=True)
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_abi_version_and_block_size():
    import sy_amd.delta as d
    from sy_amd._lib import lib

    assert lib.sydelta_abi_version() == 1
    assert d.calculate_block_size(1024) == 512
    assert d.calculate_block_size(1_000_000) == 1000
    assert d.calculate_block_size(100_000_000) == 10000
    assert d.calculate_block_size(100_000_000_000) == 128 * 1024


def test_adler32_type_matches_reference_semantics():
    import zlib

    import sy_amd.delta as d

    assert d.Adler32.hash(b"") == 1
    assert d.Adler32.hash(b"hello world") == zlib.adler32(b"hello world")
    data = b"The quick brown fox jumps over the lazy dog"
    h = d.Adler32(8)
    h.update_block(data[:8])
    for i in range(1, len(data) - 8 + 1):
        h.roll(data[i - 1], data[i + 7])
        assert h.digest() == zlib.adler32(data[i:i + 8])


def test_invalid_arguments_are_errors_not_crashes():
    import sy_amd.delta as d
    from sy_amd._lib import SyDeltaError

    with pytest.raises(SyDeltaError):
        d.compute_checksums_bytes(b"abc", 0)
    with pytest.raises(SyDeltaError) as e:
        d.compute_checksums("/nonexistent/file", 16)
    assert e.value.code == -5  # SYDELTA_E_IO, like io::Error from File::open
    with pytest.raises(SyDeltaError):
        d.generate_delta_streaming("/nonexistent/file", [], 1 << 20)


def test_empty_inputs_need_no_device(tmp_path):
    import sy_amd.delta as d

    p = tmp_path / "empty"
    p.write_bytes(b"")
    assert d.compute_checksums(p, 1024) == []  # checksum.rs:36-38


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import sy_amd.delta as d
    from sy_amd._lib import SyDeltaError

    with pytest.raises(SyDeltaError) as e:
        d.compute_checksums_bytes(b"abcdef", 4)
    assert e.value.code == -1  # SYDELTA_E_NODEV: no silent CPU fallback
