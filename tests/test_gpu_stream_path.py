"""The streamed path API: compute_checksums and
generate_delta_streaming read their file in chunks through pinned double buffers
(sydelta_api.cpp: stream_chunk_bytes, InFile, overlap).

* Parity: with small chunks (SYDELTA_STREAM_CHUNK, so files span many chunks), odd and
  large block sizes (the full-scan path above 8 KiB windows), copies crossing chunk
  boundaries, an insertion that shifts the phase, a short last block and the tail rule:
  checksums equal the C oracle's, op lists equal the oracle's generate_delta and the
  literal bytes rebuild the source (apply_delta).
* Bounded host memory: a child process signs a 2 GiB file and streams a 2 GiB edited
  copy of it through the C ABI (no Python-side op objects); its peak RSS grows by far
  less than the file size over its footprint after a 1 MiB call (the previous
  whole-file read held 2 GiB).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.late]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _case(seed: int, n: int, bs: int):
    rng = np.random.default_rng(seed)
    basis = O.synth_bytes(n, 0x5E1D0300 + seed)
    src = basis.copy()
    for p in rng.integers(0, n, 25):
        src[p] ^= 0x33
    ins = int(rng.integers(n // 3, n // 2))
    src = np.concatenate([src[:ins], rng.integers(0, 256, 7, dtype=np.uint8), src[ins:]])
    # a copied block placed across the first chunk boundary, and the basis's short last
    # block at the end (tail rule)
    k = int(rng.integers(0, n // bs - 1))
    src = np.concatenate([src, basis[k * bs:(k + 1) * bs], basis[(n // bs) * bs:]])
    return basis, src


@pytest.mark.parametrize("chunk", [1 << 20, 3 << 20])
@pytest.mark.parametrize("bs,n", [(4096, (6 << 20) + 1234), (1000 + 7, (5 << 20) + 99), (64, (2 << 20) + 5),
                                  (16384, (7 << 20) + 4321), (131072, (9 << 20) + 17)])
def test_streamed_path_api_matches_oracle(bs, n, chunk, tmp_path, monkeypatch, oracle_c, gpu):
    import sy_amd.delta as D

    monkeypatch.setenv("SYDELTA_STREAM_CHUNK", str(chunk))
    basis, src = _case(bs % 97, n, bs)
    pb, ps, po = tmp_path / "dest", tmp_path / "src", tmp_path / "out"
    basis.tofile(pb)
    src.tofile(ps)
    sigs = D.compute_checksums(pb, bs)
    w, s, z = oracle_c.compute_checksums(basis, bs)
    assert [x.weak for x in sigs] == w.tolist() and [x.strong for x in sigs] == s.tolist()
    assert [x.size for x in sigs] == z.tolist()
    delta = D.generate_delta_streaming(ps, sigs, bs)
    exp = O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs))
    got = [("C", op.offset, op.size) if isinstance(op, D.Copy) else ("D", len(op.data)) for op in delta.ops]
    assert got == [("C", a, b) if k == "C" else ("D", b) for k, a, b in exp]
    D.apply_delta(pb, delta, po)
    assert po.read_bytes() == src.tobytes()
    # the in-memory generator agrees
    assert delta == D.generate_delta(ps, sigs, bs)


@pytest.mark.parametrize("readers", ["1", "3", "16"])
def test_streamed_read_pieces(readers, tmp_path, monkeypatch, oracle_c, gpu):
    """SYDELTA_READ_THREADS (per call): each streamed chunk read in that many pieces by the
    host pool (SYDELTA_READ_PIECE lowers the smallest piece so a 1 MiB chunk splits)."""
    import sy_amd.delta as D

    monkeypatch.setenv("SYDELTA_STREAM_CHUNK", str(1 << 20))
    monkeypatch.setenv("SYDELTA_READ_THREADS", readers)
    monkeypatch.setenv("SYDELTA_READ_PIECE", "65536")
    bs = 4096
    basis, src = _case(int(readers), (3 << 20) + 777, bs)
    pb, ps = tmp_path / "dest", tmp_path / "src"
    basis.tofile(pb)
    src.tofile(ps)
    sigs = D.compute_checksums(pb, bs)
    w, s, z = oracle_c.compute_checksums(basis, bs)
    assert [x.weak for x in sigs] == w.tolist() and [x.strong for x in sigs] == s.tolist()
    delta = D.generate_delta_streaming(ps, sigs, bs)
    exp = O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs))
    got = [("C", op.offset, op.size) if isinstance(op, D.Copy) else ("D", len(op.data)) for op in delta.ops]
    assert got == [("C", a, b) if k == "C" else ("D", b) for k, a, b in exp]


@pytest.mark.parametrize("size", [0, 1, 4095, 4096, 4097])
def test_streamed_small_and_empty_files(size, tmp_path, monkeypatch, oracle_c, gpu):
    import sy_amd.delta as D

    monkeypatch.setenv("SYDELTA_STREAM_CHUNK", "65536")
    bs = 4096
    basis = O.synth_bytes(size, 5)
    pb, ps = tmp_path / "dest", tmp_path / "src"
    basis.tofile(pb)
    basis.tofile(ps)
    sigs = D.compute_checksums(pb, bs)
    assert len(sigs) == -(-size // bs)
    delta = D.generate_delta_streaming(ps, sigs, bs)
    w, s, z = oracle_c.compute_checksums(basis, bs)
    exp = O.ops_from_arrays(*oracle_c.generate_delta(basis, w, s, z, bs))
    got = [("C", op.offset, op.size) if isinstance(op, D.Copy) else ("D", len(op.data)) for op in delta.ops]
    assert got == [("C", a, b) if k == "C" else ("D", b) for k, a, b in exp]


_RSS_CHILD = r"""
import ctypes, resource, sys
sys.path.insert(0, sys.argv[1])
from sy_amd import _lib
from sy_amd._lib import check, lib
bs = 4096
# the runtime's own footprint first: one small call (a 1 MiB file), peak RSS after it
out = ctypes.POINTER(_lib.BlockChecksumC)()
n = ctypes.c_uint64(0)
check(lib.sydelta_compute_checksums(sys.argv[4].encode(), bs, ctypes.byref(out), ctypes.byref(n)))
h = ctypes.c_void_p()
check(lib.sydelta_generate_delta_streaming(sys.argv[4].encode(), out, n.value, bs, ctypes.byref(h)))
lib.sydelta_delta_free(h)
lib.sydelta_checksums_free(ctypes.cast(out, ctypes.c_void_p))
rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
out = ctypes.POINTER(_lib.BlockChecksumC)()
n = ctypes.c_uint64(0)
check(lib.sydelta_compute_checksums(sys.argv[2].encode(), bs, ctypes.byref(out), ctypes.byref(n)))
h = ctypes.c_void_p()
check(lib.sydelta_generate_delta_streaming(sys.argv[3].encode(), out, n.value, bs, ctypes.byref(h)))
st = _lib.MatchStatsC()
check(lib.sydelta_delta_stats(h, ctypes.byref(st)))
print(n.value, lib.sydelta_delta_num_ops(h), st.copy_ops, st.data_ops, st.literal_bytes, rss0,
      resource.getrusage(resource.RUSAGE_SELF).ru_maxrss)
"""


def test_streamed_path_bounded_rss(tmp_path, gpu):
    import shutil

    n = 2 << 30
    if shutil.disk_usage(tmp_path).free < 3 * n:
        pytest.skip(f"needs {3 * n >> 30} GiB free under {tmp_path}")
    pb, ps = tmp_path / "dest", tmp_path / "src"
    piece = 64 << 20
    edits = 0
    with open(pb, "wb") as fb, open(ps, "wb") as fs:
        for i in range(n // piece):
            b = O.synth_bytes(piece, 0x5E1D0400, i * piece)
            fb.write(b.tobytes())
            if i % 8 == 3:  # one substituted byte in every eighth piece
                b = b.copy()
                b[12345] ^= 0x44
                edits += 1
            fs.write(b.tobytes())
    small = tmp_path / "small"
    O.synth_bytes(1 << 20, 7).tofile(small)
    r = subprocess.run([sys.executable, "-c", _RSS_CHILD, ROOT, str(pb), str(ps), str(small)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    nsig, nops, copies, datas, lit, rss0_kib, rss_kib = map(int, r.stdout.split())
    assert nsig == n // 4096
    assert copies == nsig - edits and datas == edits and lit == 4096 * edits
    grew = rss_kib - rss0_kib
    print(f"\npeak RSS {rss_kib >> 10} MiB ({rss0_kib >> 10} MiB after a 1 MiB call, +{grew >> 10} MiB) for a "
          f"2 GiB + 2 GiB streamed path call")
    # two 64 MiB pinned chunks per buffer pair, the checksums (20 MiB) and ops: far below
    # the 2 GiB a whole-file read would hold
    assert grew < (512 << 10), (rss0_kib, rss_kib)
