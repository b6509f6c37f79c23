"""Re-entrancy: the C ABI called from many host threads at once,
as sy's sender does with up to 10 concurrent file transfers (cli.rs:178-180, each a
compute_checksums + generate_delta_streaming pair, ssh.rs:913 / sync/mod.rs:673-697).

* 10 threads, each on its own file pair: compute_checksums(dest) then
  generate_delta_streaming(source); every op list equals the C oracle's and
  apply_delta rebuilds the source.
* 10 threads on the device API (signature, Index, match, index free) over distinct
  device buffers, repeated, against the oracle.

Python threads release the GIL inside ctypes calls, so the library sees real
concurrency: per-thread streams and error state, the shared host pool, the op-array
pool and stream-ordered index allocations."""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.late]

NT = 10


def _pair(k: int, n: int, bs: int):
    basis = O.synth_bytes(n, 0x5E1D0200 + k)
    src = basis.copy()
    rng = np.random.default_rng(k)
    for p in rng.integers(0, n, 30):  # sparse byte edits
        src[p] ^= 0x5A
    ins = int(rng.integers(0, n))  # and one insertion (unaligned copies after it)
    src = np.concatenate([src[:ins], np.frombuffer(b"inserted", np.uint8), src[ins:]])
    return basis, src


def _tuples(delta, D):
    return [("C", op.offset, op.size) if isinstance(op, D.Copy) else ("D", len(op.data)) for op in delta.ops]


def test_ten_threads_path_api(tmp_path, oracle_c, gpu):
    import sy_amd.delta as D

    bs, n = 4096, 6 << 20
    pairs = [_pair(k, n + 977 * k, bs) for k in range(NT)]
    paths = []
    for k, (basis, src) in enumerate(pairs):
        pb, ps = tmp_path / f"dest{k}", tmp_path / f"src{k}"
        basis.tofile(pb)
        src.tofile(ps)
        paths.append((pb, ps))

    def one(k):
        pb, ps = paths[k]
        sigs = D.compute_checksums(pb, bs)
        return sigs, D.generate_delta_streaming(ps, sigs, bs)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(NT) as ex:
        res = list(ex.map(one, range(NT)))
    dt = time.perf_counter() - t0
    nbytes = sum(b.size + s.size for b, s in pairs)
    print(f"\n{NT} concurrent callers: {nbytes / dt / 2**30:.2f} GiB/s aggregate (files on page cache)")
    for k, (sigs, delta) in enumerate(res):
        basis, src = pairs[k]
        w, s, z = oracle_c.compute_checksums(basis, bs)
        assert [x.weak for x in sigs] == w.tolist() and [x.strong for x in sigs] == s.tolist()
        exp = [("C", a, b) if kk == "C" else ("D", b) for kk, a, b in
               O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs))]
        assert _tuples(delta, D) == exp, k
        out = tmp_path / f"out{k}"
        D.apply_delta(paths[k][0], delta, out)
        assert out.read_bytes() == src.tobytes()


def test_ten_threads_device_api(oracle_c, gpu):
    import torch

    bs = 4096
    sizes = [(3 << 20) + 4096 * k + 13 * k for k in range(NT)]
    pairs = [_pair(100 + k, sizes[k], bs) for k in range(NT)]
    dev = [(torch.from_numpy(b).cuda(), torch.from_numpy(s).cuda()) for b, s in pairs]
    torch.cuda.synchronize()
    expect = []
    for basis, src in pairs:
        w, s, z = oracle_c.compute_checksums(basis, bs)
        expect.append(O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs)))

    def one(k):
        b, s = dev[k]
        out = []
        for _ in range(3):
            w, st = gpu.signature(b, bs)
            nb = w.numel()
            idx = gpu.Index(w, st, bs, b.numel() - (nb - 1) * bs)
            d = gpu.match(idx, s)
            idx.close()
            out.append(d.tuples())
        return out

    with ThreadPoolExecutor(NT) as ex:
        res = list(ex.map(one, range(NT)))
    for k in range(NT):
        for got in res[k]:
            assert got == expect[k], k
