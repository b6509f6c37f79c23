"""GPU checks of the drop-in path across devices (VERDICT r03 "what's missing" 1).

* 10 threads call the path API at once (compute_checksums + generate_delta_streaming
  + apply_delta, as sy's --parallel transfers do, sync/mod.rs:672-697): every result
  equals the C oracle's, and the threads' bound devices are spread over the visible
  devices (all on device 0 on a one-GPU box).
* sydelta_delta_multi_device (one file chunk-sharded over devices inside the library,
  the signature slices gathered by peer copies): equal to the oracle's whole-file op list
  on a 64 MiB pair with a shift and planted copies across chunk cuts, and to the
  single-device match on a 1 GiB C5-shaped pair (apply round trip).  On a one-GPU box
  the chunks go to device 0 several times (the peer copies become device copies);
  the multi-GPU peer path is measured only where several GPUs are visible.
"""
import os
import random
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_ten_path_callers_spread_over_devices(tmp_path, oracle_c, gpu):
    import torch

    import sy_amd.delta as D

    ndev = torch.cuda.device_count()
    bs = 4096
    pairs = []
    for k in range(10):
        rng = random.Random(500 + k)
        basis = rng.randbytes((6 << 20) + 977 * k)
        src = bytearray(basis)
        for _ in range(20):
            p = rng.randrange(len(src))
            src[p] ^= 0x5A
        p = rng.randrange(len(src))
        src[p:p] = b"shift"
        pairs.append((basis, bytes(src)))
    bar = threading.Barrier(10)
    devs = [None] * 10

    def one(k):
        basis, src = pairs[k]
        d = tmp_path / f"t{k}"
        d.mkdir()
        pb, ps, po = d / "dest", d / "src", d / "out"
        pb.write_bytes(basis)
        ps.write_bytes(src)
        sigs = D.compute_checksums(pb, bs)
        delta = D.generate_delta_streaming(ps, sigs, bs)
        D.apply_delta(pb, delta, po)
        assert po.read_bytes() == src
        devs[k] = gpu.thread_device()
        bar.wait()  # every caller stays bound until all have run
        w, s, z = oracle_c.compute_checksums(np.frombuffer(basis, np.uint8), bs)
        exp = O.ops_from_arrays(*oracle_c.generate_delta(np.frombuffer(src, np.uint8), w, s, z, bs))
        got = [("C", op.offset, op.size) if isinstance(op, D.Copy) else ("D", len(op.data)) for op in delta.ops]
        assert got == [("C", a, b) if kk == "C" else ("D", b) for kk, a, b in exp], k
        return True

    with ThreadPoolExecutor(10) as ex:
        assert all(ex.map(one, range(10)))
    assert all(0 <= d < ndev for d in devs), devs
    cnt = [devs.count(d) for d in range(ndev)]
    assert max(cnt) - min(cnt) <= 1, cnt  # least-loaded binding
    print(f"path callers per device: {cnt}")


def _chunks(n, k, bs):
    cut = sorted(random.Random(n + k).sample(range(1, n // bs), k - 1)) if k > 1 else []
    return [0] + [c * bs for c in cut]


def _multi(gpu, devices, basis_t, src_t, L, bs):
    import torch

    k = len(devices)
    nb = basis_t.numel()
    bpos = _chunks(nb, k, bs)
    bch = [basis_t[bpos[g]:(bpos[g + 1] if g + 1 < k else nb)].to(f"cuda:{devices[g]}") for g in range(k)]
    npos = L - bs + 1
    spos = _chunks(npos, k, bs)
    sch = []
    for g in range(k):
        end = min(L, spos[g + 1] + bs - 1) if g + 1 < k else L
        t = torch.zeros(end - spos[g] + 16, dtype=torch.uint8, device=f"cuda:{devices[g]}")
        t[:end - spos[g]] = src_t[spos[g]:end].to(t.device)
        sch.append(t[:end - spos[g]])
    torch.cuda.synchronize()
    return gpu.delta_multi_device(devices, bch, sch, spos, L, bs)


@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_multi_device_chunked_match_equals_oracle(k, oracle_c, gpu):
    import torch

    ndev = torch.cuda.device_count()
    devices = [g % ndev for g in range(k)]
    bs = 4096
    rng = np.random.default_rng(k)
    n = 64 << 20
    basis_t = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    gpu.synth_fill(basis_t, 0x5E1D0900 + k)
    basis = basis_t.cpu().numpy()
    parts = [basis[:9 << 20], np.frombuffer(b"xyz", np.uint8), basis[9 << 20:40 << 20]]
    for j in range(30):  # planted copies of random blocks, some across chunk cuts
        b = int(rng.integers(0, n // bs))
        parts += [rng.integers(0, 256, int(rng.integers(1, 3 * bs)), dtype=np.uint8), basis[b * bs:(b + 1) * bs]]
    parts.append(basis[44 << 20:])
    src = np.concatenate(parts)
    src[rng.integers(0, src.size, 200)] ^= 0x21
    L = src.size
    src_t = torch.from_numpy(src).cuda()
    d = _multi(gpu, devices, basis_t, src_t, L, bs)
    ew, es, ez = oracle_c.compute_checksums(basis, bs, threads=8)
    assert d.tuples() == O.ops_from_arrays(*oracle_c.generate_delta(src, ew, es, ez, bs))


def test_multi_device_c5_shape_equals_single_device(gpu):
    """1 GiB, bs 8192, one substituted byte in 1 % of the blocks (the C5 edit model),
    over 4 chunks: equal to the single-device match, and apply rebuilds the source."""
    import torch

    ndev = torch.cuda.device_count()
    devices = [g % ndev for g in range(4)]
    bs = 8192
    n = 1 << 30
    basis_t = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    gpu.synth_fill(basis_t, 0x5E1D0005)
    src_t = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    gpu.synth_mutate_blocks(src_t, basis_t, 0, bs, 0x5E1D0006, 10000)
    torch.cuda.synchronize()
    d = _multi(gpu, devices, basis_t, src_t, n, bs)
    w, s = gpu.signature(basis_t, bs)
    idx = gpu.Index(w, s, bs, bs)
    ref = gpu.match(idx, src_t)
    idx.close()
    assert d.tuples() == ref.tuples()
    assert 0.005 < d.stats["data_ops"] / (n // bs) < 0.02
    out, _ = gpu.apply_device(basis_t, d, src_t)
    assert torch.equal(out[:n], src_t)
