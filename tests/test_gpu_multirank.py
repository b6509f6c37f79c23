"""The multi-rank data paths for real on one GPU: two fresh
processes, both on cuda:0, gloo for the exchange steps (the signature all-gather and
the walk chain's small gathers go through host tensors).

* C5 (chunk-sharded single file): every rank signs its share of the basis, the
  signature SoA is all-gathered, every rank builds the full index, classifies its chunk
  of window starts (sydelta_chunk_classify) and the walks are chained
  (shard.walk_chain); the per-rank op lists joined in rank order equal the C oracle's
  generate_delta over the whole file (generator.rs:116-221).
* C4 (file split): each rank matches its contiguous share of the files with one
  batched signature + index + match; every file's op list equals the oracle's.

Functional evidence only: both ranks share one GPU, so this says nothing about the
1 -> 8 GPU scaling curve, which stays unmeasured on hardware.
"""
import os
import socket
import traceback

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.late]

BS5 = 8192
CHUNK = 4 << 20  # C5 basis bytes per rank
SEED5 = 0x5E1D0005
NFILES, FSZ, BS4 = 9, 256 << 10, 4096


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _c5_rank(dist, rank, world):
    import torch

    import sy_amd.device as dev
    from sy_amd import shard

    file_len = world * CHUNK
    first = rank * CHUNK
    basis = torch.empty(CHUNK, dtype=torch.uint8, device="cuda")
    dev.synth_fill_range(basis, first, SEED5)
    p0, p1 = shard.chunk_bounds(file_len, BS5, world, rank)
    buf_end = file_len if rank == world - 1 else min(file_len, p1 + BS5 - 1)
    new = torch.empty((buf_end - first + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    src = new[:buf_end - first]
    dev.synth_fill_range(src, first, SEED5)
    dev.synth_mutate_blocks(src, src, first, BS5, SEED5 + 1, 20000)
    w, s = dev.signature(basis, BS5)
    torch.cuda.synchronize()
    # the exchange step: all-gather of the signature SoA (host tensors under gloo)
    W = [torch.empty_like(w.cpu()) for _ in range(world)]
    S = [torch.empty_like(s.cpu()) for _ in range(world)]
    dist.all_gather(W, w.cpu())
    dist.all_gather(S, s.cpu())
    w, s = torch.cat(W).cuda(), torch.cat(S).cuda()
    idx = dev.Index(w, s, BS5, BS5)
    ch = dev.Chunk(idx, new, first, file_len, p0, p1)
    gather, bcast = shard.torch_collectives(dist, "cpu")
    d, entry = shard.walk_chain(ch, rank, world, p0, gather, bcast)
    ch.close()
    idx.close()
    return {"entry": entry, "kind": np.asarray(d.kind).tolist(), "a": np.asarray(d.a, dtype=np.uint64).tolist(),
            "b": np.asarray(d.b, dtype=np.uint64).tolist(), "stats": dict(d.stats)}


def _c4_rank(rank, world):
    import bench
    import sy_amd.device as dev

    lo, hi = bench.shard_range(NFILES, world, rank)
    basis, new, files = bench.c4_files(dev, basis_bytes=FSZ, nfiles=hi - lo, first=lo)
    boff, blen, soff, slen = files
    w, s = dev.signature_batch(basis, boff, blen, BS4)
    nblk = (blen + BS4 - 1) // BS4
    last = blen - (nblk - 1) * BS4
    idx = dev.BatchIndex(w, s, nblk, last, BS4)
    out, _ = dev.match_batch(idx, new, soff, slen)
    idx.close()
    res = []
    for i, d in enumerate(out):
        res.append({"file": lo + i, "basis": basis[int(boff[i]):int(boff[i] + blen[i])].cpu().numpy().tobytes(),
                    "new": new[int(soff[i]):int(soff[i] + slen[i])].cpu().numpy().tobytes(), "ops": d.tuples()})
    return res


def _worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        c5 = _c5_rank(dist, rank, world)
        c4 = _c4_rank(rank, world)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, {"c5": c5, "c4": c4}))
    except Exception:
        q.put((rank, {"error": traceback.format_exc()}))


def test_two_ranks_on_one_gpu(oracle_c):
    import torch.multiprocessing as mp

    from oracle import oracle as O

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    for r in range(world):
        assert "error" not in res[r], res[r]["error"]
        assert procs[r].exitcode == 0
    # C5: joined per-rank op lists == the oracle over the whole file
    file_len = world * CHUNK
    basis = O.synth_bytes(file_len, SEED5)
    new = O.synth_edit_blocks(basis, 0, BS5, SEED5 + 1, 20000)
    ew, es, ez = oracle_c.compute_checksums(basis, BS5, threads=8)
    expect = O.ops_from_arrays(*oracle_c.generate_delta(new, ew, es, ez, BS5))
    joined = []
    for r in range(world):
        part = [("C" if k == 0 else "D", int(a), int(b)) for k, a, b in zip(res[r]["c5"]["kind"], res[r]["c5"]["a"],
                                                                             res[r]["c5"]["b"])]
        if joined and part and joined[-1][0] == "D" and part[0][0] == "D" and sum(joined[-1][1:]) == part[0][1]:
            joined[-1] = ("D", joined[-1][1], joined[-1][2] + part[0][2])
            part = part[1:]
        joined += part
    assert joined == expect
    assert res[0]["c5"]["entry"] == 0 and res[1]["c5"]["entry"] >= CHUNK - BS5
    assert sum(1 for k, _, _ in expect if k == "C") > 100 and any(k == "D" for k, _, _ in expect)
    # C4: every file of both ranks equals the oracle's per-file result
    files = res[0]["c4"] + res[1]["c4"]
    assert [f["file"] for f in files] == list(range(NFILES))
    for f in files:
        b = np.frombuffer(f["basis"], np.uint8)
        w, s, z = oracle_c.compute_checksums(b, BS4)
        assert f["ops"] == O.ops_from_arrays(*oracle_c.generate_delta(np.frombuffer(f["new"], np.uint8), w, s, z,
                                                                       BS4)), f["file"]
