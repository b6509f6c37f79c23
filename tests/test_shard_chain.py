"""Chunk-sharded walk chaining (sy_amd/shard.py) on CPU with gloo, world 1-4.

A stand-in chunk walks a fixed classification (hit positions -> block) with the
greedy rule of generator.rs:116-197; the chained per-rank op lists joined in rank
order must equal one walk over the whole file, including copies that cross chunk
boundaries (which force the in-order fix-up) and chunks shorter than a block."""
import os
import random
import socket

import pytest
import torch.multiprocessing as mp

from sy_amd import shard


class FakeChunk:
    def __init__(self, hits, n, p0, p1, flen, final):
        self.hits, self.n, self.p0, self.p1, self.flen, self.final = hits, n, p0, p1, flen, final
        self.walks = 0

    def walk(self, entry):
        self.walks += 1
        ops, x, lit = [], entry, entry

        def data(a, b):
            if b > a:
                ops.append(("D", a, b - a))

        while x < self.p1:
            if x in self.hits:
                data(lit, x)
                ops.append(("C", self.hits[x] * self.n, self.n))
                x += self.n
                lit = x
            else:
                x += 1
        if self.final:
            data(lit, self.flen)
            return ops, self.flen
        data(lit, self.p1)
        return ops, max(x, self.p1)


def join(parts):
    out = []
    for p in parts:
        p = list(p)
        if out and p and out[-1][0] == "D" and p[0][0] == "D" and out[-1][1] + out[-1][2] == p[0][1]:
            out[-1] = ("D", out[-1][1], out[-1][2] + p[0][2])
            p = p[1:]
        out += p
    return out


def make_case(seed):
    rng = random.Random(seed)
    n = rng.choice([4, 16, 64])
    flen = rng.randint(n, 60 * n)
    npos = flen - n + 1
    hits = {}
    for k in range(0, npos, n):  # aligned copies, some missing
        if rng.random() < 0.7:
            hits[k] = rng.randrange(100)
    for _ in range(rng.randint(0, 12)):  # unaligned hits (shifted copies)
        hits[rng.randrange(npos)] = rng.randrange(100)
    return n, flen, hits


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, seeds, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gather, bcast = shard.torch_collectives(dist, "cpu")
    out = []
    for seed in seeds:
        n, flen, hits = make_case(seed)
        p0, p1 = shard.chunk_bounds(flen, n, world, rank)
        ch = FakeChunk(hits, n, p0, p1, flen, rank == world - 1)
        ops, entry = shard.walk_chain(ch, rank, world, p0, gather, bcast)
        out.append((seed, entry, ops, ch.walks))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_walk_chain_equals_single_walk(world):
    seeds = list(range(40))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seeds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    refixed = 0
    for i, seed in enumerate(seeds):
        n, flen, hits = make_case(seed)
        whole, _ = FakeChunk(hits, n, 0, flen - n + 1, flen, True).walk(0)
        parts = [res[r][i][2] for r in range(world)]
        assert join(parts) == whole, seed
        entries = [res[r][i][1] for r in range(world)]
        assert entries[0] == 0 and entries == sorted(entries)
        refixed += sum(res[r][i][3] - 1 for r in range(world))
    assert refixed > 0  # some cases needed the in-order fix-up


def test_chunk_bounds_cover_positions():
    for flen, n in [(100, 4), (4096 * 10 + 5, 4096), (3, 4), (4, 4), (17, 16)]:
        npos = max(0, flen - n + 1)
        for world in (1, 2, 3, 8):
            b = [shard.chunk_bounds(flen, n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == npos
            assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
            assert all(x[0] % n == 0 or x[0] == npos for x in b)


def test_walk_chain_single_rank():
    n, flen, hits = make_case(3)
    ch = FakeChunk(hits, n, 0, flen - n + 1, flen, True)
    ops, entry = shard.walk_chain(ch, 0, 1, 0, lambda v: [v], lambda v, s: v)
    assert entry == 0 and ops == FakeChunk(hits, n, 0, flen - n + 1, flen, True).walk(0)[0]
