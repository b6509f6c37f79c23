"""Multi-rank plumbing of bench.py on CPU (gloo, world_size 2 and 3): file shards
cover every unit exactly once with no collective, and the job time is the max
over ranks.  The GPU data path itself has no collective."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, nunits, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = bench.shard_range(nunits, world, rank)
    t = bench.max_over_ranks(float(rank + 1), "cpu")
    q.put((rank, lo, hi, t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,nunits", [(2, 10000), (3, 10000), (2, 1), (3, 7)])
def test_shards_cover_once_and_time_is_max(world, nunits):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nunits, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    covered = []
    for rank, lo, hi, t in res:
        covered.extend(range(lo, hi))
        assert t == float(world)
    assert covered == list(range(nunits))
    sizes = [hi - lo for _, lo, hi, _ in res]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_shard_range_single_process(world):
    got = [bench.shard_range(10000, world, r) for r in range(world)]
    assert got[0][0] == 0 and got[-1][1] == 10000
    assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
