"""Host-side sharding of the delta path over ranks (one process per GPU).

* Independent files (BASELINE C4) shard with no collective: `shard_range`.
* One large file (BASELINE C5) shards by block-aligned chunks of window starts
  (`chunk_bounds`); each rank classifies its chunk against the all-gathered
  signature (sydelta_chunk_classify), then the greedy walks are chained
  (`walk_chain`): chunk g's walk must start where chunk g-1's walk left, which
  after a Copy that crosses the boundary lies inside chunk g.  Every rank first
  walks speculatively from its own first position; one all-gather of the exits
  confirms the chain when every exit lands exactly on the next chunk's start
  (block-aligned copies, the usual case); otherwise the walks from the first
  mismatch on are redone in rank order, one broadcast per hop.  The chained op
  lists joined in rank order equal the single-device result.
"""
from __future__ import annotations


def shard_range(nunits: int, world: int, rank: int):
    """Contiguous, size-balanced share of `nunits` equal units for `rank`."""
    per, extra = divmod(nunits, world)
    lo = rank * per + min(rank, extra)
    return lo, lo + per + (1 if rank < extra else 0)


def chunk_bounds(file_len: int, block_size: int, world: int, rank: int):
    """Window starts [pos_begin, pos_end) of `rank`'s chunk: whole blocks of
    positions, balanced over ranks; the last rank's chunk ends at the last full
    window (and so also owns the tail rule)."""
    npos = file_len - block_size + 1 if file_len >= block_size else 0
    nblk = -(-npos // block_size)
    lo, hi = shard_range(nblk, world, rank)
    pos_begin = min(lo * block_size, npos)
    pos_end = npos if rank == world - 1 else min(hi * block_size, npos)
    return pos_begin, pos_end


def walk_chain(chunk, rank: int, world: int, pos_begin: int, gather, bcast):
    """Chain the per-chunk greedy walks.

    chunk.walk(entry) -> (delta, exit) walks this rank's chunk from `entry`.
    gather(list[int]) -> list[list[int]] all-gathers small int lists over ranks;
    bcast(int, src) -> int broadcasts one int from rank `src`.
    Returns (delta, entry) of this rank: its part of the file's op list, which
    covers [entry, next rank's entry)."""
    delta, ex = chunk.walk(pos_begin)
    rows = gather([pos_begin, ex])
    begins = [r[0] for r in rows]
    exits = [r[1] for r in rows]
    e, entries, bad = 0, [], None
    for g in range(world):
        entries.append(e)
        if e != begins[g]:
            bad = g
            break
        e = exits[g]
    if bad is None:
        return delta, entries[rank]
    # rank order from the first chunk whose true entry differs from its start
    e = entries[bad]
    mine = entries[rank] if rank < bad else None
    for g in range(bad, world):
        if rank == g:
            mine = e
            if e != pos_begin:
                delta, ex = chunk.walk(e)
        e = bcast(ex if rank == g else 0, g)
    return delta, mine


def torch_collectives(dist, device):
    """gather/bcast callables for walk_chain over an initialised torch.distributed
    group (RCCL tensors on `device`, or gloo on CPU)."""
    import torch

    world = dist.get_world_size()

    def gather(vals):
        t = torch.tensor(vals, dtype=torch.int64, device=device)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return [[int(x) for x in o.tolist()] for o in out]

    def bcast(v, src):
        t = torch.tensor([v], dtype=torch.int64, device=device)
        dist.broadcast(t, src=src)
        return int(t.item())

    return gather, bcast
