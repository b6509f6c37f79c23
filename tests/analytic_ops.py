"""The op list of the C5 edit model in closed form (test infrastructure).

sydelta_synth_mutate_blocks (mirrored by oracle.synth_edit_blocks) substitutes one byte
in each selected block of a block-aligned file of random bytes.  The greedy walk
(generator.rs:116-221) then copies every clean block from its own aligned window and emits
each maximal run of edited blocks as one Data op: an edited block's window misses, no
window straddling it matches (random 8 KiB blocks share no weak + strong pair), and the
next clean block's aligned window matches itself.  tests/test_analytic_ops.py pins this
against the C oracle on small files."""
import numpy as np

from oracle import oracle as O


def edited_blocks(nblocks: int, seed: int, rate_ppm: int, first_block: int = 0) -> np.ndarray:
    k = np.arange(first_block, first_block + nblocks, dtype=np.uint64)
    return (O.splitmix_words(k, seed) & np.uint64(0xFFFFFFFF)) < np.uint64((rate_ppm << 32) // 1000000)


def block_edit_ops(edited: np.ndarray, bs: int):
    """(kind u8, a u64, b u64) of the walk over blocks with the given edited flags
    (kind 0 = Copy{a = offset, b = size}, 1 = Data{a = source offset, b = length})."""
    nblocks = edited.size
    prev = np.concatenate([[False], edited[:-1]])
    sb = np.nonzero(~edited | ~prev)[0]  # a Copy, or the first block of a run of edited blocks
    clean = np.nonzero(~edited)[0]
    j = np.searchsorted(clean, sb)  # the first clean block at or after each start
    run_end = np.where(j < clean.size, clean[np.minimum(j, max(clean.size - 1, 0))] if clean.size else nblocks,
                       nblocks)
    kind = np.where(edited[sb], 1, 0).astype(np.uint8)
    a = sb.astype(np.uint64) * np.uint64(bs)
    b = np.where(edited[sb], (run_end - sb) * bs, bs).astype(np.uint64)
    return kind, a, b
