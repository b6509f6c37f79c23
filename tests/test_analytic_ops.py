"""The closed-form C5 op list (tests/analytic_ops.py) equals the C oracle's greedy walk on
small files of the same edit model, so the full-size GPU test can assert the whole 64 GiB
op list against it."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.analytic_ops import block_edit_ops, edited_blocks


@pytest.mark.parametrize("bs,nblocks,ppm,seed", [(8192, 600, 10000, 0x5E1D0006), (512, 4000, 150000, 7),
                                                  (1024, 3000, 400000, 11)])
def test_block_edit_ops_match_oracle(oracle_c, bs, nblocks, ppm, seed):
    basis = O.synth_bytes(nblocks * bs, 0x5E1D0005)
    src = O.synth_edit_blocks(basis, 0, bs, seed, ppm)
    ed = edited_blocks(nblocks, seed, ppm)
    assert ed.any() and (ed[1:] & ed[:-1]).any() or ppm < 100000  # runs of edited blocks where the rate allows
    w, s, z = oracle_c.compute_checksums(basis, bs)
    kind, a, b = oracle_c.generate_delta(src, w, s, z, bs)
    ek, ea, eb = block_edit_ops(ed, bs)
    assert np.array_equal(np.asarray(kind, np.uint8), ek)
    assert np.array_equal(np.asarray(a, np.uint64), ea)
    assert np.array_equal(np.asarray(b, np.uint64), eb)
