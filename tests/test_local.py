"""Local transport block compare and change-ratio estimate,
CPU side: the oracle restatements pinned by src/delta/ratio.rs's own tests
(:200-325, identical / all changed / 25% / 80% with both thresholds / size
difference / 5 samples) and by the block-compare loop's counting rules
(local.rs:549-619: changed_blocks, literal_bytes, bytes_written)."""
import pytest

from oracle import oracle as O

MiB = 1 << 20
BS = 64 * 1024  # local.rs:384


def _ratio_case(name):
    src = bytearray(b"\x2a" * MiB)
    dst = bytes(b"\x2a" * MiB)
    if name == "all_changed":
        dst = bytes(b"\x63" * MiB)
    elif name == "partial":
        src[:256 * 1024] = b"\x63" * (256 * 1024)
    elif name == "threshold":
        src[:800 * 1024] = b"\x63" * (800 * 1024)
    elif name == "size":
        src = bytearray(b"\x2a" * (2 * MiB))
    return bytes(src), dst


def test_ratio_no_changes():  # ratio.rs:200-215
    r, sampled, changed, use, _ = O.py_estimate_change_ratio(*_ratio_case("same"), BS)
    assert changed == 0 and r == 0.0 and use


def test_ratio_all_changed():  # ratio.rs:218-234
    r, sampled, changed, use, _ = O.py_estimate_change_ratio(*_ratio_case("all_changed"), BS)
    assert changed == sampled and r == 1.0 and not use


def test_ratio_partial():  # ratio.rs:237-262
    r, sampled, changed, use, _ = O.py_estimate_change_ratio(*_ratio_case("partial"), BS)
    assert 0 < changed < sampled and 0.0 < r < 1.0 and use
    assert (sampled, changed) == (16, 4)  # 16 blocks, step 1, blocks 0..3 differ


def test_ratio_threshold():  # ratio.rs:265-289
    src, dst = _ratio_case("threshold")
    assert not O.py_estimate_change_ratio(src, dst, BS)[3]
    assert O.py_estimate_change_ratio(src, dst, BS, threshold=0.90)[3]


def test_ratio_size_difference():  # ratio.rs:292-307
    r, sampled, changed, use, _ = O.py_estimate_change_ratio(*_ratio_case("size"), BS)
    assert not use and (sampled, changed) == (0, 0) and r == 1.0


def test_ratio_small_sample_count():  # ratio.rs:310-325
    r, sampled, changed, use, _ = O.py_estimate_change_ratio(*_ratio_case("same"), BS, sample_count=5)
    assert (sampled, changed, use) == (5, 0, True)


def test_ratio_sample_positions():
    # ratio.rs:127-141: step = total_blocks / (n - 1), clamped to the last block.
    src = bytes(range(256)) * 4000  # 1,024,000 bytes -> 16 blocks (last one short)
    dst = bytearray(src)
    dst[15 * BS] ^= 1  # only the short last block differs
    r, sampled, changed, use, _ = O.py_estimate_change_ratio(src, bytes(dst), BS, sample_count=4)
    # step 16 // 3 = 5 -> blocks 0, 5, 10, 15
    assert (sampled, changed) == (4, 1)
    r, sampled, changed, use, _ = O.py_estimate_change_ratio(src, bytes(dst), BS, sample_count=3)
    # step 8 -> blocks 0, 8, 16 -> 15 (clamped)
    assert (sampled, changed) == (3, 1)


def test_ratio_empty_dest():
    # dest_size 0: size_diff 1.0 -> early return; both empty: also 1.0 (ratio.rs:105-109)
    assert O.py_estimate_change_ratio(b"x", b"", BS)[:3] == (1.0, 0, 0)
    assert O.py_estimate_change_ratio(b"", b"", BS)[:4] == (1.0, 0, 0, False)


@pytest.mark.parametrize("slen,dlen", [(0, 0), (1, 1), (BS, BS), (3 * BS + 7, 3 * BS + 7), (3 * BS + 7, 2 * BS),
                                       (2 * BS, 3 * BS + 5), (BS + 1, 0)])
def test_block_compare_counts(slen, dlen):
    src = bytes((i * 7) & 255 for i in range(slen))
    dst = bytearray(src[:dlen]) + bytes(max(0, dlen - slen))
    if dlen > BS + 10:
        dst[BS + 10] ^= 0xFF
    flags, changed, lit, written = O.py_block_compare(src, bytes(dst), BS)
    nb = -(-slen // BS)
    assert len(flags) == nb and written == slen and changed == sum(flags)
    exp = []
    for k in range(nb):
        s, d = src[k * BS:(k + 1) * BS], bytes(dst[k * BS:(k + 1) * BS])
        exp.append(int(s != d))
    assert flags == exp
    assert lit == sum(min(BS, slen - k * BS) for k in range(nb) if flags[k])


def test_ratio_paths_host_only_cases(tmp_path):
    """The path API's cases decided before any device work (ratio.rs:89-121): a missing
    file is an I/O error, a > 50 % size difference and an empty destination return
    without sampling."""
    import sy_amd._lib as L
    from sy_amd import delta

    ps, pd = tmp_path / "source.bin", tmp_path / "dest.bin"
    ps.write_bytes(b"\x2a" * (2 * MiB))
    with pytest.raises(L.SyDeltaError):
        delta.estimate_change_ratio(ps, tmp_path / "missing.bin", BS)
    with pytest.raises(L.SyDeltaError):
        delta.estimate_change_ratio(tmp_path / "missing.bin", ps, BS)
    pd.write_bytes(b"\x2a" * MiB)
    r = delta.estimate_change_ratio(ps, pd, BS)  # ratio.rs:292-307
    assert (r.change_ratio, r.blocks_sampled, r.blocks_changed, r.use_delta) == (1.0, 0, 0, False)
    assert r.change_ratio_percent() == "100.0%"
    pd.write_bytes(b"")
    r = delta.estimate_change_ratio(ps, pd, BS, threshold=0.9)
    assert (r.change_ratio, r.blocks_sampled, r.use_delta, r.threshold) == (1.0, 0, False, 0.9)
    assert r == delta.ChangeRatioResult(*O.py_estimate_change_ratio(ps.read_bytes(), b"", BS, threshold=0.9))
