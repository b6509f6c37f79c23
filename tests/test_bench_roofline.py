"""bench.py's roofline arithmetic on CPU: per-launch algorithmic bytes, the dominant
kernel, and the scan's L2-gather fraction."""
import bench


def test_roofline_scan_l2_gather():
    n = 1 << 32
    algo = bench.algo_bytes_per_step("c3", n, n, n)
    prof = {"k_scan_lds": {"ms": 192.1, "count": 10}, "k_sig_fast": {"ms": 7.0, "count": 10}}
    r = bench.roofline(prof, 10, algo, positions=n - 4095)
    assert r["kernel"] == "k_scan_lds" and r["bound"] == "l2"  # 84 % of the gather ceiling, 28 % of HBM
    assert r["algorithmic_bytes_per_launch"] == n
    assert abs(r["achieved"] - n / 19.21e-3 / 1e9) < 0.01
    assert abs(r["frac"] - r["achieved"] / bench.HBM_PEAK_GBS) < 1e-4
    g = r["l2_gather"]
    assert g["requests_per_launch"] == n - 4095
    assert abs(g["frac"] - (n - 4095) / 19.21e-3 / bench.L2_GATHER_PEAK) < 1e-4


def test_roofline_split_launches_and_no_gather():
    # two scan segments per step: each launch gets half the step's bytes
    algo = bench.algo_bytes_per_step("c3", 1 << 30, 1 << 30, 1 << 30)
    r = bench.roofline({"k_scan_lds": {"ms": 20.0, "count": 4}}, 2, algo, positions=None)
    assert r["algorithmic_bytes_per_launch"] == 1 << 29
    assert "l2_gather" not in r
    # a signature-dominated step carries no L2-gather entry
    r = bench.roofline({"k_sig_fast": {"ms": 7.0, "count": 10}}, 10, algo, positions=1 << 30)
    assert r["kernel"] == "k_sig_fast" and "l2_gather" not in r
    assert bench.roofline({}, 1, algo) is None
    assert bench.roofline({"k_unknown": {"ms": 1.0, "count": 1}}, 1, algo) is None


def test_metric_names_block_size():
    assert bench.metric_for(4096) == bench.METRIC
    assert "64 KiB" in bench.metric_for(65536)


def test_cpu_baselines_run_small():
    """The CPU baselines on small host inputs: cores from the affinity mask, the scan
    against the whole signature, the file-reading signature agreeing with the in-memory
    one, and the C4 worker pool."""
    import numpy as np

    from oracle import oracle as O

    threads, aff, quota = bench.host_cores()
    assert 1 <= threads <= aff
    bs = 4096
    basis = O.synth_bytes(8 << 20, 0x5E1D0002)
    src = basis.copy()
    rng = np.random.default_rng(1)
    m = rng.random(src.size) < 0.05
    src[m] ^= 0x5A
    r = bench.cpu_baseline(basis, src, src.size, bs, scan_bytes=1 << 20, file_bytes=2 << 20)
    assert r["value"] > 0 and r["cores"] == threads and r["affinity_cores"] == aff
    assert r["variants"]["signature_file_per_block_read_gibps"] is not None
    assert "2048 keys" in r["sample"]
    # C4: three 64 KiB pairs packed at 16-byte-aligned offsets
    fs = 64 << 10
    stride = (fs + 1 + 15) & ~15
    hb = np.zeros(3 * stride, np.uint8)
    hn = np.zeros(3 * stride, np.uint8)
    for k in range(3):
        b = O.synth_bytes(fs, 7 + k)
        hb[k * stride:k * stride + fs] = b
        hn[k * stride:k * stride + fs + 1] = np.concatenate([b[:100], [1], b[100:]])
    offs = np.arange(3, dtype=np.uint64) * stride
    files = (offs, np.full(3, fs, np.uint64), offs.copy(), np.full(3, fs + 1, np.uint64))
    c = bench.cpu_c4_baseline(hb, hn, files, bs, workers=2)
    assert c["value"] > 0 and c["cores"] == 2


def test_roofline_scan_r_modelled_requests():
    import math

    n = 1 << 32
    bits = 38400 * 32
    algo = bench.algo_bytes_per_step("c3", n, n, n)
    # 512 Ki keys: the one-hash Bloom level-1
    r = bench.roofline({"k_scan_r": {"ms": 111.7, "count": 10}}, 10, algo, positions=n, keys=1 << 19)
    g = r["l2_gather"]
    assert abs(g["requests_per_position"] - (1 - math.exp(-(1 << 19) / bits))) < 1e-4
    assert g["requests_per_launch"] == int(n * (1 - math.exp(-(1 << 19) / bits)))
    assert "level-1" in g["model"]
    # 1 Mi keys: the ribbon level-1 passes half of the positions
    r = bench.roofline({"k_scan_r": {"ms": 111.7, "count": 10}}, 10, algo, positions=n, keys=1 << 20)
    assert r["l2_gather"]["requests_per_position"] == 0.5 and "ribbon" in r["l2_gather"]["model"]
    assert r["bound"] == "l2"  # the request rate, not HBM, binds it
    # without the key count no request rate is claimed
    r2 = bench.roofline({"k_scan_r": {"ms": 111.7, "count": 10}}, 10, algo, positions=n)
    assert "l2_gather" not in r2 and r2["bound"] == "hbm"


def test_pmc_traffic_only_from_the_same_workload(tmp_path, monkeypatch):
    """PMC bytes are read only from a summary of the same workload and block size; a
    round-1-3 file (no workload field) or another workload's is never borrowed."""
    import json

    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    k = {"kernels": {"k_scan_lds": {"traffic_bytes": 2000, "bytes_per_launch": 1000}}}
    json.dump(k, open(prof / "r03_c3_pmc.json", "w"))
    json.dump(dict(k, workload="c3", block_size=4096), open(prof / "r04a_c3_pmc.json", "w"))
    assert bench.pmc_traffic("k_scan_lds", 500, "c4", 4096) == (None, None)
    assert bench.pmc_traffic("k_scan_lds", 500, "c3", 65536) == (None, None)
    assert bench.pmc_traffic("k_scan_lds", 500, "c3", 4096) == (1000, "profiles/r04a_c3_pmc.json")


def test_cpu_baselines_other_workloads_small():
    """The CPU legs of the zstd, json, xxh3, apply and local workloads on small CPU
    tensors (the bench hands them device tensors; each leg copies to the host first)."""
    import types

    import numpy as np
    import torch

    from oracle import oracle as O

    bs = 4096
    basis = torch.from_numpy(O.synth_bytes(1 << 20, 0x5E1D0005))
    new = basis.clone()
    new[5000] ^= 1
    text = torch.from_numpy(np.frombuffer(b'{"ops":[' + b'{"Copy":{"offset":4096,"size":4096}},' * 4000 + b']}',
                                          np.uint8).copy())
    z = bench.cpu_zstd_baseline(text, sample_bytes=64 << 10)
    assert z["value"] > 0 and "level 3" in z["sample"]
    j = bench.cpu_json_baseline(new, bs)
    dp = bench.cpu_dparse_baseline(new, bs)
    assert dp["value"] > 0 and dp["sample"].startswith("host parser, one Data op of 1 MiB")
    assert j["value"] > 0 and j["cores"] == 1
    offs = np.arange(4, dtype=np.uint64) * np.uint64(1 << 18)
    lens = np.full(4, 1 << 18, np.uint64)
    x = bench.cpu_xxh3_baseline(basis, offs, lens)
    assert x["value"] > 0 and x["sample"].startswith("4 file(s)")
    # a delta rebuilding `new`: blocks 0 and 2.. copied, block 1 literal
    nb = basis.numel() // bs
    kind = [0, 1] + [0] * (nb - 2)
    a = [0, bs] + [k * bs for k in range(2, nb)]
    d = types.SimpleNamespace(kind=kind, a=a, b=[bs] * nb)
    ap = bench.cpu_apply_baseline(basis, new, d, sample_bytes=1 << 20)
    assert ap["value"] > 0 and f"{nb} ops" in ap["sample"]
    lo = bench.cpu_local_baseline(new, basis, 65536, sample_bytes=1 << 20)
    assert lo["value"] > 0
    w = torch.from_numpy(np.arange(256, dtype=np.uint32).view(np.int32))
    s = torch.from_numpy(np.arange(256, dtype=np.uint64).view(np.int64))
    sj = bench.cpu_sigjson_baseline(w, s, bs)
    assert sj["value"] > 0 and sj["sample"].startswith("host writer + host parser (C calls only), 256 entries")
