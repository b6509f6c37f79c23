"""bench.py's roofline arithmetic on CPU: per-launch algorithmic bytes, the dominant
kernel, and the scan's L2-gather fraction."""
import bench


def test_roofline_scan_l2_gather():
    n = 1 << 32
    algo = bench.algo_bytes_per_step("c3", n, n, n)
    prof = {"k_scan_lds": {"ms": 192.1, "count": 10}, "k_sig_fast": {"ms": 7.0, "count": 10}}
    r = bench.roofline(prof, 10, algo, positions=n - 4095)
    assert r["kernel"] == "k_scan_lds" and r["bound"] == "hbm"
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
