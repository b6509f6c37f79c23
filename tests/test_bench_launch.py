"""bench.py --gpus N without torchrun starts N ranks (VERDICT r04 missing item 1): the
children's torchrun environment, the forwarded rank-0 line, the per-rank host-thread
share and exit-code propagation, on CPU with a stub worker (SYDELTA_BENCH_STUB: the
child prints its rank environment and exits before importing torch)."""
import json
import os
import subprocess
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(n, extra_env=None, args=()):
    env = dict(os.environ, SYDELTA_BENCH_STUB="1", SYDELTA_BENCH_FAKE_GPUS="8")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "SYDELTA_HOST_THREADS"):
        env.pop(k, None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *args], env=env,
                          capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_starts_n_ranks(n):
    p = run(n)
    assert p.returncode == 0, p.stderr
    out = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    err = [json.loads(ln) for ln in p.stderr.splitlines() if ln.startswith("{")]
    # rank 0's line on stdout, every other rank's on stderr
    assert len(out) == 1 and out[0]["RANK"] == "0"
    ranks = sorted(int(d["RANK"]) for d in out + err)
    assert ranks == list(range(n))
    cores = bench.host_cores()[0]
    for d in out + err:
        assert d["WORLD_SIZE"] == str(n)
        assert d["LOCAL_RANK"] == d["RANK"]
        assert d["MASTER_ADDR"] == "127.0.0.1"
        assert int(d["MASTER_PORT"]) > 0
        assert d["SYDELTA_HOST_THREADS"] == str(max(2, cores // n))
    assert len({d["MASTER_PORT"] for d in out + err}) == 1


def test_launcher_keeps_caller_host_threads():
    p = run(2, {"SYDELTA_HOST_THREADS": "5"})
    assert p.returncode == 0, p.stderr
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert d["SYDELTA_HOST_THREADS"] == "5"


def test_launcher_propagates_failure():
    # rank 1 exits 7 while ranks 0 and 2 would wait 60 s in a collective: the launcher
    # stops them and returns 7 well before that
    p = run(3, {"SYDELTA_BENCH_STUB_FAIL_RANK": "1"})
    assert p.returncode == 7
    assert "rank 1 exited with 7" in p.stderr


def test_launcher_refuses_too_few_gpus():
    p = run(4, {"SYDELTA_BENCH_FAKE_GPUS": "2"})
    assert p.returncode == 2
    assert "2 GPU(s) are visible" in p.stderr
    assert not p.stdout.strip()


def test_one_gpu_and_torchrun_run_in_process():
    # --gpus 1, and --gpus N under torchrun (WORLD_SIZE set): no children
    p = run(1)
    assert p.returncode == 0
    assert json.loads(p.stdout)["RANK"] is None
    p = run(2, {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"})
    assert p.returncode == 0
    assert json.loads(p.stdout)["RANK"] == "1"


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_forwards_rank0_legs(n):
    """The C4 / C5 legs ride on rank 0's line (stub: the legs' objects built by bench.c4_leg /
    c5_leg with fixed timings): forwarded to the launcher's stdout once, aggregated over all
    N ranks (C4: the 10 000 files' bytes per max-rank step; C5: N chunks of 2 x 8 GiB)."""
    p = run(n, {"SYDELTA_BENCH_STUB_LEGS": "1"}, args=("--steps", "4"))
    assert p.returncode == 0, p.stderr
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{") and '"c4"' in ln]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == n
    c4, c5 = d["c4"], d["c5"]
    assert c4["files"] == 10000 and c4["files_this_rank"] == bench.shard_range(10000, n, 0)[1]
    assert c4["ms_per_step"] == 2.0 and c4["scaling"] == "strong"
    assert abs(c4["value"] - 10000 * ((1 << 21) + 1) / 2e-3 / 2**30) < 1e-2
    assert c5["ms_per_step"] == 5.0 and c5["scaling"] == "weak"
    assert abs(c5["value"] - n * 2 * (8 << 30) / 5e-3 / 2**30) < 1e-2
    assert c5["allgather_bytes_per_rank"] == 12 * (1 << 20) * n
