"""bench.py — device-resident delta signature + rolling match on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4]

One *step* = one pass of sy's delta hot path over one batch of synthetic input
already resident in HBM:
  c3 (default, BASELINE config 3): signature of a 4 GiB basis (bs 4096) + probe-table
     build + greedy rolling match of a 4 GiB source carrying Bernoulli(5%) byte
     substitutions -> op list on the host.  Algorithmic bytes = 4 GiB + 4 GiB.
  c2 (config 2): signature only over 4 GiB.
  c4 (config 4 shape): batch of 1 MiB files (signature + per-file match).
Multi-GPU (torchrun, one rank per GPU): every rank processes its own independent
pair (file-sharded, no data-path collective) -> "scaling": "weak"; value = total
bytes of all ranks / max-over-ranks time.

The JSON line carries `roofline` for the dominant kernel (per-launch HIP-event
time measured inside the timed region, algorithmic bytes per launch, HBM peak
8 TB/s) and `cpu_baseline` (the oracle restatement of sy's CPU path, timed on a
bounded sample on this host; rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "GiB/s device-resident delta signature+match, 4 KiB blocks; % HBM-read peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=["c3", "c2", "c4"])
    ap.add_argument("--size-gib", type=float, default=4.0)
    ap.add_argument("--block-size", type=int, default=4096)
    ap.add_argument("--basis-mib", type=int, default=0,
                    help="c3 only: sign just the first M MiB of the basis (smaller index; "
                         "exercises the LDS-resident filter); 0 = the whole basis")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(bs: int):
    """sy's CPU delta path restated in C (oracle/, 'port'): rayon-style parallel
    signature on `threads` cores + single-threaded greedy scan, on a bounded sample
    of the C3 workload; returns GiB/s for the full (sig + match) byte count."""
    import numpy as np

    from oracle import oracle as O

    C = O.C()
    threads = int(os.environ.get("SYDELTA_CPU_THREADS", "16"))
    sig_n, scan_n = 512 << 20, 64 << 20
    basis = O.synth_bytes(sig_n, 0x5E1D0002)
    t0 = time.perf_counter()
    w, s, z = C.compute_checksums(basis, bs, threads=threads)
    t_sig = time.perf_counter() - t0
    # scan sample: source = basis prefix with 5% byte substitutions, probed against
    # the signature of that prefix (same per-position work as the full scan)
    rng = np.random.default_rng(0x5E1D0003)
    src = basis[:scan_n].copy()
    m = rng.random(scan_n) < 0.05
    src[m] ^= rng.integers(1, 256, int(m.sum()), dtype=np.uint8)
    nb = scan_n // bs
    t0 = time.perf_counter()
    C.generate_delta(src, w[:nb], s[:nb], z[:nb], bs)
    t_scan = time.perf_counter() - t0
    sig_rate = sig_n / t_sig          # bytes/s, `threads` threads
    scan_rate = scan_n / t_scan       # bytes/s, 1 thread (generator.rs is sequential)
    full = 4 * GIB
    t_full = full / sig_rate + full / scan_rate
    return {
        "value": round(2 * full / t_full / GIB, 5),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"signature of {sig_n >> 20} MiB on {threads} threads ({sig_rate / GIB:.3f} GiB/s) + "
                   f"single-thread rolling scan of {scan_n >> 20} MiB with 5% byte edits "
                   f"({scan_rate / 2**20:.2f} MiB/s); extrapolated to 4 GiB + 4 GiB"),
    }


def pmc_traffic(kernel: str, per_launch: int):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this
    round (profiles/*_pmc.json, written by scripts/pmc_summary.py from FETCH_SIZE and
    WRITE_SIZE passes of this same bench command), scaled to this launch's size."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        for k, v in d.get("kernels", {}).items():
            if k == kernel and "traffic_bytes" in v and v.get("bytes_per_launch"):
                best = v["traffic_bytes"] * per_launch / v["bytes_per_launch"]
    return int(best) if best else None


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import sy_amd.device as dev

    bs = args.block_size
    n = int(args.size_gib * GIB) // bs * bs
    seed_base = 0x5E1D0002 + 0x1000 * rank

    nb_bytes = min(n, (args.basis_mib << 20) // bs * bs) if args.basis_mib else n
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev.synth_fill(basis, seed_base)
    new = None
    files = None
    if args.workload in ("c3",):
        new = torch.empty(n, dtype=torch.uint8, device="cuda")
        dev.synth_mutate(new, basis, seed_base + 1, 50000)
    if args.workload == "c4":
        fsz = 1 << 20
        nfiles = n // fsz
        new = torch.empty(n, dtype=torch.uint8, device="cuda")
        dev.synth_mutate(new, basis, seed_base + 1, 16)  # ~16 substitutions per MiB file
        files = (np.arange(nfiles, dtype=np.uint64) * fsz, np.full(nfiles, fsz, np.uint64))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()

    def step():
        if args.workload == "c2":
            dev.signature(basis, bs, stream=stream)
            return None
        if args.workload == "c3":
            w, s = dev.signature(basis[:nb_bytes], bs, stream=stream)
            idx = dev.Index(w, s, bs, bs, device=local, stream=stream)
            d = dev.match(idx, new, stream=stream)
            idx.close()
            return d
        # c4: batched signature of all basis files, then one match per file
        offs, lens = files
        w, s = dev.signature_batch(basis, offs, lens, bs, stream=stream)
        per = (1 << 20) // bs
        last = None
        for f in range(len(lens)):
            idx = dev.Index(w[f * per:(f + 1) * per], s[f * per:(f + 1) * per], bs, bs, device=local, stream=stream)
            last = dev.match(idx, new[f << 20:(f + 1) << 20], stream=stream)
            idx.close()
        return last

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dev.set_profiling(True)
    dev.profile(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    dev.set_profiling(False)
    prof = dev.profile(reset=True)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    bytes_per_step = n if args.workload == "c2" else (nb_bytes + n if args.workload == "c3" else 2 * n)
    total_bytes = bytes_per_step * args.steps * world
    value = total_bytes / elapsed / GIB
    ms_per_step = elapsed / args.steps * 1e3

    # roofline of the dominant kernel: algorithmic bytes per launch / avg launch time.
    # Per step the signature kernels read the basis once and the scan reads the source
    # once; a kernel launched L times per step gets 1/L of that per launch (the scan is
    # split into segments of 2^31 positions).
    algo_step = {"k_scan": n, "k_scan_lds": n, "k_sig_fast": nb_bytes if args.workload == "c3" else n, "k_sig_batch": n,
                 "k_sig_wave": n}
    dom = max(prof, key=lambda k: prof[k]["ms"]) if prof else None
    roof = None
    if dom and dom in algo_step:
        launches_per_step = prof[dom]["count"] / args.steps
        avg_ms = prof[dom]["ms"] / max(1, prof[dom]["count"])
        per_launch = int(algo_step[dom] / launches_per_step)
        ach = per_launch / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(dom, per_launch),
                "kernel": dom, "avg_launch_ms": round(avg_ms, 4), "algorithmic_bytes_per_launch": per_launch}
    kernels = {k: {"avg_ms": round(v["ms"] / max(1, v["count"]), 4), "launches": v["count"]} for k, v in prof.items()}

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.workload == "c3":
            cpu = cpu_baseline(bs)
        sig_ms = kernels.get("k_sig_fast", {}).get("avg_ms")
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (counter-based splitmix64 bytes; Bernoulli byte substitutions)",
            "config": {
                "workload": {
                    "c3": "C3: signature(4 GiB basis) + rolling match(4 GiB source, 5% random byte edits), bs 4096",
                    "c2": "C2: signature only over 4 GiB, bs 4096",
                    "c4": "C4 shape: 1 MiB files (batched signature + per-file match)",
                }[args.workload],
                "block_size": bs,
                "basis_bytes": nb_bytes if args.workload == "c3" else n,
                "bytes_per_rank_per_step": bytes_per_step,
                "parallelism": f"file-sharded x{world} (independent pairs per rank, no collective)",
            },
            "pct_hbm_peak": round(value * GIB / 1e9 / HBM_PEAK_GBS * 100, 2),
            "roofline": roof,
            "cpu_baseline": cpu,
            "kernels": kernels,
            "signature_only_gibps": round(n / (sig_ms * 1e-3) / GIB, 2) if sig_ms else None,
            "match_stats": last.stats if last is not None else None,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
