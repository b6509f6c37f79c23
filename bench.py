"""bench.py — device-resident delta signature + rolling match on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]

One *step* = one pass of sy's delta hot path over one batch of synthetic input
already resident in HBM:
  c3 (default, BASELINE config 3): signature of a 4 GiB basis (bs 4096) + probe-table
     build + greedy rolling match of a 4 GiB source carrying Bernoulli(5%) byte
     substitutions -> op list on the host.  Algorithmic bytes = 4 GiB + 4 GiB.
  c3b (BASELINE C3's variant): the same 4 GiB basis; the source has one
     substituted byte in 5% of its 4 KiB blocks and a 1-byte insertion in 1% of them
     (every insertion shifts what follows: unaligned copies, probe + scans).
  c2 (config 2): signature only over 4 GiB.
  c4 (config 4 shape): batch of 1 MiB files (signature + per-file match).
  apply: apply_delta on the device for the C5-shaped pair of
     one rank (8 GiB, 1% edited 8 KiB blocks): Copy ops gathered from the basis, Data
     ops from the source; value = reconstructed GiB/s.
  json: serde_json text of the C3 delta (one 4 GiB literal run,
     ~3.6 characters per byte) written on the device; value = delta source GiB/s;
     cpu_baseline = the same text from libsydelta's host writer on a 256 MiB sample.
  sigjson (sy-remote.rs:146-147, ssh.rs:967-973): serde_json text of
     the C2 signature (4 GiB basis, 1 Mi entries) written on the device (the remote's
     side) and parsed back on the device (the sender's side); value = basis GiB/s
     covered; cpu_baseline = libsydelta's host writer + host parser on the same signature.
  dparse (sy-remote.rs:175): the receiver's parse of that JSON text
     on the device (literal bytes into HBM + the op list); value = literal GiB/s;
     cpu_baseline = libsydelta's host parser on a 256 MiB-literal sample.
  zstd (ssh.rs:1009-1017): the zstd frame of that JSON text (1 GiB
     source by default, ~3.6 GiB of text) on the device; value = text GiB/s;
     cpu_baseline = libzstd level 3 (compress/mod.rs:71-76) on one thread, 64 MiB sample.
  c5 (config 5): ONE file of N x 8 GiB (64 GiB at 8 GPUs), bs 8192, 1% of blocks
     with one substituted byte; chunk-sharded: each rank signs its 8 GiB of the
     basis, RCCL all-gathers the signature, builds the full index, classifies its
     8 GiB of the source and the walks are chained (sy_amd/shard.py).
  path: the drop-in path API on page-cache-warm files (host-inclusive): per step
     sydelta_compute_checksums(basis file) + sydelta_generate_delta_streaming(source
     file), both streaming their file through pinned double buffers; 1 GiB files,
     1% of blocks with one substituted byte; value = (basis + source bytes) / time.
Multi-GPU (torchrun, one rank per GPU): c3 -- every rank processes its own
independent pair (file-sharded, no data-path collective); c4 -- the files are
split over ranks; c5 -- chunks of one file.  value = total bytes of all ranks /
max-over-ranks time.

The JSON line carries `roofline` for the dominant kernel (per-launch HIP-event
time measured inside the timed region, algorithmic bytes per launch, HBM peak
8 TB/s) and `cpu_baseline` (the oracle restatement of sy's CPU path, timed on a
bounded sample on this host; rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "GiB/s device-resident delta signature+match, 4 KiB blocks; % HBM-read peak"
# Random 4/8-byte gathers from an L2-resident table, chip-wide, whatever their width or
# cache policy (profiles/r02_micro_gather2.txt: 262-281 G/s): the ceiling of a scan that
# sends one request per window start to L2.
L2_GATHER_PEAK = 265e9


def metric_for(bs: int) -> str:
    """BASELINE.json's metric, with the block size the run actually used."""
    return METRIC if bs == 4096 else METRIC.replace("4 KiB", f"{bs / 1024:g} KiB")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3",
                    choices=["c3", "c3b", "c2", "c4", "c5", "apply", "json", "dparse", "sigjson", "zstd", "local", "xxh3", "path"])
    ap.add_argument("--size-gib", type=float, default=None,
                    help="bytes per rank: c2/c3 basis and source (default 4), c5 chunk (default 8)")
    ap.add_argument("--block-size", type=int, default=None, help="default 4096 (c5: 8192)")
    ap.add_argument("--edit-ppm", type=int, default=None,
                    help="c3: byte substitution rate (default 50000 = 5%%); c5: edited-block rate (default 10000)")
    ap.add_argument("--basis-mib", type=int, default=0,
                    help="c3 only: sign just the first M MiB of the basis (smaller index; "
                         "exercises the LDS-resident filter); 0 = the whole basis")
    ap.add_argument("--files", type=int, default=None,
                    help="c4: total 1 MiB files over all ranks (10000); xxh3: files per rank (4096; 1 = one file of "
                         "--size-gib)")
    ap.add_argument("--callers", type=int, default=1,
                    help="c4: split this rank's files over K host threads, each one batched call on its own "
                         "library stream (sy runs up to 10 transfers at once, cli.rs:178-180), so one call's "
                         "host work overlaps another's kernels")
    ap.add_argument("--c4-calls", default="pairs", choices=["pairs", "three"],
                    help="c4 (and the c4 leg): one sydelta_delta_pairs_device call per batch (signature + match, "
                         "the signature of the second half beside the walks of the first, no index), or the three "
                         "calls signature_batch + index_create_batch + match_batch")
    ap.add_argument("--device-walk", action="store_true",
                    help="resolve the greedy walks on the device (K5b, SYDELTA_DEVICE_WALK=1; c4/c5/path)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--no-legs", action="store_true",
                    help="c3: skip the C4 and C5 legs that follow the headline (their objects in the line)")
    ap.add_argument("--proxy-world", type=int, default=0,
                    help="c5 on one GPU: time rank --proxy-rank of a W-rank job (the other ranks' signatures "
                         "precomputed and concatenated in place of the all-gather; index over all W chunks' keys)")
    ap.add_argument("--proxy-rank", type=int, default=0)
    a = ap.parse_args()
    if a.device_walk:
        os.environ["SYDELTA_DEVICE_WALK"] = "1"
    if a.size_gib is None:
        a.size_gib = 8.0 if a.workload in ("c5", "apply", "local") else 1.0 if a.workload in ("path", "zstd") else 4.0
    if a.files is None:
        a.files = 4096 if a.workload == "xxh3" else 10000
    if a.block_size is None:
        a.block_size = {"c5": 8192, "apply": 8192, "local": 65536}.get(a.workload, 4096)
    if a.edit_ppm is None:
        a.edit_ppm = 10000 if a.workload in ("c5", "apply", "local", "path") else 50000
    return a


def host_cores():
    """Host threads a CPU baseline may use: the affinity mask (os.sched_getaffinity),
    capped by the cgroup CPU quota when one is set (the GPU box gives a job a share of
    a large host: nproc and the mask show every core there).  Returns (threads,
    affinity count, quota or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline(basis, src, src_len: int, bs: int, scan_bytes: int = 256 << 20, file_bytes: int = 512 << 20):
    """sy's CPU delta path restated in C (oracle/, 'port') on the C3 pair itself (host
    copies of the device inputs): the signature of the WHOLE basis on the host's cores
    (checksum.rs:31-80, rayon over blocks), then the single-threaded greedy scan
    (generator.rs:116-221) of the first `scan_bytes` of the source (`src` holds at least
    that prefix) against that full signature (1 Mi keys at 4 GiB), extrapolated to the
    whole source of `src_len` bytes.  Variants: the
    per-block open/seek/read signature of checksum.rs:50-59 on a page-cache-warm file of
    `file_bytes` of the basis."""
    import tempfile

    import numpy as np

    from oracle import oracle as O

    C = O.C()
    threads, aff, quota = host_cores()
    t0 = time.perf_counter()
    w, s, z = C.compute_checksums(basis, bs, threads=threads)
    t_sig = time.perf_counter() - t0
    scan_n = min(scan_bytes, src.size)
    t0 = time.perf_counter()
    C.generate_delta(src[:scan_n], w, s, z, bs)
    t_scan = time.perf_counter() - t0
    sig_rate = basis.size / t_sig    # bytes/s, `threads` threads
    scan_rate = scan_n / t_scan      # bytes/s, 1 thread (generator.rs is sequential)
    t_full = basis.size / sig_rate + src_len / scan_rate
    # the file-reading signature (open + seek + read per block, each worker its own fd)
    fb = min(file_bytes, basis.size) // bs * bs
    file_rate = None
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp"), delete=True) as f:
        basis[:fb].tofile(f.name)
        nb = fb // bs
        fw = np.zeros(max(nb, 1), np.uint32)
        fs = np.zeros(max(nb, 1), np.uint64)
        C.L.oracle_compute_checksums_file(f.name.encode(), bs, fw.ctypes.data, fs.ctypes.data, nb, threads)  # warm
        t0 = time.perf_counter()
        got = C.L.oracle_compute_checksums_file(f.name.encode(), bs, fw.ctypes.data, fs.ctypes.data, nb, threads)
        dt = time.perf_counter() - t0
        if got == nb and np.array_equal(fw[:nb], w[:nb]):
            file_rate = fb / dt
    return {
        "value": round((basis.size + src_len) / t_full / GIB, 5),
        "unit": "GiB/s",
        "cores": threads,
        "affinity_cores": aff,
        "cgroup_quota_cores": quota,
        "kind": "port",
        "sample": (f"signature of the whole {basis.size / GIB:g} GiB basis on {threads} threads "
                   f"({sig_rate / GIB:.3f} GiB/s, {w.size} keys) + single-thread rolling scan of the first "
                   f"{scan_n >> 20} MiB of the source against it ({scan_rate / 2**20:.2f} MiB/s); "
                   f"scan extrapolated to the whole source"),
        "variants": {
            "signature_file_per_block_read_gibps": round(file_rate / GIB, 3) if file_rate else None,
            "signature_file_sample_mib": fb >> 20,
            "signature_in_memory_gibps": round(sig_rate / GIB, 3),
            "scan_single_thread_mibps": round(scan_rate / 2**20, 2),
        },
    }


def cpu_c4_baseline(basis, new, files, bs: int, workers: int = 10, sample_files: int = 500):
    """C4 on the host the way sy runs it: up to `workers` file transfers at once
    (cli.rs:178-180, --parallel default 10), each one compute_checksums of its basis +
    the sequential scan of its new file (the C oracle, which releases the GIL), over
    the first `sample_files` files; bytes = basis + new bytes of those files."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O

    C = O.C()
    boff, blen, soff, slen = files
    k = min(sample_files, len(boff))
    hb = [basis[int(boff[i]):int(boff[i] + blen[i])] for i in range(k)]
    hn = [new[int(soff[i]):int(soff[i] + slen[i])] for i in range(k)]

    def one(i):
        w, s, z = C.compute_checksums(hb[i], bs)
        C.generate_delta(hn[i], w, s, z, bs)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(one, range(k)))
    dt = time.perf_counter() - t0
    nbytes = int(blen[:k].sum() + slen[:k].sum())
    return {"value": round(nbytes / dt / GIB, 4), "unit": "GiB/s", "cores": workers, "kind": "port",
            "sample": f"{k} file pairs ({nbytes >> 20} MiB) on {workers} concurrent transfers (C oracle)"}


def cpu_json_baseline(src_dev, bs: int):
    """libsydelta's host serde_json writer (one thread) on a 256 MiB literal sample of
    the same source: the text sy's sender builds with serde_json::to_string(&delta)."""
    from sy_amd import wire

    sample = src_dev[:256 << 20].cpu().numpy()
    t0 = time.perf_counter()
    text = wire.delta_to_json([1], [0], [sample.size], sample.size, bs, sample)
    dt = time.perf_counter() - t0
    return {"value": round(sample.size / dt / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"host writer, one Data op of {sample.size >> 20} MiB ({len(text) >> 20} MiB of text)"}


def cpu_sigjson_baseline(w_dev, s_dev, bs: int):
    """libsydelta's host serde_json writer (sydelta_checksums_to_json, one thread) on the
    same signature: what sy-remote does after compute_checksums (sy-remote.rs:146-147)."""
    import numpy as np

    from sy_amd import wire

    w = w_dev.cpu().numpy().view(np.uint32)
    s = s_dev.cpu().numpy().view(np.uint64)
    idx = np.arange(w.size, dtype=np.uint64)
    sig = wire.sig_array(idx, idx * np.uint64(bs), np.full(w.size, bs, np.uint64), w, s)
    import ctypes

    from sy_amd._lib import BlockChecksumC, check, lib

    # the two C calls alone (no Python buffer handling in the timed region)
    n = lib.sydelta_checksums_to_json(sig.ctypes.data, w.size, None, 0)
    buf = np.empty(n, np.uint8)
    t0 = time.perf_counter()
    lib.sydelta_checksums_to_json(sig.ctypes.data, w.size, buf.ctypes.data, n)
    t_write = time.perf_counter() - t0
    out = ctypes.POINTER(BlockChecksumC)()
    cnt = ctypes.c_uint64()
    t0 = time.perf_counter()
    check(lib.sydelta_checksums_from_json(buf.ctypes.data, n, ctypes.byref(out), ctypes.byref(cnt)))
    t_parse = time.perf_counter() - t0
    lib.sydelta_checksums_free(out)
    assert cnt.value == w.size
    dt = t_write + t_parse
    return {"value": round(w.size * bs / dt / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"host writer + host parser (C calls only), {w.size} entries ({n >> 20} MiB of text), basis "
                      f"GiB/s covered; write {n / t_write / 1e6:.0f} MB/s, parse {n / t_parse / 1e6:.0f} MB/s"}


def cpu_dparse_baseline(src_dev, bs: int):
    """libsydelta's host serde_json parser (sydelta_delta_from_json, one thread) on the
    text of one Data op of 256 MiB of the same source (sy-remote.rs:175)."""
    from sy_amd import wire

    sample = src_dev[:256 << 20].cpu().numpy()
    text = wire.delta_to_json([1], [0], [sample.size], sample.size, bs, sample)
    t0 = time.perf_counter()
    ops, _, _ = wire.delta_from_json(text)
    dt = time.perf_counter() - t0
    assert len(ops) == 1 and len(ops[0][1]) == sample.size
    return {"value": round(sample.size / dt / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"host parser, one Data op of {sample.size >> 20} MiB ({len(text) >> 20} MiB of text)"}


def cpu_zstd_baseline(text_dev, sample_bytes: int = 64 << 20):
    """zstd level 3 -- what compress/mod.rs:71-76 runs (zstd::Encoder::new(.., 3)) -- with the
    system libzstd on one thread, on a prefix of the same Delta JSON text."""
    import ctypes.util

    import numpy as np

    z = ctypes.CDLL(ctypes.util.find_library("zstd") or "libzstd.so.1")
    z.ZSTD_compress.restype = ctypes.c_size_t
    z.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    z.ZSTD_compressBound.restype = ctypes.c_size_t
    z.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
    z.ZSTD_versionString.restype = ctypes.c_char_p
    sample = text_dev[:sample_bytes].cpu().numpy()
    cap = z.ZSTD_compressBound(sample.size)
    out = np.empty(cap, np.uint8)
    t0 = time.perf_counter()
    got = z.ZSTD_compress(out.ctypes.data, cap, sample.ctypes.data, sample.size, 3)
    dt = time.perf_counter() - t0
    return {"value": round(sample.size / dt / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"libzstd {z.ZSTD_versionString().decode()} level 3 (compress/mod.rs:71-76) on the first "
                      f"{sample.size >> 20} MiB of the same text: ratio {got / sample.size:.3f}"}


def cpu_xxh3_baseline(buf_dev, offs, lens):
    """The oracle's hash_file (python-xxhash's XXH3, one thread, 1 MiB updates as in
    integrity/xxhash3.rs:22-30) over a <= 512 MiB prefix of the same files, repeated
    for >= 3 s."""
    import numpy as np

    from oracle import oracle as O

    k = max(1, int(np.searchsorted(np.cumsum(lens), 512 << 20, side="right")))
    k = min(k, len(lens))
    end = int(offs[k - 1] + lens[k - 1])
    host = buf_dev[:end].cpu().numpy().tobytes()
    t0 = time.perf_counter()
    reps = 0
    while True:
        for o, ln in zip(offs[:k], lens[:k]):
            O.py_hash_file(host[int(o):int(o + ln)])
        reps += 1
        if time.perf_counter() - t0 >= 3.0:
            break
    dt = time.perf_counter() - t0
    nbytes = int(lens[:k].sum()) * reps
    return {"value": round(nbytes / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{k} file(s), {int(lens[:k].sum()) >> 20} MiB, hashed {reps}x (python-xxhash XXH3)"}


def cpu_apply_baseline(basis_dev, new_dev, delta, sample_bytes: int = 1 << 30):
    """The C oracle's apply_delta (applier.rs:22-56 in memory, one thread) on the ops
    that rebuild the first `sample_bytes` of the same output, repeated for >= 3 s."""
    import numpy as np

    from oracle import oracle as O

    kind = np.asarray(delta.kind, dtype=np.uint8)
    a = np.ascontiguousarray(delta.a, dtype=np.uint64)
    b = np.ascontiguousarray(delta.b, dtype=np.uint64)
    k = int(np.searchsorted(np.cumsum(b), sample_bytes, side="right"))
    kind, a, b = np.ascontiguousarray(kind[:k]), a[:k], b[:k]
    basis_end = int((a + b)[kind == 0].max()) if (kind == 0).any() else 0
    lit_end = int((a + b)[kind != 0].max()) if (kind != 0).any() else 0
    basis = basis_dev[:basis_end].cpu().numpy()
    lit = new_dev[:lit_end].cpu().numpy()
    total = int(b.sum())
    out = np.empty(max(total, 1), np.uint8)
    L = O.C().L
    reps = 0
    t0 = time.perf_counter()
    while True:
        got = L.oracle_apply_delta(basis.ctypes.data, basis.size, lit.ctypes.data, kind.ctypes.data, a.ctypes.data,
                                   b.ctypes.data, k, out.ctypes.data, out.size)
        if got != total:
            raise RuntimeError("oracle apply failed")
        reps += 1
        if time.perf_counter() - t0 >= 3.0:
            break
    dt = time.perf_counter() - t0
    return {"value": round(total * reps / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{k} ops rebuilding {total >> 20} MiB, applied {reps}x (C oracle, in memory)"}


def cpu_local_baseline(src_dev, dst_dev, bs: int, sample_bytes: int = 1 << 30):
    """The oracle's block-compare loop (local.rs:549-619, one thread) over the first
    `sample_bytes` of both files, repeated for >= 3 s; bytes compared = 2 x sample."""
    from oracle import oracle as O

    n = min(sample_bytes, src_dev.numel())
    src = src_dev[:n].cpu().numpy().tobytes()
    dst = dst_dev[:n].cpu().numpy().tobytes()
    reps = 0
    t0 = time.perf_counter()
    while True:
        O.py_block_compare(src, dst, bs)
        reps += 1
        if time.perf_counter() - t0 >= 3.0:
            break
    dt = time.perf_counter() - t0
    return {"value": round(2 * n * reps / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{n >> 20} MiB of each file in {bs >> 10} KiB blocks, compared {reps}x (bytes compared = 2x)"}


def shard_range(nunits: int, world: int, rank: int):
    """Contiguous, size-balanced share of `nunits` equal units for `rank` (the LPT
    split when all units have the same size).  No collective: every rank computes
    its own range."""
    per, extra = divmod(nunits, world)
    lo = rank * per + min(rank, extra)
    return lo, lo + per + (1 if rank < extra else 0)


def max_over_ranks(x: float, device: str) -> float:
    """The job's time is its slowest rank's (one all-reduce MAX, outside the timed region)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def c4_files(dev, basis_bytes: int, nfiles: int, first: int):
    """basis_i = 1 MiB of synthetic bytes (seed 0x5E1D0004 + i);
    new_i = basis_i with one byte inserted at a random offset and 16 random byte
    substitutions.  Files are packed at 16-byte aligned offsets in one buffer each."""
    import numpy as np
    import torch

    stride = (basis_bytes + 1 + 15) & ~15
    basis = torch.empty(max(nfiles, 1) * stride, dtype=torch.uint8, device="cuda")
    new = torch.empty_like(basis)
    rng = np.random.default_rng(0x5E1D0004 + first)
    ins = rng.integers(0, basis_bytes + 1, nfiles)
    for k in range(nfiles):
        o = k * stride
        b = basis[o:o + basis_bytes]
        dev.synth_fill(b, 0x5E1D0004 + first + k)
        p = int(ins[k])
        new[o:o + p] = b[:p]
        new[o + p] = int(rng.integers(0, 256))
        new[o + p + 1:o + basis_bytes + 1] = b[p:]
    sub = (np.arange(nfiles)[:, None] * stride + rng.integers(0, basis_bytes + 1, (nfiles, 16))).reshape(-1)
    idx = torch.from_numpy(sub.astype(np.int64)).cuda()
    new[idx] = new[idx] ^ torch.from_numpy(rng.integers(1, 256, sub.size).astype(np.uint8)).cuda()
    offs = np.arange(nfiles, dtype=np.uint64) * stride
    return basis, new, (offs, np.full(nfiles, basis_bytes, np.uint64), offs.copy(),
                        np.full(nfiles, basis_bytes + 1, np.uint64))


def host_inclusive(dev, bs: int, size: int, stream_dev: int):
    """Rate including pinned-host <-> HBM copies: a C3-shaped pair
    of `size` bytes starts in pinned host memory; the basis goes H2D and is signed
    while the source's H2D runs on a second stream; then index + match, op list on
    the host.  Reported beside `value`, never as it."""
    import torch

    hb = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    hn = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    db = torch.empty(size, dtype=torch.uint8, device="cuda")
    dn = torch.empty(size, dtype=torch.uint8, device="cuda")
    dev.synth_fill(db, 0x5E1D0012)
    dev.synth_mutate(dn, db, 0x5E1D0013, 50000)
    hb.copy_(db)
    hn.copy_(dn)
    torch.cuda.synchronize()
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    best = None
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s1):
            db.copy_(hb, non_blocking=True)
        with torch.cuda.stream(s2):
            dn.copy_(hn, non_blocking=True)
        w, s = dev.signature(db, bs, stream=s1)
        idx = dev.Index(w, s, bs, bs, device=stream_dev, stream=s1)
        s1.wait_stream(s2)
        d = dev.match(idx, dn, stream=s1)
        idx.close()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    t0 = time.perf_counter()
    db.copy_(hb)
    torch.cuda.synchronize()
    h2d = size / (time.perf_counter() - t0) / 1e9
    return {"value": round(2 * size / best / GIB, 3), "unit": "GiB/s",
            "sample": f"{size >> 20} MiB basis + {size >> 20} MiB source (5% byte edits) from pinned host memory, "
                      f"H2D of the source overlapped with the signature, op list to host; best of 3",
            "h2d_GBps": round(h2d, 2), "ops": len(d.kind)}


def _pmc_order(path: str):
    """Chronological order of profiles/r<round><tag>_*_pmc.json: round, then the tag as
    the scripts name them (r03, r03b .. r03z, r03aa ..: shorter tags first)."""
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (0, 0, "")


def _pmc_files(workload: str, block_size: int):
    """profiles/*_pmc.json of this workload and block size, oldest first.  A summary
    records both (scripts/pmc_summary.py workload=.. block_size=..); files without them
    (round 1-3) or of another workload are never borrowed."""
    import glob

    out = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")), key=_pmc_order):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload") == workload and d.get("block_size") == block_size:
            out.append((f, d))
    return out


def pmc_traffic(kernel: str, per_launch: int, workload: str, block_size: int):
    """(HBM bytes per launch of `kernel`, source file) from the newest committed rocprofv3
    PMC summary of the same workload and block size (FETCH_SIZE and WRITE_SIZE passes of
    this bench command), scaled to this launch's size; (None, None) when there is none."""
    best, src = None, None
    for f, d in _pmc_files(workload, block_size):
        v = d.get("kernels", {}).get(kernel)
        if v and "traffic_bytes" in v and v.get("bytes_per_launch"):
            best, src = v["traffic_bytes"] * per_launch / v["bytes_per_launch"], os.path.basename(f)
    return (int(best), "profiles/" + src) if best else (None, None)


def pmc_counters(kernel: str, workload: str, block_size: int):
    """Raw per-launch counters (TCC/TCP request counts) of `kernel` from the newest
    profiles/*_pmc.json of the same workload and block size, with that launch's
    algorithmic bytes."""
    best = None
    for f, d in _pmc_files(workload, block_size):
        v = d.get("kernels", {}).get(kernel)
        if v and v.get("counters") and v.get("bytes_per_launch"):
            best = dict(v["counters"], bytes_per_launch=v["bytes_per_launch"], source=os.path.basename(f))
    return best


def algo_bytes_per_step(workload: str, n: int, nb_bytes: int, src_bytes: int) -> dict:
    """Algorithmic HBM bytes per step of each kernel that can dominate a workload.  Per
    step the signature kernels read the basis once and the scan reads the source once
    (SURVEY.md section 8(d))."""
    return {"k_scan": src_bytes, "k_scan_lds": src_bytes, "k_scan_w": src_bytes, "k_scan_r": src_bytes,
            "k_scan_g": src_bytes,
            "k_walk_files": src_bytes,  # c4: every source byte read once (the walk's classification + ops)
            "k_sig_fast": nb_bytes if workload in ("c3", "c3b") else n,
            "k_sig_batch": n, "k_sig_wave": n, "k_probe": src_bytes,
            "k_apply": 2 * n,  # apply: every output byte read once and written once
            "k_json_write": n,  # json: every literal byte read once (text written: ~3.6x)
            "k_zstd_block": src_bytes,  # zstd: every text byte read once
            "k_dparse": src_bytes,  # dparse: the text read once + the literal bytes written
            "k_sigjson_write": src_bytes,  # sigjson: 12 B per entry read + the text written once
            "k_sigparse": src_bytes + 28 * (n // 4096),  # sigjson (bs 4096): the text read once + 40 B per entry written
            "k_block_cmp": 2 * n,  # local: both files read once
            "k_xxh_pieces": n}  # xxh3: every file byte read once


def roofline(prof: dict, steps: int, algo_step: dict, positions=None, keys=None, workload="c3", block_size=4096):
    """Roofline of the dominant kernel: algorithmic bytes per launch / its average launch
    time (HIP events on the launch stream, sydelta_profile).  A kernel launched L times
    per step gets 1/L of its per-step bytes per launch (the scan is split into segments
    of 2^31 positions).

    For the scan in global-filter mode (k_scan_lds / k_scan over an index whose Bloom
    filter lives in L2) the binding resource is not HBM but the L2 request rate: one
    random filter-word request per window start.  `l2_gather` reports that rate against
    L2_GATHER_PEAK (the measured chip-wide ceiling of random L2 gathers,
    profiles/r02_micro_gather2.txt) when the step's scanned positions are known.  For
    the level-1 scans (k_scan_r / k_scan_g: 38400 words = 1228800 bits; round 3's k_scan_w:
    2^19 bits) only the positions that pass the level-1 filter in LDS send a request; that
    fraction is modelled as 1 - exp(-keys / bits) for the one-hash Bloom and 1/2 for the
    ribbon, and the entry says so.

    `bound` is "l2" when the L2 request rate binds the kernel (its l2_gather fraction,
    measured or modelled, exceeds its HBM fraction); achieved / peak / frac stay the HBM
    figures the metric is quoted in."""
    import math

    dom = max(prof, key=lambda k: prof[k]["ms"]) if prof else None
    if not dom or dom not in algo_step:
        return None
    launches_per_step = prof[dom]["count"] / steps
    avg_ms = prof[dom]["ms"] / max(1, prof[dom]["count"])
    per_launch = int(algo_step[dom] / launches_per_step)
    ach = per_launch / (avg_ms * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic(dom, per_launch, workload, block_size)
    roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
            "kernel": dom, "avg_launch_ms": round(avg_ms, 4), "algorithmic_bytes_per_launch": per_launch}
    # level-1 filter bits per key (one hash)
    l1_bits = {"k_scan_w": 1 << 19, "k_scan_r": 38400 * 32, "k_scan_g": 38400 * 32}
    if positions and (dom in ("k_scan_lds", "k_scan") or (dom in l1_bits and keys)):
        # the ribbon level-1 (sydelta_internal.hpp: 852000..1100000 keys unless SYDELTA_L1
        # forces a layout) passes ~1/2 of the positions whatever the key count
        l1_env = os.environ.get("SYDELTA_L1", "")
        # and only a scan of >= 2^31 positions builds it (sydelta_internal.hpp: kRibMinScan)
        ribbon = dom in l1_bits and keys and (l1_env == "ribbon" or (l1_env != "bloom" and 852000 <= keys <= 1100000
                                                                     and positions >= 1 << 31))
        per_pos = 1.0 if dom not in l1_bits else 0.5 if ribbon else 1.0 - math.exp(-keys / float(l1_bits[dom]))
        req = positions * per_pos / launches_per_step  # filter-word requests per launch
        rate = req / (avg_ms * 1e-3)
        roof["l2_gather"] = {"requests_per_launch": int(req), "achieved": round(rate / 1e9, 2),
                             "peak": round(L2_GATHER_PEAK / 1e9, 1), "unit": "G requests/s",
                             "frac": round(rate / L2_GATHER_PEAK, 4),
                             "requests_per_position": round(per_pos, 4),
                             "model": ("one per window start" if dom not in l1_bits else
                                       "window starts x ribbon level-1 pass rate 1/2" if ribbon else
                                       f"window starts x level-1 pass rate 1-exp(-keys/{l1_bits[dom]})")}
        pc = pmc_counters(dom, workload, block_size)
        if pc and pc.get("TCC_REQ_sum"):
            # measured: every L2 request of the launch (filter words, staged bytes, table
            # lookups) per scanned byte, from the rocprofv3 TCC pass of the same command
            rq = pc["TCC_REQ_sum"] / pc["bytes_per_launch"]
            roof["l2_gather"]["measured"] = {
                "tcc_requests_per_position": round(rq, 4),
                "tcc_hit_rate": round(pc["TCC_HIT_sum"] / max(1.0, pc["TCC_HIT_sum"] + pc["TCC_MISS_sum"]), 4),
                "tcc_requests_per_s_G": round(rq * per_launch / (avg_ms * 1e-3) / 1e9, 2),
                "frac": round(rq * per_launch / (avg_ms * 1e-3) / L2_GATHER_PEAK, 4),
                "source": "profiles/" + pc["source"]}
        lf = roof["l2_gather"].get("measured", roof["l2_gather"])["frac"]
        if lf > roof["frac"]:
            roof["bound"] = "l2"
    return roof


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus() -> int:
    """Devices this process may use, counted without initialising the GPU (on this image
    torch.cuda.device_count() does not start the HIP runtime).  SYDELTA_BENCH_FAKE_GPUS
    overrides it for the launcher's CPU tests."""
    fake = os.environ.get("SYDELTA_BENCH_FAKE_GPUS")
    if fake is not None:
        return int(fake)
    import torch

    return torch.cuda.device_count()


def launch_ranks(nranks: int, argv) -> int:
    """`bench.py --gpus N` without a launcher: start N child processes of this script, one
    per GPU, each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (the
    torchrun contract) and SYDELTA_HOST_THREADS = max(2, host cores // N) so the ranks'
    host pools do not oversubscribe the host (sy's transfers share one host too,
    sync/mod.rs:673-697).  Nothing here touches the GPU and nothing execs: the children
    are ordinary subprocesses.  Rank 0's stdout (the JSON line) is forwarded to ours,
    the other ranks' stdout to our stderr.  The first rank to fail ends the job: the
    others are terminated (they would wait in a collective) and its exit code is ours."""
    import subprocess
    import threading

    have = visible_gpus()
    if have < nranks:
        print(f"bench.py: --gpus {nranks} asks for {nranks} ranks but {have} GPU(s) are visible", file=sys.stderr)
        return 2
    cores = host_cores()[0]
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=port)
        env.setdefault("SYDELTA_HOST_THREADS", str(max(2, cores // nranks)))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE, text=True, bufsize=1))

    def pump(p, out):
        for ln in p.stdout:
            out.write(ln)
            out.flush()

    pumps = [threading.Thread(target=pump, args=(p, sys.stdout if r == 0 else sys.stderr), daemon=True)
             for r, p in enumerate(procs)]
    for t in pumps:
        t.start()
    rc = 0
    live = set(range(nranks))
    while live:
        for r in sorted(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    for p in procs:  # every child has exited; collect and close the pipes
        p.wait()
    for t in pumps:
        t.join(timeout=5)
    return rc


C4_FILES = 10000  # BASELINE config 4


def time_steps(step, steps: int, warmup: int, world: int):
    """W untimed steps, then exactly K timed ones bracketed by a barrier + synchronize on
    both sides; the max over ranks.  Returns (seconds, the last step's result)."""
    import torch
    import torch.distributed as dist

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for _ in range(steps):
        last = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        el = max_over_ranks(el, "cuda")
    return el, last


def c4_step(dev, basis, new, files, bs: int, device: int, strm, calls: str = "pairs"):
    """One batch of files = (boff, blen, soff, slen): the signature of every basis and the match
    of every source (K10 walks every file on the device) -- one sydelta_delta_pairs_device call
    (calls "pairs"), or batched signature, per-file index and batched match (three calls); strm
    None = the calling thread's library stream (the call then synchronizes before returning)."""
    boff, blen, soff, slen = files
    if calls == "pairs":
        res = dev.delta_pairs_handle(basis, boff, blen, new, soff, slen, bs, stream=strm)
        tot = res.stats
        res.close()
        return tot
    w, s = dev.signature_batch(basis, boff, blen, bs, stream=strm)
    nblk = (blen + bs - 1) // bs
    last = blen - (nblk - 1) * bs
    idx = dev.BatchIndex(w, s, nblk, last, bs, device=device, stream=strm)
    # the per-file op lists stay in the library's batch (host memory), as the Rust caller
    # would read them through the accessors
    res = dev.match_batch_handle(idx, new, soff, slen, stream=strm)
    idx.close()
    tot = res.stats
    res.close()
    return tot


def c5_setup(dev, n: int, bs: int, edit_ppm: int, world: int, rank: int):
    """BASELINE config 5: one file of world * n bytes; rank owns basis bytes [rank n,
    (rank+1) n) and window starts [rank n, (rank+1) n) of the source (+ the next bs-1 bytes
    as halo).  Counter-based generators give every rank the same bytes for the same file
    offsets."""
    import torch

    from sy_amd import shard

    file_len = world * n
    first = rank * n
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev.synth_fill_range(basis, first, 0x5E1D0005)
    p0, p1 = shard.chunk_bounds(file_len, bs, world, rank)
    buf_end = file_len if rank == world - 1 else min(file_len, p1 + bs - 1)
    new = torch.empty((buf_end - first + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    src_view = new[:buf_end - first]
    dev.synth_fill_range(src_view, first, 0x5E1D0005)
    dev.synth_mutate_blocks(src_view, src_view, first, bs, 0x5E1D0006, edit_ppm)
    return dict(basis=basis, new=new, file_len=file_len, first=first, p0=p0, p1=p1)


def c5_proxy_signature(dev, c5: dict, n: int, bs: int, world: int, rank: int):
    """The whole file's signature SoA of a `world`-rank C5 job as rank `rank` would hold it
    after the all-gather: every other rank's chunk generated and signed here (untimed) into
    its slot; rank's own slot is written by each timed step."""
    import torch

    nb = n // bs
    W = torch.empty(world * nb, dtype=torch.int32, device="cuda")
    S = torch.empty(world * nb, dtype=torch.int64, device="cuda")
    tmp = c5["basis"]
    for g in range(world):
        if g == rank:
            continue
        dev.synth_fill_range(tmp, g * n, 0x5E1D0005)
        w, s = dev.signature(tmp, bs)
        W[g * nb:(g + 1) * nb].copy_(w.view(torch.int32))
        S[g * nb:(g + 1) * nb].copy_(s.view(torch.int64))
    dev.synth_fill_range(tmp, rank * n, 0x5E1D0005)  # the rank's own basis chunk again
    torch.cuda.synchronize()
    return W, S


def c4_leg(args, world: int, el: float, files_this_rank: int, bytes_this_rank: int, last: dict) -> dict:
    """The line's "c4" object: the job's aggregate over all ranks' files (el = max over ranks)."""
    total = C4_FILES * ((1 << 20) + (1 << 20) + 1)  # basis + source bytes of all ranks' files per step
    return {"workload": "C4: 10000 x 1 MiB files (1-byte insertion + 16 substitutions each), bs 4096, file-sharded "
                        "(no collective); " + ("one signature+match call per batch" if args.c4_calls == "pairs"
                                               else "three calls"),
            "value": round(total * args.steps / el / GIB, 3), "unit": "GiB/s", "scaling": "strong",
            "ms_per_step": round(el / args.steps * 1e3, 4), "files": C4_FILES, "files_this_rank": files_this_rank,
            "bytes_this_rank_per_step": bytes_this_rank,
            "copy_ops_this_rank": int(last["copy_ops"]), "literal_bytes_this_rank": int(last["literal_bytes"])}


def c5_leg(args, world: int, el: float, ag_ms: float, st: dict) -> dict:
    """The line's "c5" object: one 8 GiB chunk per rank (el = max over ranks)."""
    n5, bs5 = 8 << 30, 8192
    return {"workload": f"C5: one {world * n5 / GIB:.0f} GiB file, bs {bs5}, 1% of blocks with one substituted byte; "
                        f"signature + RCCL all-gather + index + chunk walk, chunk-sharded",
            "value": round(world * 2 * n5 * args.steps / el / GIB, 3), "unit": "GiB/s", "scaling": "weak",
            "ms_per_step": round(el / args.steps * 1e3, 4), "bytes_per_rank_per_step": 2 * n5,
            "allgather_ms": round(ag_ms, 4), "allgather_bytes_per_rank": 12 * (n5 // bs5) * world if world > 1 else 0,
            "copy_ops_this_rank": int(st["copy_ops"]), "literal_bytes_this_rank": int(st["literal_bytes"])}


def run_legs(args, dev, world: int, rank: int, device: int, stream) -> dict:
    """The north star's multi-GPU configs beside the C3 headline, so the driver's
    `--gpus N` run measures them (BASELINE.json configs 4 and 5):
      c4: this rank's shard_range of 10 000 x 1 MiB file pairs (no collective; strong
          scaling: the total is fixed, each rank's share shrinks with N);
      c5: one 8 GiB chunk per rank of one N x 8 GiB file, bs 8192, 1 % edited blocks:
          signature, RCCL all-gather of the signature SoA, the full index, the chunk's
          walk chained over ranks (weak scaling); the all-gather also timed alone.
    Same steps / warmup as the headline, barrier-bracketed, max over ranks; no CPU
    baseline (the c4 / c5 workloads report theirs at N=1)."""
    import torch
    import torch.distributed as dist

    out = {}
    # ---- C4
    lo, hi = shard_range(C4_FILES, world, rank)
    basis, new, files = c4_files(dev, basis_bytes=1 << 20, nfiles=hi - lo, first=lo)
    torch.cuda.synchronize()
    el, last = time_steps(lambda: c4_step(dev, basis, new, files, 4096, device, stream, args.c4_calls), args.steps,
                          args.warmup, world)
    out["c4"] = c4_leg(args, world, el, hi - lo, int(files[1].sum() + files[3].sum()), last)
    del basis, new, files, last
    torch.cuda.empty_cache()
    # ---- C5
    n5, bs5, ppm5 = 8 << 30, 8192, 10000
    c5 = c5_setup(dev, n5, bs5, ppm5, world, rank)
    from sy_amd import shard

    gather, bcast = shard.torch_collectives(dist, "cuda") if world > 1 else ((lambda v: [v]), (lambda v, src: v))
    nb = n5 // bs5
    W = torch.empty(world * nb, dtype=torch.int32, device="cuda") if world > 1 else None
    S = torch.empty(world * nb, dtype=torch.int64, device="cuda") if world > 1 else None

    def c5_step():
        w, s = dev.signature(c5["basis"], bs5, stream=stream)
        if world > 1:  # the one exchange step: RCCL all-gather of the signature SoA
            dist.all_gather_into_tensor(W, w.view(torch.int32))
            dist.all_gather_into_tensor(S, s.view(torch.int64))
            w, s = W.view(w.dtype), S.view(s.dtype)
        idx = dev.Index(w, s, bs5, bs5, device=device, stream=stream)
        ch = dev.Chunk(idx, c5["new"], c5["first"], c5["file_len"], c5["p0"], c5["p1"], stream=stream)
        d, _ = shard.walk_chain(ch, rank, world, c5["p0"], gather, bcast)
        ch.close()
        idx.close()
        return d.stats

    el, st = time_steps(c5_step, args.steps, args.warmup, world)
    ag_ms = 0.0
    if world > 1:
        w0, s0 = dev.signature(c5["basis"], bs5)
        torch.cuda.synchronize()

        def ag():
            dist.all_gather_into_tensor(W, w0.view(torch.int32))
            dist.all_gather_into_tensor(S, s0.view(torch.int64))

        ag_el, _ = time_steps(ag, args.steps, 1, world)
        ag_ms = ag_el / args.steps * 1e3
    out["c5"] = c5_leg(args, world, el, ag_ms, st)
    del c5, W, S
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if os.environ.get("SYDELTA_BENCH_STUB"):
        # launcher test hook (tests/test_bench_launch.py): report the rank environment, no GPU
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                       "MASTER_PORT", "SYDELTA_HOST_THREADS")}), flush=True)
        if os.environ.get("SYDELTA_BENCH_STUB_LEGS") and int(os.environ.get("RANK", "0")) == 0:
            # the legs' objects as rank 0 builds them (fixed timings: 2 ms C4, 5 ms C5 per step)
            st = {"copy_ops": 1, "literal_bytes": 2}
            lo, hi = shard_range(C4_FILES, world, 0)
            print(json.dumps({"metric": METRIC, "n_gpus": world,
                              "c4": c4_leg(args, world, 2e-3 * args.steps, hi - lo, 0, st),
                              "c5": c5_leg(args, world, 5e-3 * args.steps, 0.1, st)}), flush=True)
        fail = os.environ.get("SYDELTA_BENCH_STUB_FAIL_RANK")
        if fail is not None:
            if int(fail) == int(os.environ.get("RANK", "0")):
                time.sleep(0.5)
                sys.exit(7)
            time.sleep(60)  # the other ranks would wait in a collective for the failed one
        return
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; n_gpus reports WORLD_SIZE", file=sys.stderr)
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import sy_amd.device as dev
    import ctypes

    from sy_amd import _lib
    from sy_amd._lib import check, lib

    bs = args.block_size
    n = int(args.size_gib * GIB) // bs * bs
    seed_base = 0x5E1D0002 + 0x1000 * rank

    nb_bytes = min(n, (args.basis_mib << 20) // bs * bs) if args.basis_mib else n
    basis = None
    if args.workload not in ("c4", "path"):
        basis = torch.empty(n, dtype=torch.uint8, device="cuda")
        if args.workload != "c5":
            dev.synth_fill(basis, seed_base)
    new = None
    files = None
    if args.workload in ("c3",):
        new = torch.empty(n, dtype=torch.uint8, device="cuda")
        dev.synth_mutate(new, basis, seed_base + 1, args.edit_ppm)
    if args.workload == "c3b":
        import numpy as np

        ed = torch.empty(n, dtype=torch.uint8, device="cuda")
        dev.synth_mutate_blocks(ed, basis, 0, 4096, seed_base + 1, 50000)
        rng = np.random.default_rng(seed_base + 2)
        nblk4 = n // 4096
        ins = np.sort(rng.choice(nblk4, nblk4 // 100, replace=False)) * 4096 + rng.integers(0, 4096, nblk4 // 100)
        extra = torch.from_numpy(rng.integers(0, 256, ins.size, dtype=np.uint8)).cuda()
        cuts = np.concatenate([[0], ins, [n]])
        # piece i of the edited basis lands i bytes later (the insertions before it); one
        # copy per piece and one scatter of the inserted bytes (torch.cat of the 21 K pieces
        # crashed under rocprofv3's counter collection)
        new = torch.empty(n + ins.size, dtype=torch.uint8, device="cuda")
        for i in range(ins.size + 1):
            a0, a1 = int(cuts[i]), int(cuts[i + 1])
            new[a0 + i:a1 + i].copy_(ed[a0:a1])
        new[torch.from_numpy(ins + np.arange(ins.size)).cuda()] = extra
        del ed
    c5 = None
    apply_d = None
    json_d = None
    if args.workload in ("json", "zstd", "dparse"):
        from sy_amd import wire

        dev.synth_fill(basis, seed_base)
        new = torch.empty(n, dtype=torch.uint8, device="cuda")
        dev.synth_mutate(new, basis, seed_base + 1, args.edit_ppm)
        w, s = dev.signature(basis, bs)
        idx = dev.Index(w, s, bs, bs, device=local)
        json_d = dev.match(idx, new)
        idx.close()
        json_h = wire._delta_handle(json_d.kind, json_d.a, json_d.b, json_d.source_size, bs)
        json_len = ctypes.c_uint64()
        check(lib.sydelta_delta_to_json_device(json_h, new.data_ptr(), n, None, 0, ctypes.byref(json_len), None))
        json_out = torch.empty(json_len.value + 16, dtype=torch.uint8, device="cuda")
        zstd_len = json_len.value
        if args.workload in ("zstd", "dparse"):  # the text to compress / parse, written once
            check(lib.sydelta_delta_to_json_device(json_h, new.data_ptr(), n, json_out.data_ptr(), json_out.numel(),
                                                   ctypes.byref(json_len), None))
            if args.workload == "zstd":
                zstd_out = torch.empty(int(lib.sydelta_zstd_bound(zstd_len)) + 16, dtype=torch.uint8, device="cuda")
            else:
                dp_lit = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    if args.workload == "sigjson":
        from sy_amd import wire

        sj_w, sj_s = dev.signature(basis, bs)
        sj_len = int(wire.checksums_to_json_device(sj_w, sj_s, bs, bs).numel())
        sj_out = torch.empty(sj_len + 16, dtype=torch.uint8, device="cuda")
        sj_recs = torch.empty(sj_w.numel() * 40, dtype=torch.uint8, device="cuda")
    if args.workload == "apply":
        dev.synth_fill_range(basis, 0, 0x5E1D0005)
        new = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
        dev.synth_fill_range(new[:n], 0, 0x5E1D0005)
        dev.synth_mutate_blocks(new[:n], new[:n], 0, bs, 0x5E1D0006, args.edit_ppm)
        w, s = dev.signature(basis, bs)
        idx = dev.Index(w, s, bs, bs, device=local)
        apply_d = dev.match(idx, new, length=n)
        idx.close()
        apply_out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    if args.workload == "local":
        # local transport: the new file (source) against the existing one (dest), both
        # resident; 1% of 64 KiB blocks carry one substituted byte.
        dev.synth_fill_range(basis, 0, 0x5E1D0007)
        new = torch.empty(n, dtype=torch.uint8, device="cuda")
        dev.synth_fill_range(new, 0, 0x5E1D0007)
        dev.synth_mutate_blocks(new, new, 0, bs, 0x5E1D0008, args.edit_ppm)
        local_flags = torch.empty(n // bs, dtype=torch.uint8, device="cuda")
    if args.workload == "xxh3":
        # integrity verify (integrity/mod.rs:104): whole-file XXH3-64 of every file
        if args.files == 1:
            xxh_offs, xxh_lens = np.zeros(1, np.uint64), np.full(1, n, np.uint64)
        else:
            fsz = n // args.files
            xxh_offs = np.arange(args.files, dtype=np.uint64) * np.uint64(fsz)
            xxh_lens = np.full(args.files, fsz, dtype=np.uint64)
    proxy = args.workload == "c5" and args.proxy_world > 1 and world == 1
    if args.workload == "c5":
        from sy_amd import shard

        del basis
        cw, cr = (args.proxy_world, args.proxy_rank) if proxy else (world, rank)
        c5 = c5_setup(dev, n, bs, args.edit_ppm, cw, cr)
        basis, new = c5["basis"], c5["new"]
        if world > 1:
            gather, bcast = shard.torch_collectives(dist, "cuda")
        else:
            gather, bcast = (lambda v: [v]), (lambda v, src: v)
        c5.update(gather=gather, bcast=bcast, shard=shard, world=cw, rank=cr)
        if proxy:  # rank cr of a cw-rank job: the others' signatures in place of the all-gather
            c5["W"], c5["S"] = c5_proxy_signature(dev, c5, n, bs, cw, cr)
    path_files = None
    if args.workload == "path":
        import tempfile

        from oracle import oracle as O

        tmpd = tempfile.mkdtemp(prefix=f"sydelta_bench_r{rank}_", dir=os.environ.get("TMPDIR", "/tmp"))
        pb, ps = os.path.join(tmpd, "basis"), os.path.join(tmpd, "source")
        piece = 64 << 20
        with open(pb, "wb") as fb, open(ps, "wb") as fs:
            for i in range(0, n, piece):
                b = O.synth_bytes(min(piece, n - i), 0x5E1D0500 + rank, i)
                fb.write(b.tobytes())
                fs.write(O.synth_edit_blocks(b, i, bs, 0x5E1D0501, args.edit_ppm).tobytes())
        for f in (pb, ps):  # page-cache warm
            with open(f, "rb") as fh:
                while fh.read(64 << 20):
                    pass
        path_files = (tmpd, pb, ps)
    if args.workload == "c4":
        # BASELINE config 4: files [lo, hi) of --files 1 MiB files go to this rank
        # (equal sizes, so contiguous ranges are the bytes-balanced LPT split).
        fsz = 1 << 20
        lo, hi = shard_range(args.files, world, rank)
        files = c4_files(dev, basis_bytes=fsz, nfiles=hi - lo, first=lo)
        basis, new, files = files
        n = int(files[1].sum())  # basis bytes of this rank
    torch.cuda.synchronize()
    # The step's calls get a stream of their own.  torch's default stream is the legacy
    # NULL stream (handle 0), which the C ABI reads as "no stream": each call would run on
    # the library's thread stream and synchronize before returning, so the host could not
    # queue the next call (the index build, the probe) while the signature kernel runs.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)

    def c4_batch(fs, strm):
        return c4_step(dev, basis, new, fs, bs, local, strm, args.c4_calls)

    c4_pool, c4_groups = None, []
    if args.workload == "c4" and args.callers > 1:
        from concurrent.futures import ThreadPoolExecutor

        nf = len(files[0])
        c4_groups = [shard_range(nf, args.callers, g) for g in range(args.callers)]
        c4_groups = [g for g in c4_groups if g[1] > g[0]]
        c4_pool = ThreadPoolExecutor(len(c4_groups))

    def step():
        if args.workload == "path":
            sig = ctypes.POINTER(_lib.BlockChecksumC)()
            nsig = ctypes.c_uint64(0)
            check(lib.sydelta_compute_checksums(path_files[1].encode(), bs, ctypes.byref(sig), ctypes.byref(nsig)))
            h = ctypes.c_void_p()
            try:
                check(lib.sydelta_generate_delta_streaming(path_files[2].encode(), sig, nsig.value, bs,
                                                           ctypes.byref(h)))
                st = _lib.MatchStatsC()
                check(lib.sydelta_delta_stats(h, ctypes.byref(st)))
            finally:
                lib.sydelta_checksums_free(ctypes.cast(sig, ctypes.c_void_p))
                if h:
                    lib.sydelta_delta_free(h)
            return {k: getattr(st, k) for k, _ in _lib.MatchStatsC._fields_}
        if args.workload == "c2":
            dev.signature(basis, bs, stream=stream)
            return None
        if args.workload in ("c3", "c3b"):
            w, s = dev.signature(basis[:nb_bytes], bs, stream=stream)
            idx = dev.Index(w, s, bs, bs, device=local, stream=stream)
            d = dev.match(idx, new, stream=stream)
            idx.close()
            return d
        if args.workload == "apply":
            _, st = dev.apply_device(basis, apply_d, new, out=apply_out, stream=stream)
            return st
        if args.workload == "xxh3":
            h = dev.xxh3_batch(basis, xxh_offs, xxh_lens, stream=stream)
            return {"files": len(h), "hash0": f"{int(h[0]):016x}"}
        if args.workload == "local":
            # the local delta decision (ratio.rs) then the block compare (local.rs)
            r = dev.estimate_change_ratio(new, basis, bs, stream=stream)
            st = _lib.BlockCompareStatsC()
            check(lib.sydelta_block_compare_device(local, new.data_ptr(), n, basis.data_ptr(), n, bs,
                                                   local_flags.data_ptr(), int(stream.cuda_stream), ctypes.byref(st)))
            return {"changed_blocks": st.changed_blocks, "literal_bytes": st.literal_bytes,
                    "change_ratio": r["change_ratio"], "use_delta": r["use_delta"]}
        if args.workload == "zstd":
            got = ctypes.c_uint64()
            check(lib.sydelta_zstd_compress_device(local, json_out.data_ptr(), zstd_len, zstd_out.data_ptr(),
                                                   zstd_out.numel(), ctypes.byref(got), int(stream.cuda_stream)))
            return {"text_bytes": zstd_len, "frame_bytes": got.value, "ratio": round(got.value / zstd_len, 4)}
        if args.workload == "sigjson":
            ln = ctypes.c_uint64()
            check(lib.sydelta_checksums_to_json_device(sj_w.data_ptr(), sj_s.data_ptr(), sj_w.numel(), bs, bs,
                                                       sj_out.data_ptr(), sj_out.numel(), ctypes.byref(ln),
                                                       int(stream.cuda_stream)))
            got = ctypes.c_uint64()
            check(lib.sydelta_checksums_from_json_device(sj_out.data_ptr(), ln.value, sj_recs.data_ptr(),
                                                         sj_w.numel(), ctypes.byref(got), int(stream.cuda_stream)))
            return {"json_bytes": ln.value, "entries": sj_w.numel(), "parsed": got.value}
        if args.workload == "dparse":
            ln = ctypes.c_uint64()
            h = ctypes.c_void_p()
            check(lib.sydelta_delta_from_json_device(json_out.data_ptr(), zstd_len, dp_lit.data_ptr(), dp_lit.numel(),
                                                     ctypes.byref(ln), ctypes.byref(h), int(stream.cuda_stream)))
            nops = int(lib.sydelta_delta_num_ops(h))
            lib.sydelta_delta_free(h)
            return {"text_bytes": zstd_len, "literal_bytes": ln.value, "ops": nops}
        if args.workload == "json":
            ln = ctypes.c_uint64()
            check(lib.sydelta_delta_to_json_device(json_h, new.data_ptr(), n, json_out.data_ptr(), json_out.numel(),
                                                   ctypes.byref(ln), int(stream.cuda_stream)))
            return {"json_bytes": ln.value, "ops": len(json_d.kind)}
        if args.workload == "c5":
            w, s = dev.signature(basis, bs, stream=stream)
            if proxy:  # this rank's slot of the whole signature (the all-gather's result, untimed)
                nb = w.numel()
                c5["W"][cr * nb:(cr + 1) * nb].copy_(w.view(torch.int32))
                c5["S"][cr * nb:(cr + 1) * nb].copy_(s.view(torch.int64))
                w, s = c5["W"].view(w.dtype), c5["S"].view(s.dtype)
            if world > 1:  # the one exchange step: RCCL all-gather of the signature SoA
                W = torch.empty(world * w.numel(), dtype=w.dtype, device="cuda")
                S = torch.empty(world * s.numel(), dtype=s.dtype, device="cuda")
                dist.all_gather_into_tensor(W, w)
                dist.all_gather_into_tensor(S, s)
                w, s = W, S
            idx = dev.Index(w, s, bs, bs, device=local, stream=stream)
            ch = dev.Chunk(idx, new, c5["first"], c5["file_len"], c5["p0"], c5["p1"], stream=stream)
            if proxy:
                d, _ = ch.walk(c5["p0"])  # (its chain entry is its start: block-aligned copies)
            else:
                d, entry = c5["shard"].walk_chain(ch, rank, world, c5["p0"], c5["gather"], c5["bcast"])
            ch.close()
            idx.close()
            return d
        # c4: batched signature of all basis files, per-file index, one batched match
        if c4_pool is None:
            return c4_batch(files, stream)
        parts = list(c4_pool.map(lambda g: c4_batch(tuple(x[g[0]:g[1]] for x in files), None), c4_groups))
        return {k: sum(p[k] for p in parts) for k in parts[0]}

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
    busy = prof.pop("__busy__", None)  # the union of the timed launches (library profiler)
    if world > 1:
        elapsed = max_over_ranks(elapsed, "cuda")

    if args.workload == "c2":
        bytes_per_step = n
    elif args.workload in ("c3", "c3b"):
        bytes_per_step = nb_bytes + new.numel()
    elif args.workload == "c5":
        bytes_per_step = 2 * n
    elif args.workload == "apply":
        bytes_per_step = n  # reconstructed bytes
    elif args.workload == "local":
        bytes_per_step = 2 * n  # both files compared
    elif args.workload == "xxh3":
        bytes_per_step = int(xxh_lens.sum())
    elif args.workload == "zstd":
        bytes_per_step = zstd_len  # JSON text compressed
    elif args.workload == "dparse":
        bytes_per_step = n  # literal bytes recovered from the text
    elif args.workload == "json":
        bytes_per_step = n  # delta source bytes covered by the text
    elif args.workload == "sigjson":
        bytes_per_step = n  # basis bytes covered by the signature text
    elif args.workload == "path":
        bytes_per_step = 2 * n  # basis file signed + source file matched
    else:
        bytes_per_step = int(files[1].sum() + files[3].sum())
    total_bytes = bytes_per_step * args.steps * world
    value = total_bytes / elapsed / GIB
    ms_per_step = elapsed / args.steps * 1e3

    src_bytes = (int(files[3].sum()) if args.workload == "c4" else new.numel() if args.workload == "c3b" else
                 zstd_len if args.workload == "zstd" else zstd_len + n if args.workload == "dparse" else
                 sj_len + 12 * (n // bs) if args.workload == "sigjson" else n)
    algo_step = algo_bytes_per_step(args.workload, n, nb_bytes, src_bytes)
    stats = (last if isinstance(last, dict) else last.stats) if last is not None else None
    positions = stats.get("positions") if isinstance(stats, dict) and args.workload in ("c3", "c3b") else None
    roof = roofline(prof, args.steps, algo_step, positions,
                    keys=nb_bytes // bs if args.workload in ("c3", "c3b") else None, workload=args.workload,
                    block_size=bs)
    if roof is not None and busy and busy.get("ms"):
        # the step's kernel-busy time: the union of every timed launch of the step (overlapping
        # launches of several callers' streams counted once), against the step's algorithmic
        # bytes -- the roofline of the step as a whole, which per-launch times overstate when
        # callers overlap
        ub = busy["ms"] / args.steps
        roof["kernel_busy"] = {"union_ms_per_step": round(ub, 4), "step_ms": round(elapsed / args.steps * 1e3, 4),
                               "busy_frac_of_step": round(ub / (elapsed / args.steps * 1e3), 4),
                               "achieved": round(bytes_per_step / (ub * 1e-3) / 1e9, 2), "unit": "GB/s",
                               "frac": round(bytes_per_step / (ub * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                               "bytes_per_step": bytes_per_step}
        if args.workload == "c4" and len(c4_groups) > 1:
            roof["per_launch_overlap"] = ("the dominant kernel's launches of several callers overlap: its per-launch "
                                          "figures overstate its time; kernel_busy is the step's roofline")
    if roof is not None and roof.get("kernel") == "k_scan_r" and positions and args.workload == "c3":
        # the C3 ceiling: every position tested, a level-1 filter of at most
        # 1.17 bits per key in LDS passes >= 0.444 of them (information bound), each pass one
        # L2 request for its level-2 word, + 0.016 for the source rows + 0.008 for the table
        # lookups; the chip serves ~270 G random L2 requests/s.  The rest of the step as measured.
        step_ms = elapsed / args.steps * 1e3
        rest = step_ms - roof["avg_launch_ms"] * (prof["k_scan_r"]["count"] / args.steps)
        ceil = {}
        for name, rpp in (("information_bound", 0.468), ("ribbon_as_built", 0.528)):
            scan = positions * rpp / 270e9 * 1e3
            st = scan + rest
            ceil[name] = {"requests_per_position": rpp, "scan_ms": round(scan, 3), "step_ms": round(st, 3),
                          "value_GiBps": round(bytes_per_step / (st * 1e-3) / GIB, 1),
                          "hbm_frac": round(bytes_per_step / (st * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        roof["ceiling"] = dict(ceil, model="L2 request rate 270 G/s x requests per position; the rest of the step "
                                           "as measured (DESIGN.md §6.6)", value_frac_of_bound=round(
                                               (bytes_per_step / (step_ms * 1e-3) / GIB) /
                                               ceil["information_bound"]["value_GiBps"], 4))
    kernels = {k: {"avg_ms": round(v["ms"] / max(1, v["count"]), 4), "launches": v["count"]} for k, v in prof.items()}

    legs = None
    if args.workload == "c3" and not args.no_legs:
        # the headline's buffers go first (the legs need ~20 GiB for C4, ~17 GiB for C5)
        cpu_src = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu_src = (basis[:nb_bytes].cpu().numpy(), new[:min(new.numel(), 256 << 20)].cpu().numpy(), new.numel())
        basis = new = last = None
        torch.cuda.empty_cache()
        legs = run_legs(args, dev, world, rank, local, stream)

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.workload in ("c3", "c3b"):
            if legs is not None:
                cpu = cpu_baseline(*cpu_src, bs)
            else:
                cpu = cpu_baseline(basis[:nb_bytes].cpu().numpy(), new[:min(new.numel(), 256 << 20)].cpu().numpy(),
                                   new.numel(), bs)
        if world == 1 and not args.no_cpu_baseline and args.workload == "c4":
            k = min(500, len(files[0]))  # the sampled files' bytes only
            cpu = cpu_c4_baseline(basis[:int(files[0][k - 1] + files[1][k - 1])].cpu().numpy(),
                                  new[:int(files[2][k - 1] + files[3][k - 1])].cpu().numpy(), files, bs, sample_files=k)
        if world == 1 and not args.no_cpu_baseline and args.workload == "zstd":
            cpu = cpu_zstd_baseline(json_out[:zstd_len])
        if world == 1 and not args.no_cpu_baseline and args.workload == "sigjson":
            cpu = cpu_sigjson_baseline(sj_w, sj_s, bs)
        if world == 1 and not args.no_cpu_baseline and args.workload == "dparse":
            cpu = cpu_dparse_baseline(new, bs)
        if world == 1 and not args.no_cpu_baseline and args.workload == "json":
            cpu = cpu_json_baseline(new, bs)
        if world == 1 and not args.no_cpu_baseline and args.workload == "xxh3":
            cpu = cpu_xxh3_baseline(basis, xxh_offs, xxh_lens)
        if world == 1 and not args.no_cpu_baseline and args.workload == "apply":
            cpu = cpu_apply_baseline(basis, new, apply_d)
        if world == 1 and not args.no_cpu_baseline and args.workload == "local":
            cpu = cpu_local_baseline(new, basis, bs)
        hinc = None
        if world == 1 and not args.no_host_inclusive and args.workload == "c3" and not proxy:
            hinc = host_inclusive(dev, bs, min(n, 1 << 30), local)
        sig_ms = kernels.get("k_sig_fast", {}).get("avg_ms")
        line = {
            "metric": metric_for(bs),
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "c4" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": (f"synthetic (counter-based splitmix64 bytes; one substituted byte in {args.edit_ppm / 1e4:g}% of {bs // 1024} KiB blocks)"
                     if args.workload in ("c5", "apply", "local", "path") else
                     "synthetic (counter-based splitmix64 bytes; Bernoulli byte substitutions)"),
            "config": {
                "workload": {
                    "c3": "C3: signature(4 GiB basis) + rolling match(4 GiB source, 5% random byte edits), bs 4096",
                    "c3b": "C3b: signature(4 GiB basis) + rolling match(4 GiB source: one substituted byte in 5% "
                           "of 4 KiB blocks, a 1-byte insertion in 1%), bs 4096",
                    "c2": "C2: signature only over 4 GiB, bs 4096",
                    "c4": f"C4: {args.files} x 1 MiB files (1-byte insertion + 16 substitutions each), "
                          + ("signature + match of every pair in one call (sydelta_delta_pairs_device)"
                             if args.c4_calls == "pairs" else "batched signature + per-file index + batched match")
                          + ", file-sharded over ranks",
                    "c5": (f"C5 rank proxy: rank {args.proxy_rank} of a {args.proxy_world}-rank job on one GPU -- its "
                           f"{n / GIB:.0f} GiB chunk of one {args.proxy_world * n / GIB:.0f} GiB file, bs {bs}, "
                           f"{args.edit_ppm / 1e4:g}% of blocks with one substituted byte: signature of its chunk + "
                           f"index over the whole file's {args.proxy_world * (n // bs)} keys (the other ranks' "
                           f"signatures precomputed in place of the all-gather, untimed) + its chunk's walk; value = "
                           f"this rank's bytes / its step time" if proxy else
                           f"C5: one {world * n / GIB:.0f} GiB file, bs {bs}, {args.edit_ppm / 1e4:g}% of blocks with "
                           f"one substituted byte; signature + all-gather + index + chunk match, chunk-sharded"),
                    "apply": f"apply_delta on the device: {n / GIB:.0f} GiB reconstructed from a bs {bs} delta "
                             f"({args.edit_ppm / 1e4:g}% of blocks edited), per rank",
                    "xxh3": (f"integrity: whole-file XXH3-64 of {args.files} x {n // max(1, args.files) >> 20} MiB "
                             f"files per rank" if args.files != 1 else
                             f"integrity: whole-file XXH3-64 of one {n / GIB:.0f} GiB file"),
                    "local": f"local transport: change-ratio sample + block compare of two {n / GIB:.0f} GiB files, "
                             f"bs {bs}, {args.edit_ppm / 1e4:g}% of blocks edited",
                    "sigjson": f"serde_json text of the C2 signature ({n / GIB:g} GiB basis, {n // bs} entries) "
                               f"written and parsed back on the device",
                    "dparse": f"the C3 delta's serde_json text ({n / GIB:g} GiB source, one literal run) parsed on "
                              f"the device: literal bytes to HBM + the op list",
                    "json": f"serde_json text of the C3 delta ({n / GIB:.0f} GiB source, one literal run) on the device",
                    "zstd": f"zstd frame (Huffman literals + FSE-coded sequences, 128 KiB blocks) of the C3 delta's JSON text ({n / GIB:g} GiB source, "
                            f"one literal run) on the device; value = text bytes/s",
                    "path": f"path API on page-cache-warm files: compute_checksums({n / GIB:g} GiB basis) + "
                            f"generate_delta_streaming({n / GIB:g} GiB source, {args.edit_ppm / 1e4:g}% of {bs} B "
                            f"blocks edited), host-inclusive",
                }[args.workload],
                "block_size": bs,
                "basis_bytes": nb_bytes if args.workload in ("c3", "c3b") else n,
                "bytes_per_rank_per_step": bytes_per_step,
                "parallelism": (f"chunk-sharded x{world} (RCCL all-gather of the signature, chained walks)"
                                if args.workload == "c5" else
                                f"file-sharded x{world} (independent pairs per rank, no collective)"),
                **({"files": args.files, "files_this_rank": len(files[0]), "callers_per_rank": max(1, len(c4_groups))}
                   if args.workload == "c4" else {}),
                "walk": ("device (K10 per file / file segment)" if args.workload == "c4" else
                         "device (K10 per chunk segment, two pipelined parts)" if args.workload == "c5" else
                         "device (K5b)" if args.device_walk else "host threads"),
            },
            "pct_hbm_peak": round(value * GIB / 1e9 / HBM_PEAK_GBS * 100, 2),
            "roofline": roof,
            "cpu_baseline": cpu,
            "host_inclusive": hinc,
            **({"cpu_baseline_note": "rank 0 at N=1 only: a world > 1 run reports no CPU baseline and no "
                                     "host-inclusive rate"} if world > 1 else {}),
            **(legs or {}),
            "kernels": kernels,
            "signature_only_gibps": round(n / (sig_ms * 1e-3) / GIB, 2) if sig_ms else None,
            "match_stats": stats,
        }
        print(json.dumps(line), flush=True)
    if path_files:
        import shutil

        shutil.rmtree(path_files[0], ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
