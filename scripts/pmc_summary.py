"""Summarise rocprofv3 output of scripts/gpu_check.sh into profiles/.

    python scripts/pmc_summary.py gpurun_out/<tag> profiles/<tag> [workload=c3] [block_size=4096] \
        [kernel=bytes_per_launch ...]

Writes <dst>_kernel_stats.csv (the --kernel-trace --stats summary, verbatim) and
<dst>_pmc.json: per kernel, average duration and HBM bytes per launch from the
FETCH_SIZE / WRITE_SIZE passes, corrected as MI355X_MICROARCH.md §HBM says
(FETCH_SIZE is in KiB and counts every L2 -> fabric read request as 64 B; WRITE_SIZE
in KiB, exact -> x1024).  Read bytes, calibrated per access pattern
(profiles/r05zb_fetch_calibration.json, tools/micro_fetch_cal.hip): a kernel that streams
its algorithmic bytes (kernel=bytes below) in whole 128-B lines sends one 128-B request per
line; every other request it sends is a partial-line miss of 64 B (gathers of filter
words, table buckets).  So read bytes = 128 x min(requests, bytes/128) + 64 x the rest.
Without a byte count a kernel's requests are taken as 128-B ones (x2, the streaming
calibration).  Requests the Infinity Cache serves are counted as well (the counters do not
separate them), so for IC-resident tables this is traffic beyond L2, an upper bound on HBM.  bench.py reads the
_pmc.json whose workload and block size match its own run to fill roofline.traffic
(a file without them, or of another workload, is never borrowed).
"""
import collections
import csv
import json
import os
import shutil
import sys


ALIASES = {"k_probe_rows": "k_probe"}  # rocprof kernel name -> sydelta_profile name


def norm(name):
    return name.split("(")[0].replace("void ", "").replace("sydelta::", "").split("<")[0].strip()


def per_kernel(path, counter=None):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if counter is not None and r["Counter_Name"] != counter:
            continue
        name = norm(r["Kernel_Name"])
        agg[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def counters(path):
    names = set()
    for r in csv.DictReader(open(path)):
        names.add(r["Counter_Name"])
    return sorted(names)


def main(src, dst, sizes=()):
    sizes = dict(kv.split("=") for kv in sizes)
    workload = sizes.pop("workload", None)
    block_size = sizes.pop("block_size", None)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, dst + "_kernel_stats.csv")
    dur = {}
    for r in csv.DictReader(open(stats)):
        name = norm(r["Name"])
        if name in dur:  # template instances of one kernel: keep the busier one
            if int(r["Calls"]) * float(r["AverageNs"]) <= dur[name]["calls"] * dur[name]["avg_ms"] * 1e6:
                continue
        dur[name] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
    fetch = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    extra = {}  # raw per-launch averages of the other passes (TCC / TCP request counts)
    for p in ("tcc", "tcp"):
        f = os.path.join(src, "pmc_" + p, "run_counter_collection.csv")
        if os.path.exists(f):
            for c in counters(f):
                for k, v in per_kernel(f, c).items():
                    extra.setdefault(k, {})[c] = round(v, 1)
    out = {}
    for k in dur:
        if k.startswith("void rocprim") or k.startswith("__amd"):
            continue
        f = fetch.get(k)
        w = write.get(k)
        out[k] = dict(dur[k])
        if f is not None:
            out[k]["fetch_kib_raw"] = round(f, 3)
            req = f * 1024 / 64  # EA read requests (FETCH_SIZE tallies 64 B each)
            out[k]["read_requests"] = int(req)
            if k in sizes:
                full = min(req, int(sizes[k]) / 128)
                out[k]["full_line_requests"] = int(full)
                out[k]["partial_line_requests"] = int(req - full)
                out[k]["hbm_read_bytes"] = int(128 * full + 64 * (req - full))
            else:
                out[k]["hbm_read_bytes"] = int(128 * req)
        if w is not None:
            out[k]["hbm_write_bytes"] = int(w * 1024)
        if f is not None and w is not None:
            out[k]["traffic_bytes"] = out[k]["hbm_read_bytes"] + out[k]["hbm_write_bytes"]
        if k in extra:
            out[k]["counters"] = extra[k]
        if k in sizes:
            out[k]["bytes_per_launch"] = int(sizes[k])
            if "traffic_bytes" in out[k]:
                out[k]["traffic_over_algorithmic"] = round(out[k]["traffic_bytes"] / int(sizes[k]), 3)
    for k, alias in ALIASES.items():  # the library profiler's name of the same kernel (bench.py's lookup)
        if k in out and alias not in out:
            out[alias] = dict(out[k], rocprof_name=k)
    meta = {"source": src, "workload": workload, "block_size": int(block_size) if block_size else None,
            "correction": ("FETCH_SIZE KiB x1024 / 64 = read requests; read bytes = 128 x the full-line requests of the "
                           "kernel's streamed bytes + 64 x the partial-line rest (x2 without a byte count); WRITE_SIZE "
                           "KiB x1024 (profiles/r05zb_fetch_calibration.json)"),
            "kernels": out}
    json.dump(meta, open(dst + "_pmc.json", "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
