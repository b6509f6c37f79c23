"""FETCH_SIZE calibration summary: tools/micro_fetch_cal.hip's known
accesses against rocprofv3's per-kernel FETCH_SIZE (and TCC EA request counts).

    python scripts/fetch_cal.py gpurun_out/<tag> profiles/<tag>_fetch_calibration.json

For each kernel: FETCH bytes (KiB x 1024, uncorrected), the accesses and distinct 32/64/128-B
lines the host counted, and FETCH bytes per distinct line -- the factor that turns a
pattern's FETCH into lines fetched from beyond L2 (HBM or the Infinity Cache).
"""
import collections
import csv
import json
import re
import sys


def per_kernel(path, counter=None):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if counter and r["Counter_Name"] != counter:
            continue
        agg[r["Kernel_Name"].split("(")[0].replace("void ", "").strip()].append(float(r["Counter_Value"]))
    return agg


def main(src, dst):
    counts = {}
    for line in open(f"{src}/counts.txt"):
        m = re.match(r"(\S+)( \(.*\))? accesses (\d+) bytes_requested (\d+)(.*)", line.strip())
        if not m:
            continue
        d = {"accesses": int(m.group(3)), "bytes_requested": int(m.group(4))}
        for k, v in re.findall(r"lines(\d+) (\d+)", m.group(5)):
            d["lines" + k] = int(v)
        counts[m.group(1)] = d
    fetch = per_kernel(f"{src}/pmc_fetch/run_counter_collection.csv")
    out = {}
    for name, vals in fetch.items():
        key = next((k for k in counts if k.split("<")[0] in name and (("<" not in k) or k.split("<")[1][0] in name)),
                   None)
        if key is None:
            continue
        if key == "k_cal_stream":  # first launch: the 1 GiB stream (the second is the 16 MiB warm-up)
            vals = vals[:1]
        c = counts[key]
        fb = vals[0] * 1024
        e = {"fetch_bytes_raw": fb, **c, "fetch_over_requested": round(fb / c["bytes_requested"], 4)}
        for L in (32, 64, 128):
            if f"lines{L}" in c:
                e[f"fetch_bytes_per_line{L}"] = round(fb / c[f"lines{L}"], 2)
        out[key] = e
    try:
        for cn in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"):
            for name, vals in per_kernel(f"{src}/pmc_ea/run_counter_collection.csv", cn).items():
                for k in out:
                    if k.split("<")[0] in name and (("<" not in k) or k.split("<")[1][0] in name):
                        out[k][cn] = vals[0]
    except FileNotFoundError:
        pass
    json.dump({"source": src, "kernels": out}, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
