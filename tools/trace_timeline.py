"""Timeline of the kernels of one bench step from a rocprofv3 kernel trace (measurement
only): each kernel's start and end relative to the step's first kernel, and the idle gaps.

    python tools/trace_timeline.py <kernel_trace.csv> [--first k_sig_fast] [--step -2]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--first", default="k_sig_fast", help="kernel that opens a step")
    ap.add_argument("--step", type=int, default=-2, help="which step (python index over the steps found)")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         f"q{r.get('Queue_Id', '?')} s{r.get('Stream_Id', '?')} " + name.split("(")[0][:60]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.first in r[2]]
    i0 = starts[a.step]
    i1 = starts[a.step + 1] if a.step + 1 < len(starts) and a.step != -1 else len(rows)
    t0 = rows[i0][0]
    busy_end = t0
    idle = 0
    for s, e, name in rows[i0:i1]:
        gap = max(0, s - busy_end)
        idle += gap
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  gap {gap / 1e3:7.1f}  {name}")
        busy_end = max(busy_end, e)
    nxt = rows[i1][0] if i1 < len(rows) else busy_end
    print(f"step span to the next step's first kernel: {(nxt - t0) / 1e3:.1f} us; GPU idle inside: {idle / 1e3:.1f} us;"
          f" idle after the last kernel: {(nxt - busy_end) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
