"""GPU busy time from a rocprofv3 kernel trace (kernel_trace.csv): the union of kernel
intervals against the span they cover, per window of `--windows` equal slices (the
bench's steps when warmup is short), and the largest idle gaps with the kernels around
them.  Used to tell host-bound steps from device-bound ones (C4 with 10 callers).

    python scripts/trace_busy.py <dir holding *kernel_trace.csv> [--skip-first N] [--gaps 10]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--skip-first", type=int, default=0, help="drop the first N kernels (warmup)")
    ap.add_argument("--gaps", type=int, default=12)
    ap.add_argument("--since", default="", help="start at the first kernel whose name contains this, after skip")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60],
                             r.get("Queue_Id", ""), r.get("Stream_Id", "")))
    rows.sort()
    rows = rows[a.skip_first:]
    if a.since:
        k = next((i for i, r in enumerate(rows) if a.since in r[2]), 0)
        rows = rows[k:]
    if not rows:
        print("no kernels")
        return
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
    gaps = []
    prev_name = rows[0][2]
    for s, e, name, q, st in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_e - t0, prev_name, name))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = name if e >= cur_e else prev_name
    busy += cur_e - cur_s
    span = t1 - t0
    print(f"{len(rows)} kernels over {span / 1e6:.3f} ms: busy {busy / 1e6:.3f} ms ({100 * busy / span:.1f} %), "
          f"idle {(span - busy) / 1e6:.3f} ms in {len(gaps)} gaps")
    queues = sorted({(r[3], r[4]) for r in rows})
    print(f"queues/streams used: {len(queues)}")
    per = {}
    for s, e, name, q, st in rows:
        per.setdefault(name, [0, 0])
        per[name][0] += 1
        per[name][1] += e - s
    for name, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:12]:
        print(f"  {name:60s} {c:6d} launches {t / 1e6:9.3f} ms summed")
    gaps.sort(reverse=True)
    print("largest idle gaps (ms, at ms, after -> before):")
    for g, at, p, n in gaps[:a.gaps]:
        print(f"  {g / 1e6:8.3f} at {at / 1e6:9.3f}  {p[:40]} -> {n[:40]}")


if __name__ == "__main__":
    main()
