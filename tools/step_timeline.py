"""One step's launches per queue from a rocprofv3 kernel trace: start / end relative to the
step start, duration, grid -- plus, for each queue, the time between two anchor kernels
(default: the main queue's wait for the side queue's D step).  Used to read the D step's
critical path (DESIGN.md §"D step").

    python tools/step_timeline.py <run_kernel_trace.csv> [--step -2] [--marker ...]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-2, help="which marker-to-marker span (python index)")
    ap.add_argument("--marker", default="conv_c8r_kernel<7, 7, 1, 1>")
    ap.add_argument("--min-us", type=float, default=0.0, help="hide launches shorter than this")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                 r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60],
                 r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("Workgroup_Size", "")) for r in rows)
    marks = [k[0] for k in ks if a.marker in k[3]]
    spans = list(zip(marks, marks[1:]))
    t0, t1 = spans[a.step]
    by_q = collections.defaultdict(list)
    for s, e, q, n, g, wg in ks:
        if t0 <= s < t1:
            by_q[q].append((s, e, n, g, wg))
    print(f"step span {(t1 - t0) / 1e3:.1f} us")
    for q, v in sorted(by_q.items(), key=lambda kv: -len(kv[1])):
        busy = sum(e - s for s, e, *_ in v) / 1e3
        print(f"\n== queue {q}: {len(v)} launches, busy {busy:.1f} us")
        prev = None
        for s, e, n, g, wg in v:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            prev = e
            d = (e - s) / 1e3
            if d < a.min_us and gap < 5:
                continue
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {d:8.1f}  gap {gap:7.1f}  grid {g:>9} wg {wg:>4}  {n}")


if __name__ == "__main__":
    main()
