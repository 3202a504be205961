"""Kernel names and mean durations of a tools/bench_conv.py run traced by rocprofv3: one line
per (kernel, grid) in order of first appearance (the cases run one after another), with its
launch count and mean duration -- which kernel each training shape's fwd / dgrad / wgrad runs.

    python tools/case_kernels.py <kernel_trace.csv> [--iters 10]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70],
                   r.get("Grid_Size_X", "")) for r in csv.DictReader(open(a.trace)))
    rows = [r for r in rows if "at::native" not in r[2] and "elementwise" not in r[2]]
    # (kernel, grid) in order of first appearance: the cases run one after another
    agg = {}
    for s, e, n, g in rows:
        c, t = agg.get((n, g), (0, 0))
        agg[(n, g)] = (c + 1, t + e - s)
    for (n, g), (c, t) in agg.items():
        print(f"{c:4d} x {t / c / 1e3:8.1f} us  grid {g:>9}  {n}")


if __name__ == "__main__":
    main()
