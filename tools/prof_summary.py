"""Summarise a rocprofv3 --kernel-trace CSV: per-step totals by kernel and by
(kernel, grid, VGPR) so individual layers can be told apart.

    python tools/prof_summary.py <run_kernel_trace.csv> --steps 7 [--by-grid] [--top 40]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=7)
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    agg = collections.defaultdict(lambda: [0, 0.0])
    tot = 0.0
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
        key = (name, r["Grid_Size_X"], r["LDS_Block_Size"]) if a.by_grid else (name,)
        agg[key][0] += 1
        agg[key][1] += d
        tot += d
    print(f"kernel time per step: {tot / a.steps / 1e3:.3f} ms")
    print("| ms/step | % | launches/step | avg us | kernel |")
    print("|---:|---:|---:|---:|---|")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"| {t / a.steps / 1e3:.3f} | {100 * t / tot:.1f} | {n / a.steps:.1f} | {t / n:.1f} | `{' '.join(k)}` |")


if __name__ == "__main__":
    main()
