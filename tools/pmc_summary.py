"""Aggregate rocprofv3 --pmc CSVs: mean counter value per (kernel, grid size).

    python tools/pmc_summary.py <dir-with-run_counter_collection.csv> [...] [--filter conv]
"""
import argparse
import collections
import csv
import os


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return agg, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    merged = collections.defaultdict(dict)
    for d in a.dirs:
        agg, dur = load(d)
        for k, cs in agg.items():
            for c, v in cs.items():
                merged[k][c] = sum(v) / len(v)
            merged[k]["n"] = len(dur[k])
    for k, cs in sorted(merged.items()):
        if a.filter not in k[0]:
            continue
        print(k[0], "grid", k[1], {c: (round(v, 1) if v < 1e6 else f"{v:.4g}") for c, v in sorted(cs.items())})


if __name__ == "__main__":
    main()
