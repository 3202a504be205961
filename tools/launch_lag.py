"""Host enqueue vs GPU start for one step: joins a rocprofv3 HIP runtime trace with its kernel
trace on the correlation id.  Per launch: when the host call started / returned, when the
kernel started on its queue, and the lead (kernel start - host return; negative means the
GPU was waiting for the host).  Host calls that block for long are flagged -- a launch that
returns late is the host waiting for queue space or a synchronisation.

    python tools/launch_lag.py <kernel_trace.csv> <hip_api_trace.csv> [--step -2]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ktrace")
    ap.add_argument("apitrace")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--marker", default="conv_c8r_kernel<7, 7, 1, 1>")
    ap.add_argument("--block-us", type=float, default=20.0, help="flag host calls longer than this")
    a = ap.parse_args()
    ks = list(csv.DictReader(open(a.ktrace)))
    api = list(csv.DictReader(open(a.apitrace)))
    by_corr = {r["Correlation_Id"]: r for r in api}
    rows = []
    for r in ks:
        h = by_corr.get(r["Correlation_Id"])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                     r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:56],
                     int(h["Start_Timestamp"]) if h else None, int(h["End_Timestamp"]) if h else None))
    rows.sort(key=lambda x: x[4] if x[4] is not None else x[0])
    marks = sorted(x[0] for x in rows if a.marker in x[3])
    t0, t1 = list(zip(marks, marks[1:]))[a.step]
    # host calls of the step: from the marker's host call to the next marker's
    hm = sorted(x[4] for x in rows if a.marker in x[3] and x[4] is not None)
    h0, h1 = [(p, q) for p, q in zip(hm, hm[1:])][a.step]
    print(f"GPU step span {(t1 - t0) / 1e3:.1f} us; host enqueue span {(h1 - h0) / 1e3:.1f} us; "
          f"host starts the step {(t0 - h0) / 1e3:.1f} us before the GPU does")
    blocked = collections.Counter()
    for s, e, q, n, hs, he in rows:
        if hs is None or not (h0 <= hs < h1):
            continue
        lead = (s - he) / 1e3
        hd = (he - hs) / 1e3
        flag = "  <-- host blocked" if hd > a.block_us else ""
        if hd > a.block_us:
            blocked[n] += hd
        print(f"host {(hs - t0) / 1e3:9.1f} +{hd:7.1f}  gpu {(s - t0) / 1e3:9.1f}  lead {lead:8.1f}  q{q}  {n}{flag}")
    # other (non-launch) host calls in the step that took long: syncs, event waits, copies
    print("\nlong non-launch HIP calls in the step:")
    for r in api:
        hs, he = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if h0 <= hs < h1 and (he - hs) / 1e3 > a.block_us and "Launch" not in r["Function"]:
            print(f"  host {(hs - t0) / 1e3:9.1f} +{(he - hs) / 1e3:7.1f}  {r['Function']}")
    if blocked:
        print("\nhost time blocked inside launches, by kernel:")
        for n, v in blocked.most_common(10):
            print(f"  {v:8.1f} us  {n}")


if __name__ == "__main__":
    main()
