"""Per-stream busy time, idle gaps and overlap from a rocprofv3 kernel trace, over the last
--steps steps (a step = the span between consecutive launches of --marker, default the
generator's first conv: the dense-K 7x7 kernel).

    python tools/stream_gaps.py <run_kernel_trace.csv> [--steps 5]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="conv_c8r_kernel<7, 7, 1, 1>")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace))]
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                 r["Kernel_Name"].replace("(anonymous namespace)::", "")) for r in rows))
    marks = [k[0] for k in ks if a.marker in k[3]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker launches")
    t0, t1 = marks[-a.steps - 1], marks[-1]
    span = (t1 - t0) / a.steps / 1e3
    by_q = collections.defaultdict(list)
    for s, e, q, n in ks:
        if t0 <= s < t1:
            by_q[q].append((s, e, n))
    print(f"step span (marker to marker): {span:.1f} us")
    allint = []
    for q, v in sorted(by_q.items()):
        busy = sum(e - s for s, e, _ in v) / a.steps / 1e3
        gaps = collections.Counter()
        gsum = 0.0
        for (s0, e0, n0), (s1, e1, n1) in zip(v, v[1:]):
            g = (s1 - e0) / 1e3
            if g > 0:
                gsum += g
                gaps[(n0.split("(")[0][:40], n1.split("(")[0][:40])] += g
        print(f"queue {q}: {len(v) / a.steps:.0f} launches/step, busy {busy:.1f} us/step, "
              f"gaps {gsum / a.steps:.1f} us/step")
        for (n0, n1), g in gaps.most_common(8):
            print(f"    {g / a.steps:7.1f} us/step after {n0} -> {n1}")
        allint += [(s, e) for s, e, _ in v]
    allint.sort()
    cover, cur_s, cur_e = 0, None, None
    for s, e in allint:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                cover += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    cover += cur_e - cur_s
    print(f"GPU busy (any queue): {cover / a.steps / 1e3:.1f} us/step of {span:.1f}")


if __name__ == "__main__":
    main()
