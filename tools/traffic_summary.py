"""HBM traffic per launch from rocprofv3 --pmc passes (tools/gpu_traffic.sh).

FETCH_SIZE / WRITE_SIZE are in KB per dispatch.  Per MI355X_MICROARCH.md (HBM
section) FETCH_SIZE counts HALF the bytes of wide coalesced reads on gfx950
(TCC_EA0_RDREQ x 64 B for 128-B requests), so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane stores.  Prints one JSON object:
{kernel_family: {"fetch_kb_raw", "write_kb", "hbm_bytes", "launches"}}.
"""
import collections
import csv
import json
import os
import sys

FAMILIES = {"fwd": ("conv_pp_kernel<3, 3, 256, false, false, false, false>",),
            "dgrad": ("conv_pp_kernel<3, 3, 256, false, false, false, false>", "reflect_ring_kernel"),
            "wgrad": ("wgrad_pc_kernel<8>", "wgrad_pc_reduce")}


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    p = os.path.join(d, "run_counter_collection.csv")
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main(root):
    out = {}
    for fam, names in FAMILIES.items():
        f = per_kernel(os.path.join(root, f"fetch_{fam}"), "FETCH_SIZE")
        w = per_kernel(os.path.join(root, f"write_{fam}"), "WRITE_SIZE")
        fk = wk = 0.0
        n = 0
        for name in names:
            fv = [v for k, vs in f.items() if name in k for v in vs]
            wv = [v for k, vs in w.items() if name in k for v in vs]
            if not fv or not wv:
                continue
            fv, wv = fv[1:] or fv, wv[1:] or wv   # drop the cold first launch
            fk += sum(fv) / len(fv)
            wk += sum(wv) / len(wv)
            n = max(n, len(fv))
        out[fam] = {"fetch_kb_raw": round(fk, 1), "write_kb": round(wk, 1),
                    "hbm_bytes": round((2 * fk + wk) * 1024), "launches": n}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
