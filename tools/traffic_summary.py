"""HBM traffic and MFMA counters per launch from rocprofv3 --pmc passes (tools/gpu_traffic.sh).

Each pass runs tools/bench_conv.py on ONE family of the resblock conv (fwd+stats,
dgrad incl. the reflect ring, wgrad incl. its reduce), so every kernel of the pass
that is not a torch setup kernel or the weight pack belongs to that family; the
family's per-launch figure is the sum over its kernels of each kernel's mean over
its dispatches (the first, cold dispatch dropped).

FETCH_SIZE / WRITE_SIZE are in KB per dispatch.  Per MI355X_MICROARCH.md (HBM
section) FETCH_SIZE counts HALF the bytes of wide coalesced reads on gfx950
(TCC_EA0_RDREQ x 64 B for 128-B requests), so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane stores.  Prints one JSON object:
{family: {"kernels", "fetch_kb_raw", "write_kb", "hbm_bytes", "alg_bytes", "ratio",
          "launches", [SQ counters per launch]}}.
"""
import collections
import csv
import json
import os
import sys

FAMILIES = ("fwd", "dgrad", "wgrad")
SKIP = ("at::", "weight_pack", "elementwise", "distribution", "fill", "copy")
# algorithmic bytes of one resblock launch at B=16, 64x64x256 bf16: x + y (or dY + dX,
# or x + dY) 2 x 33.55 MB, plus the 1.18 MB bf16 weight image (fp32 dW for wgrad: 2.36 MB)
ALG = {"fwd": 2 * 16 * 64 * 64 * 256 * 2 + 256 * 256 * 9 * 2,
       "dgrad": 2 * 16 * 64 * 64 * 256 * 2 + 256 * 256 * 9 * 2,
       "wgrad": 2 * 16 * 64 * 64 * 256 * 2 + 256 * 256 * 9 * 4}


def kernel_name(k):
    """'void (anonymous namespace)::conv_pp_kernel<3, 3, 256, ...>(irgan_conv_desc, ...)' ->
    'conv_pp_kernel<3, 3, 256, ...>' (the template arguments name the variant)."""
    k = k.replace("(anonymous namespace)::", "")
    if k.startswith("void "):
        k = k[5:]
    depth, end = 0, len(k)
    for i, ch in enumerate(k):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            end = i
            break
    return k[:end][:120]


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    p = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(p):
        return vals
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == counter and not any(s in r["Kernel_Name"] for s in SKIP):
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def fam_mean(vals):
    tot, n, names = 0.0, 0, []
    for k, vs in vals.items():
        vs = vs[1:] or vs   # drop the cold first dispatch
        tot += sum(vs) / len(vs)
        n = max(n, len(vs))
        names.append(kernel_name(k))
    return tot, n, names


def main(root):
    out = {}
    for fam in FAMILIES:
        fk, n, names = fam_mean(per_kernel(os.path.join(root, f"fetch_{fam}"), "FETCH_SIZE"))
        wk, _, _ = fam_mean(per_kernel(os.path.join(root, f"write_{fam}"), "WRITE_SIZE"))
        hb = round((2 * fk + wk) * 1024)
        out[fam] = {"kernels": sorted(names), "fetch_kb_raw": round(fk, 1), "write_kb": round(wk, 1),
                    "hbm_bytes": hb, "alg_bytes": ALG[fam], "ratio": round(hb / ALG[fam], 3), "launches": n}
        for sq in ("sq1", "sq2"):
            p = os.path.join(root, f"{sq}_{fam}", "run_counter_collection.csv")
            if not os.path.exists(p):
                continue
            ctr = collections.defaultdict(lambda: collections.defaultdict(list))
            for r in csv.DictReader(open(p)):
                if not any(s in r["Kernel_Name"] for s in SKIP):
                    ctr[r["Counter_Name"]][r["Kernel_Name"]].append(float(r["Counter_Value"]))
            for c, per in ctr.items():
                out[fam][c] = round(fam_mean(per)[0], 1)
        if "SQ_INSTS_MFMA" in out[fam]:
            # one 16x16x32 bf16 MFMA = 16384 FLOP; 77.3 GFLOP per launch at B=16
            out[fam]["mfma_flop_over_alg"] = round(out[fam]["SQ_INSTS_MFMA"] * 16384 / (2 * 16 * 64 * 64 * 256 * 256 * 9),
                                                   3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in out[fam] and "GRBM_GUI_ACTIVE" in out[fam]:
            pass   # the busy fraction needs the CU count: see DESIGN.md section 3
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
