"""Per-launch HBM bytes and SQ counters of the 64-channel conv family from tools/gpu_pmc_c64.sh
(the same counter handling as tools/traffic_summary.py: FETCH_SIZE doubled per the gfx950
correction, plus WRITE_SIZE; the cold first dispatch dropped).  Algorithmic bytes at B=16:
the operands read once and the output written once, bf16."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic_summary import fam_mean, per_kernel  # noqa: E402

MB = 16 * 256 * 256 * 2          # one bf16 channel of a 256^2 B=16 map, bytes
ALG = {"down1_fwds": 64 * MB + 128 * MB, "down1_fwd": 64 * MB + 128 * MB, "vgg12_fwd": 64 * MB + 64 * MB,
       "vgg21_fwd": (64 * MB + 128 * MB) // 4, "up2_fwds": 192 * MB + 64 * MB,
       "up2_dgrad": 64 * MB + 192 * MB, "up2_wgrad": 192 * MB + 64 * MB}
FLOP = {"down1_fwds": 64 * 128, "down1_fwd": 64 * 128, "vgg12_fwd": 64 * 64, "vgg21_fwd": 64 * 128 // 4,
        "up2_fwds": 192 * 64, "up2_dgrad": 192 * 64, "up2_wgrad": 192 * 64}   # x 2 * 16 * 256^2 * 9


def main(root):
    out = {}
    for case, alg in ALG.items():
        fk, n, names = fam_mean(per_kernel(os.path.join(root, f"fetch_{case}"), "FETCH_SIZE"))
        wk, _, _ = fam_mean(per_kernel(os.path.join(root, f"write_{case}"), "WRITE_SIZE"))
        hb = round((2 * fk + wk) * 1024)
        e = {"kernels": sorted(names), "hbm_bytes": hb, "alg_bytes": alg, "ratio": round(hb / alg, 3),
             "flop": 2 * 16 * 256 * 256 * 9 * FLOP[case], "launches": n}
        for sq in ("sq1", "sq2"):
            for cnt in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                        "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_MFMA",
                        "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAVES", "GRBM_GUI_ACTIVE"):
                v = per_kernel(os.path.join(root, f"{sq}_{case}"), cnt)
                if v:
                    e[cnt] = round(fam_mean(v)[0])
        out[case] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
