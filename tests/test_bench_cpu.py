"""bench.py's host-side contract pieces (no GPU): the workload label names a BASELINE config only
for that config's exact per-GPU shape, the algorithmic FLOPs per image are SURVEY.md 8d's
measured figures, and the roofline's traffic figure comes from the newest committed PMC file."""
import os

import bench


def test_workload_label_names_only_exact_baseline_shapes():
    assert bench.workload_label(256, 256, 16, "bf16", 1).endswith("(BASELINE configs[1])")
    assert bench.workload_label(256, 256, 16, "bf16", 8).endswith("(BASELINE configs[2])")
    assert bench.workload_label(512, 640, 4, "bf16", 8).endswith("(BASELINE configs[3] per-GPU shape)")
    assert bench.workload_label(256, 256, 32, "fp8", 8).endswith("(BASELINE configs[4] per-GPU shape)")
    for args in ((256, 256, 32, "bf16", 1), (256, 256, 16, "fp8", 1), (512, 512, 4, "bf16", 1), (64, 64, 2, "bf16", 1)):
        assert "BASELINE" not in bench.workload_label(*args), args


def test_min_gflop_per_img_is_the_survey_figure():
    assert bench.min_gflop_per_img(256, 256) == 534.85
    assert bench.min_gflop_per_img(512, 640) == 2680.06
    assert bench.min_gflop_per_img(64, 64) == 33.05
    assert abs(bench.min_gflop_per_img(128, 128) - 534.85 / 4) < 1e-9


def test_pmc_traffic_reads_the_newest_committed_file():
    p = bench.pmc_file()
    assert p and os.path.basename(p).startswith("r") and p.endswith("_pmc_traffic.json")
    for fam in ("fwd", "dgrad", "wgrad"):
        t = bench.pmc_traffic(fam)
        # at least the algorithmic bytes of one ResnetBlock conv (x read, y written: 2 x 33.5 MB)
        assert t is not None and t >= 67e6, (fam, t)
