"""tools/pmc_summary.py windows the PMC / kernel-trace dispatches to bench.py's timed steps
(steps delimited by k_stereo_points), so roofline.traffic and the algorithmic bytes describe
the same launches."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_summary  # noqa: E402

STEP = "void gfpl::k_stereo_points<512, true>(gfpl::KParams, int)"
LINES_INIT = "void gfpl::k_stereo_lines<1, true, 512>(gfpl::KParams)"
LINES = "void gfpl::k_stereo_lines<2, false, 512>(gfpl::KParams)"


def _rows():
    """init (stereo lines only), then 6 steps of (stereo points, stereo lines), then a detection kernel"""
    rows, d = [], 1
    rows.append((d, LINES_INIT, 1000.0)); d += 1
    for j in range(1, 7):
        rows.append((d, STEP, 10.0 * j)); d += 1
        rows.append((d, LINES, 100.0 * j)); d += 1
    rows.append((d, "void gfpl::k_orb_blur(gfpl::OrbArgs)", 7.0))
    return rows


def test_counter_window(tmp_path):
    p = tmp_path / "fetch" / "run_counter_collection.csv"
    p.parent.mkdir()
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for d, k, v in _rows():
            w.writerow([d, k, "FETCH_SIZE", v])
            w.writerow([d, k, "WRITE_SIZE", 1.0])
    dst = tmp_path / "pmc.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(tmp_path), "64", str(dst),
                    "cfg2", "3", "2"], check=True, capture_output=True)
    out = json.loads(dst.read_text())
    assert (out["batch"], out["workload"], out["steps"], out["warmup"]) == (64, "cfg2", 3, 2)
    ks = out["kernels"]
    # timed steps 3, 4, 5 only (warm-up steps 1-2, the init dispatch and step 6 excluded)
    assert ks["k_stereo_points"]["FETCH_SIZE"] == 40.0 and ks["k_stereo_points"]["dispatches"] == 3
    assert ks["k_stereo_lines"]["FETCH_SIZE"] == 400.0 and ks["k_stereo_lines"]["window"] == "timed"
    assert ks["k_stereo_points"]["hbm_bytes_per_launch"] == (2 * 40.0 + 1.0) * 1024
    assert ks["k_orb_blur"]["window"] == "all"


def test_trace_window(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for d, k, v in _rows():
            w.writerow([d, k, 1000, 1000 + int(v * 1e6)])
    res = pmc_summary.trace(str(p), 3, 2)
    assert res["k_stereo_points"] == {"launches": 3, "avg_ms": 40.0}
    assert "k_orb_blur" not in res
