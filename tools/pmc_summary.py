#!/usr/bin/env python3
"""Per-kernel PMC summary of a bench run's rocprofv3 --pmc passes, over the bench's timed window.

    pmc_summary.py DIR BATCH DST WORKLOAD STEPS WARMUP

Reads every *counter_collection.csv under DIR (one directory per pass) and averages each
counter per dispatch per kernel over the TIMED steps only: a dispatch belongs to step j when
it comes after the j-th k_stereo_points dispatch of its run (every insertStereoPair starts
with it; j = 0 is the initial frame), and the window is steps WARMUP+1 .. WARMUP+STEPS — the
launches bench.py's HIP-event times, algorithmic bytes and counts average.  Kernels with no
dispatch in the window (detection, initialisation) are averaged over all their dispatches
and flagged `window: "all"`.  Writes DST with the HBM traffic per launch, bytes = 2 x
FETCH_SIZE + WRITE_SIZE (KB units from rocprofv3; FETCH_SIZE doubled per
MI355X_MICROARCH.md §HBM: gfx950 reports half of the bytes of wide coalesced reads), and the
window (batch, workload, steps, warmup) that bench.py's load_pmc checks.

    pmc_summary.py --trace KERNEL_TRACE_CSV STEPS WARMUP

prints the mean kernel durations of a --kernel-trace run over the same window (for the
rocprofv3 --stats cross-check of `roofline.avg_launch_ms`).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

STEP_KERNEL = "k_stereo_points"


def short(name: str) -> str:
    m = re.search(r"gfpl(?:::|\d+)(k_\w+?)(?:E|I|<|\(|$)", name)
    if m:
        return m.group(1)
    m = re.search(r"(k_[a-z0-9_]+)", name)
    return m.group(1) if m else name[:60]


def step_of(dispatch_ids_of_step_kernel, d):
    """Number of step-kernel dispatches with id <= d (the step a dispatch belongs to)."""
    lo, hi = 0, len(dispatch_ids_of_step_kernel)
    while lo < hi:
        mid = (lo + hi) // 2
        if dispatch_ids_of_step_kernel[mid] <= d:
            lo = mid + 1
        else:
            hi = mid
    return lo


def windowed(rows, steps, warmup, value):
    """rows: dicts of one run with Dispatch_Id and Kernel_Name -> {kernel: (values in window, all values)}"""
    sk = sorted({int(r["Dispatch_Id"]) for r in rows if short(r["Kernel_Name"]) == STEP_KERNEL})
    out = defaultdict(lambda: ([], []))
    for r in rows:
        d = int(r["Dispatch_Id"])
        k = short(r["Kernel_Name"])
        v = value(r)
        out[k][1].append((d, v))
        if warmup + 1 <= step_of(sk, d) <= warmup + steps:
            out[k][0].append((d, v))
    return out


def summary(d, batch, workload, steps, warmup):
    # kernel -> counter -> [(in-window values), (all values)] per dispatch
    vals = defaultdict(lambda: defaultdict(lambda: ([], [])))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        per = defaultdict(dict)   # (dispatch, kernel) -> {counter: summed value}
        for r in rows:
            key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
            c = r["Counter_Name"]
            per[key][c] = per[key].get(c, 0.0) + float(r.get("Counter_Value") or 0)
        disp_rows = [{"Dispatch_Id": k[0], "Kernel_Name": k[1], "c": v} for k, v in per.items()]
        counters = {c for v in per.values() for c in v}
        for c in counters:
            w = windowed([r for r in disp_rows if c in r["c"]], steps, warmup, lambda r, c=c: r["c"][c])
            for k, (win, alld) in w.items():
                vals[k][c][0].extend(win)
                vals[k][c][1].extend(alld)
    out = {"batch": batch, "workload": workload, "steps": steps, "warmup": warmup,
           "window": f"dispatches of steps {warmup + 1}..{warmup + steps} (after the warm-up), "
                     f"steps delimited by {STEP_KERNEL}",
           "kernels": {}}
    for k in sorted(vals):
        row, used = {}, "timed"
        for c, (win, alld) in vals[k].items():
            src = win if win else alld
            if not win:
                used = "all"
            row[c] = sum(v for _, v in src) / max(1, len(src))
        row["dispatches"] = max(len(w if w else a) for w, a in vals[k].values())
        row["window"] = used
        if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            row["hbm_bytes_per_launch"] = (2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024.0
            # FETCH_SIZE as counted for dword-aligned gathers (tools/probe/fetch_calib.hip,
            # profiles/r04_fcal: 0.95 known bytes per counted byte, against 2.00 for 16-B streams)
            row["hbm_bytes_per_launch_gather_cal"] = (row["FETCH_SIZE"] / 0.95 + row["WRITE_SIZE"]) * 1024.0
        if row.get("SQ_WAVES"):
            row["valu_insts_per_wave"] = row.get("SQ_INSTS_VALU", 0) / row["SQ_WAVES"]
            row["lds_insts_per_wave"] = row.get("SQ_INSTS_LDS", 0) / row["SQ_WAVES"]
        if row.get("SQ_WAVE_CYCLES"):
            w = row["SQ_WAVE_CYCLES"]
            row["frac_wait_any"] = row.get("SQ_WAIT_ANY", 0) / w
            row["frac_wait_inst"] = row.get("SQ_WAIT_INST_ANY", 0) / w if "SQ_WAIT_INST_ANY" in row else None
            row["frac_active"] = row.get("SQ_ACTIVE_INST_ANY", 0) / w if "SQ_ACTIVE_INST_ANY" in row else None
            # MI355X_MICROARCH.md §rocprofv3: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES
            if row["frac_wait_inst"] is not None and row["frac_active"] is not None:
                row["cycle_closure"] = row["frac_wait_any"] + row["frac_wait_inst"] + row["frac_active"]
            # mean resident waves per SIMD: wave-cycles (quad-cycles x 4) over the kernel's cycles
            # (GRBM_GUI_ACTIVE summed over the 8 XCDs) x 1024 SIMDs
            if row.get("GRBM_GUI_ACTIVE"):
                row["occupancy_waves_per_simd"] = 4.0 * w / (row["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
        out["kernels"][k] = row
    return out


def trace(path, steps, warmup):
    with open(path) as fh:
        rows = list(csv.DictReader(fh))
    w = windowed(rows, steps, warmup, lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    res = {}
    for k, (win, alld) in sorted(w.items()):
        if win:
            res[k] = {"launches": len(win), "avg_ms": sum(v for _, v in win) / len(win)}
    return res


def main():
    if sys.argv[1] == "--trace":
        res = trace(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
        print(json.dumps({"window": f"steps {int(sys.argv[4]) + 1}..{int(sys.argv[4]) + int(sys.argv[3])}",
                          "kernels": res}, indent=1))
        return
    d, batch, dst, workload, steps, warmup = sys.argv[1:7]
    out = summary(d, int(batch), workload, int(steps), int(warmup))
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    keys = ["dispatches", "window", "hbm_bytes_per_launch", "hbm_bytes_per_launch_gather_cal", "valu_insts_per_wave", "lds_insts_per_wave", "SQ_WAVES",
            "frac_wait_any", "frac_wait_inst", "frac_active", "cycle_closure", "occupancy_waves_per_simd",
            "SQ_LDS_BANK_CONFLICT"]
    for k, row in out["kernels"].items():
        print(k, {x: (round(row[x], 3) if isinstance(row.get(x), float) else row.get(x)) for x in keys if x in row})
    print("wrote", dst)


if __name__ == "__main__":
    main()
