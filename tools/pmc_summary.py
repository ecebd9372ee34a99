#!/usr/bin/env python3
"""Per-kernel PMC summary of tools/pmc.sh output.

Reads every *counter_collection.csv under the given directory, averages each
counter per dispatch per kernel, and writes profiles/pmc_latest.json with the
HBM traffic per launch: bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB units from
rocprofv3; FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM: gfx950 reports half
of the bytes of wide coalesced reads).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"gfpl(?:::|\d+)(k_\w+?)(?:E|I|<|\(|$)", name)
    if m:
        return m.group(1)
    m = re.search(r"(k_[a-z0-9_]+)", name)
    return m.group(1) if m else name[:60]


def main():
    d = sys.argv[1]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else None
    workload = sys.argv[4] if len(sys.argv) > 4 else "cfg2"
    vals = defaultdict(lambda: defaultdict(dict))   # kernel -> counter -> {dispatch: value}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                c = row.get("Counter_Name")
                v = float(row.get("Counter_Value", 0) or 0)
                disp = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[k][c][disp] = vals[k][c].get(disp, 0.0) + v
    out = {"batch": batch, "workload": workload, "kernels": {}}
    for k in sorted(vals):
        row = {c: sum(v.values()) / max(1, len(v)) for c, v in vals[k].items()}
        row["dispatches"] = max(len(v) for v in vals[k].values())
        if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            row["hbm_bytes_per_launch"] = (2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024.0
        if row.get("SQ_WAVES"):
            row["valu_insts_per_wave"] = row.get("SQ_INSTS_VALU", 0) / row["SQ_WAVES"]
            row["lds_insts_per_wave"] = row.get("SQ_INSTS_LDS", 0) / row["SQ_WAVES"]
        if row.get("SQ_WAVE_CYCLES"):
            w = row["SQ_WAVE_CYCLES"]
            row["frac_wait_any"] = row.get("SQ_WAIT_ANY", 0) / w
            row["frac_wait_inst"] = row.get("SQ_WAIT_INST_ANY", 0) / w
            row["frac_active"] = row.get("SQ_ACTIVE_INST_ANY", 0) / w if "SQ_ACTIVE_INST_ANY" in row else None
        out["kernels"][k] = row
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(root, "profiles", "pmc_latest.json")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    # human-readable
    keys = ["dispatches", "hbm_bytes_per_launch", "valu_insts_per_wave", "lds_insts_per_wave", "SQ_WAVES",
            "frac_wait_any", "frac_wait_inst", "frac_active", "SQ_LDS_BANK_CONFLICT"]
    for k, row in out["kernels"].items():
        print(k, {x: (round(row[x], 3) if isinstance(row.get(x), float) else row.get(x)) for x in keys if x in row})
    print("wrote", dst)


if __name__ == "__main__":
    main()
