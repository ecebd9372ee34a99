#!/usr/bin/env python3
"""Per-kernel register / LDS / scratch table of the HIP library (DESIGN.md §4 register notes).

Compiles every gf-pl-slam_amd/csrc/*.hip for the device only with the product flags of the
Makefile plus `-Rpass-analysis=kernel-resource-usage` and tabulates the compiler's remarks
(VGPRs, AGPRs, SGPRs, VGPR / SGPR spills, scratch bytes per lane, LDS bytes per block, the
occupancy the compiler derives from them).  Runs on the CPU (hipcc cross-compiles).

usage: python3 tools/kernel_resources.py [out.md]
"""
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-Iinclude",
         "--cuda-device-only", "-c", "-Rpass-analysis=kernel-resource-usage", "-o", os.devnull]
FIELDS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("TotalSGPRs", "sgpr"), ("VGPRs Spill", "vspill"),
          ("SGPRs Spill", "sspill"), ("ScratchSize [bytes/lane]", "scratch"),
          ("LDS Size [bytes/block]", "lds"), ("Occupancy [waves/SIMD]", "occ")]


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                             check=True).stdout.split("\n")
        return [re.sub(r"\(.*", "", o).replace("gfpl::", "") for o in out[:len(names)]]
    except (OSError, subprocess.CalledProcessError):
        return names


def resources(src):
    r = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + [src], cwd=ROOT, capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{src}: hipcc failed\n{r.stderr[-2000:]}")
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1), "file": os.path.basename(src)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([^:]+): (\S+) \[-Rpass", line)
        if m and cur is not None:
            for key, short in FIELDS:
                if m.group(1).strip() == key:
                    cur[short] = m.group(2)
    return rows


def main():
    rows = []
    for src in sorted(glob.glob(os.path.join(ROOT, "gf-pl-slam_amd/csrc/*.hip"))):
        rows += resources(os.path.relpath(src, ROOT))
    for r, d in zip(rows, demangle([r["name"] for r in rows])):
        r["kernel"] = d
    lines = ["| file | kernel | VGPR | AGPR | SGPR | VGPR spill | SGPR spill | scratch B/lane | LDS B/block | waves/SIMD |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        lines.append("| " + " | ".join([r["file"], f"`{r['kernel']}`"] +
                                       [r.get(s, "?") for _, s in FIELDS]) + " |")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
