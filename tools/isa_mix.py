#!/usr/bin/env python3
"""Instruction mix of one kernel's ISA (hipcc -S output), from its first
depth-1 loop header to the end of the function: f64 VALU / other VALU / DPP /
SALU / LDS / VMEM counts.  Usage: tools/isa_mix.py file.s kernel_symbol"""
import collections
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = lines[start:end]
    hdr = next((i for i, l in enumerate(body) if "Loop Header: Depth=1" in l), 0)
    cnt = collections.Counter()
    for l in body[hdr:]:
        t = l.strip().split()
        if not t or t[0].startswith(";") or t[0].startswith("."):
            continue
        op = t[0]
        if op.startswith("v_"):
            cat = "v_f64" if "f64" in op else ("v_dpp" if "dpp" in l else "v_other")
        elif op.startswith("s_"):
            cat = "salu"
        elif op.startswith("ds_"):
            cat = "lds"
        elif op.startswith(("global", "scratch", "buffer", "flat")):
            cat = "vmem"
        else:
            cat = "other"
        cnt[cat] += 1
    print(f"{sym}: {end - start} lines, loop body from +{hdr}: {dict(cnt)}")


if __name__ == "__main__":
    main()
