#!/bin/bash
# SQ counters of the LSD kernels (tools/bench_lsd.py), one pass per counter set.
# Usage: bash tools/pmc_lsd.sh [out_dir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/lsdsq}
mkdir -p $OUT && rm -rf $OUT/*
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $OUT/p$i -o p$i -f csv -- \
      python3 tools/bench_lsd.py --images 1024 --steps 1 --warmup 0 --cpu-sample 0 --check 0 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, os, re, sys
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(dict))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        m = re.search(r"(k_lsd_[a-z0-9_]+)", row.get("Kernel_Name", ""))
        if not m: continue
        d = (f, row.get("Dispatch_Id"))
        vals[m.group(1)][row["Counter_Name"]][d] = vals[m.group(1)][row["Counter_Name"]].get(d, 0.0) + float(row["Counter_Value"] or 0)
for k, cs in vals.items():
    avg = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    w = max(avg.get("SQ_WAVES", 1), 1)
    print(k, "waves", int(w), " ".join(f"{c[3:]}={avg[c] / w:.4g}" for c in sorted(avg) if c != "SQ_WAVES"))
PY
