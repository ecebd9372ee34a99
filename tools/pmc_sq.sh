#!/bin/bash
# SQ counters (instruction mix / stall breakdown) of one short bench run, two passes.
# Usage: B=4096 bash tools/pmc_sq.sh [out_dir]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B=${B:-4096}
OUT=${1:-gpurun_out/sq}
mkdir -p $OUT && rm -rf $OUT/*
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $P -d $OUT/p$i -o p$i -f csv -- \
      python3 bench.py --batch $B --steps 2 --warmup 1 --no-cpu > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT $B $OUT/sq.json > /dev/null && python3 - "$OUT/sq.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, r in d.items():
    if not k.startswith("k_"): continue
    w = max(r.get("SQ_WAVES", 1), 1)
    keys = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
            "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS",
            "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VMEM_RD"]
    print(k, "waves", int(w), " ".join(f"{c[3:]}={r.get(c, 0) / w:.4g}" for c in keys))
PY
