#!/bin/bash
# Batch-size sweep of bench.py (sequences per GPU); one JSON line per B.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/bsweep.jsonl
: > $out
for B in "$@"; do
  timeout -k 10 400 python bench.py --batch $B --steps 4 --warmup 1 --no-cpu > gpurun_out/bsweep_$B.log 2>&1 || { echo "B=$B failed rc=$?"; tail -5 gpurun_out/bsweep_$B.log; exit 1; }
  tail -1 gpurun_out/bsweep_$B.log >> $out
  python -c "import json,sys; d=json.loads(open('gpurun_out/bsweep_$B.log').read().strip().splitlines()[-1]); print($B, round(d['value']), round(d['ms_per_step'],2), d['stage_ms'], d['gen_s'])"
done
