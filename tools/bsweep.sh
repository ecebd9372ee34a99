#!/bin/bash
# Batch-size sweep of bench.py (sequences per GPU, SURVEY §8(d) config 2: B swept 1…16384);
# one JSON line per B in gpurun_out/bsweep.jsonl.  Detection, host-fed and CPU legs are off:
# the sweep is about the tracking step's latency / throughput against B.
# usage: tools/bsweep.sh [steps] B1 B2 ...
set -o pipefail
mkdir -p gpurun_out
steps=$1; shift
out=gpurun_out/bsweep.jsonl
: > $out
for B in "$@"; do
  timeout -k 10 400 python bench.py --batch $B --steps $steps --warmup 3 --no-cpu --no-detect --no-host-fed --no-b1 \
      --parity-seqs $(( B < 4 ? B : 4 )) > gpurun_out/bsweep_$B.log 2>&1 || { echo "B=$B failed rc=$?"; tail -5 gpurun_out/bsweep_$B.log; exit 1; }
  tail -1 gpurun_out/bsweep_$B.log >> $out
  python -c "import json,sys; d=json.loads(open('gpurun_out/bsweep_$B.log').read().strip().splitlines()[-1]); print($B, round(d['value']), round(d['ms_per_step'],3), d['stage_ms'], d['kernel_ms'], d['parity_sampled']['mismatches'])"
done
