#!/bin/bash
# Round-4 session P: line-cut search balance (wave durations from the -DGFPL_CUT_CLOCK build) at
# B = 16384, the bench workload.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04p
mkdir -p $O
export GFPL_LIB_DIR=$(realpath build/ab_clock)
timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 2 \
    --dump-records $O/records.npy > $O/bench_clock.log 2>&1 || { tail -5 $O/bench_clock.log; exit 1; }
unset GFPL_LIB_DIR
python tools/cut_balance.py $O/records.npy | tee $O/balance.json
