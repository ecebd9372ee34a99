#!/bin/bash
# Round-4 session AE: the exact-sum flush served by the whole wave (64 lines per round) —
# parity (exact / mixed / proven steps), A/B, and the per-wave durations against their exact-step counts.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "passed|failed|Error" $O/pytest.log | tail -5; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/ab_bench.sh $O 20 default build/ab_head default build/ab_head
export GFPL_LIB_DIR=$(realpath build/ab_clock)
timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 2 \
    --dump-records $O/records.npy > $O/bench_clock.log 2>&1 || { tail -5 $O/bench_clock.log; exit 1; }
unset GFPL_LIB_DIR
python tools/cut_balance.py $O/records.npy | tee $O/balance.json
