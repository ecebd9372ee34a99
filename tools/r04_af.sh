#!/bin/bash
# Round-4 session AF: the exact-sum flush with eight entries per pass (the r = 0 infos read from HBM
# in the chain) — parity, A/B against four per pass, per-wave durations of both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "passed|failed|Error" $O/pytest.log | tail -5; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/ab_bench.sh $O 20 default build/ab_f4 default build/ab_f4
for v in ab_clock ab_clock4; do
  export GFPL_LIB_DIR=$(realpath build/$v)
  timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 2 \
      --dump-records $O/records_$v.npy > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 1; }
  echo "$v $(python tools/cut_balance.py $O/records_$v.npy | head -1 | cut -c1-200)"
done
unset GFPL_LIB_DIR
