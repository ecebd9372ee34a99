#!/bin/bash
# Round-4 session S: line-cut search waves exchanging their progress with their SIMD partner
# (GFPL_CUT_FAIR 2) — parity, A/B against the quarter-step priority (1), the per-wave durations;
# k_cut_prep without its comparison-data stores (timing probe, 3 steps).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "passed|failed|Error" $O/pytest.log | tail -5; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/ab_bench.sh $O 20 default build/ab_fair1 default
export GFPL_LIB_DIR=$(realpath build/ab_clock)
timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 2 \
    --dump-records $O/records.npy > $O/bench_clock.log 2>&1 || { tail -5 $O/bench_clock.log; exit 1; }
python tools/cut_balance.py $O/records.npy | tee $O/balance.json
export GFPL_LIB_DIR=$(realpath build/ab_prepprobe)
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 0 \
    > $O/bench_prepprobe.log 2>&1 || { tail -5 $O/bench_prepprobe.log; exit 1; }
unset GFPL_LIB_DIR
python -c "import json; d=json.loads(open('$O/bench_prepprobe.log').read().strip().splitlines()[-1]); print('prepprobe', d['kernel_ms'])"
