#!/bin/bash
# Round-4 session AA: k_cut_prep's staged record slices read four at a time — parity, A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "passed|failed|Error" $O/pytest.log | tail -5; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/ab_bench.sh $O 20 default build/ab_head default build/ab_head
