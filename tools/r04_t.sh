#!/bin/bash
# Round-4 session T: k_cut_prep records stored 16 B per lane; k_pose issue priority by GN progress
# (variant) — parity, A/B against the previous library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "passed|failed|Error" $O/pytest.log | tail -5; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/ab_bench.sh $O 20 default build/ab_stage0 build/ab_head build/ab_posefair default
