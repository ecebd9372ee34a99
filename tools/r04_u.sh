#!/bin/bash
# Round-4 session U: issue priority by phase in k_stereo_points / k_cut_prep and by GN progress in
# k_pose (default on), k_cut_finish's invCovPose staged through LDS — parity, A/B per change.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_detector_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "passed|failed|Error" $O/pytest.log | tail -5; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/ab_bench.sh $O 20 default build/ab_nosp build/ab_noprepprio build/ab_nofin default
