#!/bin/bash
# Round-4 session AC: k_stereo_points setup — record fields kept in registers (no second read of
# the right keypoints), one block scan for both histograms — parity, A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_detector_gpu.py tests/test_pipeline_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "passed|failed|Error" $O/pytest.log | tail -5; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash tools/ab_bench.sh $O 20 default build/ab_head default build/ab_head
