#!/bin/bash
# Round-4 session D: line-cut certification diagnostics, then A/B of the cut search with the
# agreement test off (diagnostic build) against the product build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 300 python tools/cut_diag.py --batch 64 --frames 4 --lines 24 > $O/cut_diag.log 2>&1 || { tail -20 $O/cut_diag.log; exit 1; }
cat $O/cut_diag.log | cut -c1-400
timeout -k 10 600 python -u -m pytest tests/test_detector_gpu.py tests/test_pipeline_gpu.py tests/test_gpu_parity.py -x -q -m gpu \
   -k "stress or out_of_range or images_to_poses or detector" --timeout 300 --timeout-method thread > $O/pytest_fix.log 2>&1
tail -3 $O/pytest_fix.log
bash tools/ab_bench.sh $O/ab 8 build/agree_off default
