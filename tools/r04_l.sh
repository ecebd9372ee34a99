#!/bin/bash
# Round-4 session L: LSD after moving the compact indices to the sort — LSD tests, 1024 / 2048 bench, kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lsd_gpu.py tests/test_pipeline_gpu.py tests/test_detector_gpu.py -v -m gpu --timeout 500 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"
grep -E "passed|failed" $O/pytest.log | tail -2
for n in 1024 2048; do
  timeout -k 10 300 python tools/bench_lsd.py --images $n --steps 5 --cpu-sample 0 --check 8 > $O/lsd_$n.log 2>&1 || { tail -5 $O/lsd_$n.log; exit 1; }
  tail -1 $O/lsd_$n.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o lsd -f csv -- python3 tools/bench_lsd.py --images 2048 \
    --steps 3 --cpu-sample 0 --check 2 > $O/lsd_prof.log 2>&1 || { tail -5 $O/lsd_prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/lsd_kernel_stats.csv \;
cut -d, -f1-4 $O/lsd_kernel_stats.csv | head -8
