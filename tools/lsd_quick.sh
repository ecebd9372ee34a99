#!/bin/bash
# LSD GPU check: parity tests, bench line, rocprofv3 kernel stats (run under gpurun)
set -o pipefail
OUT=${1:-gpurun_out/lsd}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_lsd_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u tools/bench_lsd.py --images ${IMAGES:-1024} > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/tools/bench_lsd.py --images ${IMAGES:-1024} --steps 3 --cpu-sample 0 --check 0 > $R/$OUT/prof.log 2>&1 || exit 1
cut -d, -f1-4 $(find $R/$OUT/prof -name "*kernel_stats.csv") | head -7
