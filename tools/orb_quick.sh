#!/bin/bash
# ORB row on the GPU: parity tests, throughput line, rocprof kernel stats.
# Usage: bash tools/orb_quick.sh [OUT=gpurun_out/orb]
set -o pipefail
OUT=${OUT:-gpurun_out/orb}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_orb_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_orb.py ${ORB_ARGS} > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o orb -- python3 tools/bench_orb.py --cpu-sample 0 --check 0 --steps 5 ${ORB_ARGS} > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
find $OUT/prof -name "orb_kernel_stats.csv" | xargs cat | cut -d, -f1-4 | cut -c1-120
