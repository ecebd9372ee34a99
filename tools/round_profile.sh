#!/bin/bash
# Full measurement session on one GPU box:
#   1. GPU parity tests
#   2. PMC traffic passes (FETCH_SIZE, WRITE_SIZE; --kernel-trace only) on the bench
#      workload -> profiles/pmc_latest.json (read by bench.py's roofline.traffic)
#   3. the default bench line (with CPU baseline)
#   4. rocprofv3 --kernel-trace --stats of the same bench command
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/round
rm -rf $OUT && mkdir -p $OUT/pmc
BENCH_ARGS="$@"
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 500 rocprofv3 --kernel-trace --pmc $c -d $OUT/pmc/$c -o $c -f csv -- \
      python3 bench.py --no-cpu --steps 2 --warmup 1 $BENCH_ARGS > $OUT/pmc/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $OUT/pmc/$c.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/pmc ${PMC_BATCH:-16384} profiles/pmc_latest.json ${PMC_WORKLOAD:-cfg2} > $OUT/pmc/summary.txt && cp profiles/pmc_latest.json $OUT/pmc_latest.json || exit 1
timeout -k 10 600 python3 bench.py $BENCH_ARGS > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof -f csv -- python3 bench.py $BENCH_ARGS > $OUT/bench_rocprof.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/bench_rocprof.log; exit 1; }
tail -1 $OUT/bench_rocprof.log
ls $OUT/prof
