#!/bin/bash
# Full measurement session on one GPU box (every GPU step under its own time limit,
# chained so the script stops at the first failure):
#   1. GPU parity tests (skip with SKIP_TESTS=1)
#   2. PMC passes on the bench workload at the bench's own --steps/--warmup (FETCH_SIZE,
#      WRITE_SIZE, SQ instruction / cycle counters; --kernel-trace only, one group per pass;
#      no CPU baseline / parity / host-fed / detection so the step kernels run only in the
#      init + warm-up + timed steps) -> $OUT/pmc_latest.json, windowed to the timed steps by
#      tools/pmc_summary.py, copied to profiles/pmc_latest.json (read by bench.py:
#      roofline.traffic, roofline_valu)
#   3. the default bench line (CPU baseline + sampled parity)
#   4. rocprofv3 --kernel-trace --stats of the same bench command (+ the kernel durations
#      over the timed window: $OUT/trace_window.json)
# Usage: bash tools/round_profile.sh [bench args...]   (env: SKIP_TESTS=1, OUT=..., STEPS, WARMUP;
#   PHASE=pmc: steps 1-2 only, PHASE=bench: steps 3-4 only — at B = 65536 the whole session exceeds
#   one GPU call's limit)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/round}
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
WORKLOAD=${PMC_WORKLOAD:-cfg2}
PHASE=${PHASE:-all}
[ "$PHASE" = bench ] || rm -rf $OUT
mkdir -p $OUT/pmc
BENCH_ARGS="--steps $STEPS --warmup $WARMUP --workload $WORKLOAD $@"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
pmc() {   # name counters...
  local name=$1; shift
  timeout -k 10 500 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/pmc/$name -o $name -f csv -- \
      python3 bench.py --no-cpu --parity-seqs 0 --no-detect --no-host-fed --no-b1 --proven-steps 0 $BENCH_ARGS > $OUT/pmc/$name.log 2>&1 \
    || { echo "pmc $name failed"; tail -5 $OUT/pmc/$name.log; return 1; }
}
if [ "$PHASE" != bench ]; then
pmc fetch FETCH_SIZE && \
pmc write WRITE_SIZE && \
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY && \
pmc sq2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
B=$(python3 -c "import json,sys; print(json.loads([l for l in open('$OUT/pmc/fetch.log') if l.startswith('{')][-1])['config']['sequences_per_gpu'])") || exit 1
python3 tools/pmc_summary.py $OUT/pmc $B $OUT/pmc_latest.json $WORKLOAD $STEPS $WARMUP > $OUT/pmc/summary.txt \
  && cp $OUT/pmc_latest.json profiles/pmc_latest.json || exit 1
fi
[ "$PHASE" = pmc ] && exit 0
timeout -k 10 900 python3 bench.py $BENCH_ARGS > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof -f csv -- python3 bench.py --no-cpu --parity-seqs 0 --no-b1 $BENCH_ARGS > $OUT/bench_rocprof.log 2>&1 \
  || { echo "rocprof failed"; tail -5 $OUT/bench_rocprof.log; exit 1; }
tail -1 $OUT/bench_rocprof.log
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/bench_kernel_stats.csv \;
python3 tools/pmc_summary.py --trace $(find $OUT/prof -name "*kernel_trace.csv" | head -1) $STEPS $WARMUP > $OUT/trace_window.json
ls $OUT
