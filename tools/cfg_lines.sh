#!/bin/bash
# BASELINE configs[2..4] bench lines (cfg3 KITTI, cfg4 EuRoC MH_01 ground truth, cfg5 stress) with
# sampled parity, then the LSD bench and its rocprofv3 kernel statistics.  Each step time-limited.
set -o pipefail
OUT=${OUT:-gpurun_out/cfg}
BATCH=${BATCH:-32768}   # cfg3 / cfg4 (bench.py's 65536 default would spend most of a GPU call generating inputs)
mkdir -p $OUT
for w in cfg3 cfg4; do
  timeout -k 10 400 python3 bench.py --workload $w --batch $BATCH --steps 20 --warmup 5 --no-cpu --no-detect --no-host-fed > $OUT/${w}_bench.log 2>&1 \
    || { echo "$w failed"; tail -5 $OUT/${w}_bench.log; exit 1; }
  tail -1 $OUT/${w}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', round(d['value']), round(d['ms_per_step'],2), d['parity_sampled']['frames'], d['parity_sampled']['mismatches'])"
done
timeout -k 10 500 python3 bench.py --workload cfg5 --steps 8 --warmup 2 --batch 16384 --no-cpu --no-detect --no-host-fed > $OUT/cfg5_bench.log 2>&1 \
  || { echo "cfg5 failed"; tail -5 $OUT/cfg5_bench.log; exit 1; }
tail -1 $OUT/cfg5_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg5', round(d['value']), round(d['ms_per_step'],2), d['parity_sampled']['frames'], d['parity_sampled']['mismatches'], d['stage_ms'])"
bash tools/lsd_quick.sh $OUT/lsd
