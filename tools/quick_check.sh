#!/bin/bash
# Quick GPU-box check after a kernel change: the tracker and LSD parity suites, a short bench line
# (sampled parity) and the LSD bench.  Every step time-limited; stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_lsd_gpu.py tests/test_pipeline_gpu.py -x -q -m gpu \
    --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-detect --no-host-fed --parity-seqs 8 > $OUT/bench.log 2>&1 \
    || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],2), d['parity_sampled']['mismatches'], d['stage_ms'], d['kernel_ms'])"
timeout -k 10 200 python tools/bench_lsd.py --images 1024 --steps 3 --warmup 1 --cpu-sample 0 --check 4 > $OUT/lsd.log 2>&1 \
    || { tail -5 $OUT/lsd.log; exit 1; }
tail -1 $OUT/lsd.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lsd', round(d['value']), round(d['ms_per_call'],2), d['parity_sampled'])"
