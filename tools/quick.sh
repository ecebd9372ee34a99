#!/bin/bash
# GPU parity tests + a short bench line (stage / kernel ms).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu "$@" > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['stage_ms'], d['kernel_ms'])"
