#!/bin/bash
# One GPU-box session: parity tests, then the default bench (each step time-limited).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "Error|assert|mismatch|differ" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?
tail -1 gpurun_out/bench.log
exit $rc
