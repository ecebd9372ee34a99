#!/bin/bash
# GPU parity tests (optionally a -k filter) + a short bench line with sampled parity.
# Usage: bash tools/quick.sh [-k expr] [-- bench args]   Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
K=""
if [ "$1" == "-k" ]; then K="$2"; shift 2; fi
[ "$1" == "--" ] && shift
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu ${K:+-k "$K"} --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 4 --warmup 1 --no-cpu "$@" > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['parity_sampled']['frames'], d['parity_sampled']['mismatches'], d['parity_sampled']['first'], d['stage_ms'], d['kernel_ms'])"
