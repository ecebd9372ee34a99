#!/bin/bash
# Round-4 session A: the whole -m gpu suite, then the default bench line (no detection legs).
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 1050 python -u -m pytest tests -v -m gpu --maxfail=6 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -8 $O/pytest_gpu.log
grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-detect > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms'], d['cut_search'], d['parity_sampled']['mismatches'], d['host_fed'], d['counts_per_seq_step'])"
bash tools/ab_bench.sh $O/ab 10 build/base default
