#!/bin/bash
# Round-4 session N: the whole -m gpu suite, smoke, the default bench line, then LSD at
# 3072 / 4096 images per call and images -> poses with LSD at 2048 frames per step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --maxfail=6 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms'], d['roofline']['frac'], d['latency_b1_ms'], d['cpu_baseline']['value'], d['parity_sampled'])"
for n in 3072 4096; do
  timeout -k 10 300 python tools/bench_lsd.py --images $n --steps 5 --cpu-sample 0 --check 4 > $O/lsd_$n.log 2>&1 \
    || { tail -5 $O/lsd_$n.log; exit 1; }
  tail -1 $O/lsd_$n.log | cut -c1-300
done
timeout -k 10 500 python tools/pipe_rate.py --batch 2048 --steps 3 --lsd 1 > $O/pipe_2048.log 2>&1 || { tail -5 $O/pipe_2048.log; exit 1; }
tail -1 $O/pipe_2048.log | cut -c1-600
