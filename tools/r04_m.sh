#!/bin/bash
# Round-4 session M: the whole -m gpu suite, smoke, and the default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --maxfail=6 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['stage_ms'], d['kernel_ms'], d['roofline']['frac'], d['latency_b1_ms'], d['cpu_baseline']['value'], d['parity_sampled'])"
