#!/bin/bash
# Round-4 session I: proven vs measured line cut on the bench workload (+ the proven-mode tests).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "proven or certified or bench_config" -s --timeout 500 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"
grep -E "passed|failed|proven mode" $O/pytest.log | tail -3
for mode in proof measured; do
  flag=""; [ $mode = proof ] && flag="--cut-proof"
  timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 4 $flag > $O/bench_$mode.log 2>&1 || { tail -5 $O/bench_$mode.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$mode.log').read().strip().splitlines()[-1]); print('$mode', round(d['value']), d['kernel_ms'], d['stage_ms']['line_cut'], d['cut_search']['exact_frac'], d['parity_sampled']['mismatches'])"
done
