#!/bin/bash
# Round-4 session E: the certified cut search against its margin (exact fraction, lines without a
# usable bound), then the bench's cut search at three margins.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 300 python tools/cut_diag.py --batch 128 --frames 4 --certify 1e-9,1e-8,1e-7,1e-6,1e-5,1e-4,1e-3 > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
grep cut_certify $O/sweep.log
for t in 1e-6 1e-5 1e-4; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 4 \
      --cut-certify $t > $O/bench_$t.log 2>&1 || { tail -5 $O/bench_$t.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$t.log').read().strip().splitlines()[-1]); print('$t', round(d['value']), d['kernel_ms'], d['cut_search']['exact_frac'], d['cut_search']['lines_unbounded_frac'], d['parity_sampled']['mismatches'])"
done
