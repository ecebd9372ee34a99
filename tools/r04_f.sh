#!/bin/bash
# Round-4 session F: cut search in measured mode (default) vs the per-step LDS operand reload
# (A/B build), proven mode at its default margin, then the GPU suite on the cut / detector tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04f
mkdir -p $O
bash tools/ab_bench.sh $O/ab 8 build/lds_ops default || exit 1
timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 4 \
    --cut-proof > $O/bench_proof.log 2>&1 || { tail -5 $O/bench_proof.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_proof.log').read().strip().splitlines()[-1]); print('proof', round(d['value']), d['kernel_ms'], d['cut_search'], d['parity_sampled']['mismatches'])"
timeout -k 10 900 python -u -m pytest tests -v -m gpu --maxfail=6 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head
