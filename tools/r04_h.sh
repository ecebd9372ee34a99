#!/bin/bash
# Round-4 session H: proven-mode line cut — diagnostics, margin sweep, GPU tests, bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 300 python tools/cut_diag.py --batch 64 --frames 4 --lines 12 --proof 1 > $O/cut_diag.log 2>&1 || { tail -20 $O/cut_diag.log; exit 1; }
cut -c1-300 $O/cut_diag.log | head -20
timeout -k 10 300 python tools/cut_diag.py --batch 128 --frames 4 --proof 1 --certify 1e-10,1e-9,1e-8,1e-7 > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
grep cut_certify $O/sweep.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "proven or certified or bench_config" -s --timeout 500 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"
grep -E "passed|failed|proven mode" $O/pytest.log | tail -5
timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 4 \
    --cut-proof > $O/bench_proof.log 2>&1 || { tail -5 $O/bench_proof.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_proof.log').read().strip().splitlines()[-1]); print('proof', round(d['value']), d['kernel_ms'], d['cut_search'], d['parity_sampled']['mismatches'])"
