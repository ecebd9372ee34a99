#!/bin/bash
# Round-4 session X2 (final tree): proven-mode line, the batch sweep and the cfg3 / cfg4 / cfg5 lines on the
# round's final kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04x2
mkdir -p $O
timeout -k 10 400 python bench.py --cut-proof --steps 20 --warmup 5 --no-cpu --no-detect --no-host-fed --no-b1 > $O/proof_bench.log 2>&1 \
  || { tail -5 $O/proof_bench.log; exit 1; }
tail -1 $O/proof_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('proof', round(d['value']), d['kernel_ms'], d['cut_search'])"
bash tools/bsweep.sh 20 1 8 64 512 4096 16384 || exit 1
mv gpurun_out/bsweep* $O/
OUT=$O bash tools/cfg_lines.sh || exit 1
