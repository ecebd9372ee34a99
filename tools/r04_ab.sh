#!/bin/bash
# Round-4 session AB: proven-mode line cut with the next record's first 48 doubles prefetched into
# LDS (CUT_PF_PROOF 3) — proven-mode parity tests, A/B of the proven bench line against no prefetch.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "proven or certified or cut" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "passed|failed|Error" $O/pytest.log | tail -5; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
for d in default build/ab_pf1 default build/ab_pf1; do
  tag=$(basename $d)
  if [ "$d" = default ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$(realpath $d); fi
  timeout -k 10 300 python bench.py --cut-proof --steps 20 --warmup 3 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 4 > $O/ab_$tag.log 2>&1 \
    || { echo "$tag failed"; tail -5 $O/ab_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/ab_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']), d['kernel_ms'], d['cut_search']['exact_frac'], d['parity_sampled']['mismatches'])"
done
unset GFPL_LIB_DIR
