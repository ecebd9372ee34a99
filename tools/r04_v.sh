#!/bin/bash
# Round-4 session V: LSD region growth with issue priority by seed progress — LSD tests, A/B at
# 3072 and 2048 images per call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lsd_gpu.py -x -v -m gpu --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "passed|failed|Error" $O/pytest.log | tail -5; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
for d in default build/ab_nolsdprio default; do
  tag=$(basename $d)
  if [ "$d" = default ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$(realpath $d); fi
  for n in 3072 2048; do
    timeout -k 10 300 python tools/bench_lsd.py --images $n --steps 5 --cpu-sample 0 --check 2 > $O/lsd_${tag}_$n.log 2>&1 \
      || { tail -5 $O/lsd_${tag}_$n.log; exit 1; }
    echo "$tag $n $(tail -1 $O/lsd_${tag}_$n.log | cut -c1-170)"
  done
done
unset GFPL_LIB_DIR
