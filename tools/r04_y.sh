#!/bin/bash
# Round-4 session Y: LSD sort with CAP / 4 at 128 VGPRs (eight images per CU) for batches above six
# images per CU (variant) — parity sampled by bench_lsd, A/B at 3072 and 2048 images per call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04y
mkdir -p $O
for d in default build/ab_t3 default build/ab_t3; do
  tag=$(basename $d)
  if [ "$d" = default ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$(realpath $d); fi
  for n in 3072 2048; do
    timeout -k 10 300 python tools/bench_lsd.py --images $n --steps 5 --cpu-sample 0 --check 4 > $O/lsd_${tag}_$n.log 2>&1 \
      || { tail -5 $O/lsd_${tag}_$n.log; exit 1; }
    echo "$tag $n $(tail -1 $O/lsd_${tag}_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['parity_sampled'])")"
  done
done
unset GFPL_LIB_DIR
