#!/bin/bash
# A/B of LSD library variants (tools/variant.sh builds) on the GPU box: bench_lsd images/s and
# sampled parity per variant ("base" = the in-tree library).  Usage: bash tools/lsd_ab.sh dir...
set -o pipefail
mkdir -p gpurun_out/lsd_ab
for v in "$@"; do
  if [ "$v" = base ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$v; fi
  tag=$(basename $v)
  timeout -k 10 200 python tools/bench_lsd.py --images ${IMAGES:-1024} --steps 3 --warmup 1 --cpu-sample 0 --check 2 \
      > gpurun_out/lsd_ab/$tag.log 2>&1 || { echo "$tag failed rc=$?"; tail -5 gpurun_out/lsd_ab/$tag.log; exit 1; }
  tail -1 gpurun_out/lsd_ab/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_call'],2), d['parity_sampled'])"
done
