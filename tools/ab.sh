#!/bin/bash
# A/B timing of library variants on the GPU box: tools/ab.sh dir1 dir2 ...
# ("base" = the in-tree library; env BATCH, WORKLOAD).  One short bench per variant, each
# time-limited, no parity sampling (probe variants compute wrong results on purpose).
set -o pipefail
mkdir -p gpurun_out/ab
B=${BATCH:-16384}
for v in "$@"; do
  if [ "$v" = base ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$v; fi
  tag=$(basename $v)
  timeout -k 10 300 python bench.py --batch $B --steps 3 --warmup 1 --no-cpu --no-detect --no-host-fed --parity-seqs 0 \
      --workload ${WORKLOAD:-cfg2} > gpurun_out/ab/$tag.log 2>&1 || { echo "$tag failed rc=$?"; tail -5 gpurun_out/ab/$tag.log; exit 1; }
  tail -1 gpurun_out/ab/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],2), d['stage_ms'], d['kernel_ms'])"
done
