#!/bin/bash
# A/B of kernel variants on the bench workload: one short bench per library directory
# (GFPL_LIB_DIR; "default" = the in-tree gf-pl-slam_amd/lib), tracking step only.
# usage: tools/ab_bench.sh OUTDIR STEPS DIR1 DIR2 ...
set -o pipefail
out=$1; steps=$2; shift 2
mkdir -p $out
for d in "$@"; do
  tag=$(basename $d)
  if [ "$d" = default ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$(realpath $d); fi
  timeout -k 10 300 python bench.py --steps $steps --warmup 3 --no-cpu --no-detect --no-host-fed --no-b1 --proven-steps 0 \
      --parity-seqs 4 > $out/ab_$tag.log 2>&1 || { echo "$tag failed"; tail -5 $out/ab_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$out/ab_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']), round(d['ms_per_step'],3), d['stage_ms'], d['kernel_ms'], d['cut_search'].get('exact_frac'), d['parity_sampled']['mismatches'])"
done
unset GFPL_LIB_DIR
