#!/bin/bash
# A/B of kernel variants on the bench workload: one short bench per library directory
# (GFPL_LIB_DIR; "default" = the in-tree gf-pl-slam_amd/lib), tracking step only.
# usage: tools/ab_bench.sh OUTDIR STEPS DIR1 DIR2 ...
set -o pipefail
out=$1; steps=$2; shift 2
mkdir -p $out
rm -f $out/.ab_keys
for d in "$@"; do
  tag=$(basename $d)
  if [ "$d" = default ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$(realpath $d); fi
  timeout -k 10 300 python bench.py --steps $steps --warmup 3 --batch 16384 --distinct 16384 --no-cpu --no-detect --no-host-fed --no-b1 --proven-steps 0 \
      --parity-seqs 4 > $out/ab_$tag.log 2>&1 || { echo "$tag failed"; tail -5 $out/ab_$tag.log; exit 1; }
  python -c "
import json; d=json.loads(open('$out/ab_$tag.log').read().strip().splitlines()[-1])
key=(d['host']['distinct_sequences_per_rank'], d['cut_search']['steps'])
print('$tag', round(d['value']), round(d['ms_per_step'],3), d['stage_ms'], d['kernel_ms'], d['cut_search'].get('exact_frac'),
      d['parity_sampled']['mismatches'], 'distinct', key[0], 'greedy_steps', key[1])
open('$out/.ab_keys','a').write(repr(key) + chr(10))
ks=set(open('$out/.ab_keys').read().split(chr(10))) - {''}
if len(ks) > 1: print('WARNING: A/B runs differ in inputs or line-cut paths:', ks)
"
done
unset GFPL_LIB_DIR
