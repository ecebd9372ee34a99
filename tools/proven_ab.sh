#!/bin/bash
# Proven-mode A/B (cut_proof 1) of library dirs at B = 16384 under rocprofv3 --kernel-trace --stats:
# the line cut's stage time, the line and the proof kernels' average durations.
# usage: tools/proven_ab.sh NAME DIR1 DIR2 ...   ("default" = the in-tree library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
for d in "$@"; do
  tag=$(basename $d)
  if [ "$d" = default ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$(realpath $d); fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o prof -f csv -- python3 bench.py --batch 16384 \
      --distinct 16384 --steps 8 --warmup 3 --cut-proof 1 --no-cpu --no-detect --no-host-fed --no-b1 --proven-steps 0 \
      --parity-seqs 8 > $O/proven_$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/proven_$tag.log; exit 1; }
  st=$(find $O/prof_$tag -name "*kernel_stats.csv" | head -1)
  python3 -c "
import json, csv
d=json.loads([l for l in open('$O/proven_$tag.log') if l.startswith('{')][-1])
ks={r['Name'].split('(')[0].replace('void ','').replace('gfpl::',''): round(float(r['AverageNs'])/1e6,3) for r in csv.DictReader(open('$st')) if 'cut' in r['Name']}
print('$tag', round(d['value']), round(d['ms_per_step'],3), 'line_cut', d['stage_ms']['line_cut'], ks, 'parity', d['parity_sampled']['frames'], d['parity_sampled']['mismatches'])"
  find $O/prof_$tag -name "*kernel_trace.csv" -delete
done
