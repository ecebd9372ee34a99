#!/bin/bash
# FETCH_SIZE per kernel (WRITE_SIZE needs its own pass) for the default build and experimental builds
# (GFPL_LIB_DIR=<dir>), B sequences, one short bench run each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B=${B:-16384}
mkdir -p gpurun_out/fv && rm -rf gpurun_out/fv/*
for v in base "$@"; do
  n=$(basename $v)
  if [ $v != base ]; then export GFPL_LIB_DIR=$v; else unset GFPL_LIB_DIR; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/fv/$n -o $n -f csv -- \
      python3 bench.py --batch $B --steps 2 --warmup 1 --no-cpu > gpurun_out/fv/$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/fv/$n.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/fv/$n $B gpurun_out/fv/$n.json > /dev/null
  python3 -c "
import json; d=json.load(open('gpurun_out/fv/$n.json'))['kernels']
print('$n', {k: round(2*v.get('FETCH_SIZE',0)*1024/1e9,2) for k,v in d.items() if k.startswith('k_stereo') or k.startswith('k_pose') or k.startswith('k_cross')})"
done
