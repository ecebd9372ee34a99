#!/bin/bash
# FETCH_SIZE / WRITE_SIZE (separate passes) per kernel for library variants:
#   B=4096 bash tools/pmc_ab.sh base build/x ...   ("base" = the in-tree library)
set -o pipefail
B=${B:-4096}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" = base ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$v; fi
  tag=$(basename $v)
  OUT=gpurun_out/pmcab/$tag
  rm -rf $OUT && mkdir -p $OUT
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d $OUT/$c -o $c -f csv -- \
        python3 bench.py --batch $B --steps 2 --warmup 1 --no-cpu > $OUT/$c.log 2>&1 || { echo "$tag $c failed"; tail -5 $OUT/$c.log; exit 1; }
  done
  echo "== $tag"
  python3 tools/pmc_summary.py $OUT $B $OUT/pmc.json | grep -E "k_stereo|k_pose|k_cut_search|k_cross" || true
done
