#!/bin/bash
# SQ counters of the default build and an experimental build (GFPL_LIB_DIR=$1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B=${B:-4096}
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
mkdir -p gpurun_out/cmp && rm -rf gpurun_out/cmp/*
for v in base exp; do
  if [ $v = exp ]; then export GFPL_LIB_DIR=$1; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $CTRS -d gpurun_out/cmp/$v -o $v -f csv -- \
      python3 bench.py --batch $B --steps 2 --warmup 1 --no-cpu > gpurun_out/cmp/$v.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/cmp/$v $B gpurun_out/cmp/$v.json | grep -E "^k_" | cut -c1-220 | sed "s/^/$v /"
done
