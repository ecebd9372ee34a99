#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, --kernel-trace only,
# as MI355X_MICROARCH.md §rocprofv3 prescribes), then the per-kernel summary.
set -o pipefail
B=${1:-4096}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc/$name -o $name -f csv -- \
      python3 bench.py --batch $B --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc/$name.log 2>&1
}
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
run sq2 SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT && \
python3 tools/pmc_summary.py gpurun_out/pmc $B gpurun_out/pmc/pmc_latest.json > gpurun_out/pmc/summary.txt
rc=$?
cat gpurun_out/pmc/summary.txt
exit $rc
