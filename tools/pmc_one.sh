#!/bin/bash
# One PMC pass (counters given as args) over a short bench run; summary to stdout.
set -o pipefail
B=${B:-4096}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc1
rm -rf gpurun_out/pmc1/*
timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc1/run -o run -f csv -- \
    python3 bench.py --batch $B --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc1/run.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/pmc1 $B gpurun_out/pmc1/pmc.json
