#!/bin/bash
# Round-4 session AG: LSD at 3072 images per call on the final tree — bench line and rocprofv3
# kernel statistics.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ag
mkdir -p $O
timeout -k 10 300 python tools/bench_lsd.py --images 3072 --steps 5 --cpu-sample 8 --check 8 > $O/lsd_3072.log 2>&1 || { tail -5 $O/lsd_3072.log; exit 1; }
tail -1 $O/lsd_3072.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o lsd -f csv -- python3 tools/bench_lsd.py --images 3072 \
    --steps 3 --cpu-sample 0 --check 2 > $O/lsd_prof.log 2>&1 || { tail -5 $O/lsd_prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/lsd_kernel_stats_3072.csv \;
cut -d, -f1-4 $O/lsd_kernel_stats_3072.csv | head -8
