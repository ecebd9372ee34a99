#!/bin/bash
# Round-4 LSD session: throughput at 1024 / 2048 images per call, the rocprofv3 kernel
# statistics at 2048, and images -> poses with LSD on the device (B = 1024 frames).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04lsd
mkdir -p $O
for n in 1024 2048; do
  timeout -k 10 300 python tools/bench_lsd.py --images $n --steps 5 --cpu-sample 4 --check 8 > $O/lsd_$n.log 2>&1 \
    || { tail -5 $O/lsd_$n.log; exit 1; }
  tail -1 $O/lsd_$n.log | cut -c1-400
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o lsd -f csv -- python3 tools/bench_lsd.py --images 2048 \
    --steps 3 --cpu-sample 0 --check 2 > $O/lsd_prof.log 2>&1 || { tail -5 $O/lsd_prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/lsd_kernel_stats.csv \;
cut -d, -f1-4 $O/lsd_kernel_stats.csv | head -8
timeout -k 10 400 python tools/pipe_rate.py --batch 1024 --steps 3 --lsd 2 > $O/pipe.log 2>&1 || { tail -5 $O/pipe.log; exit 1; }
tail -1 $O/pipe.log | cut -c1-600
