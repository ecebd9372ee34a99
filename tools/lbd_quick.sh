#!/bin/bash
# LBD row on the GPU: parity tests, throughput line, rocprof kernel stats.
set -o pipefail
OUT=${OUT:-gpurun_out/lbd}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_lbd_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_lbd.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o lbd -- python3 tools/bench_lbd.py --cpu-sample 0 --check 0 --steps 5 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
python3 -c "
import csv,glob
for f in glob.glob('$OUT/prof/**/lbd_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Name'].split('(')[0][:30], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
