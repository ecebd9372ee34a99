set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/lsdpmc; rm -rf $OUT; mkdir -p $OUT
for P in FETCH_SIZE WRITE_SIZE; do
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $OUT/$P -o $P -f csv -- python3 tools/bench_lsd.py --images 1024 --steps 1 --warmup 0 --cpu-sample 0 --check 0 > $OUT/$P.log 2>&1 || { echo fail $P; tail -3 $OUT/$P.log; exit 1; }
done
python3 - <<'PY'
import csv,glob,re
from collections import defaultdict
v=defaultdict(lambda: defaultdict(list))
for f in glob.glob('gpurun_out/lsdpmc/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        m=re.search(r'(k_lsd_[a-z_]+)',r['Kernel_Name'])
        if m: v[m.group(1)][r['Counter_Name']].append(float(r['Counter_Value']))
for k,c in v.items(): print(k, {n: round(sum(x)/len(x)/1e6,3) for n,x in c.items()}, 'GB (KB units /1e6)')
PY
