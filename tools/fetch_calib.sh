#!/bin/bash
# FETCH_SIZE calibration for the SAD's access pattern (tools/probe/fetch_calib.hip): one PMC pass,
# then bytes-per-FETCH_SIZE-unit per kernel against the known byte counts the probe prints.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fcal
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/fcal/pmc -o fcal -f csv -- \
    ./tools/probe/fetch_calib 1024 > gpurun_out/fcal/probe.log 2>&1 || { tail -5 gpurun_out/fcal/probe.log; exit 1; }
python3 - <<'PY'
import csv, glob, json
known = json.loads([l for l in open("gpurun_out/fcal/probe.log") if l.startswith("{")][-1])
rows = []
for f in glob.glob("gpurun_out/fcal/pmc/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
per = {}
for r in rows:
    k = r["Kernel_Name"]
    for n in ("k_stream", "k_gather", "k_rows"):
        if n in k:
            per.setdefault(n, []).append(float(r["Counter_Value"]) * 1024.0)
res = {}
for n, b in (("k_stream", known["stream_bytes"]), ("k_gather", known["gather_bytes"]),
             ("k_rows", known["rows_distinct_line_bytes"])):
    v = per.get(n, [])
    if v:
        fs = sum(v) / len(v)
        res[n] = {"fetch_size_bytes": fs, "known_bytes": b, "known_over_fetch": b / fs}
res["rows_loaded_bytes"] = known["rows_loaded_bytes"]
print(json.dumps(res, indent=1))
json.dump(res, open("gpurun_out/fcal/fetch_calib.json", "w"), indent=1)
PY
