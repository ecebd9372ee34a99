"""bench.py keeps the driver's JSON contract (one line on rank 0 with the metric,
roofline and CPU-baseline objects) — a tiny run on the GPU box."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--batch", "128", "--steps", "2",
                        "--warmup", "1", "--cpu-seconds", "0.5", "--cpu-threads", "2", "--parity-seqs", "4"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k, t in [("metric", str), ("value", float), ("unit", str), ("n_gpus", int), ("steps", int),
                 ("warmup", int), ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str),
                 ("dtype", str), ("data", str), ("config", dict), ("roofline", dict), ("cpu_baseline", dict)]:
        assert isinstance(d[k], t), k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["value"] > 0 and "vs_baseline" in d
    assert "workload" in d["config"]
    rf = d["roofline"]
    assert rf["bound"] in ("hbm", "mfma") and rf["unit"] in ("GB/s", "TFLOP/s")
    assert rf["achieved"] > 0 and rf["peak"] > 0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    assert "traffic" in rf
    ps = d["parity_sampled"]
    assert ps["sequences"] == 4 and ps["frames"] == 4 * 4 and ps["mismatches"] == 0, ps
    hf = d["host_fed"]
    assert 0 < hf["value"] < d["value"] and hf["upload_GBps"] > 0
    c = d["counts_per_seq_step"]
    assert c["S_p"] > 0 and c["S_l"] > 0 and c["M_p"] > 0 and c["M_o"] >= c["S_p"]
    assert d["roofline"]["window"] and "traffic_note" in d["roofline"]
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0 and cb["sample"]
