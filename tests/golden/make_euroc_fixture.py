"""Extract the first N ground-truth poses + timestamps of the EuRoC sequences
the BASELINE configs 1 and 4 name (config/asl/gt-ass/{mh_01..mh_05,v1_01..v1_03})
from the reference's data files into gf-pl-slam_amd/data/euroc_gt.json (used by the
golden fixtures, the EuRoC parity tests and bench.py's cfg4 workload).

Run in the build container (the reference is not on the GPU box):
    python tests/golden/make_euroc_fixture.py /root/reference
The output is data (3x4 row-major T_w<-c rows, timestamps in seconds).
"""
import json
import os
import sys

N = 64
SEQS = ["mh_01", "mh_02", "mh_03", "mh_04", "mh_05", "v1_01", "v1_02", "v1_03"]


def main(ref):
    out = {"source": "config/asl/gt-ass/<seq>/{groundtruth,associations}.txt", "n": N, "seqs": {}}
    for s in SEQS:
        d = os.path.join(ref, "config", "asl", "gt-ass", s)
        with open(os.path.join(d, "groundtruth.txt")) as f:
            rows = [[float(x) for x in ln.split()] for ln in f if ln.strip()][:N]
        with open(os.path.join(d, "associations.txt")) as f:
            ts = [int(ln.split()[0]) / 1e9 for ln in f if ln.strip()][:N]
        assert all(len(r) == 12 for r in rows)
        out["seqs"][s] = {"T_wc_3x4": rows, "t": ts}
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dst = os.path.join(root, "gf-pl-slam_amd", "data", "euroc_gt.json")
    with open(dst, "w") as f:
        json.dump(out, f)
    print("wrote", dst)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
