"""Extract the first 512 ground-truth poses + timestamps of the EuRoC sequences
the BASELINE configs 1 and 4 name (config/asl/gt-ass/{mh_01..mh_05,v1_01..v1_03})
from the reference's data files into gf-pl-slam_amd/data/euroc_gt.npz (used by the
golden fixtures, the EuRoC parity tests and bench.py's cfg4 workload): float64 arrays
<seq>_T [512][12] and <seq>_t [512], the first 25 s of each trajectory at 20 Hz.

Run in the build container (the reference is not on the GPU box):
    python tests/golden/make_euroc_fixture.py /root/reference
The output is data (3x4 row-major T_w<-c rows, timestamps in seconds).
"""
import os
import sys

import numpy as np

N_NPZ = 512
SEQS = ["mh_01", "mh_02", "mh_03", "mh_04", "mh_05", "v1_01", "v1_02", "v1_03"]


def main(ref):
    arrs = {}
    for s in SEQS:
        d = os.path.join(ref, "config", "asl", "gt-ass", s)
        with open(os.path.join(d, "groundtruth.txt")) as f:
            rows = [[float(x) for x in ln.split()] for ln in f if ln.strip()][:N_NPZ]
        with open(os.path.join(d, "associations.txt")) as f:
            ts = [int(ln.split()[0]) / 1e9 for ln in f if ln.strip()][:N_NPZ]
        assert all(len(r) == 12 for r in rows) and len(rows) == len(ts) == N_NPZ
        arrs[s + "_T"] = np.array(rows, np.float64)
        arrs[s + "_t"] = np.array(ts, np.float64)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dst = os.path.join(root, "gf-pl-slam_amd", "data", "euroc_gt.npz")
    np.savez(dst, **arrs)
    print("wrote", dst)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
