#!/usr/bin/env python3
"""k_stereo_points phase split from a bench clock dump (bench.py --dump-records with a library
built with -DGFPL_SP_CLOCK): per workgroup (sequence) the 100 MHz wall clock at the kernel start,
after the setup (counting sorts), the band scan, the SAD-job tile sort, the sub-pixel SAD and the
end (emission sort, stores).  usage: python3 tools/sp_phases.py records_clk.npy"""
import json
import sys

import numpy as np

c = np.load(sys.argv[1]).astype(np.float64)[:, :6]
ok = (c > 0).all(1)
c = c[ok]
d = np.diff(c, axis=1) / 100.0   # us
names = ["setup", "band_scan", "sad_sort", "sad", "emission"]
life = c[:, 5] - c[:, 0]
out = {"workgroups": int(c.shape[0]), "lifetime_us_mean": float(life.mean() / 100.0),
       "phase_us_mean": {n: round(float(d[:, i].mean()), 2) for i, n in enumerate(names)},
       "phase_share": {n: round(float(d[:, i].mean() * 100.0 / life.mean()), 3) for i, n in enumerate(names)},
       "kernel_span_us": float((c[:, 5].max() - c[:, 0].min()) / 100.0)}
print(json.dumps(out))
