#!/usr/bin/env python3
"""k_stereo_points phase split from a bench clock dump (bench.py --dump-records with a library
built with -DGFPL_SP_CLOCK): per workgroup (sequence) the 100 MHz wall clock at the kernel start,
after the setup (counting sorts), the band scan, the SAD-job tile sort, the sub-pixel SAD and the
end (emission sort, stores).  With --lines (a -DGFPL_SL_CLOCK build): k_stereo_lines' train-row staging,
knn pass, medians, triangulation + emission.  usage: python3 tools/sp_phases.py records_clk.npy [--lines]"""
import json
import sys

import numpy as np

lines = "--lines" in sys.argv   # a -DGFPL_SL_CLOCK build: k_stereo_lines' phases instead
npc = 5 if lines else 6
c = np.load([a for a in sys.argv[1:] if not a.startswith("--")][0]).astype(np.float64)[:, :npc]
ok = (c > 0).all(1)
c = c[ok]
d = np.diff(c, axis=1) / 100.0   # us
names = ["staging", "knn", "medians", "triangulation_emission"] if lines else ["setup", "band_scan", "sad_sort", "sad", "emission"]
life = c[:, npc - 1] - c[:, 0]
out = {"workgroups": int(c.shape[0]), "lifetime_us_mean": float(life.mean() / 100.0),
       "phase_us_mean": {n: round(float(d[:, i].mean()), 2) for i, n in enumerate(names)},
       "phase_share": {n: round(float(d[:, i].mean() * 100.0 / life.mean()), 3) for i, n in enumerate(names)},
       "kernel_span_us": float((c[:, npc - 1].max() - c[:, 0].min()) / 100.0)}
print(json.dumps(out))
