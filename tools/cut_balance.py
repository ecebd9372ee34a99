#!/usr/bin/env python3
"""Line-cut search balance from a bench step-record dump (bench.py --dump-records, a library built
with -DGFPL_CUT_CLOCK: slot 19 = the k_cut_search wave's duration in 100 MHz wall-clock ticks).
Per wave (8 consecutive sequences): duration, the groups' greedy steps (slot 16) and matched
lines (slot 14).  usage: python3 tools/cut_balance.py records.npy"""
import json
import sys

import numpy as np

r = np.load(sys.argv[1])
B = r.shape[0] // 8 * 8
w = r[:B].reshape(-1, 8, r.shape[1])
dur = w[:, 0, 19].astype(np.float64) / 100.0          # us
steps = w[:, :, 16].astype(np.float64)
lines = w[:, :, 14].astype(np.float64)
q = lambda a: {k: round(float(v), 2) for k, v in zip(("min", "p10", "p50", "p90", "max", "mean"),
                                                     list(np.percentile(a, [0, 10, 50, 90, 100])) + [a.mean()])}
out = {"waves": int(w.shape[0]), "wave_us": q(dur), "seq_steps": q(steps.ravel()), "wave_max_steps": q(steps.max(1)),
       "wave_sum_steps": q(steps.sum(1)), "seq_lines": q(lines.ravel()),
       "corr_dur_vs_max_steps": float(np.corrcoef(dur, steps.max(1))[0, 1]),
       "corr_dur_vs_sum_steps": float(np.corrcoef(dur, steps.sum(1))[0, 1]),
       "mean_over_max_dur": float(dur.mean() / dur.max()),
       "group_idle_frac": float(1.0 - steps.sum() / (steps.max(1).sum() * 8))}
print(json.dumps(out))
