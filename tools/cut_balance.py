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

# the clock build's per-wave start / end / hardware ids (gfpl_debug_clocks, records_clk.npy)
import os  # noqa: E402
ck = sys.argv[1].replace(".npy", "") + "_clk.npy"
if os.path.exists(ck):
    c = np.load(ck)[:B].reshape(-1, 8, 8)[:, 0, :]
    t0, t1, hw, xcc = c[:, 0].astype(np.float64), c[:, 1].astype(np.float64), c[:, 2], c[:, 3]
    if (t0 > 0).all():
        st = (t0 - t0.min()) / 100.0
        en = (t1 - t0.min()) / 100.0
        half = np.arange(len(st)) >= len(st) // 2
        slot = hw & 0xF
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 0xF
        key = (xcc & 0xF) * 1024 + ((hw >> 13) & 7) * 256 + ((hw >> 12) & 1) * 128 + cu * 8 + simd
        _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
        print(json.dumps({"start_us": {"first_half_mean": float(st[~half].mean()), "second_half_mean": float(st[half].mean()),
                                       "max": float(st.max())},
                          "end_us": {"first_half_mean": float(en[~half].mean()), "second_half_mean": float(en[half].mean()),
                                     "max": float(en.max())},
                          "waves_per_simd": {str(k): int(v) for k, v in zip(*np.unique(cnt, return_counts=True))},
                          "dur_by_slot": {str(int(s)): round(float(dur[slot == s].mean()), 1) for s in np.unique(slot)},
                          "dur_by_simd": {str(int(s)): round(float(dur[simd == s].mean()), 1) for s in np.unique(simd)},
                          "dur_first_vs_second_on_simd": [round(float(dur[np.array([st[i] <= st[inv == inv[i]].min() for i in range(len(st))])].mean()), 1),
                                                          round(float(dur[np.array([st[i] > st[inv == inv[i]].min() for i in range(len(st))])].mean()), 1)]}))
