"""Synthetic keylines for the LBD tests: segments inside the image with fractional
endpoints, the LSD wrapper's angle = atan2(ey - sy, ex - sx) in float
(src/LSDDetector_custom.cpp:285), octave 0."""
import numpy as np

import gfpl


def synth_keylines(n, w, h, seed, min_len=2.0, max_len=200.0, border=False):
    rng = np.random.default_rng(seed)
    kl = np.zeros(n, gfpl.KEYLINE_DT)
    for i in range(n):
        while True:
            sx, sy = rng.uniform(0, w - 1), rng.uniform(0, h - 1)
            a = rng.uniform(-np.pi, np.pi)
            ln = rng.uniform(min_len, max_len)
            ex, ey = sx + ln * np.cos(a), sy + ln * np.sin(a)
            if border:
                ex, ey = min(max(ex, 0.0), w - 1.0), min(max(ey, 0.0), h - 1.0)
            if 0 <= ex <= w - 1 and 0 <= ey <= h - 1:
                break
        kl[i] = (np.float32(sx), np.float32(sy), np.float32(ex), np.float32(ey),
                 np.arctan2(np.float32(ey) - np.float32(sy), np.float32(ex) - np.float32(sx)).astype(np.float32), 0)
    return kl
