#!/usr/bin/env python3
"""Proven line cut diagnostics (cut_proof 1): run n sequences x F frames of the bench workload, and
after each insert read k_cut_verify's per-sequence reason mask and worst E / R0 (scr.dbg slots 4, 5;
DESIGN.md §3): how many sequences the after-the-fact proof leaves for the eager redo, and why.
usage: python tools/verify_diag.py [n] [F]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))
import gfpl  # noqa: E402

REASONS = {1: "replay", 2: "v'<=0 or r_v", 256: "forced", 512: "exact recheck disagrees"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0, cut_proof=1)
    cam = gfpl.make_camera("vga", cfg)
    H = gfpl.HostFrames(cam, gfpl.synth_params(respawn=16), n, F, 2048, 512)
    D = gfpl.DeviceFrames(H)
    ctx = gfpl.Context(cam, cfg)
    h = gfpl.StereoFrameHandler(ctx, n, 2048, 512)
    h.initialize(D.frames(0))
    masks, worst, terms, xchk = [], [], [], []
    for k in range(1, F):
        h.insertStereoPair(D.frames(k))
        d = h.debug_clocks()
        masks.append(d[:, 4].copy())
        worst.append(d[:, 5].copy().view(np.float64))
        terms.append(d[:, :4].copy().view(np.float64))
        xchk.append(d[:, 6].copy())
        print("frame", k, h.last_step_cut_proof(), flush=True)
        h.optimizePose()
        h.updateFrame()
    m = np.concatenate(masks)
    w = np.concatenate(worst)
    x = np.concatenate(xchk)
    print("sequences x frames", len(m), "redone", int((m != 0).sum()), "steps re-checked exactly", int(x.sum()),
          "sequences with a re-check", int((x > 0).sum()))
    for bit, name in REASONS.items():
        print(f"  {name:12s} {int(((m & bit) != 0).sum())}")
    ok = w[(m == 0)]
    t = np.concatenate(terms)
    top = np.argsort(-w)[:12]
    print("worst proven steps: E/R0 and its terms (eps_S, K0 rest, A1/B1, v') / R0")
    for i in top:
        print(f"  {w[i]:.3g}  " + "  ".join(f"{x:.3g}" for x in t[i]), "mask", int(m[i]))
    med = np.median(t, axis=0)
    print("median terms", [float(f"{x:.3g}") for x in med])
    print("worst E/R0 over proven sequences: max", float(ok.max()) if len(ok) else None,
          "quantiles", np.quantile(w, [0.5, 0.9, 0.99, 0.999]).tolist())


if __name__ == "__main__":
    main()
