#!/usr/bin/env python3
"""Line-cut certification diagnostics on the bench workload (cfg2): a small batch stepped a few
frames; per step the greedy steps, the exact-fallback steps and the lines without a usable
agreement bound (gfpl_last_step_track_counts), then sequence 0's per-line agreement bounds
(R0, A1, A2, B1, B2, EV: CutCmp::eb, record slots 77-79) beside v's(0), v'e(0) and the
bound E at t = 0 (gfpl_debug_cut_records).  GPU; prints JSON lines."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--lines", type=int, default=24)
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--certify", default="", help="comma-separated cut_certify values to sweep (counts only)")
    ap.add_argument("--proof", type=int, default=1, help="gfpl_config.cut_proof")
    a = ap.parse_args()
    import torch
    import gfpl
    import bench
    cam_name, synth_over, _ = bench.WORKLOADS[a.workload]
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0, cut_proof=a.proof)
    cam = gfpl.make_camera(cam_name, cfg)
    sp = gfpl.synth_params(**synth_over, pyr_from_l0=1)
    KP, KL = 2048, 512
    if a.certify:
        H = gfpl.HostFrames(cam, sp, a.batch, a.frames + 1, KP, KL, seq0=0, threads=8)
        for tau in [float(x) for x in a.certify.split(",")]:
            c2 = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0,
                                     cut_certify=tau, cut_proof=a.proof)
            ctx = gfpl.Context(cam, c2)
            h = gfpl.StereoFrameHandler(ctx, a.batch, KP, KL)

            def up(k):
                h.upload_wait(h.upload_async(H.frames(k), 0, k % 2))
                return h.staged_frames(k % 2)
            h.initialize(up(0))
            tot = {"steps": 0, "exact_steps": 0, "lines_unbounded": 0}
            ml = 0.0
            for k in range(1, a.frames + 1):
                h.frameStep(up(k))
                tc = h.last_step_track_counts()
                for n in tot:
                    tot[n] += tc[n]
                ml += h.last_step_counts()["M_l"] * a.batch
            print(json.dumps({"cut_certify": tau, **tot, "exact_frac": tot["exact_steps"] / max(1, tot["steps"]),
                              "lines_unbounded_frac": tot["lines_unbounded"] / max(1.0, ml)}), flush=True)
            h.close()
            ctx.close()
        return
    ctx = gfpl.Context(cam, cfg)
    h = gfpl.StereoFrameHandler(ctx, a.batch, KP, KL)
    H = gfpl.HostFrames(cam, sp, a.batch, a.frames + 1, KP, KL, seq0=0, threads=8)

    def staged(k):
        h.upload_wait(h.upload_async(H.frames(k), 0, k % 2))
        return h.staged_frames(k % 2)
    h.initialize(staged(0))
    for k in range(1, a.frames + 1):
        h.frameStep(staged(k))
        torch.cuda.synchronize()
        tc = h.last_step_track_counts()
        cnt = h.last_step_counts()
        print(json.dumps({"frame": k, **tc, "M_l_mean": cnt["M_l"],
                          "exact_frac": tc["exact_steps"] / max(1, tc["steps"])}), flush=True)
    # records of the cut of the last insert: slot 77-79 = eb (6 floats); PD_VS 36, PD_VE 41
    n = min(a.lines, KL)
    rec = h.debug_cut_records(0, n)
    eb = rec[:, 77:80].copy().view(np.float32).reshape(n, 6)
    for m in range(n):
        vs0, ve0 = rec[m, 36], rec[m, 41]
        e = eb[m]
        E0 = (e[1] + e[2] / vs0) / vs0 + (e[3] + e[4] / ve0) / ve0 if vs0 > 0 and ve0 > 0 else float("nan")
        print(json.dumps({"line": m, "R0": float(e[0]), "A1": float(e[1]), "A2": float(e[2]), "B1": float(e[3]),
                          "B2": float(e[4]), "EV": float(e[5]), "vs0": vs0, "ve0": ve0, "E_at_0": E0,
                          "pd_ok": rec[m, 46], "err_floats": rec[m, 48:55].copy().view(np.float32).tolist()}))
    h.close()
    ctx.close()


if __name__ == "__main__":
    main()
