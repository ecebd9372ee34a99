#!/usr/bin/env python3
"""LSD line detection throughput (detector part): gfpl_lsd_detect over a
batch of grey images resident in HBM (StereoFrame detects lines on 2 images per stereo frame):
half staircase stereo scenes (gfpl.pipeline), half gfpl_synth_image textures.  One JSON line:
images/s on the GPU, segments / keylines / gradient-defined pixels per image, sampled parity,
the CPU oracle on a bounded sample (one core)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def images(W, H, n):
    from gfpl import pipeline as P
    import gfpl
    out = []
    for i in range(n):
        if i % 2 == 0:
            l, r, _, _ = P.synth_stereo_steps(i // 4, (i // 2) % 8, W, H)
            out.append(l if (i // 2) % 2 == 0 else r)
        else:
            out.append(gfpl.synth_image(i, i % 5, W, H))
        if i % 1024 == 1023:
            print(f"[bench_lsd] {i + 1} of {n} images generated", file=sys.stderr, flush=True)
    return np.stack(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cam", default="vga")
    ap.add_argument("--images", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=16)
    ap.add_argument("--check", type=int, default=8)
    a = ap.parse_args()
    import torch
    import gfpl
    c = gfpl.CAMERAS[a.cam]
    W, H, n = c["width"], c["height"], a.images
    imgs = images(W, H, n)
    prm = gfpl.LsdParams.reference(W, H)
    cap = 320
    det = gfpl.LSDDetector(W, H, prm, max_images=n, kl_cap=cap)
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(imgs).to(dev)
    d_kl = torch.zeros(n * cap * gfpl.KEYLINE_DT.itemsize, dtype=torch.uint8, device=dev)
    d_n = torch.zeros(n, dtype=torch.int32, device=dev)
    d_r = torch.zeros(n * cap, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    for _ in range(a.warmup):
        det.detect_batch(d_img, n, d_kl, d_n, d_r)
    times = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        det.detect_batch(d_img, n, d_kl, d_n, d_r)   # synchronises
        times.append(time.perf_counter() - t0)
    ms = 1e3 * float(np.mean(times))
    cnt = d_n.cpu().numpy()
    out = {"metric": "LSD images/s (LSDDetectorC::detect + lsdNFeatures filter)", "value": n / (ms * 1e-3),
           "unit": "images/s", "images_per_call": n, "ms_per_call": ms, "keylines_per_image": float(cnt.mean()),
           "config": {"workload": f"{a.cam} {W}x{H}, LSD_REFINE_STD scale 1, 300 keylines kept",
                      "data": "synthetic (staircase stereo scenes + gfpl_synth_image textures)"}}
    import oracle as O
    if a.check:
        kl = d_kl.cpu().numpy().view(gfpl.KEYLINE_DT).reshape(n, cap)
        bad = 0
        for i in range(min(a.check, n)):
            rk, _, _ = O.lsd_detect(imgs[i], prm)
            bad += int(cnt[i] != len(rk) or kl[i, :cnt[i]].tobytes() != rk.tobytes())
        out["parity_sampled"] = {"images": min(a.check, n), "mismatches": bad}
    if a.cpu_sample:
        t0 = time.perf_counter()
        segs = 0
        for i in range(a.cpu_sample):
            segs += len(O.lsd_detect(imgs[i], prm)[2])
        dt = time.perf_counter() - t0
        out["segments_per_image"] = segs / a.cpu_sample
        out["cpu_baseline"] = {"value": a.cpu_sample / dt, "unit": "images/s", "cores": 1, "kind": "port",
                               "sample": f"{a.cpu_sample} images of the batch through the CPU oracle"}
    # share of pixels with a defined gradient angle (norm > rho): the region-growing work
    prec, rho, _ = O.lsd_constants(W, H)
    g = imgs[:8].astype(np.int32)
    DA = g[:, 1:, 1:] - g[:, :-1, :-1]
    BC = g[:, :-1, 1:] - g[:, 1:, :-1]
    out["defined_px_frac"] = float((np.sqrt(((DA + BC) ** 2 + (DA - BC) ** 2) / 4.0) > rho).mean())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
