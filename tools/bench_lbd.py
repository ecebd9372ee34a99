#!/usr/bin/env python3
"""LBD descriptor throughput (descriptor part): gfpl_lbd_compute over a
batch of synthetic grey images resident in HBM with lsdNFeatures = 300 synthetic keylines
each (StereoFrame computes them for 2 images per stereo frame).  One JSON line: images/s and
keylines/s on the GPU, sampled parity, the CPU oracle on a bounded sample (one core)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cam", default="vga")
    ap.add_argument("--images", type=int, default=256)
    ap.add_argument("--lines", type=int, default=300)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-sample", type=int, default=4)
    ap.add_argument("--check", type=int, default=2)
    a = ap.parse_args()
    import torch
    import gfpl
    c = gfpl.CAMERAS[a.cam]
    W, H, n, m = c["width"], c["height"], a.images, a.lines
    imgs = np.stack([gfpl.synth_image(i, i % 5, W, H) for i in range(n)])
    kls = np.stack([gfpl.synth_keylines(m, W, H, 1000 + i, max_len=150.0) for i in range(n)])
    lbd = gfpl.BinaryDescriptor(W, H, max_images=n, kl_cap=m)
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(imgs).to(dev)
    d_kl = torch.from_numpy(np.ascontiguousarray(kls).view(np.uint8).reshape(-1)).to(dev)
    d_n = torch.full((n,), m, dtype=torch.int32, device=dev)
    d_desc = torch.zeros(n * m * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for _ in range(a.warmup):
        lbd.compute_batch(d_img, n, d_kl, d_n, d_desc)
    times = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lbd.compute_batch(d_img, n, d_kl, d_n, d_desc)   # synchronises
        times.append(time.perf_counter() - t0)
    ms = 1e3 * float(np.mean(times))
    out = {"metric": "LBD images/s (BinaryDescriptor::compute, 300 keylines per image)", "value": n / (ms * 1e-3),
           "unit": "images/s", "keylines_per_s": n * m / (ms * 1e-3), "images_per_call": n, "ms_per_call": ms,
           "config": {"workload": f"{a.cam} {W}x{H}, {m} octave-0 keylines per image, 9 bands x 7 rows",
                      "data": "synthetic (gfpl_synth_image + random segments)"}}
    import oracle as O
    if a.check:
        got = d_desc.cpu().numpy().reshape(n, m, 32)
        bad = sum(int(not (got[i] == O.lbd_compute(imgs[i], kls[i])[0]).all()) for i in range(min(a.check, n)))
        out["parity_sampled"] = {"images": min(a.check, n), "mismatches": bad}
    if a.cpu_sample:
        t0 = time.perf_counter()
        for i in range(a.cpu_sample):
            O.lbd_compute(imgs[i], kls[i])
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": a.cpu_sample / dt, "unit": "images/s", "cores": 1, "kind": "port",
                               "sample": f"{a.cpu_sample} images of the batch through the CPU oracle"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
