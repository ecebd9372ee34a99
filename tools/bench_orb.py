#!/usr/bin/env python3
"""ORB extraction throughput: gfpl_orb_extract over a batch of
synthetic grey images resident in HBM, as ORBextractor::operator() (src/ORBextractor.cc:
1043-1105) is run per image by StereoFrame (2 per stereo frame).

Prints one JSON line: images/s on the GPU (inputs resident, outputs left on the device),
ms per batch, keypoints per image, and the CPU oracle timed on a bounded sample of the same
images (one core) as the reference-side restatement.  Per-kernel times come from
`rocprofv3 --kernel-trace --stats -- python3 tools/bench_orb.py ...`."""
from __future__ import annotations

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
    ap.add_argument("--images", type=int, default=256, help="images per gfpl_orb_extract call")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--nlevels", type=int, default=4)
    ap.add_argument("--scale", type=float, default=1.2)
    ap.add_argument("--cpu-sample", type=int, default=8, help="images timed on the CPU oracle (0: skip)")
    ap.add_argument("--check", type=int, default=2, help="images of the batch compared with the oracle")
    a = ap.parse_args()

    import torch
    import gfpl
    c = gfpl.CAMERAS[a.cam]
    W, H, n = c["width"], c["height"], a.images
    # distinct images: synthetic scenes with sensor noise
    imgs = np.stack([gfpl.synth_image(i, i % 7, W, H) for i in range(n)])
    orb = gfpl.ORBextractor(a.nfeatures, a.scale, a.nlevels, 20, 7, W, H, max_images=n)
    dev = torch.device("cuda", 0)
    kc = orb.kp_cap
    d_img = torch.from_numpy(imgs).to(dev)
    kps = torch.zeros(n * kc * gfpl.KEYPOINT_DT.itemsize, dtype=torch.uint8, device=dev)
    desc = torch.zeros(n * kc * 32, dtype=torch.uint8, device=dev)
    nkp = torch.zeros(n, dtype=torch.int32, device=dev)
    ang = torch.zeros(n * kc, dtype=torch.float32, device=dev)
    rsp = torch.zeros(n * kc, dtype=torch.float32, device=dev)
    stride = (orb.pyramid_bytes + 255) // 256 * 256
    pyr = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for _ in range(a.warmup):
        orb.extract(d_img, n, kps, desc, nkp, ang, rsp, pyr, stride)
    times = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        orb.extract(d_img, n, kps, desc, nkp, ang, rsp, pyr, stride)   # synchronises
        times.append(time.perf_counter() - t0)
    ms = 1e3 * float(np.mean(times))
    nk = nkp.cpu().numpy()
    out = {"metric": "ORB images/s (ORBextractor::operator(), keypoints+descriptors+pyramid)",
           "value": n / (ms * 1e-3), "unit": "images/s", "images_per_call": n, "ms_per_call": ms,
           "ms_min": 1e3 * float(np.min(times)), "kp_per_image": float(nk.mean()),
           "config": {"workload": f"{a.cam} {W}x{H}, nfeatures {a.nfeatures}, {a.nlevels} levels, "
                                  f"scale {a.scale}, FAST 20/7", "data": "synthetic (gfpl_synth_image)"}}
    if a.check or a.cpu_sample:
        import oracle as O
        if a.check:
            k = kps.cpu().numpy().view(gfpl.KEYPOINT_DT).reshape(n, kc)
            d = desc.cpu().numpy().reshape(n, kc, 32)
            bad = 0
            for i in range(min(a.check, n)):
                o = O.orb_extract(imgs[i], a.nfeatures, a.scale, a.nlevels, kp_cap=kc)
                m = len(o["kps"])
                bad += int(nk[i] != m or not (k[i, :m] == o["kps"]).all() or not (d[i, :m] == o["desc"]).all())
            out["parity_sampled"] = {"images": min(a.check, n), "mismatches": bad}
        if a.cpu_sample:
            t0 = time.perf_counter()
            for i in range(a.cpu_sample):
                O.orb_extract(imgs[i], a.nfeatures, a.scale, a.nlevels, kp_cap=kc)
            dt = time.perf_counter() - t0
            out["cpu_baseline"] = {"value": a.cpu_sample / dt, "unit": "images/s", "cores": 1, "kind": "port",
                                   "sample": f"{a.cpu_sample} images of the batch through the CPU oracle"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
