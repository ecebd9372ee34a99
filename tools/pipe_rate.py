"""Images-to-poses rates alone (bench.py's pipeline_rate, the `detection` block's
images_to_poses / images_to_poses_lsd), for iterating on the detectors without the full bench."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))

import bench  # noqa: E402
import gfpl  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--lsd", type=int, default=1, help="1: LSD on the device, 0: given keylines, 2: both")
    a = ap.parse_args()
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0)
    cam = gfpl.make_camera("vga", cfg)
    out = {}
    for lsd in ((a.lsd == 1,) if a.lsd < 2 else (False, True)):
        out["images_to_poses_lsd" if lsd else "images_to_poses"] = bench.pipeline_rate(cam, cfg, B=a.batch,
                                                                                       steps=a.steps, lsd=lsd, progress=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
