"""Line-cut move statistics from the oracle's analysis build (round 5, DESIGN.md §4 k_cut_search_w).

Builds oracle/ with -DGFPL_ORACLE_CUT_STATS into /tmp/ostats (never the in-tree liboracle.so, which is
the timed CPU baseline), tracks 8 bench-config (cfg2) sequences over 6 frames, and prints the move
classes: (sign of the start-ratio change + 1) * 3 + (sign of the end-ratio change + 1), then the
single-ratio repeats and the line count.  The per-line move strings land in /tmp/gfplo_cut_paths.txt,
which tools/grid_shapes.py reads.  CPU only."""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))

LIB = "/tmp/ostats/liboracle.so"


def main():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    src = [os.path.join(ROOT, "oracle", f) for f in
           ("gfpl_oracle.cpp", "gfpl_orb_oracle.cpp", "gfpl_lbd_oracle.cpp", "gfpl_lsd_oracle.cpp")]
    subprocess.run(["g++", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-march=x86-64-v3",
                    "-I" + os.path.join(ROOT, "include"), "-DGFPL_ORACLE_CUT_STATS", *src, "-o", LIB, "-lpthread"],
                   check=True)
    import bench
    import gfpl
    import oracle as O
    join = os.path.join
    os.path.join = lambda *a: LIB if join(*a).endswith("liboracle.so") else join(*a)
    try:
        L = O.lib()
    finally:
        os.path.join = join
    L.gfplo_cut_stats.argtypes = [C.c_void_p]
    cam_name, synth_over, _ = bench.WORKLOADS["cfg2"]
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0)
    cam = gfpl.make_camera(cam_name, cfg)
    sp = gfpl.synth_params(**synth_over, pyr_from_l0=1)
    n, nf, KP, KL = 8, 6, 2048, 512
    H = gfpl.HostFrames(cam, sp, n, nf + 1, KP, KL, seq0=0, threads=8)
    hs = [O.OracleHandler(cam, cfg, KP, KL) for _ in range(n)]
    for b, h in enumerate(hs):
        h.initialize(H.frames(0), b)
    for k in range(1, nf + 1):
        for b, h in enumerate(hs):
            h.insertStereoPair(H.frames(k), b)
            h.optimizePose()
            h.updateFrame()
    import numpy as np
    o = np.zeros(8, np.int64)
    L.gfplo_cut_stats(o.ctypes.data)   # (prints the gap histogram and the move classes on stderr)
    print("lines, steps, valid evals, bit-distinct evals, unmoved lines, setup logdets, moves back:", o.tolist())


if __name__ == "__main__":
    main()
