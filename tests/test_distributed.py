"""World-size-2 rehearsal of bench.py's multi-GPU path on CPU (gloo).

Sequences shard across ranks with no data-path collective: each rank tracks
its own sequences; the camera/config block is broadcast from rank 0 and the
timing / frame counters are reduced.  Here the tracker is the CPU oracle (the
GPU path runs the same per-rank code on cuda:<local_rank> with nccl=RCCL).
"""
import os
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, F = 2, 3


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import gfpl
    import oracle as O
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga" if rank == 0 else "euroc", cfg)   # rank 1 starts with the wrong camera
    if rank == 1:
        cfg.max_iters = 99
    bench.broadcast_setup(cam, cfg, dist, "cpu")
    sp = gfpl.synth_params(n_kp=500, n_kl=120, n_world_pts=700, n_world_lines=170, seed=21)
    s0 = bench.shard_first_seq(rank, B)
    H = gfpl.HostFrames(cam, sp, B, F, 512, 128, seq0=s0, threads=1)
    poses = []
    for b in range(B):
        h = O.OracleHandler(cam, cfg, 512, 128)
        h.initialize(H.frames(0), b)
        for k in range(1, F):
            h.insertStereoPair(H.frames(k), b); h.optimizePose(); h.updateFrame()
        poses.append(h.read_frame(gfpl.PREV).get("Tfw"))
    t, n = bench.reduce_job(0.5 + rank, B * (F - 1), dist, "cpu")
    q.put((rank, cam.width, cfg.max_iters, s0, np.stack(poses), t, n))
    dist.destroy_process_group()


def test_two_rank_sharded_tracking():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, w0, it0, s00, P0, t0, n0), (r1, w1, it1, s01, P1, t1, n1) = res
    assert w0 == w1 == 640 and it0 == it1 == 5            # rank 0's camera/config everywhere
    assert (s00, s01) == (0, B)                           # disjoint shards
    assert t0 == t1 == 1.5 and n0 == n1 == 2 * B * (F - 1)   # MAX time, SUM frames
    assert not np.allclose(P0, P1)                        # different sequences
    # single-process run of the same global sequence ids gives identical results
    sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import gfpl
    import oracle as O
    cfg = gfpl.default_config(); cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(n_kp=500, n_kl=120, n_world_pts=700, n_world_lines=170, seed=21)
    H = gfpl.HostFrames(cam, sp, 2 * B, F, 512, 128, threads=1)
    for b in range(2 * B):
        h = O.OracleHandler(cam, cfg, 512, 128)
        h.initialize(H.frames(0), b)
        for k in range(1, F):
            h.insertStereoPair(H.frames(k), b); h.optimizePose(); h.updateFrame()
        ref = (P0 if b < B else P1)[b % B]
        assert np.array_equal(h.read_frame(gfpl.PREV).get("Tfw"), ref)
