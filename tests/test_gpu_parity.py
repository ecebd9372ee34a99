"""GPU (HIP, through the C ABI) vs CPU oracle parity of the tracking path.

Bar (BASELINE.json north_star): matched indices / Hamming / every discrete
decision bit-exact; poses within 1e-6 relative.  The kernels evaluate the
oracle's operation order, so the double-precision
feature state is compared bit-for-bit as well.
"""
import ctypes as C

import numpy as np
import pytest

import gfpl
import oracle as O
from parity import compare_core, compare_pose, compare_prev_matched, compare_track

pytestmark = pytest.mark.gpu


def _run_sequence(cam_name, cfg_over, n_seq, n_frames, kp_cap, kl_cap, synth_over=None, seed=1):
    cfg = gfpl.default_config(**cfg_over)
    cam = gfpl.make_camera(cam_name, cfg)
    sp = gfpl.synth_params(seed=seed, **(synth_over or {}))
    H = gfpl.HostFrames(cam, sp, n_seq, n_frames, kp_cap, kl_cap)
    D = gfpl.DeviceFrames(H)
    ctx = gfpl.Context(cam, cfg)
    g = gfpl.StereoFrameHandler(ctx, n_seq, kp_cap, kl_cap)
    orc = [O.OracleHandler(cam, cfg, kp_cap, kl_cap) for _ in range(n_seq)]
    report = {"core": [], "track": [], "prev": [], "pose": [], "pose_exact": [], "counts": []}
    g.initialize(D.frames(0))
    for b, o in enumerate(orc):
        o.initialize(H.frames(0), b)
        report["core"] += compare_core(g.read_frame(gfpl.PREV, b), o.read_frame(gfpl.PREV), f"init s{b} ")
    for k in range(1, n_frames):
        g.insertStereoPair(D.frames(k))
        for b, o in enumerate(orc):
            o.insertStereoPair(H.frames(k), b)
            tag = f"f{k} s{b} "
            gc, oc = g.read_frame(gfpl.CURR, b), o.read_frame(gfpl.CURR)
            report["core"] += compare_core(gc, oc, tag)
            tg, to = g.read_track(b), o.read_track()
            report["track"] += compare_track(tg, to, tag + "insert ")
            report["counts"].append((oc.n_pt, oc.n_ls, len(to["matched_pt"]), len(to["matched_ls"])))
            if not compare_track(tg, to):
                report["prev"] += compare_prev_matched(g.read_frame(gfpl.PREV, b), o.read_frame(gfpl.PREV), to, tag)
        g.optimizePose()
        for b, o in enumerate(orc):
            o.optimizePose()
            tag = f"f{k} s{b} "
            bad, exact = compare_pose(g.read_frame(gfpl.CURR, b), o.read_frame(gfpl.CURR), what=tag)
            report["pose"] += bad
            report["pose_exact"].append(exact)
            tg, to = g.read_track(b), o.read_track()
            report["track"] += compare_track(tg, to, tag + "pose ")
            if not compare_track(tg, to):
                report["prev"] += compare_prev_matched(g.read_frame(gfpl.PREV, b), o.read_frame(gfpl.PREV), to, tag + "pose ")
        g.updateFrame()
        for o in orc:
            o.updateFrame()
    return report


def _check(rep):
    msgs = rep["core"] + rep["track"] + rep["prev"] + rep["pose"]
    assert not msgs, "\n".join(msgs[:40])
    # real work happened
    assert all(c[0] > 0 and c[1] > 0 for c in rep["counts"]), rep["counts"]


@pytest.fixture(scope="module")
def vga_default():
    return _run_sequence("vga", {}, n_seq=3, n_frames=5, kp_cap=2048, kl_cap=512)


def test_vga_default_config_parity(vga_default):
    _check(vga_default)


def test_vga_default_pose_bitexact(vga_default):
    # stronger than the 1e-6 bar: same op order -> identical bits
    assert all(vga_default["pose_exact"]), vga_default["pose_exact"]


def test_bench_config_parity():
    # harness overrides of SURVEY §8(d): 10 + 10 GN iterations, no early stop
    rep = _run_sequence("vga", dict(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0),
                        n_seq=2, n_frames=4, kp_cap=2048, kl_cap=512, seed=7)
    _check(rep)


def test_kitti_camera_parity():
    rep = _run_sequence("kitti", dict(max_iters=10, max_iters_ref=10), n_seq=2, n_frames=4, kp_cap=2048,
                        kl_cap=512, synth_over=dict(dt=0.1, v_fwd=8.0, z_min=4.0, z_max=40.0), seed=3)
    _check(rep)


def test_small_counts_parity():
    # ragged small frames: 300 ORB + 60 LBD per side
    rep = _run_sequence("euroc", {}, n_seq=2, n_frames=4, kp_cap=512, kl_cap=128,
                        synth_over=dict(n_kp=300, n_kl=60, n_world_pts=400, n_world_lines=90), seed=11)
    _check(rep)


def test_knn2_hamming_parity():
    import torch
    rng = np.random.default_rng(5)
    q = rng.integers(0, 256, (700, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    t[17] = t[3]      # exact ties -> lower train index first (ledger T1)
    q[5] = t[3]
    cfg = gfpl.default_config()
    ctx = gfpl.Context(gfpl.make_camera("vga", cfg), cfg)
    for cell in (1, 2):
        qd, td = torch.from_numpy(q).cuda(), torch.from_numpy(t).cuda()
        idx = torch.zeros((700, 2), dtype=torch.int32, device="cuda")
        dist = torch.zeros((700, 2), dtype=torch.float32, device="cuda")
        assert ctx.knn2(qd, 700, td, 300, cell, idx, dist) == 0
        ctx.synchronize()
        rc, oi, od = O.knn2(q, t, cell)
        assert rc == 0
        assert np.array_equal(idx.cpu().numpy(), oi)
        assert np.array_equal(dist.cpu().numpy(), od)
    # U4: fewer than two train rows
    assert ctx.knn2(qd, 700, td, 1, 1, idx, dist) == -4
