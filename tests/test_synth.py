"""The synthetic input generator: deterministic, within capacity, detections
inside the margins the sub-pixel SAD needs, descriptors with the intended
Hamming statistics."""
import numpy as np
import pytest

import gfpl


def test_counts_margins_and_octaves():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(seed=1)
    H = gfpl.HostFrames(cam, sp, 2, 2, 2048, 512)
    assert (H.n_kp_l == 2000).all() and (H.n_kp_r == 2000).all()
    assert (H.n_kl_l == 500).all() and (H.n_kl_r == 500).all()
    kp = H.kp_l[0, 0, :2000]
    assert kp["x"].min() >= 40 - 1.5 and kp["x"].max() <= 640 - 41 + 1.5
    assert set(np.unique(kp["octave"])) <= {0, 1, 2, 3}
    assert np.all(H.time_stamp[1] - H.time_stamp[0] > 0.049)


def test_descriptor_statistics():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    H = gfpl.HostFrames(cam, gfpl.synth_params(seed=2), 1, 1, 2048, 512)
    dl, dr = H.pdesc_l[0, 0, :2000], H.pdesc_r[0, 0, :2000]
    # random pairs ~128 bits apart
    x = np.unpackbits(np.bitwise_xor(dl[:500], dr[500:1000]), axis=1).sum(1)
    assert 110 < x.mean() < 146


def test_seq_offset_equals_global_id():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(n_kp=300, n_kl=60, n_world_pts=400, n_world_lines=90, seed=4)
    A = gfpl.HostFrames(cam, sp, 3, 2, 512, 128)
    B = gfpl.HostFrames(cam, sp, 1, 2, 512, 128, seq0=2)
    for a, b in zip(A.arrays(), B.arrays()):
        assert np.array_equal(a[:, 2], b[:, 0])


def test_frames_independent_of_chunking():
    """bench.py stages inputs frame by frame (DeviceFrames.generate): a frame must
    not depend on which other frames were generated with it."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(seed=3, n_kp=300, n_kl=60, n_world_pts=400, n_world_lines=90)
    whole = gfpl.HostFrames(cam, sp, 3, 4, 512, 128, seq0=5)
    one = gfpl.HostFrames(cam, sp, 3, 1, 512, 128, seq0=5, frame0=2)
    for a, b in zip(whole.arrays(), one.arrays()):
        assert np.array_equal(a[2], b[0])
    assert gfpl.input_bytes_per_frame(cam, 512, 128) == sum(a[0].nbytes for a in one.arrays()) // 3


def test_respawn_keeps_the_scene_stationary():
    """bench.py's workloads re-spawn landmarks (gfpl_synth `respawn`): the true (landmark)
    detections stay at 90 % of the budget at every frame (10 % distractors),
    where the fixed pool of respawn = 0 drains as the camera moves on."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    cfg = gfpl.default_config()
    for wl, (cam_name, over, _) in bench.WORKLOADS.items():
        cam = gfpl.make_camera(cam_name, cfg)
        keep = []
        if wl == "cfg4":
            T, t = gfpl.euroc_traj("mh_02", 61)
            keep += [T, t]
            over = dict(over, traj=T.ctypes.data, n_traj=len(t), traj_t=t.ctypes.data)
        sp = gfpl.synth_params(**over)
        for k in (0, 1, 7, 20, 33, 60):
            for s in (0, 5):
                n_kp, n_kl = gfpl.synth_true_counts(cam, sp, s, k)
                assert n_kp >= 0.9 * sp.n_kp - 1 and n_kl >= 0.9 * sp.n_kl - 1, (wl, k, s, n_kp, n_kl)
    # the fixed pool drains (the round-2 bench workload: 1800 -> < 1000 true keypoints by frame 25)
    cam = gfpl.make_camera("vga", cfg)
    assert gfpl.synth_true_counts(cam, gfpl.synth_params(), 0, 25)[0] < 1000


def test_respawn_zero_is_the_fixed_pool():
    """respawn = 0 keeps the round-1/2 generator bit for bit (the golden fixtures depend on it)."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(seed=3, n_kp=300, n_kl=60, n_world_pts=400, n_world_lines=90)
    assert sp.respawn == 0
    A = gfpl.HostFrames(cam, sp, 2, 3, 512, 128)
    sp2 = gfpl.synth_params(seed=3, n_kp=300, n_kl=60, n_world_pts=400, n_world_lines=90, respawn=4)
    R = gfpl.HostFrames(cam, sp2, 2, 3, 512, 128)
    assert not np.array_equal(A.kp_l, R.kp_l)


def test_trajectory_frames_are_not_wrapped():
    """A frame past the loaded ground-truth trajectory is refused (it used to wrap to pose 0)."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("euroc", cfg)
    T, t = gfpl.euroc_traj("v1_03", 4)
    sp = gfpl.synth_params(traj=T.ctypes.data, n_traj=len(t), traj_t=t.ctypes.data, respawn=16)
    gfpl.HostFrames(cam, sp, 1, 4, 2048, 512)
    with pytest.raises(gfpl.GfplError):
        gfpl.HostFrames(cam, sp, 1, 5, 2048, 512)
    with pytest.raises(ValueError):
        gfpl.euroc_traj("mh_01", gfpl.EUROC_MAX_POSES + 1)


def test_level0_pyramids_are_the_orb_resize_chain():
    """pyr_from_l0 = 1: levels 1.. of the right pyramid are cv::resize INTER_LINEAR of the level
    above (ComputePyramid, src/ORBextractor.cc:1107-1132) — byte-equal to the ORB oracle's
    restatement, hence to the device's k_orb_resize (tests/test_orb_gpu.py); pyr_from_l0 = 2
    writes level 0 only, byte-equal to mode 1's level 0, with the same detections."""
    import oracle as O
    for name in ("vga", "kitti", "euroc"):
        cfg = gfpl.default_config()
        cam = gfpl.make_camera(name, cfg)
        W0, H0 = int(cam.lvl_cols[0]), int(cam.lvl_rows[0])
        h1 = gfpl.HostFrames(cam, gfpl.synth_params(respawn=16, pyr_from_l0=1), 2, 2, 2048, 512)
        h2 = gfpl.HostFrames(cam, gfpl.synth_params(respawn=16, pyr_from_l0=2), 2, 2, 2048, 512)
        for f in range(2):
            for b in range(2):
                pyr = h1.pyr_r[f, b]
                lv = lambda l: pyr[int(cam.lvl_offset[l]):int(cam.lvl_offset[l]) + int(cam.lvl_cols[l]) * int(cam.lvl_rows[l])] \
                    .reshape(int(cam.lvl_rows[l]), int(cam.lvl_cols[l]))
                for l in range(1, int(cam.n_levels)):
                    want = O.orb_resize(np.ascontiguousarray(lv(l - 1)), int(cam.lvl_cols[l]), int(cam.lvl_rows[l]))
                    assert (lv(l) == want).all(), (name, f, b, l)
                assert (h2.pyr_r[f, b, :W0 * H0] == pyr[:W0 * H0]).all() and not h2.pyr_r[f, b, W0 * H0:].any()
        for a1, a2 in zip(h1.arrays()[:12], h2.arrays()[:12]):
            assert (a1 == a2).all()


def test_level0_patches_survive_the_pyramid():
    """The magnified level-0 stamps leave each true keypoint's patch at its octave level, so the
    sub-pixel refinement (both windows from the right pyramid, ledger Q1) keeps most stereo points:
    on the oracle, >= 85% of the per-level stamping's stereo points (VGA, 1800 true keypoints)."""
    import oracle as O
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    n = {}
    for mode in (0, 1):
        h = gfpl.HostFrames(cam, gfpl.synth_params(respawn=16, pyr_from_l0=mode), 1, 1, 2048, 512)
        o = O.OracleHandler(cam, cfg, 2048, 512)
        o.initialize(h.frames(0), 0)
        n[mode] = o.read_frame(gfpl.PREV).n_pt
    assert n[1] >= 0.85 * n[0] and n[1] > 1200, n
