"""C++ host mirror (gf-pl-slam_amd/host/stvo.h): the app/plslam_mod.cpp-style
driver runs the StVO classes over the C ABI; its per-frame poses must equal the
CPU oracle's on the same synthetic sequence."""
import json
import os
import subprocess

import numpy as np
import pytest

import gfpl
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "gf-pl-slam_amd", "bin", "plslam_gpu")


def test_driver_fails_loudly_without_gpu():
    if not os.path.exists(BIN):
        pytest.skip("host mirror not built")
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([BIN, "--frames", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "no HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("camera,seq", [("vga", 3), ("kitti", 1)])
def test_host_mirror_matches_oracle(camera, seq, tmp_path):
    n = 6
    r = subprocess.run([BIN, "--camera", camera, "--frames", str(n), "--seq", str(seq), "--json",
                        "--out", str(tmp_path / "run")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == n - 1
    cfg = gfpl.default_config()
    cam = gfpl.make_camera(camera, cfg)
    over = dict(dt=0.1, v_fwd=8.0, z_min=4.0, z_max=40.0) if camera == "kitti" else {}
    H = gfpl.HostFrames(cam, gfpl.synth_params(**over), 1, n, 2048, 512, seq0=seq)
    o = O.OracleHandler(cam, cfg, 2048, 512)
    o.initialize(H.frames(0), 0)
    T_kf_w, poses = np.eye(4), []
    for k in range(1, n):
        o.insertStereoPair(H.frames(k), 0)
        tr = o.read_track()
        o.optimizePose()
        g = lines[k - 1]
        assert g["frame"] == k
        c = o.read_frame(gfpl.CURR)
        assert g["n_pt"] == c.n_pt and g["n_ls"] == c.n_ls
        assert g["matched_pt"] == len(tr["matched_pt"]) and g["matched_ls"] == len(tr["matched_ls"])
        assert g["n_inliers"] == o.read_track()["n_inliers"]
        # the app's keyframe step (app/plslam_mod.cpp:424-447), chain of MapHandler::addKeyFrame
        T_base = T_kf_w
        kf = o.needNewKF()
        assert bool(g["kf"]) == kf, k
        if kf:
            T_kf_w = T_kf_w @ c.get("Tfw")
            o.currFrameIsKF()
            c = o.read_frame(gfpl.CURR)
        # %.17g round-trips doubles exactly: the pose is bit-identical
        assert np.array_equal(np.array(g["Tfw"]), c.get("Tfw").reshape(-1)), k
        assert np.array_equal(np.array(g["DT"]), c.get("DT").reshape(-1)), k
        assert g["err_norm"] == float(c.s.err_norm)
        poses.append(T_base @ o.read_frame(gfpl.PREV).get("Tfw"))   # updateFrame_ECCV18 (:864-922)
        o.updateFrame()
    traj = (tmp_path / "run_AllFrameTrajectory.txt").read_text().splitlines()
    assert traj[0] == "#TimeStamp Tx Ty Tz Qx Qy Qz Qw" and len(traj) == n   # header + n-1 poses
    assert all(len(t.split()) == 7 for t in traj[1:])
    for t, T in zip(traj[1:], poses):
        assert np.allclose([float(x) for x in t.split()[:3]], T[:3, 3], atol=2e-7)
