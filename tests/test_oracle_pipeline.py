"""CPU oracle end to end on synthetic sequences: sensible tracking, the
reference's guards on empty / tiny inputs, and determinism."""
import numpy as np

import gfpl
import oracle as O
from parity import make_ragged


def _run(H, cam, cfg, b, kp, kl):
    h = O.OracleHandler(cam, cfg, kp, kl)
    h.initialize(H.frames(0), b)
    out = []
    for k in range(1, H.F):
        h.insertStereoPair(H.frames(k), b)
        tr = h.read_track()
        h.optimizePose()
        c = h.read_frame(gfpl.CURR)
        out.append((c.n_pt, c.n_ls, len(tr["matched_pt"]), len(tr["matched_ls"]), c.get("DT"),
                    h.read_track()["num_frame_loss"], c.s.err_norm))
        h.updateFrame()
    return out


def test_tracks_synthetic_motion():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(seed=3)
    H = gfpl.HostFrames(cam, sp, 1, 4, 2048, 512)
    for n_pt, n_ls, mp_, ml, DT, loss, err in _run(H, cam, cfg, 0, 2048, 512):
        assert 1200 < n_pt <= 2000 and 300 < n_ls <= 500
        assert mp_ == 500 and ml == 300                  # reference caps (src/config.cpp:94-95)
        assert loss == 0 and 0 <= err < 1.0
        # forward 0.5 m/s at 20 Hz: prev<-curr translation ~ +2.5 cm along z
        assert abs(DT[2, 3] - 0.025) < 3e-3 and abs(DT[0, 3]) < 3e-3


def test_ragged_inputs_follow_reference_guards():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(n_kp=600, n_kl=150, n_world_pts=800, n_world_lines=200, seed=13)
    H = make_ragged(gfpl.HostFrames(cam, sp, 5, 3, 1024, 256))
    r1 = _run(H, cam, cfg, 1, 1024, 256)
    assert r1[1][0] == 0 and r1[1][2] == 0          # no left kps at frame 2 -> no points, no point matches
    r2 = _run(H, cam, cfg, 2, 1024, 256)
    assert r2[0][1] == 0 and r2[0][3] == 0          # one right line -> no stereo lines
    r3 = _run(H, cam, cfg, 3, 1024, 256)
    assert r3[1][:4] == (0, 0, 0, 0)
    assert np.array_equal(r3[1][4], np.eye(4)) and r3[1][5] == 0   # too few features: identity, still tracked
    r4 = _run(H, cam, cfg, 4, 1024, 256)
    assert r4[0][0] <= 30 and r4[0][1] <= 3


def test_deterministic():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("kitti", cfg)
    sp = gfpl.synth_params(seed=8, dt=0.1, v_fwd=8.0, z_min=4.0, z_max=40.0)
    H1 = gfpl.HostFrames(cam, sp, 1, 3, 2048, 512)
    H2 = gfpl.HostFrames(cam, sp, 1, 3, 2048, 512)
    for a, b in zip(H1.arrays(), H2.arrays()):
        assert np.array_equal(a, b)
    a, b = _run(H1, cam, cfg, 0, 2048, 512), _run(H2, cam, cfg, 0, 2048, 512)
    for x, y in zip(a, b):
        assert x[:4] == y[:4] and np.array_equal(x[4], y[4])
