"""The image-input boundary (gfpl_detector_*, include/gfpl.h): StereoFrame's detection from a
grey stereo pair on the device — ORB, LSD, LBD of both images — feeding the tracker through the
detector's gfpl_frames views, against the oracle chain (ORB / LSD / LBD oracles -> tracker
oracle) on the same images.  Reference: StereoFrameHandler::initialize / insertStereoPair(
const Mat& img_l, const Mat& img_r, int idx, double ts) (include/stereoFrameHandler.h:48-53,
src/stereoFrame.cpp:148-172, 411-450, 1128-1227; app/plslam_mod.cpp:377,387).  Also drives the
C++ mirror (plslam_gpu --images) from image files."""
import json
import os
import subprocess

import numpy as np
import pytest

import gfpl
import oracle as O
from gfpl.pipeline import synth_stereo_steps
from parity import compare_core, compare_pose, compare_track
from test_pipeline_gpu import _host_frames

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "gf-pl-slam_amd", "bin", "plslam_gpu")
NFEAT, KP, KL = 2000, 2320, 320
BARS = 600   # the dense scene: ~2000 ORB keypoints and 300 LSD keylines per image (the north-star load)


def _oracle_scene(L, R):
    return (L, R, O.lsd_detect(L)[0], O.lsd_detect(R)[0])


def test_detector_images_to_poses_match_the_oracle_chain():
    """B = 2 staircase sequences x 4 frames: device images -> gfpl_detect_stereo_async ->
    initialize / frameStep, with the detection of frame k + 1 enqueued before the step on frame k
    (the views' ready / consumed events alone order them); detections byte-equal to the oracles',
    stereo features, matched lists and poses bit-equal to the oracle tracker's."""
    import torch
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    B, F = 2, 4
    W, H = int(cam.width), int(cam.height)
    dev = torch.device("cuda", 0)
    ctx = gfpl.Context(cam, cfg, stream=torch.cuda.current_stream(dev).cuda_stream)
    det = gfpl.StereoDetector(ctx, B, KP, KL, gfpl.DetectorParams.reference(cam, cfg, nfeatures=NFEAT))
    g = gfpl.StereoFrameHandler(ctx, B, KP, KL)
    orc = [O.OracleHandler(cam, cfg, KP, KL) for _ in range(B)]

    def detect(k):
        imgs = [synth_stereo_steps(b, k, W, H, bars=BARS)[:2] for b in range(B)]
        left = torch.from_numpy(np.stack([i[0] for i in imgs])).to(dev)
        right = torch.from_numpy(np.stack([i[1] for i in imgs])).to(dev)
        ts = torch.full((B,), 0.05 * k, dtype=torch.float64, device=dev)
        return imgs, det.detect(left, right, ts)

    bad, counts = [], []
    imgs, fr = detect(0)
    for k in range(F):
        scenes = [_oracle_scene(L, R) for L, R in imgs]
        hfr, harr = _host_frames(cam, scenes, KP, KL, 0.05 * k)
        # the detections of every sequence, read back through gfpl_read_detections
        for b in range(B):
            d = det.read(fr, b)
            for side, s in enumerate("lr"):
                n_kp, n_kl = int(harr[side][b]), int(harr[6 + side][b])
                assert len(d["kp_" + s]) == n_kp and len(d["kl_" + s]) == n_kl, (k, b, s)
                assert d["kp_" + s].tobytes() == harr[2 + side][b, :n_kp].tobytes(), (k, b, s)
                assert (d["pdesc_" + s] == harr[4 + side][b, :n_kp]).all(), (k, b, s)
                assert d["kl_" + s].tobytes() == harr[8 + side][b, :n_kl].tobytes(), (k, b, s)
                assert (d["ldesc_" + s] == harr[10 + side][b, :n_kl]).all(), (k, b, s)
        cur = fr
        if k + 1 < F:
            imgs, fr = detect(k + 1)   # enqueued before the tracker reads frame k
        if k == 0:
            g.initialize(cur)
            for b, o in enumerate(orc):
                o.initialize(hfr, b)
            continue
        g.frameStep(cur)
        for b, o in enumerate(orc):
            o.insertStereoPair(hfr, b)
            o.optimizePose()
            tr = o.read_track()
            counts.append((len(tr["matched_pt"]), len(tr["matched_ls"])))
            o.updateFrame()
            gp, op = g.read_frame(gfpl.PREV, b), o.read_frame(gfpl.PREV)
            bad += compare_core(gp, op, f"f{k} s{b} ")
            bad += compare_pose(gp, op, what=f"f{k} s{b} ")[0]
            bad += compare_track(g.read_last_track(b), tr, f"f{k} s{b} ")
    det.status()
    assert not bad, "\n".join(bad[:30])
    assert all(c[0] > 100 and c[1] > 100 for c in counts), counts   # tracking at the dense scene's load
    g.close()
    det.close()


def test_detector_host_images_views_and_lifetime():
    """gfpl_detect_stereo_host (host images) equals the device form; at most `sets` views may be
    outstanding (GFPL_E_STATE otherwise, gfpl_detector_discard frees one); a context is not
    destroyed while a detector (or an ORB / LSD / LBD object) built on it lives."""
    import torch
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    W, H = int(cam.width), int(cam.height)
    dev = torch.device("cuda", 0)
    ctx = gfpl.Context(cam, cfg)
    det = gfpl.StereoDetector(ctx, 1, KP, KL, gfpl.DetectorParams.reference(cam, cfg, nfeatures=NFEAT), sets=2)
    L, R = synth_stereo_steps(5, 2, W, H)[:2]
    f_host = det.detect_host(L, R, 0.1)
    a = det.read(f_host, 0)
    f_dev = det.detect(torch.from_numpy(L[None].copy()).to(dev), torch.from_numpy(R[None].copy()).to(dev),
                       torch.tensor([0.1], dtype=torch.float64, device=dev), n=1)
    b = det.read(f_dev, 0)
    for k in a:
        assert a[k].tobytes() == b[k].tobytes(), k
    ol = O.orb_extract(L, nfeatures=NFEAT, kp_cap=KP)
    assert a["kp_l"].tobytes() == ol["kps"].tobytes() and (a["pdesc_l"] == ol["desc"]).all()
    # two views outstanding: the third detection would overwrite the first one's buffers
    with pytest.raises(gfpl.GfplError):
        det.detect_host(L, R, 0.2)
    det.discard(f_host)
    f3 = det.detect_host(L, R, 0.2)
    assert det.read(f3, 0)["kl_r"].tobytes() == a["kl_r"].tobytes()
    det.status()
    # the context is refused while the detector lives (its streams and camera are used)
    with pytest.raises(gfpl.GfplError):
        ctx.close()
    det.close()
    orb = gfpl.ORBextractor(500, 1.2, 3, 20, 7, W, H, ctx=ctx)
    with pytest.raises(gfpl.GfplError):
        ctx.close()
    orb.close()
    ctx.close()


def _write_pgm(path, img):
    h, w = img.shape
    with open(path, "wb") as f:
        f.write(f"P5\n# gfpl test\n{w} {h}\n255\n".encode())
        f.write(np.ascontiguousarray(img, np.uint8).tobytes())


def test_host_mirror_from_images_matches_the_oracle_chain(tmp_path):
    """The C++ mirror driven by images (plslam_gpu --images: StVO::StereoFrame(img_l, img_r, idx,
    cam, ts) -> initialize / insertStereoPair -> optimizePose -> needNewKF -> updateFrame_ECCV18),
    bit-exact against the oracle chain on the same image files."""
    n = 5
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    W, H = int(cam.width), int(cam.height)
    for side in ("left", "right"):
        (tmp_path / side).mkdir()
    imgs = [synth_stereo_steps(7, k, W, H, bars=BARS)[:2] for k in range(n)]
    ts = [1403636579.763555527 + 0.05 * k for k in range(n)]
    for k, (L, R) in enumerate(imgs):
        _write_pgm(tmp_path / "left" / f"{k:06d}.pgm", L)
        _write_pgm(tmp_path / "right" / f"{k:06d}.pgm", R)
    (tmp_path / "times.txt").write_text("".join(f"{t:.9f}\n" for t in ts))
    r = subprocess.run([BIN, "--camera", "vga", "--images", str(tmp_path), "--frames", str(n + 3), "--json",
                        "--orb-features", str(NFEAT), "--out", str(tmp_path / "run")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == n - 1   # stops at the first missing pair
    tsf = [float(f"{t:.9f}") for t in ts]
    o = O.OracleHandler(cam, cfg, KP, KL)
    hfr, harr = _host_frames(cam, [_oracle_scene(*imgs[0])], KP, KL, tsf[0])
    o.initialize(hfr, 0)
    for k in range(1, n):
        hfr, harr = _host_frames(cam, [_oracle_scene(*imgs[k])], KP, KL, tsf[k])
        o.insertStereoPair(hfr, 0)
        tr = o.read_track()
        o.optimizePose()
        g = lines[k - 1]
        c = o.read_frame(gfpl.CURR)
        assert g["frame"] == k and g["n_pt"] == c.n_pt and g["n_ls"] == c.n_ls, (k, g, c.n_pt, c.n_ls)
        assert g["matched_pt"] == len(tr["matched_pt"]) and g["matched_ls"] == len(tr["matched_ls"])
        kf = o.needNewKF()
        assert bool(g["kf"]) == kf, k
        if kf:
            o.currFrameIsKF()
            c = o.read_frame(gfpl.CURR)
        assert g["time_stamp"] == tsf[k]
        assert np.array_equal(np.array(g["Tfw"]), c.get("Tfw").reshape(-1)), k
        assert np.array_equal(np.array(g["DT"]), c.get("DT").reshape(-1)), k
        assert g["err_norm"] == float(c.s.err_norm)
        o.updateFrame()
    # the log's detection counts are the image detections (points_l / lines_l sizes)
    log = (tmp_path / "run_Log.txt").read_text().splitlines()[1:]
    assert len(log) == n - 1
    for k, t in enumerate(log, start=1):
        f = t.split(" ")
        n_kp_l = len(O.orb_extract(imgs[k][0], nfeatures=NFEAT, kp_cap=KP)["kps"])
        assert int(f[11]) == n_kp_l and int(f[12]) == len(O.lsd_detect(imgs[k][0])[0]), (k, f[11:13])
    # tracking at the dense scene's load (2000 ORB + 300 LSD per image; stereo points stop at ~5 px of
    # disparity, ledger Q1, so the 2 px band carries them)
    assert lines[-1]["matched_pt"] > 100 and lines[-1]["matched_ls"] > 100, lines[-1]


def test_detector_inputs_reusable_once_detect_returns():
    """gfpl_detect_stereo_async copies the caller's device images on the detector's stream and
    orders the context's stream after that copy: overwriting the same input tensors on the
    context's stream right after detect() returns leaves the detections those of the first
    images (include/gfpl.h, gfpl_detect_stereo_async)."""
    import torch
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    W, H = int(cam.width), int(cam.height)
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    ctx = gfpl.Context(cam, cfg, stream=s.cuda_stream)
    det = gfpl.StereoDetector(ctx, 1, KP, KL, gfpl.DetectorParams.reference(cam, cfg, nfeatures=NFEAT), sets=2)
    L, R = synth_stereo_steps(3, 1, W, H)[:2]
    L2, R2 = synth_stereo_steps(4, 2, W, H)[:2]
    ref = det.read(det.detect_host(L, R, 0.1), 0)
    left = torch.from_numpy(L[None].copy()).to(dev)
    right = torch.from_numpy(R[None].copy()).to(dev)
    ts = torch.tensor([0.1], dtype=torch.float64, device=dev)
    nl = torch.from_numpy(L2[None].copy()).to(dev)
    nr = torch.from_numpy(R2[None].copy()).to(dev)
    torch.cuda.synchronize()
    fr = det.detect(left, right, ts, n=1)
    with torch.cuda.stream(s):   # the next frame written into the same buffers at once
        left.copy_(nl)
        right.copy_(nr)
        ts.fill_(0.2)
    got = det.read(fr, 0)
    for k in ref:
        assert got[k].tobytes() == ref[k].tobytes(), k
    det.status()
    det.close()
    ctx.close()


def test_camera_and_cut_config_state_rules():
    """gfpl_set_camera is refused (GFPL_E_STATE) while a seqbatch or a detector object of the
    context lives; gfpl_set_config rejects a cut step that is not a positive finite number and
    an unordered cut range (GFPL_E_INVALID)."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    ctx = gfpl.Context(cam, cfg)
    L = ctx.L
    for bad in (0.0, -0.05, float("nan"), float("inf")):
        c = gfpl.default_config()
        c.cut_step = bad
        assert L.gfpl_set_config(ctx.h, gfpl.C.byref(c)) == -1, bad
    c = gfpl.default_config()
    c.cut_rng[0], c.cut_rng[1] = 0.5, 0.25
    assert L.gfpl_set_config(ctx.h, gfpl.C.byref(c)) == -1
    assert L.gfpl_set_config(ctx.h, gfpl.C.byref(gfpl.default_config())) == 0
    assert L.gfpl_set_camera(ctx.h, gfpl.C.byref(cam)) == 0          # nothing built on it yet
    h = gfpl.StereoFrameHandler(ctx, 2, 256, 64)
    assert L.gfpl_set_camera(ctx.h, gfpl.C.byref(cam)) == -6
    h.close()
    orb = gfpl.ORBextractor(500, 1.2, 3, 20, 7, int(cam.width), int(cam.height), ctx=ctx)
    assert L.gfpl_set_camera(ctx.h, gfpl.C.byref(cam)) == -6
    orb.close()
    assert L.gfpl_set_camera(ctx.h, gfpl.C.byref(cam)) == 0
    ctx.close()
