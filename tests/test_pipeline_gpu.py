"""Images in, poses out on the GPU (gfpl.pipeline): ORB and LBD detection on the device feeding
StereoFrameHandler through gfpl_frames views of their outputs, against the oracle pipeline
(ORB oracle, LBD oracle, tracker oracle) on the same images — bit-exact stereo features,
matched lists and poses (SURVEY.md §8(f)1-2 joined to rows a-e)."""
import numpy as np
import pytest

import gfpl
import oracle as O
from gfpl.pipeline import ImagePipeline, synth_stereo_scene, synth_stereo_steps
from parity import compare_core, compare_pose, compare_track

pytestmark = pytest.mark.gpu


def _host_frames(cam, scenes, kp_cap, kl_cap, ts):
    B = len(scenes)
    n_kp_l = np.zeros(B, np.int32); n_kp_r = np.zeros(B, np.int32)
    kp_l = np.zeros((B, kp_cap), gfpl.KEYPOINT_DT); kp_r = np.zeros((B, kp_cap), gfpl.KEYPOINT_DT)
    pd_l = np.zeros((B, kp_cap, 32), np.uint8); pd_r = np.zeros((B, kp_cap, 32), np.uint8)
    n_kl_l = np.zeros(B, np.int32); n_kl_r = np.zeros(B, np.int32)
    kl_l = np.zeros((B, kl_cap), gfpl.KEYLINE_DT); kl_r = np.zeros((B, kl_cap), gfpl.KEYLINE_DT)
    ld_l = np.zeros((B, kl_cap, 32), np.uint8); ld_r = np.zeros((B, kl_cap, 32), np.uint8)
    pyr = np.zeros((B, int(cam.pyr_bytes)), np.uint8)
    for b, (L, R, kll, klr) in enumerate(scenes):
        ol = O.orb_extract(L, kp_cap=kp_cap, nlevels=int(cam.n_levels))
        orr = O.orb_extract(R, kp_cap=kp_cap, nlevels=int(cam.n_levels))
        n_kp_l[b], n_kp_r[b] = len(ol["kps"]), len(orr["kps"])
        kp_l[b, :n_kp_l[b]], pd_l[b, :n_kp_l[b]] = ol["kps"], ol["desc"]
        kp_r[b, :n_kp_r[b]], pd_r[b, :n_kp_r[b]] = orr["kps"], orr["desc"]
        pb = int(sum(cam.lvl_cols[l] * cam.lvl_rows[l] for l in range(cam.n_levels)))
        pyr[b, :pb] = orr["pyramid"][:pb]
        n_kl_l[b], n_kl_r[b] = len(kll), len(klr)
        kl_l[b, :len(kll)], kl_r[b, :len(klr)] = kll, klr
        ld_l[b, :len(kll)] = O.lbd_compute(L, kll)[0]
        ld_r[b, :len(klr)] = O.lbd_compute(R, klr)[0]
    arrs = [n_kp_l, n_kp_r, kp_l, kp_r, pd_l, pd_r, n_kl_l, n_kl_r, kl_l, kl_r, ld_l, ld_r, pyr,
            np.full(B, ts, np.float64)]
    return gfpl.make_frames(B, kp_cap, kl_cap, arrs), arrs


@pytest.mark.parametrize("disparity", [3, 12, "steps"])
def test_images_to_poses_match_the_oracle_pipeline(disparity):
    """The plane scene at two depths, and the staircase of bands at disparities 2 / 12 / 20 / 8
    ("steps": points from the far band, lines from the near ones, tx = 0.05 m a frame).  The reference's sub-pixel stereo refinement reads both
    SAD windows from the right pyramid (ledger Q1), so a point's refinement only finds its
    self-match when the disparity is within the +-4 px search (3 px: points track, their
    disparities collapse to the 0.01 clamp); at 12 px the points mostly fail the refinement
    while the lines (whose covariance gate wants near depth) track."""
    import torch
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    B, F, KL = 2, 4, 320
    W, H = int(cam.width), int(cam.height)
    ctx = gfpl.Context(cam, cfg)
    pipe = ImagePipeline(ctx, cam, B, KL)
    KP = pipe.kp_cap
    g = gfpl.StereoFrameHandler(ctx, B, KP, KL)
    orc = [O.OracleHandler(cam, cfg, KP, KL) for _ in range(B)]
    dev = torch.device("cuda", 0)
    bad, counts = [], []
    for k in range(F):
        scenes = [synth_stereo_steps(b, k, W, H) if disparity == "steps" else
                  synth_stereo_scene(b, k, W, H, disparity=disparity) for b in range(B)]
        left = torch.from_numpy(np.stack([s[0] for s in scenes])).to(dev)
        right = torch.from_numpy(np.stack([s[1] for s in scenes])).to(dev)
        kl = [np.zeros((B, KL), gfpl.KEYLINE_DT) for _ in range(2)]
        n = [np.zeros(B, np.int32) for _ in range(2)]
        for b, s in enumerate(scenes):
            for side in range(2):
                n[side][b] = len(s[2 + side])
                kl[side][b, :n[side][b]] = s[2 + side]
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
        fr = pipe.detect(left, right, to(kl[0]), torch.from_numpy(n[0]).to(dev), to(kl[1]),
                         torch.from_numpy(n[1]).to(dev), torch.full((B,), 0.05 * k, dtype=torch.float64, device=dev))
        hfr, harr = _host_frames(cam, scenes, KP, KL, 0.05 * k)
        pipe.status()   # capacity errors raise
        pipe.synchronize()   # every device output (the time stamps' copy included) is complete
        # the device detections are the oracle's, byte for byte (valid rows; the device
        # buffers keep stale rows past each count)
        d = [t.cpu().numpy() for t in fr._keep]
        for side in range(2):
            nk_d, nl_d = d[0 + side], d[6 + side]
            assert (nk_d == harr[0 + side]).all() and (nl_d == harr[6 + side]).all(), (k, side)
            kd = d[2 + side].view(gfpl.KEYPOINT_DT).reshape(B, KP)
            pdd = d[4 + side].reshape(B, KP, 32)
            ldd = d[10 + side].reshape(B, KL, 32)
            for b in range(B):
                n1, n2 = int(nk_d[b]), int(nl_d[b])
                assert (kd[b, :n1] == harr[2 + side][b, :n1]).all(), (k, side, b)
                assert (pdd[b, :n1] == harr[4 + side][b, :n1]).all(), (k, side, b)
                assert (ldd[b, :n2] == harr[10 + side][b, :n2]).all(), (k, side, b)
        assert (d[12].reshape(B, -1) == harr[12]).all(), k
        torch.cuda.synchronize()
        if k == 0:
            g.initialize(fr)
            for b, o in enumerate(orc):
                o.initialize(hfr, b)
            continue
        g.frameStep(fr)
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
    assert not bad, "\n".join(bad[:30])
    if disparity == "steps":
        assert all(c[0] > 30 and c[1] > 100 for c in counts), counts
    else:
        assert all((c[0] if disparity == 3 else c[1]) > 100 for c in counts), counts
    pipe.close()


def test_images_to_poses_with_lsd_on_device():
    """Every detector on the device (ImagePipeline.detect_images: LSD -> LBD, ORB) against the
    oracle chain (LSD oracle -> LBD oracle, ORB oracle, tracker oracle) on the staircase scene."""
    import torch
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    B, F, KL = 2, 4, 320
    W, H = int(cam.width), int(cam.height)
    ctx = gfpl.Context(cam, cfg)
    pipe = ImagePipeline(ctx, cam, B, KL, lsd=True)
    KP = pipe.kp_cap
    g = gfpl.StereoFrameHandler(ctx, B, KP, KL)
    orc = [O.OracleHandler(cam, cfg, KP, KL) for _ in range(B)]
    dev = torch.device("cuda", 0)
    bad, counts = [], []
    for k in range(F):
        imgs = [synth_stereo_steps(b, k, W, H)[:2] for b in range(B)]
        scenes = [(L, R, O.lsd_detect(L)[0], O.lsd_detect(R)[0]) for L, R in imgs]
        left = torch.from_numpy(np.stack([s[0] for s in scenes])).to(dev)
        right = torch.from_numpy(np.stack([s[1] for s in scenes])).to(dev)
        fr = pipe.detect_images(left, right, torch.full((B,), 0.05 * k, dtype=torch.float64, device=dev))
        hfr, harr = _host_frames(cam, scenes, KP, KL, 0.05 * k)
        pipe.status()
        pipe.synchronize()
        d = [t.cpu().numpy() for t in fr._keep]
        for side in range(2):
            nl_d = d[6 + side]
            assert (nl_d == harr[6 + side]).all(), (k, side, nl_d, harr[6 + side])
            kld = d[8 + side].view(gfpl.KEYLINE_DT).reshape(B, KL)
            ldd = d[10 + side].reshape(B, KL, 32)
            for b in range(B):
                n2 = int(nl_d[b])
                assert kld[b, :n2].tobytes() == harr[8 + side][b, :n2].tobytes(), (k, side, b)
                assert (ldd[b, :n2] == harr[10 + side][b, :n2]).all(), (k, side, b)
        torch.cuda.synchronize()
        if k == 0:
            g.initialize(fr)
            for b, o in enumerate(orc):
                o.initialize(hfr, b)
            continue
        g.frameStep(fr)
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
    assert not bad, "\n".join(bad[:30])
    assert all(c[1] > 5 for c in counts), counts
    pipe.close()


def test_detection_overlapped_with_tracking_parity():
    """The bench's order: the detection of frame k + 1 is enqueued (its own stream, the other
    buffer set) before the tracking step of frame k, with no host synchronisation between
    them — the gfpl_frames ready / consumed events alone order them.  Poses, stereo features
    and matched lists equal the oracle chain's, frame by frame."""
    import torch
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10)
    cam = gfpl.make_camera("vga", cfg)
    B, F, KL = 3, 6, 320
    W, H = int(cam.width), int(cam.height)
    ctx = gfpl.Context(cam, cfg)
    pipe = ImagePipeline(ctx, cam, B, KL)
    KP = pipe.kp_cap
    g = gfpl.StereoFrameHandler(ctx, B, KP, KL)
    orc = [O.OracleHandler(cam, cfg, KP, KL) for _ in range(B)]
    dev = torch.device("cuda", 0)
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    def inputs(k):
        scenes = [synth_stereo_steps(b, k, W, H) for b in range(B)]
        kl = [np.zeros((B, KL), gfpl.KEYLINE_DT) for _ in range(2)]
        n = [np.zeros(B, np.int32) for _ in range(2)]
        for b, sc in enumerate(scenes):
            for side in range(2):
                n[side][b] = len(sc[2 + side])
                kl[side][b, :n[side][b]] = sc[2 + side]
        dev_in = (to(np.stack([x[0] for x in scenes])), to(np.stack([x[1] for x in scenes])),
                  to(kl[0].view(np.uint8).reshape(-1)), to(n[0]), to(kl[1].view(np.uint8).reshape(-1)), to(n[1]),
                  torch.full((B,), 0.05 * k, dtype=torch.float64, device=dev))
        return scenes, dev_in

    sc0, in0 = inputs(0)
    g.initialize(pipe.detect(*in0))
    hfr0, _ = _host_frames(cam, sc0, KP, KL, 0.0)
    for b, o in enumerate(orc):
        o.initialize(hfr0, b)
    scenes, nxt = inputs(1)
    fr_next = pipe.detect(*nxt)
    bad = []
    for k in range(1, F):
        cur, cur_scenes = fr_next, scenes
        if k + 1 < F:
            scenes, nxt = inputs(k + 1)
            fr_next = pipe.detect(*nxt)     # enqueued before the step on frame k
        g.frameStep(cur)
        hfr, _ = _host_frames(cam, cur_scenes, KP, KL, 0.05 * k)
        for b, o in enumerate(orc):
            o.insertStereoPair(hfr, b)
            o.optimizePose()
            tr = o.read_track()
            o.updateFrame()
            gp, op = g.read_frame(gfpl.PREV, b), o.read_frame(gfpl.PREV)
            bad += compare_core(gp, op, f"f{k} s{b} ")
            bad += compare_pose(gp, op, what=f"f{k} s{b} ")[0]
            bad += compare_track(g.read_last_track(b), tr, f"f{k} s{b} ")
    pipe.status()
    assert not bad, "\n".join(bad[:30])
    g.close()
    pipe.close()
