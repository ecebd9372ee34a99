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
from parity import compare_core, compare_pose, compare_prev_matched, compare_track, make_ragged

pytestmark = pytest.mark.gpu


def _run_sequence(cam_name, cfg_over, n_seq, n_frames, kp_cap, kl_cap, synth_over=None, seed=1, mutate=None,
                  dev_hook=None):
    cfg = gfpl.default_config(**cfg_over)
    cam = gfpl.make_camera(cam_name, cfg)
    sp = gfpl.synth_params(seed=seed, **(synth_over or {}))
    H = gfpl.HostFrames(cam, sp, n_seq, n_frames, kp_cap, kl_cap)
    if mutate:
        H = mutate(H)
    D = gfpl.DeviceFrames(H)
    if dev_hook:
        dev_hook(cam, H, D)
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


def _check(rep, need_work=True):
    msgs = rep["core"] + rep["track"] + rep["prev"] + rep["pose"]
    assert not msgs, "\n".join(msgs[:40])
    # real work happened
    if need_work:
        assert all(c[0] > 0 and c[1] > 0 for c in rep["counts"]), rep["counts"]


@pytest.fixture(scope="module")
def vga_default():
    return _run_sequence("vga", {}, n_seq=3, n_frames=5, kp_cap=2048, kl_cap=512)


def test_vga_default_config_parity(vga_default):
    _check(vga_default)


def test_vga_default_pose_bitexact(vga_default):
    # stronger than the 1e-6 bar: same op order -> identical bits
    assert all(vga_default["pose_exact"]), vga_default["pose_exact"]


@pytest.mark.parametrize("wave_max,w8_max", [("0", "0"), ("4096", "0"), ("4096", "4096")])
def test_bench_config_parity(monkeypatch, wave_max, w8_max):
    # harness overrides of SURVEY §8(d): 10 + 10 GN iterations, no early stop; both line-cut searches,
    # the three pose layouts (one wave per sequence; the small-batch 4 and 8 waves per sequence) and both
    # stereo layouts (8 and 16 waves per sequence)
    monkeypatch.setenv("GFPL_CUT_WAVE_MAX_B", wave_max)
    monkeypatch.setenv("GFPL_POSE_MULTI_MAX_B", wave_max)
    monkeypatch.setenv("GFPL_POSE_W8_MAX_B", w8_max)
    monkeypatch.setenv("GFPL_SP_WIDE_MAX_B", wave_max)   # 0: the bench batch's 8-wave stereo kernels, else 16
    rep = _run_sequence("vga", dict(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0),
                        n_seq=2, n_frames=4, kp_cap=2048, kl_cap=512, seed=7)
    _check(rep)


@pytest.mark.parametrize("n_seq", [1, 8])
def test_small_batch_parity(n_seq):
    """The small-batch kernels at the batch sizes they serve by default (B <= 256: the wave line-cut
    search and the 8-wave k_pose), bench config, against the oracle — B = 1 is the reference app's
    one stream per process (app/plslam_mod.cpp:387-411)."""
    rep = _run_sequence("vga", dict(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0),
                        n_seq=n_seq, n_frames=4, kp_cap=2048, kl_cap=512, seed=11)
    _check(rep)


def test_cut_progress_partner_slots():
    """k_cut_search's progress exchange pairs each wave with wave slot ^ 1 of its SIMD (k_cut.hip
    cut_prog_slots).  At B = 16384 (2048 search waves over 1024 SIMDs, two resident per SIMD) every
    wave's HW_ID / XCC_ID (debug slots 6 / 7, measured mode) is read back: each SIMD holding two waves
    must hold them in slots s and s ^ 1.  Input: 64 distinct generated sequences tiled over the batch."""
    B, n_dist, KP, KL = 16384, 64, 2048, 512
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0)
    cam = gfpl.make_camera("vga", cfg)
    ctx = gfpl.Context(cam, cfg)
    h = gfpl.StereoFrameHandler(ctx, B, KP, KL)
    hb = gfpl.HostBatch(cam, gfpl.synth_params(pyr_from_l0=2), n_dist, KP, KL, seq0=0, pinned=True)

    def stage(k):
        hb.fill(k, 8, seq0=0, n=n_dist)
        for s0 in range(0, B, n_dist):
            h.upload_wait(h.upload_async(hb.frames(n_dist), s0, 0, l0_stride=int(cam.pyr_bytes)))
        return h.staged_frames(0)

    h.initialize(stage(0))
    h.frameStep(stage(1))
    d = h.debug_clocks()[::8]   # one row per search wave (8 sequences each)
    hw, xcc = d[:, 6].astype(np.int64), d[:, 7].astype(np.int64)
    simd = ((((xcc & 7) * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 15)) * 4 + ((hw >> 4) & 3)
    slot = hw & 15
    per = {}
    for s_, w_ in zip(simd.tolist(), slot.tolist()):
        per.setdefault(s_, []).append(w_)
    pairs = [v for v in per.values() if len(v) == 2]
    print(f"{len(per)} SIMDs, {len(pairs)} with two waves, slot sets {sorted(set(tuple(sorted(v)) for v in pairs))[:8]}")
    assert len(pairs) > 0.5 * len(per)
    bad = [v for v in pairs if v[0] != (v[1] ^ 1)]
    assert not bad, f"{len(bad)} SIMDs whose two waves are not partner slots, e.g. {bad[:4]}"


@pytest.mark.parametrize("proof,wave_max", [(1, "0"), (1, "4096"), (2, "0"), (3, "0")])
def test_proven_cut_parity(monkeypatch, proof, wave_max):
    """Proven-mode line cut against the oracle: cut_proof 1 — the recorded measured
    search proven after the fact by k_cut_verify (the reference's own endpoint variances at every
    compared ratio, the two running invCov_sums), unproven sequences redone eagerly; 2 — the eager
    proven search for every sequence (v'-tables, exact running sum, per-step bound); 3 — every
    sequence sent through the redo path (the fallback of mode 1).  Both searches record: the
    8-sequence-per-wave one and the small-batch one (GFPL_CUT_WAVE_MAX_B)."""
    monkeypatch.setenv("GFPL_CUT_WAVE_MAX_B", wave_max)
    rep = _run_sequence("vga", dict(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0,
                                    cut_proof=proof),
                        n_seq=3, n_frames=5, kp_cap=2048, kl_cap=512, seed=9)
    _check(rep)


def test_outlier_workload_parity():
    """cfg2o: 10% of the true observations displaced 3-8 px per frame (synth outlier_frac), so
    removeOutliers (src/stereoFrameHandler.cpp:2058-2116) flags more than the MAD tail and the
    stage-2 restart sees a changed list; pyramids resized from level 0 (pyr_from_l0 = 1)."""
    rep = _run_sequence("vga", dict(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0),
                        n_seq=3, n_frames=5, kp_cap=2048, kl_cap=512,
                        synth_over=dict(respawn=16, outlier_frac=0.1, pyr_from_l0=1), seed=17)
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


@pytest.mark.parametrize("nq,nt", [(33, 2), (5, 2049), (1000, 3000), (64, 31)])
def test_knn2_hamming_shapes(nq, nt):
    """gfpl_knn2_hamming (MFMA path) on ragged tile shapes and a train set that spans
    several LDS chunks, with planted ties, against the oracle's BFMatcher restatement."""
    import torch
    rng = np.random.default_rng(nq * 7 + nt)
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    t[nt - 1] = t[0]                 # a tie across the whole train range
    q[nq // 2] = t[nt // 2]          # an exact match
    cfg = gfpl.default_config()
    ctx = gfpl.Context(gfpl.make_camera("vga", cfg), cfg)
    qd, td = torch.from_numpy(q).cuda(), torch.from_numpy(t).cuda()
    for cell in (1, 2):
        idx = torch.zeros((nq, 2), dtype=torch.int32, device="cuda")
        dist = torch.zeros((nq, 2), dtype=torch.float32, device="cuda")
        assert ctx.knn2(qd, nq, td, nt, cell, idx, dist) == 0
        ctx.synchronize()
        rc, oi, od = O.knn2(q, t, cell)
        assert rc == 0
        assert np.array_equal(idx.cpu().numpy(), oi), cell
        assert np.array_equal(dist.cpu().numpy(), od), cell


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


@pytest.mark.parametrize("layout", ["small_batch", "bench_batch"])
def test_ragged_inputs_parity(layout, monkeypatch):
    # empty / one-line / tiny detection sets (ledger U4, U5 guards), through the small-batch kernels
    # (B = 5: 8-wave k_cut_prep / k_pose, the wave search, 16-wave stereo) and through the ones the
    # bench batch runs (every small-batch threshold forced to 0)
    if layout == "bench_batch":
        for v in ("GFPL_CUT_WAVE_MAX_B", "GFPL_CUT_PREP_W8_MAX_B", "GFPL_POSE_MULTI_MAX_B", "GFPL_POSE_W8_MAX_B",
                  "GFPL_SP_WIDE_MAX_B"):
            monkeypatch.setenv(v, "0")
    rep = _run_sequence("vga", {}, n_seq=5, n_frames=3, kp_cap=1024, kl_cap=256,
                        synth_over=dict(n_kp=600, n_kl=150, n_world_pts=800, n_world_lines=200), seed=13,
                        mutate=make_ragged)
    _check(rep, need_work=False)


def test_stage_entry_points_from_oracle_state():
    """Each stage entry point on its own, started from the oracle's state
    written through gfpl_write_frame (as the reference's simulators build
    frames through public members, src/simulate_line_cut.cpp:62-212)."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(seed=17)
    KP, KL = 2048, 512
    H = gfpl.HostFrames(cam, sp, 1, 3, KP, KL)
    D = gfpl.DeviceFrames(H)
    o = O.OracleHandler(cam, cfg, KP, KL)
    o.initialize(H.frames(0), 0)
    o.insertStereoPair(H.frames(1), 0)
    o.optimizePose()
    o.updateFrame()
    ctx = gfpl.Context(cam, cfg)
    g = gfpl.StereoFrameHandler(ctx, 1, KP, KL)
    g.write_frame(gfpl.PREV, 0, o.read_frame(gfpl.PREV))
    o.begin_frame(H.frames(2), 0)
    bad = []
    g.stereoPoints(D.frames(2)); o.stereoPoints()
    g.stereoLines(D.frames(2)); o.stereoLines()
    bad += compare_core(g.read_frame(gfpl.CURR, 0), o.read_frame(gfpl.CURR), "stereo ")
    g.estimateStereoUncertainty(); o.estimateStereoUncertainty()
    g.crossFrameMatchingPoints(); o.crossFrameMatchingPoints()
    g.crossFrameMatchingLines(); o.crossFrameMatchingLines()
    tg, to = g.read_track(0), o.read_track()
    bad += compare_track(tg, to, "cross ")
    g.estimateProjUncertainty_submodular(); o.estimateProjUncertainty_submodular()
    bad += compare_prev_matched(g.read_frame(gfpl.PREV, 0), o.read_frame(gfpl.PREV), to, "cut ")
    g.optimizePose(); o.optimizePose()
    pb, exact = compare_pose(g.read_frame(gfpl.CURR, 0), o.read_frame(gfpl.CURR), what="pose ")
    bad += pb
    assert not bad, "\n".join(bad[:30])
    assert exact
    assert len(to["matched_pt"]) > 100 and len(to["matched_ls"]) > 50


def test_pose_only_noise_free_parity():
    """optimizePose alone on a written noise-free problem (all residuals ~0:
    the MAD outlier pass is degenerate — a decision-heavy case)."""
    from test_oracle_known_answers import _noise_free_problem
    for it, mine in ((5, 1e-7), (10, 0.0)):
        cfg = gfpl.default_config(max_iters=it, max_iters_ref=it, min_error=mine, min_error_change=mine)
        cam = gfpl.make_camera("vga", cfg)
        prev, curr, tr = _noise_free_problem(O.expmap_se3(np.array([0.02, -0.01, 0.025, 0.01, -0.02, 0.015])),
                                             cfg, cam)
        o = O.OracleHandler(cam, cfg, 256, 64)
        o.write_frame(gfpl.PREV, prev); o.write_frame(gfpl.CURR, curr); o.write_track(tr)
        ctx = gfpl.Context(cam, cfg)
        g = gfpl.StereoFrameHandler(ctx, 1, 256, 64)
        g.write_frame(gfpl.PREV, 0, prev); g.write_frame(gfpl.CURR, 0, curr); g.write_track(0, tr)
        o.optimizePose(); g.optimizePose()
        bad, exact = compare_pose(g.read_frame(gfpl.CURR, 0), o.read_frame(gfpl.CURR))
        assert not bad and exact, bad
        assert compare_track(g.read_track(0), o.read_track()) == []


def test_stress_config_parity():
    """BASELINE configs[4]: 1920x1080 stereo, 8000 ORB + 2000 LBD per side, line cut on."""
    rep = _run_sequence("stress", {}, n_seq=3, n_frames=8, kp_cap=8192, kl_cap=2048,
                        synth_over=dict(n_kp=8000, n_kl=2000, n_world_pts=10400, n_world_lines=2800,
                                        z_max=12.0), seed=19)
    _check(rep)
    assert rep["counts"][0][0] > 3000 and rep["counts"][0][1] > 500, rep["counts"]


def test_cross_points_nan_and_far_projections():
    """Cross-frame point matching on hostile state (written through gfpl_write_frame):
    NaN / infinite / far projections of previous points and NaN / far current
    observations.  The reference's `norm() > 10` gate lets NaN through
    (src/stereoFrameHandler.cpp:536); the GPU grid must keep exactly that."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    KP, KL = 2048, 512
    H = gfpl.HostFrames(cam, gfpl.synth_params(seed=23), 1, 3, KP, KL)
    o = O.OracleHandler(cam, cfg, KP, KL)
    o.initialize(H.frames(0), 0)
    o.insertStereoPair(H.frames(1), 0)
    o.optimizePose()
    o.updateFrame()
    o.begin_frame(H.frames(2), 0)
    o.stereoPoints(); o.stereoLines(); o.estimateStereoUncertainty()
    prev, curr = o.read_frame(gfpl.PREV), o.read_frame(gfpl.CURR)
    P = prev.get("pt_P")
    pl = curr.get("pt_pl")
    assert len(P) > 40 and len(pl) > 40
    P[5] = np.nan                     # NaN projection -> passes the gate in the reference
    P[7] = (0.0, 0.0, 0.0)            # 0/0 -> NaN
    P[9] = (1e12, 0.0, 1.0)           # far off-image
    P[11] = (np.inf, 0.0, 1.0)
    P[13] = (-3.0, 1.0, -2.0)         # behind the camera, finite projection
    pl[3] = np.nan                    # NaN observation -> every prev point passes the gate
    pl[4] = (1e7, 1e7)
    pl[6] = (-1e9, 5.0)
    ctx = gfpl.Context(cam, cfg)
    g = gfpl.StereoFrameHandler(ctx, 1, KP, KL)
    for w, f in ((gfpl.PREV, prev), (gfpl.CURR, curr)):
        o.write_frame(w, f)
        g.write_frame(w, 0, f)
    g.crossFrameMatchingPoints(); o.crossFrameMatchingPoints()
    tg, to = g.read_track(0), o.read_track()
    bad = compare_track(tg, to, "cross ")
    bad += compare_prev_matched(g.read_frame(gfpl.PREV, 0), o.read_frame(gfpl.PREV), to, "cross ")
    bad += compare_core(g.read_frame(gfpl.CURR, 0), o.read_frame(gfpl.CURR), "cross curr ")
    assert not bad, "\n".join(bad[:30])
    assert len(to["matched_pt"]) > 100


def test_optimize_pose_explicit_initial_guess():
    """optimizePose(Matrix4d DT_ini) with a guess other than prev_frame->DT (per sequence)."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    KP, KL = 2048, 512
    H = gfpl.HostFrames(cam, gfpl.synth_params(seed=29), 2, 3, KP, KL)
    D = gfpl.DeviceFrames(H)
    ctx = gfpl.Context(cam, cfg)
    g = gfpl.StereoFrameHandler(ctx, 2, KP, KL)
    orc = [O.OracleHandler(cam, cfg, KP, KL) for _ in range(2)]
    g.initialize(D.frames(0))
    for b, o in enumerate(orc):
        o.initialize(H.frames(0), b)
    guesses = np.stack([np.eye(4), O.expmap_se3(np.array([0.01, 0.0, -0.02, 0.0, 0.01, 0.0]))])
    for k in (1, 2):
        g.insertStereoPair(D.frames(k))
        g.optimizePose(guesses)
        for b, o in enumerate(orc):
            o.insertStereoPair(H.frames(k), b)
            o.optimizePose(guesses[b])
            bad, exact = compare_pose(g.read_frame(gfpl.CURR, b), o.read_frame(gfpl.CURR), what=f"f{k} s{b} ")
            assert not bad and exact, bad
            assert compare_track(g.read_track(b), o.read_track()) == []
        g.updateFrame()
        for o in orc:
            o.updateFrame()


@pytest.mark.parametrize("seq", gfpl.EUROC_SEQS)
def test_euroc_ground_truth_trajectory_parity(seq):
    """BASELINE configs[3]: the EuRoC rig on each of the eight ground-truth trajectories
    (config/asl/gt-ass/{mh_01..mh_05, v1_01..v1_03}), bench cfg4's scene (re-spawned
    landmarks), 10+10 GN iterations."""
    T, t = gfpl.euroc_traj(seq, 6)
    rep = _run_sequence("euroc", dict(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0),
                        n_seq=2, n_frames=6, kp_cap=2048, kl_cap=512,
                        synth_over=dict(z_min=2.0, z_max=12.0, respawn=16, traj=T.ctypes.data, n_traj=len(t),
                                        traj_t=t.ctypes.data), seed=31 + gfpl.EUROC_SEQS.index(seq))
    _check(rep)
    assert all(rep["pose_exact"])


@pytest.mark.parametrize("wl", ["cfg2", "cfg3"])
def test_bench_workload_parity(wl):
    """The bench's own scenes (stationary, landmarks re-spawned: bench.WORKLOADS) over
    frames 0..7, so re-spawned landmarks enter and leave the matched sets."""
    import bench
    cam_name, over, _ = bench.WORKLOADS[wl]
    rep = _run_sequence(cam_name, dict(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0),
                        n_seq=2, n_frames=8, kp_cap=2048, kl_cap=512, synth_over=over, seed=41)
    _check(rep)
    assert all(rep["pose_exact"])


@pytest.mark.parametrize("level0", [False, True])
def test_async_double_buffered_upload_parity(level0):
    """gfpl_upload_frames_async: frames uploaded chunk by chunk from host memory into the two
    staging buffers on the copy stream, frame k + 1 copied while the step on frame k runs
    (the staging events order them); poses and matched lists equal the oracle's.  level0:
    gfpl_upload_frames_l0_async copies only level 0 of each right pyramid (the host frames
    hold level 0 alone, pyr_from_l0 = 2) and the device builds levels 1.. — byte-equal to the
    host's ComputePyramid restatement (pyr_from_l0 = 1), which the oracle tracks on."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    B, F, KP, KL = 5, 5, 2048, 512
    H = gfpl.HostFrames(cam, gfpl.synth_params(seed=43, respawn=16, pyr_from_l0=1 if level0 else 0), B, F, KP, KL)
    Hup = gfpl.HostFrames(cam, gfpl.synth_params(seed=43, respawn=16, pyr_from_l0=2), B, F, KP, KL) if level0 else H
    g = gfpl.StereoFrameHandler(gfpl.Context(cam, cfg), B, KP, KL)
    orc = [O.OracleHandler(cam, cfg, KP, KL) for _ in range(B)]

    def upload(k, slot):
        # two chunks of 3 + 2 sequences
        ts = [g.upload_async(gfpl.make_frames(n, KP, KL, [a[k, s0:s0 + n] for a in Hup.arrays()]), s0, slot,
                             l0_stride=int(cam.pyr_bytes) if level0 else 0)
              for s0, n in ((0, 3), (3, 2))]
        return ts[-1]

    g.upload_wait(upload(0, 0))
    if level0:   # the device-built pyramids are the host restatement's, byte for byte
        import torch
        st = g.staged_frames(0)
        pb = int(cam.pyr_bytes)
        used = int(cam.lvl_offset[int(cam.n_levels) - 1]) + int(cam.lvl_cols[int(cam.n_levels) - 1]) * \
            int(cam.lvl_rows[int(cam.n_levels) - 1])
        buf = np.zeros(B * pb, np.uint8)
        torch.cuda.synchronize()
        assert gfpl.hiplib().gfpl_copy_to_host(g.ctx.h, buf.ctypes.data, st.pyr_r, B * pb) == 0
        got = buf.reshape(B, pb)[:, :used]
        assert (got == H.pyr_r[0][:, :used]).all()
    g.initialize(g.staged_frames(0))
    upload(1, 1)
    for k in range(1, F):
        if k + 1 < F:
            upload(k + 1, (k + 1) % 2)   # waits (on the GPU) for the step that last read that buffer
        g.frameStep(g.staged_frames(k % 2))
        for b, o in enumerate(orc):
            if k == 1:
                o.initialize(H.frames(0), b)
            o.insertStereoPair(H.frames(k), b)
            o.optimizePose()
            tr = o.read_track()
            o.updateFrame()
            gp, op = g.read_frame(gfpl.PREV, b), o.read_frame(gfpl.PREV)
            bad = compare_core(gp, op, f"f{k} s{b} ") + compare_track(g.read_last_track(b), tr, f"f{k} s{b} ")
            pb, exact = compare_pose(gp, op, what=f"f{k} s{b} ")
            assert not bad and not pb and exact, (bad + pb)[:10]


# ---- certified line-cut search: the chosen ratios are the reference's
@pytest.mark.parametrize("margin", [0.0, 1e-3])
def test_line_cut_exact_and_mixed_steps_parity(margin):
    # 0: every step evaluated with the reference's LLT; 1e-3: a large share of the
    # steps fall back to it, mixed with certified steps inside the same lines
    rep = _run_sequence("vga", dict(cut_certify=margin, max_iters=10, max_iters_ref=10, min_error=0.0,
                                    min_error_change=0.0), n_seq=2, n_frames=3, kp_cap=2048, kl_cap=512, seed=11)
    _check(rep)


def test_cut_certify_margin_validated():
    cam = gfpl.make_camera("vga", gfpl.default_config())
    for bad in (1e-12, -1.0, 1.0):
        with pytest.raises(gfpl.GfplError):
            gfpl.Context(cam, gfpl.default_config(cut_certify=bad))


@pytest.mark.parametrize("wave_max", ["0", "4096"])
def test_line_cut_certified_matches_exact_at_scale(monkeypatch, wave_max):
    """512 sequences x 3 frames on the GPU three times — the margined search in measured mode,
    in proven mode (gfpl_config.cut_proof: a margined decision only under the proven per-step
    agreement bound) and exact steps only — cut ratios, invCovPose of every
    matched line and the poses bit-identical; proven mode certifies most steps."""
    monkeypatch.setenv("GFPL_CUT_WAVE_MAX_B", wave_max)   # 0: the 8-sequence-per-wave search, else one per wave
    monkeypatch.setenv("GFPL_POSE_MULTI_MAX_B", wave_max)  # 0: one wave per sequence in k_pose, else four
    monkeypatch.setenv("GFPL_POSE_W8_MAX_B", "0")         # (eight: test_bench_config_parity)
    n, F, KP, KL = 512, 3, 2048, 512
    base = dict(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0)
    cam = gfpl.make_camera("vga", gfpl.default_config(**base))
    H = gfpl.HostFrames(cam, gfpl.synth_params(seed=21), n, F, KP, KL)
    D = gfpl.DeviceFrames(H)
    out = []
    proven = {"steps": 0, "exact_steps": 0, "lines_unbounded": 0}
    verified = {"redone": 0, "steps_proven": 0, "vref_evals": 0, "lines": 0}
    for margin, proof in ((1e-9, 0), (1e-9, 2), (1e-9, 1), (0.0, 0)):
        ctx = gfpl.Context(cam, gfpl.default_config(cut_certify=margin, cut_proof=proof, **base))
        h = gfpl.StereoFrameHandler(ctx, n, KP, KL)
        h.initialize(D.frames(0))
        res = []
        for k in range(1, F):
            h.insertStereoPair(D.frames(k))
            if proof == 2:
                tc = h.last_step_track_counts()
                for key in proven:
                    proven[key] += tc[key]
            if proof == 1:
                vc = h.last_step_cut_proof()
                for key in verified:
                    verified[key] += vc[key]
            h.optimizePose()
            for b in range(n):
                tr = h.read_track(b)
                pf = h.read_frame(gfpl.PREV, b)
                ml = tr["matched_ls"]
                res.append((ml.copy(), pf.get("ls_cut")[ml].copy(), pf.get("ls_invcov")[ml].copy(),
                            h.read_frame(gfpl.CURR, b).get("Tfw")))
            h.updateFrame()
        out.append(res)
    for other in (out[1], out[2], out[3]):
        n_lines = 0
        for (ma, ca, ia, ta), (mb, cb, ib, tb) in zip(out[0], other):
            assert np.array_equal(ma, mb)
            assert np.array_equal(ca.view(np.uint64), cb.view(np.uint64))
            assert np.array_equal(ia.view(np.uint64), ib.view(np.uint64))
            assert np.array_equal(ta.view(np.uint64), tb.view(np.uint64))
            n_lines += len(ma)
        assert n_lines > 100 * n
    print("eager proven mode:", proven, "verified proven mode:", verified)
    assert proven["steps"] > 0 and proven["exact_steps"] < 0.05 * proven["steps"], proven
    # the recorded search is proven for (nearly) every sequence: a redo is the exception
    assert verified["steps_proven"] > 0.9 * proven["steps"] and verified["redone"] <= 0.01 * n * (F - 1), verified


# ---- keyframe decision: needNewKF / currFrameIsKF
def test_need_new_kf_and_curr_frame_is_kf_parity():
    """3 sequences x 8 frames with the app's order (insert, optimizePose, needNewKF,
    currFrameIsKF when needed, updateFrame; app/plslam_mod.cpp:387-477): decisions,
    entropy ratios, accumulated covariances and the curr frame after a keyframe are
    bit-identical to the oracle.  maxKFNumFrames = 3 and minEntropyRatio = 0.97 make
    both gates fire."""
    n, F = 3, 8
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, max_kf_num_frames=3, min_entropy_ratio=0.97)
    cam = gfpl.make_camera("vga", cfg)
    H = gfpl.HostFrames(cam, gfpl.synth_params(seed=17), n, F, 2048, 512)
    D = gfpl.DeviceFrames(H)
    g = gfpl.StereoFrameHandler(gfpl.Context(cam, cfg), n, 2048, 512)
    orc = [O.OracleHandler(cam, cfg, 2048, 512) for _ in range(n)]
    g.initialize(D.frames(0))
    for b, o in enumerate(orc):
        o.initialize(H.frames(0), b)
    n_kf = 0
    for k in range(1, F):
        g.insertStereoPair(D.frames(k))
        g.optimizePose()
        flags = g.needNewKF()
        for b, o in enumerate(orc):
            o.insertStereoPair(H.frames(k), b)
            o.optimizePose()
            fo = o.needNewKF()
            sg, so = g.read_kf_state(b), o.read_kf_state()
            assert bool(flags[b]) == fo, (k, b, sg, so)
            for key in ("entropy_first_prevKF", "entropy_ratio"):
                assert np.float64(sg[key]).view(np.uint64) == np.float64(so[key]).view(np.uint64), (k, b, key)
            assert np.array_equal(sg["cov_prevKF_currF"].view(np.uint64), so["cov_prevKF_currF"].view(np.uint64))
            assert sg["num_frame_since_kf"] == so["num_frame_since_kf"]
            if fo:
                o.currFrameIsKF()
        g.currFrameIsKF(flags)
        n_kf += int(flags.sum())
        for b, o in enumerate(orc):
            report = compare_core(g.read_frame(gfpl.CURR, b), o.read_frame(gfpl.CURR), f"f{k} s{b} kf ")
            assert not report, report[:10]
            assert compare_pose(g.read_frame(gfpl.CURR, b), o.read_frame(gfpl.CURR))[1]
            sg, so = g.read_kf_state(b), o.read_kf_state()
            assert (sg["prev_f_iskf"], sg["num_frame_since_kf"]) == (so["prev_f_iskf"], so["num_frame_since_kf"])
        g.updateFrame()
        for o in orc:
            o.updateFrame()
    assert n_kf >= n


def _odd_octaves(H):
    """~3% of the left and right keypoints of every tracked frame get octaves outside
    the pyramid (negative, >= n_levels, beyond int8): the stereo band scan's
    out-of-range segment and the int8 / HBM octave fallback."""
    rng = np.random.default_rng(5)
    for f in range(1, H.F):
        for b in range(H.B):
            for arr, n in ((H.kp_r, int(H.n_kp_r[f, b])), (H.kp_l, int(H.n_kp_l[f, b]))):
                idx = rng.choice(n, max(1, n // 30), replace=False)
                arr["octave"][f, b, idx] = rng.choice([-1, 4, 5, 7, 200, -128, -100000], len(idx))
    return H


@pytest.mark.parametrize("kp_cap", [2048, 4096])
def test_out_of_range_octaves_parity(kp_cap):
    # 2048: the per-octave segmented band scan; 4096: the single sorted list (1024 threads)
    rep = _run_sequence("vga", {}, n_seq=3, n_frames=3, kp_cap=kp_cap, kl_cap=256,
                        synth_over=dict(n_kp=900, n_kl=150, n_world_pts=1200, n_world_lines=200), seed=17,
                        mutate=_odd_octaves)
    _check(rep)


def test_line_cut_ill_conditioned_s_parity():
    """Near-singular S in the certified cut search: budgets of 2 points and 4-6 lines
    leave S = invCov_sum - info_m(0,0) built from a handful of rank-1 / rank-2 terms,
    so its LLT pivots collapse; such lines must fall back to the reference's exact
    steps (GFPL_CUT_MIN_PIVOT, k_cut.hip) and the ratios / poses equal the oracle."""
    for pts, lns in ((2, 4), (3, 6), (0 + 1, 5)):
        rep = _run_sequence("vga", dict(cut_certify=1e-9, max_point_match_num=pts, max_line_match_num=lns,
                                        max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0),
                            n_seq=6, n_frames=3, kp_cap=1024, kl_cap=256,
                            synth_over=dict(n_kp=700, n_kl=160, n_world_pts=900, n_world_lines=220), seed=37 + lns)
        _check(rep)


def test_pose_long_match_lists_parity():
    """Matched lists above 512 entries (the gazebo budget maxPointMatchNum = 1000,
    src/config.cpp:89; 600 lines) take k_pose's sorted-MAD path (residuals in LDS),
    lists of up to 512 the register selection (wave_select) — both must give the oracle's
    std::sort medians, hence the same outlier flags and poses."""
    rep = _run_sequence("vga", dict(max_point_match_num=1000, max_line_match_num=600),
                        n_seq=2, n_frames=4, kp_cap=2048, kl_cap=1024,
                        synth_over=dict(n_kp=2000, n_kl=1000, n_world_pts=2600, n_world_lines=1300), seed=43)
    _check(rep)
    assert max(c[2] for c in rep["counts"]) > 512 and max(c[3] for c in rep["counts"]) > 512, rep["counts"]


def test_match_budget_raise_after_seqbatch_refused():
    """A seqbatch sizes matched_pt / matched_ls and the cut / pose scratch from the
    config's budgets at creation: a larger budget while it lives is refused
    (GFPL_E_CAPACITY), a smaller one is accepted, and after the seqbatch is gone the
    larger one is accepted again; the context refuses destruction while it lives."""
    L = gfpl.hiplib()
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    ctx = gfpl.Context(cam, cfg)
    h = gfpl.StereoFrameHandler(ctx, 2, 512, 128)
    raised = gfpl.default_config(max_point_match_num=1000)   # the gazebo value, src/config.cpp:89
    assert L.gfpl_set_config(ctx.h, C.byref(raised)) == -5
    raised = gfpl.default_config(max_line_match_num=301)
    assert L.gfpl_set_config(ctx.h, C.byref(raised)) == -5
    lower = gfpl.default_config(max_point_match_num=100, max_line_match_num=50)
    assert L.gfpl_set_config(ctx.h, C.byref(lower)) == 0
    assert L.gfpl_destroy(ctx.h) == -6
    h.close()
    raised = gfpl.default_config(max_point_match_num=1000)
    assert L.gfpl_set_config(ctx.h, C.byref(raised)) == 0
