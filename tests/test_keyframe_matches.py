"""Keyframe consumer: MapHandler::lookForCommonMatches keyframe-pair stage
(src/mapHandler.cpp:199-470) — gfpl_kf_common_matches (GPU, C ABI) against the
oracle restatement, and the oracle against constructed known answers.

Bar: the accepted (kf0 row, kf1 row) pairs and their order are integer results,
compared exactly.
"""
import numpy as np
import pytest

import gfpl
import oracle as O


def _proj(cam, P):
    return np.array([cam.cx + (cam.fx * P[0]) / P[2], cam.cy + (cam.fy * P[1]) / P[2]])


def _pose(rx, ry, rz, t):
    cx, sx, cy, sy, cz, sz = np.cos(rx), np.sin(rx), np.cos(ry), np.sin(ry), np.cos(rz), np.sin(rz)
    R = (np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]]) @ np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
         @ np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]]))
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, t
    return T


def _inv(T):
    o = np.eye(4)
    o[:3, :3] = T[:3, :3].T
    o[:3, 3] = -T[:3, :3].T @ T[:3, 3]
    return o


def known_pair(cam, n_pt=300, n_ls=120, seed=3, bad_frac=0.1, flips=8, same_pose_lines=True):
    """Two keyframes whose true correspondences, gate failures and expected
    accepted pairs are known by construction."""
    rng = np.random.default_rng(seed)
    kp, kl = max(n_pt, 2), max(n_ls, 2)
    f0, f1 = gfpl.FrameHost(kp, kl), gfpl.FrameHost(kp, kl)
    f0.s.n_pt = f1.s.n_pt = n_pt
    f0.s.n_ls = f1.s.n_ls = n_ls
    T0 = _pose(0.01, -0.02, 0.015, [0.1, -0.05, 0.2])
    T1 = T0.copy() if same_pose_lines else _pose(0.02, 0.01, -0.01, [0.3, 0.0, 0.25])
    if not same_pose_lines:
        pass
    DT = _inv(T1) @ T0

    def flipped(d):
        d = d.copy()
        for b in rng.choice(256, flips, replace=False):
            d[b // 8] ^= np.uint8(1 << (b % 8))
        return d

    exp_pt = []
    perm = rng.permutation(n_pt)
    for i in range(n_pt):
        d = rng.integers(0, 256, 32, dtype=np.uint8)
        P = np.array([rng.uniform(-2, 2), rng.uniform(-1.5, 1.5), rng.uniform(2, 8)])
        f0.arr["pdesc"][i] = d
        f0.arr["pt_P"][i] = P
        f0.arr["pt_sigma2"][i] = 1.0 / 1.44 ** rng.integers(1, 4)
        j = perm[i]
        f1.arr["pdesc"][j] = flipped(d)
        Pc = DT[:3, :3] @ P + DT[:3, 3]
        off = 0.0 if rng.random() > bad_frac else 12.0
        f1.arr["pt_pl"][j] = _proj(cam, Pc) + np.array([off, -0.3 * off])
        if off == 0.0:
            exp_pt.append((i, j))
    exp_ls = []
    perm = rng.permutation(n_ls)
    for i in range(n_ls):
        d = rng.integers(0, 256, 32, dtype=np.uint8)
        sP = np.array([rng.uniform(-2, 2), rng.uniform(-1.5, 1.5), rng.uniform(2, 8)])
        eP = sP + rng.uniform(-0.8, 0.8, 3)
        eP[2] = max(eP[2], 1.5)
        su, eu = _proj(cam, DT[:3, :3] @ sP + DT[:3, 3]), _proj(cam, DT[:3, :3] @ eP + DT[:3, 3])
        le = np.cross([su[0], su[1], 1.0], [eu[0], eu[1], 1.0])
        le = le / np.hypot(le[0], le[1])
        bad = rng.random() < bad_frac
        if bad:
            le[2] += 6.0
        f0.arr["ldesc"][i] = d
        f0.arr["ls_sP"][i], f0.arr["ls_eP"][i], f0.arr["ls_le"][i] = sP, eP, le
        f0.arr["ls_sigma2"][i] = 1.0
        j = perm[i]
        f1.arr["ldesc"][j] = flipped(d)
        if not bad:
            exp_ls.append((i, j))
    return f0, T0, f1, T1, np.array(exp_pt, np.int32).reshape(-1, 2), np.array(exp_ls, np.int32).reshape(-1, 2)


def test_oracle_known_answer():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    f0, T0, f1, T1, ep, el = known_pair(cam)
    pp, lp = O.kf_common_matches(cam, cfg, gfpl.KeyFrameView(f0, T0), gfpl.KeyFrameView(f1, T1))
    assert len(ep) > 200 and len(el) > 80
    np.testing.assert_array_equal(pp, ep)
    np.testing.assert_array_equal(lp, el)


def test_oracle_ratio_and_mutual_rejections():
    """Duplicate kf1 descriptors: d0 == d1 gives ratio 1 > maxRatio12P (points) and
    d1 - d0 = 0 below the MAD threshold (lines); those pairs are dropped (and the
    features whose true partner row was overwritten lose their match)."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    f0, T0, f1, T1, ep, el = known_pair(cam, n_pt=64, n_ls=64, bad_frac=0.0, seed=5)
    q, t = ep[7]
    f1.arr["pdesc"][(t + 1) % 64] = f1.arr["pdesc"][t]
    ql, tl = el[9]
    f1.arr["ldesc"][(tl + 1) % 64] = f1.arr["ldesc"][tl]
    pp, lp = O.kf_common_matches(cam, cfg, gfpl.KeyFrameView(f0, T0), gfpl.KeyFrameView(f1, T1))
    for got, exp, pair in ((pp, ep, (q, t)), (lp, el, (ql, tl))):
        g = set(map(tuple, got.tolist()))
        assert pair not in g and g <= set(map(tuple, exp.tolist())) and len(g) == len(exp) - 2


def test_oracle_too_few_rows():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    f0, T0, f1, T1, _, el = known_pair(cam, n_pt=1, n_ls=5)
    pp, lp = O.kf_common_matches(cam, cfg, gfpl.KeyFrameView(f0, T0), gfpl.KeyFrameView(f1, T1))
    assert len(pp) == 0
    np.testing.assert_array_equal(lp, el)


def _tracked_keyframes(cam_name="vga", frames=(1, 4), seed=11):
    """Two keyframes of one oracle-tracked synthetic sequence (their Tfw as T_kf_w)."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera(cam_name, cfg)
    sp = gfpl.synth_params(seed=seed)
    n = max(frames) + 1
    H = gfpl.HostFrames(cam, sp, 1, n, 2048, 512)
    o = O.OracleHandler(cam, cfg, 2048, 512)
    o.initialize(H.frames(0), 0)
    out = {}
    for k in range(1, n):
        o.insertStereoPair(H.frames(k), 0)
        o.optimizePose()
        o.updateFrame()
        if k in frames:
            fh = o.read_frame(gfpl.PREV)
            out[k] = (fh, fh.get("Tfw"))
    (a, ta), (b, tb) = out[frames[0]], out[frames[1]]
    return cam, cfg, a, ta, b, tb


@pytest.mark.gpu
def test_gpu_kf_common_matches_known_answer():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    ctx = gfpl.Context(cam, cfg)
    for seed, n_pt, n_ls in [(3, 300, 120), (4, 3000, 1500), (6, 70, 2)]:
        f0, T0, f1, T1, ep, el = known_pair(cam, n_pt=n_pt, n_ls=n_ls, seed=seed)
        gp, gl = ctx.lookForCommonMatches(gfpl.KeyFrameView(f0, T0, "cuda"), gfpl.KeyFrameView(f1, T1, "cuda"))
        op, ol = O.kf_common_matches(cam, cfg, gfpl.KeyFrameView(f0, T0), gfpl.KeyFrameView(f1, T1))
        np.testing.assert_array_equal(gp, op)
        np.testing.assert_array_equal(gl, ol)
        np.testing.assert_array_equal(gp, ep)
        np.testing.assert_array_equal(gl, el)


@pytest.mark.gpu
@pytest.mark.parametrize("cam_name", ["vga", "kitti"])
def test_gpu_kf_common_matches_tracked_keyframes(cam_name):
    cam, cfg, a, ta, b, tb = _tracked_keyframes(cam_name)
    ctx = gfpl.Context(cam, cfg)
    gp, gl = ctx.lookForCommonMatches(gfpl.KeyFrameView(a, ta, "cuda"), gfpl.KeyFrameView(b, tb, "cuda"))
    op, ol = O.kf_common_matches(cam, cfg, gfpl.KeyFrameView(a, ta), gfpl.KeyFrameView(b, tb))
    assert len(op) > 50 and len(ol) > 10, (len(op), len(ol))
    np.testing.assert_array_equal(gp, op)
    np.testing.assert_array_equal(gl, ol)


@pytest.mark.gpu
def test_gpu_kf_common_matches_too_few_rows():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    ctx = gfpl.Context(cam, cfg)
    f0, T0, f1, T1, _, _ = known_pair(cam, n_pt=1, n_ls=0)
    gp, gl = ctx.lookForCommonMatches(gfpl.KeyFrameView(f0, T0, "cuda"), gfpl.KeyFrameView(f1, T1, "cuda"))
    assert len(gp) == 0 and len(gl) == 0


# ----------------------------------------------------------- local-map stage --
def known_local_map(cam, n_pt=200, n_ls=80, seed=21, flips=8):
    """A local map seen from kf1 (T_kf_w = T1) and kf1's unmatched features, with
    the expected (map row, kf1 row) pairs of src/mapHandler.cpp:472-772 by
    construction: some map rows project outside the image (filtered out), some
    kf1 observations are offset beyond maxKFEpipP / maxKFEpipL, and one line has a
    large NEGATIVE residual, which the reference's signed test accepts."""
    rng = np.random.default_rng(seed)
    T1 = _pose(0.02, -0.01, 0.03, [0.4, -0.1, 0.3])
    Twf = _inv(T1)
    Tfw = T1   # world point = T1 @ camera point

    def world(pc):
        return Tfw[:3, :3] @ pc + Tfw[:3, 3]

    def flipped(d):
        d = d.copy()
        for b in rng.choice(256, flips, replace=False):
            d[b // 8] ^= np.uint8(1 << (b % 8))
        return d

    def in_view(pc):
        u = _proj(cam, pc)
        return 0 < u[0] < cam.width and 0 < u[1] < cam.height and pc[2] > 0

    f1 = gfpl.FrameHost(max(n_pt, 2), max(n_ls, 2))
    f1.s.n_pt, f1.s.n_ls = n_pt, n_ls
    pdesc, P, exp_pt = [], [], []
    perm = rng.permutation(n_pt)
    for i in range(n_pt):
        out = rng.random() < 0.1
        pc = np.array([rng.uniform(-2, 2), rng.uniform(-1.5, 1.5), rng.uniform(2, 8)])
        if out:
            pc[0] = pc[2] * 3.0   # far right of the image
        d = rng.integers(0, 256, 32, dtype=np.uint8)
        pdesc.append(d)
        P.append(world(pc))
        j = perm[i]
        f1.arr["pdesc"][j] = flipped(d)
        off = 0.3 if rng.random() > 0.15 else 4.0
        f1.arr["pt_pl"][j] = _proj(cam, pc) + np.array([off, 0.0]) if not out else np.array([10.0, 10.0])
        if in_view(pc) and off < 1.0:
            exp_pt.append((i, j))
    ldesc, L, exp_ls = [], [], []
    perm = rng.permutation(n_ls)
    for i in range(n_ls):
        out = rng.random() < 0.1
        sc = np.array([rng.uniform(-1.5, 1.5), rng.uniform(-1, 1), rng.uniform(2, 8)])
        ec = sc + np.array(rng.uniform(-0.5, 0.5, 3))
        ec[2] = max(ec[2], 1.5)
        if out:
            ec[0] = ec[2] * 3.0
        d = rng.integers(0, 256, 32, dtype=np.uint8)
        ldesc.append(d)
        L.append(np.concatenate([world(sc), world(ec)]))
        su, eu = _proj(cam, sc), _proj(cam, ec)
        le = np.cross([su[0], su[1], 1.0], [eu[0], eu[1], 1.0])
        le = le / np.hypot(le[0], le[1])
        kind = rng.random()
        if kind < 0.1:
            le[2] += 5.0     # residuals +5: rejected
        elif kind < 0.15:
            le[2] -= 5.0     # residuals -5: accepted by the signed test
        j = perm[i]
        f1.arr["ldesc"][j] = flipped(d)
        f1.arr["ls_le"][j] = le
        if in_view(sc) and in_view(ec) and not (kind < 0.1):
            exp_ls.append((i, j))
    m_args = (np.array(pdesc), np.array(P), np.array(ldesc), np.array(L))
    return m_args, f1, T1, np.array(exp_pt, np.int32).reshape(-1, 2), np.array(exp_ls, np.int32).reshape(-1, 2)


def test_oracle_local_map_known_answer():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    m_args, f1, T1, ep, el = known_local_map(cam)
    pp, lp = O.kf_local_map_matches(cam, cfg, gfpl.MapView(*m_args), gfpl.KeyFrameView(f1, T1))
    assert len(ep) > 100 and len(el) > 40
    np.testing.assert_array_equal(pp, ep)
    np.testing.assert_array_equal(lp, el)


@pytest.mark.gpu
def test_gpu_kf_local_map_matches():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    ctx = gfpl.Context(cam, cfg)
    for seed, n_pt, n_ls, ep_p, ep_l in [(21, 200, 80, 1.0, 1.0), (22, 2500, 900, 1.0, 1.0), (23, 300, 120, 4.5, 0.5)]:
        m_args, f1, T1, ep, el = known_local_map(cam, n_pt, n_ls, seed)
        gp, gl = ctx.lookForLocalMapMatches(gfpl.MapView(*m_args, device="cuda"), gfpl.KeyFrameView(f1, T1, "cuda"),
                                            ep_p, ep_l)
        op, ol = O.kf_local_map_matches(cam, cfg, gfpl.MapView(*m_args), gfpl.KeyFrameView(f1, T1), ep_p, ep_l)
        np.testing.assert_array_equal(gp, op)
        np.testing.assert_array_equal(gl, ol)
        if ep_p == 1.0:
            np.testing.assert_array_equal(gp, ep)
            np.testing.assert_array_equal(gl, el)
