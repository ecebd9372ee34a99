"""Pin the CPU oracle with hand-derived known answers.

The reference cannot be built here and has no usable tests of its own, so the
oracle's building blocks are checked against closed forms / numpy, and the
whole GN stage against a noise-free problem whose answer is known exactly.
"""
import ctypes as C

import numpy as np
import pytest

import gfpl
import oracle as O


# ------------------------------------------------------------- Hamming --
@pytest.mark.parametrize("byte,h1,h2", [(0xFF, 8, 4), (0x55, 4, 4), (0x03, 2, 1), (0xAA, 4, 4),
                                        (0x01, 1, 1), (0x02, 1, 1), (0xC0, 2, 1), (0x00, 0, 0)])
def test_hamming_known_bytes(byte, h1, h2):
    a = np.zeros(32, np.uint8)
    b = np.full(32, byte, np.uint8)
    assert O.hamming(a, b, 1) == 32 * h1          # descriptorDistance / NORM_HAMMING
    assert O.hamming(a, b, 2) == 32 * h2          # NORM_HAMMING2: non-zero 2-bit cells


def test_hamming_random_matches_numpy():
    rng = np.random.default_rng(0)
    for _ in range(50):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        x = np.bitwise_xor(a, b)
        h1 = int(np.unpackbits(x).sum())
        cells = ((x | (x >> 1)) & 0x55)
        h2 = int(np.unpackbits(cells.astype(np.uint8)).sum())
        assert O.hamming(a, b, 1) == h1
        assert O.hamming(a, b, 2) == h2


def test_knn2_tie_rule_lower_train_index_first():
    # cv::batchDistance insertion: d < dist[K-1], shift while dist[k] > d
    t = np.zeros((5, 32), np.uint8)
    t[0, 0] = 0b111   # d=3
    t[1, 0] = 0b1     # d=1
    t[2, 0] = 0b10    # d=1 (tie with 1)
    t[3, 0] = 0b1     # d=1 (tie)
    t[4, 0] = 0b11    # d=2
    q = np.zeros((1, 32), np.uint8)
    rc, idx, dist = O.knn2(q, t, 1)
    assert rc == 0
    assert idx.tolist() == [[1, 2]] and dist.tolist() == [[1.0, 1.0]]
    rc, _, _ = O.knn2(q, t[:1], 1)
    assert rc == -4   # U4: fewer than two train rows


def test_knn2_matches_bruteforce():
    rng = np.random.default_rng(3)
    q = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (60, 32), dtype=np.uint8)
    t[10] = t[20]
    for cell in (1, 2):
        rc, idx, dist = O.knn2(q, t, cell)
        for i in range(len(q)):
            d = np.array([O.hamming(q[i], t[j], cell) for j in range(len(t))])
            order = np.lexsort((np.arange(len(t)), d))   # (dist, index)
            assert idx[i].tolist() == order[:2].tolist()
            assert dist[i].tolist() == d[order[:2]].astype(np.float32).tolist()


# ------------------------------------------------------ pinned libm (N3) --
def _ulp_diff(a, b):
    a = np.float64(a); b = np.float64(b)
    ia = np.array(a).view(np.int64); ib = np.array(b).view(np.int64)
    return abs(int(ia) - int(ib))


def test_log_within_one_ulp():
    rng = np.random.default_rng(1)
    xs = np.concatenate([np.exp(rng.uniform(-700, 700, 3000)), rng.uniform(0.5, 2.0, 3000),
                         np.array([1.0, 2.0, 0.5, 1e-310, 5e-324, 1.7976931348623157e308])])
    for x in xs:
        assert _ulp_diff(O.log(float(x)), np.log(x)) <= 1, x
    assert O.log(1.0) == 0.0
    assert O.log(0.0) == -np.inf
    assert np.isnan(O.log(-1.0))
    assert O.log(np.inf) == np.inf


def test_sin_cos_within_one_ulp():
    rng = np.random.default_rng(2)
    xs = np.concatenate([rng.uniform(-4, 4, 3000), rng.uniform(-1e5, 1e5, 1000),
                         np.array([1e-9, 1e-6, np.pi / 4, np.pi / 2, np.pi, 3.0])])
    for x in xs:
        assert _ulp_diff(O.sin(float(x)), np.sin(x)) <= 1, x
        assert _ulp_diff(O.cos(float(x)), np.cos(x)) <= 1, x


# ---------------------------------------------------------- small dense --
def _spd(rng, n=6, cond=1e3):
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    w = np.exp(rng.uniform(0, np.log(cond), n))
    return (Q * w) @ Q.T


def test_logdet_spd_matches_numpy():
    rng = np.random.default_rng(4)
    for _ in range(200):
        A = _spd(rng) * rng.uniform(1e-3, 1e6)
        s, ld = np.linalg.slogdet(A)
        assert s > 0
        assert abs(O.logdet6(A) - ld) <= 1e-9 * max(1.0, abs(ld))


def test_logdet_reads_lower_triangle_only():
    rng = np.random.default_rng(5)
    A = _spd(rng)
    B = A.copy()
    B[np.triu_indices(6, 1)] = 12345.0   # garbage above the diagonal
    assert O.logdet6(A) == O.logdet6(B)


def test_logdet_partial_failure_semantics():
    # ledger Q11: LLT stops at the first non-positive pivot k; diag entries
    # k..5 keep their input values, so logdet mixes L_ii (i<k) with a_jj (j>=k)
    A = np.diag([4.0, 9.0, 2.0, 3.0, 5.0, 7.0])
    A[2, 1] = A[1, 2] = 10.0          # pivot 2: 2 - (10/3)^2 < 0
    L00, L11 = 2.0, 3.0
    expect = 2 * (np.log(L00) + np.log(L11) + np.log(2.0) + np.log(3.0) + np.log(5.0) + np.log(7.0))
    assert abs(O.logdet6(A) - expect) < 1e-12


def test_ldlt_solve_spd_and_indefinite():
    rng = np.random.default_rng(6)
    for _ in range(100):
        H = _spd(rng, cond=1e6)
        g = rng.normal(size=6)
        x = O.ldlt_solve6(H, g)
        assert np.allclose(H @ x, g, rtol=1e-8, atol=1e-8)
    Q, _ = np.linalg.qr(rng.normal(size=(6, 6)))
    H = (Q * np.array([3.0, -2.0, 1.0, -5.0, 0.5, 4.0])) @ Q.T     # indefinite -> pivoting
    g = rng.normal(size=6)
    assert np.allclose(H @ O.ldlt_solve6(H, g), g, atol=1e-9)
    assert np.all(O.ldlt_solve6(np.zeros((6, 6)), g) == 0.0)       # all-zero diagonal


def test_inverses_match_numpy():
    rng = np.random.default_rng(7)
    for _ in range(50):
        A = rng.normal(size=(6, 6))
        assert np.allclose(O.inverse6(A), np.linalg.inv(A), rtol=1e-9, atol=1e-9)
        B = rng.normal(size=(4, 4))
        assert np.allclose(O.inverse4(B), np.linalg.inv(B), rtol=1e-9, atol=1e-9)


def test_jacobi_rotation_shortcuts_are_bit_identical():
    """eig_sym's device rotation (gfpl_device.hpp) skips two sqrt / div chains where they cannot
    change a bit of the oracle's (oracle/gfpl_oracle.cpp eig_sym): 1 / (|th| + sqrt(th^2 + 1)) is
    0.5 / |th| for 2^27 <= |th| <= 1e150, and t^2 + 1 == 1 gives c = 1."""
    rng = np.random.default_rng(27)
    e = rng.uniform(27, 498, 2_000_000)
    th = np.exp2(e) * rng.uniform(1, 2, e.size)
    th = np.concatenate([th[th <= 1e150], 2.0 ** 27 + np.arange(4096) * 2.0 ** -25, [1e150]])
    assert np.array_equal(1.0 / (th + np.sqrt(th * th + 1.0)), 0.5 / th)
    t = np.concatenate([np.exp2(rng.uniform(-600, -20, 1_000_000)), [2.0 ** -27, 2.0 ** -26]])
    tt1 = t * t + 1.0
    assert np.all((1.0 / np.sqrt(tt1))[tt1 == 1.0] == 1.0)


def _jacobi(A, fast):
    """oracle/gfpl_oracle.cpp eig_sym (fast=False) and the device's eig_sym (gfpl_device.hpp: the
    rotation shortcuts and the early exit), in Python doubles (IEEE, correctly rounded sqrt)."""
    import math
    n = A.shape[0]
    a = [float(x) for x in A.ravel()]
    for _ in range(50):
        off = 0.0
        for p in range(n):
            for q in range(p + 1, n):
                off = off + a[p * n + q] * a[p * n + q]
        if not off > 0.0:
            break
        if fast:
            thr, fin = math.inf, True
            for i in range(n):
                e = (np.float64(a[i * n + i]).view(np.uint64) >> np.uint64(52)) & np.uint64(0x7FF)
                e = int(e)
                fin = fin and e != 0x7FF
                thr = min(thr, 0.0 if e == 0 else math.ldexp(1.0, 2 * (e - 1076) - 6))
            if fin and off < thr:
                break
        for p in range(n - 1):
            for q in range(p + 1, n):
                apq = a[p * n + q]
                if apq == 0.0:
                    continue
                app, aqq = a[p * n + p], a[q * n + q]
                th = (aqq - app) / (2.0 * apq)
                if abs(th) > 1e150:
                    t = 0.5 / th
                elif fast and abs(th) >= 2.0 ** 27:
                    t = 0.5 / abs(th)
                    t = -t if th < 0.0 else t
                else:
                    t = 1.0 / (abs(th) + math.sqrt(th * th + 1.0))
                    t = -t if th < 0.0 else t
                tt1 = t * t + 1.0
                c = 1.0 if (fast and tt1 == 1.0) else 1.0 / math.sqrt(tt1)
                s_ = t * c
                for k in range(n):
                    if k in (p, q):
                        continue
                    akp, akq = a[k * n + p], a[k * n + q]
                    nkp, nkq = c * akp - s_ * akq, s_ * akp + c * akq
                    a[k * n + p] = a[p * n + k] = nkp
                    a[k * n + q] = a[q * n + k] = nkq
                a[p * n + p] = app - t * apq
                a[q * n + q] = aqq + t * apq
                a[p * n + q] = a[q * n + p] = 0.0
    return sorted(a[i * n + i] for i in range(n))


def test_jacobi_early_exit_keeps_the_oracles_bits():
    """The device eig_sym stops once no later rotation can move a diagonal entry; its eigenvalues
    equal the oracle's full sweep bit for bit (random, near-degenerate, diagonal, widely scaled)."""
    rng = np.random.default_rng(45)
    for trial in range(600):
        n = 3 if trial % 2 else 6
        kind = trial % 6
        A = rng.normal(size=(n, n))
        A = A @ A.T if kind < 2 else A + A.T
        if kind == 2:   # near-degenerate: a repeated eigenvalue plus a tiny perturbation
            Q = np.linalg.qr(rng.normal(size=(n, n)))[0]
            A = Q @ np.diag([1.0] * (n - 1) + [2.0]) @ Q.T + 1e-13 * (lambda M: M + M.T)(rng.normal(size=(n, n)))
        if kind == 3:
            A = np.diag(rng.normal(size=n)) + np.triu(1e-170 * rng.normal(size=(n, n)), 1)
            A = np.triu(A) + np.triu(A, 1).T
        if kind == 4:
            A = A * 10.0 ** rng.uniform(-150, 150)
        if kind == 5:
            A[0, :] = 0.0
            A[:, 0] = 0.0
        got, ref = _jacobi(A, True), _jacobi(A, False)
        assert [np.float64(x).view(np.uint64) for x in got] == [np.float64(x).view(np.uint64) for x in ref], (trial, got, ref)


def test_eig_sym_matches_numpy():
    rng = np.random.default_rng(8)
    for n in (3, 6):
        for _ in range(100):
            A = rng.normal(size=(n, n)); A = A + A.T
            w = O.eig_sym(A)
            assert np.allclose(w, np.linalg.eigvalsh(A), rtol=1e-10, atol=1e-10)


def test_se3_identities():
    assert np.array_equal(O.expmap_se3(np.zeros(6)), np.eye(4))
    rng = np.random.default_rng(9)
    for _ in range(50):
        x = rng.normal(size=6) * [1, 1, 1, 0.5, 0.5, 0.5]
        T = O.expmap_se3(x)
        R = T[:3, :3]
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-12)
        assert np.allclose(O.inverse_se3(T) @ T, np.eye(4), atol=1e-12)
        # Rodrigues closed form
        w = x[3:]; th = np.linalg.norm(w); k = w / th
        K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        assert np.allclose(R, np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K, atol=1e-12)


# ------------------------------------------------ GN known answer --
def _noise_free_problem(T_cp, cfg, cam, n_pt=120, n_ls=40, seed=0):
    """prev frame with points / lines, curr observations generated by T_cp exactly."""
    rng = np.random.default_rng(seed)
    KP, KL = 256, 64
    prev = gfpl.FrameHost(KP, KL)
    fx, fy, cx, cy = cam.fx, cam.fy, cam.cx, cam.cy

    def proj(P):
        return np.array([cx + fx * P[0] / P[2], cy + fy * P[1] / P[2]])

    P = np.stack([rng.uniform(-2, 2, n_pt), rng.uniform(-1.5, 1.5, n_pt), rng.uniform(3, 8, n_pt)], 1)
    prev.s.n_pt = n_pt
    a = prev.arr
    a["pt_P"][:n_pt] = P
    for i in range(n_pt):
        Pc = T_cp[:3, :3] @ P[i] + T_cp[:3, 3]
        a["pt_pl_obs"][i] = proj(Pc)
        a["pt_pl"][i] = proj(P[i])
    a["pt_sigma2"][:n_pt] = 1.0
    a["pt_inlier"][:n_pt] = 1
    a["pt_idx"][:n_pt] = np.arange(n_pt)
    S = np.stack([rng.uniform(-2, 2, n_ls), rng.uniform(-1.5, 1.5, n_ls), rng.uniform(3, 8, n_ls)], 1)
    E = S + rng.normal(size=(n_ls, 3)) * 0.5
    prev.s.n_ls = n_ls
    a["ls_sP"][:n_ls] = S
    a["ls_eP"][:n_ls] = E
    for i in range(n_ls):
        s = proj(T_cp[:3, :3] @ S[i] + T_cp[:3, 3]); e = proj(T_cp[:3, :3] @ E[i] + T_cp[:3, 3])
        le = np.cross([s[0], s[1], 1.0], [e[0], e[1], 1.0])
        a["ls_le_obs"][i] = le / np.hypot(le[0], le[1])
    a["ls_sigma2"][:n_ls] = 1.0
    a["ls_inlier"][:n_ls] = 1
    for n in ("Tfw", "DT"):
        np.ctypeslib.as_array(getattr(prev.s, n))[:] = np.eye(4).ravel()
    prev.s.time_stamp = 1.0
    curr = gfpl.FrameHost(KP, KL)
    curr.s.time_stamp = 1.05
    tr = gfpl.TrackHost()
    tr.n_matched_pt, tr.n_matched_ls = n_pt, n_ls
    for i in range(n_pt):
        tr.matched_pt[i] = i
    for i in range(n_ls):
        tr.matched_ls[i] = i
    tr.n_inliers_pt, tr.n_inliers_ls, tr.n_inliers = n_pt, n_ls, n_pt + n_ls
    return prev, curr, tr


def test_gn_noise_free_recovers_pose():
    # the reference stops once the mean robust squared residual < minError
    # (1e-7 px^2, src/stereoFrameHandler.cpp:2042), so the recovered pose is
    # exact to ~1e-6, not to machine precision
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    x = np.array([0.02, -0.01, 0.025, 0.01, -0.02, 0.015])
    T_cp = O.expmap_se3(x)
    prev, curr, tr = _noise_free_problem(T_cp, cfg, cam)
    h = O.OracleHandler(cam, cfg, 256, 64)
    h.write_frame(gfpl.PREV, prev)
    h.write_frame(gfpl.CURR, curr)
    h.write_track(tr)
    h.optimizePose()
    c = h.read_frame(gfpl.CURR)
    # curr.DT = inverse_se3(DT_opt) and DT_opt = T_cp (src/stereoFrameHandler.cpp:1986)
    assert np.allclose(c.get("DT"), np.linalg.inv(T_cp), atol=1e-5)
    assert np.allclose(c.get("Tfw"), np.linalg.inv(T_cp), atol=1e-5)
    assert 0.0 <= c.s.err_norm < 1e-7
    assert h.read_track()["num_frame_loss"] == 0


def test_gn_too_few_features_gives_identity():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    prev, curr, tr = _noise_free_problem(O.expmap_se3(np.full(6, 0.01)), cfg, cam, n_pt=6, n_ls=4)
    h = O.OracleHandler(cam, cfg, 256, 64)
    h.write_frame(gfpl.PREV, prev); h.write_frame(gfpl.CURR, curr); h.write_track(tr)
    h.optimizePose()   # n_inliers = 10 is not > minFeatures (src/stereoFrameHandler.cpp:1953)
    c = h.read_frame(gfpl.CURR)
    assert np.array_equal(c.get("DT"), np.eye(4))
    assert np.all(c.get("DT_cov") == 0.0)


def test_motion_gate_rejects_large_step():
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10)
    cam = gfpl.make_camera("vga", cfg)
    T_cp = O.expmap_se3(np.array([0.0, 0.0, 0.6, 0.0, 0.0, 0.0]))   # 0.6 m in 0.05 s > 10 m/s
    prev, curr, tr = _noise_free_problem(T_cp, cfg, cam)
    h = O.OracleHandler(cam, cfg, 256, 64)
    h.write_frame(gfpl.PREV, prev); h.write_frame(gfpl.CURR, curr); h.write_track(tr)
    h.optimizePose()
    c = h.read_frame(gfpl.CURR)
    assert np.array_equal(c.get("DT"), np.eye(4))     # rolled back (src/stereoFrameHandler.cpp:2004-2011)
    assert c.s.err_norm == -1.0


def test_line_cut_zero_covariance_never_moves():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    prev, curr, tr = _noise_free_problem(np.eye(4), cfg, cam, n_pt=30, n_ls=5)
    np.ctypeslib.as_array(curr.s.Tfw)[:] = np.eye(4).ravel()
    h = O.OracleHandler(cam, cfg, 256, 64)
    h.write_frame(gfpl.PREV, prev); h.write_frame(gfpl.CURR, curr); h.write_track(tr)
    h.estimateProjUncertainty_submodular()   # covS = covE = 0: variances 0 -> no finite metric
    p = h.read_frame(gfpl.PREV)
    assert np.all(p.get("ls_cut")[:5] == 0.0)


# ------------------------------------------------- keyframe decision ----
def test_det6_matches_numpy_and_permutation_sign():
    rng = np.random.default_rng(5)
    for _ in range(30):
        A = rng.normal(size=(6, 6))
        assert O.det6(A) == pytest.approx(np.linalg.det(A), rel=1e-10)
    # a permutation matrix of odd parity has determinant exactly -1, even +1
    P = np.eye(6)[[1, 0, 2, 3, 4, 5]]
    assert O.det6(P) == -1.0
    assert O.det6(np.eye(6)[[1, 2, 0, 3, 4, 5]]) == 1.0
    assert O.det6(np.diag([2.0, 3.0, 0.5, 1.0, 4.0, 0.25])) == 3.0
    assert O.det6(np.zeros((6, 6))) == 0.0


def test_need_new_kf_entropy_and_frame_count(tmp_path):
    """needNewKF on a short synthetic sequence: the first decision after a keyframe
    compares the accumulated covariance with the first one (ratio 1 at the first
    call), the frame-count gate fires after maxKFNumFrames, and currFrameIsKF
    resets the state (src/stereoFrameHandler.cpp:2309-2379)."""
    cfg = gfpl.default_config(max_iters=5, max_iters_ref=5, max_kf_num_frames=2)
    cam = gfpl.make_camera("vga", cfg)
    H = gfpl.HostFrames(cam, gfpl.synth_params(seed=2), 1, 6, 2048, 512)
    o = O.OracleHandler(cam, cfg, 2048, 512)
    o.initialize(H.frames(0), 0)
    st = o.read_kf_state()
    assert st["prev_f_iskf"] == 1 and st["num_frame_since_kf"] == 0
    assert np.array_equal(st["T_prevKF"], np.eye(4)) and not st["cov_prevKF_currF"].any()
    seen = []
    for k in range(1, 6):
        o.insertStereoPair(H.frames(k), 0)
        o.optimizePose()
        f = o.needNewKF()
        st = o.read_kf_state()
        cov = o.read_frame(gfpl.CURR).get("DT_cov")
        e = 3.0 * (1.0 + np.log(2.0 * np.pi)) + 0.5 * np.log(np.linalg.det(cov))
        if k == 1:
            assert st["entropy_first_prevKF"] == pytest.approx(e, rel=1e-9)
            assert st["entropy_ratio"] == pytest.approx(1.0, rel=1e-9) or st["entropy_ratio"] < 1.0
        seen.append((st["num_frame_since_kf"], f))
        if f:
            o.currFrameIsKF()
            s2 = o.read_kf_state()
            assert s2["num_frame_since_kf"] == 0 and s2["prev_f_iskf"] == 1
            assert np.array_equal(o.read_frame(gfpl.CURR).get("Tfw"), np.eye(4))
        o.updateFrame()
    # the frame-count gate (numFrameSinceKeyframe > 2) fires no later than the 3rd frame after a KF
    assert any(f for _, f in seen)
    assert all(n <= 3 for n, _ in seen)


def _gate_bound(C, th):
    """k_stereo.hip eig_gate_bound: 1 / 0 when bounds settle "largest eigenvalue < th", else -1."""
    import math
    c = [float(x) for x in C.ravel()]
    if not all(math.isfinite(x) for x in c):
        return -1
    M = max(abs(x) for x in c)
    G = max((c[4 * i] + abs(c[3 * i + (i + 1) % 3])) + abs(c[3 * i + (i + 2) % 3]) for i in range(3))
    D = max(c[4 * i] for i in range(3))
    if D >= th:
        return 0
    if G + 4e-9 * M < th:
        return 1
    return -1


def test_line_gate_bounds_agree_with_the_eigenvalues():
    """The stereo line gate (src/stereoFrame.cpp:743-751) decided from bounds gives eig_sym's
    decision whenever the bounds settle it: endpoint-covariance-like 3x3 matrices (a dominant
    viewing-ray direction plus isotropic noise) with th swept across their largest eigenvalue."""
    rng = np.random.default_rng(9)
    settled = [0, 0]
    for trial in range(3000):
        v = rng.normal(size=3)
        C = np.outer(v, v) * 10.0 ** rng.uniform(-6, 2) + np.diag(rng.uniform(0, 1e-3, 3))
        C = (C + C.T) / 2.0
        lam = _jacobi(C, True)[2]
        th = lam * (1.0 + rng.choice([-1.0, 1.0]) * 10.0 ** rng.uniform(-14, 0.5))
        g = _gate_bound(C, th)
        if g >= 0:
            settled[g] += 1
            assert g == (1 if lam < th else 0), (trial, lam, th, g)
    assert min(settled) > 50   # (both outcomes exercised)
