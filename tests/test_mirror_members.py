"""The C++ mirror's StereoFrame members that MapHandler / StereoFrameHandler call on frames
(include/stereoFrame.h:104-148): BFMatcher-backed matchPointFeatures / matchLineFeatures /
*_radius, point / lineDescriptorMAD, the budget thresholds and the frame-level
extractInitialStereoFeatures / extractStereoFeatures_ORBSLAM / estimateStereoUncertainty.

CPU: the MapHandler-shaped caller (tests/mirror_maphandler.cpp: std::async(&StereoFrame::
matchPointFeatures, kf0, bfm, ...) as src/mapHandler.cpp:223-226) compiles against stvo.h and
fails loudly without a GPU; the oracle's radiusMatch rows and match statistics equal an
independent numpy / Python statement of the reference's sorts.
GPU: the caller's outputs equal the oracle's, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

import gfpl
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "gf-pl-slam_amd", "bin", "mirror_maphandler")
SRC = os.path.join(ROOT, "tests", "mirror_maphandler.cpp")


def test_maphandler_shaped_caller_compiles_against_the_mirror(tmp_path):
    """The std::async(&StereoFrame::matchPointFeatures, kf0, bfm, d1, d2, ref(m)) pattern of
    src/mapHandler.cpp:223-226 and every frame member it uses compile against stvo.h."""
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                        SRC], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


def test_maphandler_shaped_caller_fails_loudly_without_gpu(tmp_path):
    if not os.path.exists(BIN):
        pytest.skip("mirror caller not built (make host)")
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([BIN, "--out", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3 and "no HIP device" in r.stderr


def _desc(n, seed, base=None, flips=0):
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 256, (n, 32), dtype=np.uint8) if base is None else base.copy()
    for i in range(len(d)):
        for _ in range(flips):
            d[i, rng.integers(0, 32)] ^= np.uint8(1 << int(rng.integers(0, 8)))
    return d


def _ham(a, b, cell):
    x = np.bitwise_xor(a, b)
    if cell == 2:
        x = (x | (x >> 1)) & 0x55
    return int(np.unpackbits(x).sum())


def test_oracle_radius_rows_match_a_python_statement():
    """radiusMatch (ledger T1: distance <= maxDistance; T2: equal distances in train order)."""
    t = _desc(60, 1)
    q = np.concatenate([_desc(20, 2, base=t[:20], flips=6), _desc(8, 3)])
    for cell, r in ((1, 50.0), (1, 3.0), (2, 40.0), (1, 0.0)):
        off, idx, dist = O.radius_match(q, t, r, cell)
        for i in range(len(q)):
            ds = [(_ham(q[i], t[j], cell), j) for j in range(len(t))]
            want = sorted([x for x in ds if x[0] <= r], key=lambda x: x[0])   # Python's sort is stable
            got = list(zip(dist[off[i]:off[i + 1]].astype(int), idx[off[i]:off[i + 1]]))
            assert got == want, (cell, r, i)


def _select(v, k):
    key = [(1, 0.0) if x != x else (0, x) for x in v]   # NaN above every number (ledger U12)
    s = sorted(range(len(v)), key=lambda i: key[i])
    return v[s[k]]


def _stats_py(kind, d0, d1, max_num):
    n = len(d0)
    f = np.float32
    nn = 1.4826 * float(_select([f(abs(f(float(x) - 0.0))) for x in d0], n // 2))
    if kind == 1:
        nn12 = 1.4826 * float(_select([f(abs(f(float(f(b - a)) - 0.0))) for a, b in zip(d0, d1)], n // 2))
    else:
        with np.errstate(divide="ignore", invalid="ignore"):
            r = [f(a / b) for a, b in zip(d0, d1)]
        med = float(_select(r, n - 1 - n // 2))   # the descending order's element n/2
        nn12 = 1.4826 * float(_select([f(abs(f(float(x) - med))) for x in r], n // 2))
    thr = float(_select([f(x) for x in d0], min(max_num, n) - 1))
    return nn, nn12, thr


def test_oracle_match_stats_match_a_python_statement():
    """lineDescriptorMAD / pointDescriptorMAD / *BudgetThres (src/stereoFrame.cpp:1259-1341)."""
    rng = np.random.default_rng(7)
    for n in (1, 2, 5, 64, 301):
        d0 = rng.integers(0, 90, n).astype(np.float32)
        d1 = (d0 + rng.integers(0, 40, n)).astype(np.float32)
        if n > 4:
            d0[2] = d1[2] = 0.0   # 0 / 0: a NaN ratio
        for kind in (0, 1):
            for mx in (1, 3, 300, 500):
                got = O.match_stats(kind, d0, d1, mx)
                want = _stats_py(kind, d0, d1, mx)
                assert all((a == b) or (a != a and b != b) for a, b in zip(got, want)), (n, kind, mx, got, want)


def _rows(a, name):
    off = a[name + "_off"]
    return off, a[name + "_t"], a[name + "_d"]


@pytest.mark.gpu
@pytest.mark.parametrize("seq", [0, 5])
def test_mirror_frame_members_match_the_oracle(tmp_path, seq):
    """mirror_maphandler on GPU vs the oracle: frame-level stereo extraction of frames 0 / 1 and the
    line covariances of frame 0 (every field bitwise), knn-2 both ways (two std::async tasks on one
    BFMatcher), radius rows both ways, HAMMING2 radius rows of the lines, the MAD statistics and
    budget thresholds."""
    r = subprocess.run([BIN, "--out", str(tmp_path), "--seq", str(seq)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    import json
    names = json.loads(r.stdout.strip().splitlines()[-1])["arrays"]
    dt = {"pt": np.float64, "ls": np.float64, "pti": np.int32, "lsi": np.int32, "pdesc": np.uint8, "ldesc": np.uint8,
          "off": np.int32, "q": np.int32, "t": np.int32, "d": np.float32, "stats": np.float64}
    a = {n: np.fromfile(tmp_path / (n + ".bin"), dt[n.split("_")[-1]]) for n in names}

    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    KP, KL = 2048, 512
    H = gfpl.HostFrames(cam, gfpl.synth_params(), 1, 2, KP, KL, seq0=seq)
    o = O.OracleHandler(cam, cfg, KP, KL)
    o.initialize(H.frames(0), 0)
    o.estimateStereoUncertainty()
    f0 = o.read_frame(gfpl.PREV)
    o.begin_frame(H.frames(1), 0)
    o.stereoPoints()
    o.stereoLines()
    f1 = o.read_frame(gfpl.CURR)
    for tag, f in (("f0", f0), ("f1", f1)):
        n_pt, n_ls = int(f.s.n_pt), int(f.s.n_ls)
        pt = a[tag + "_pt"].reshape(-1, 7)
        ls = a[tag + "_ls"].reshape(-1, 35)
        assert len(pt) == n_pt and len(ls) == n_ls, (tag, len(pt), n_pt, len(ls), n_ls)
        want_pt = np.concatenate([f.get("pt_pl"), f.get("pt_disp")[:, None], f.get("pt_P"),
                                  f.get("pt_sigma2")[:, None]], axis=1)
        assert pt.tobytes() == want_pt.tobytes(), tag
        assert (a[tag + "_pti"].reshape(-1, 2) == np.stack([f.get("pt_idx"), f.get("pt_level")], 1)).all(), tag
        want_ls = np.concatenate([f.get("ls_spl"), f.get("ls_epl"), f.get("ls_sdisp")[:, None],
                                  f.get("ls_edisp")[:, None], f.get("ls_angle")[:, None], f.get("ls_sP"),
                                  f.get("ls_eP"), f.get("ls_le"), f.get("ls_sigma2")[:, None],
                                  f.get("ls_covS").reshape(-1, 9), f.get("ls_covE").reshape(-1, 9)], axis=1)
        if tag == "f0":
            assert np.abs(want_ls[:, 17:]).sum() > 0   # the covariances were estimated
        assert ls.tobytes() == want_ls.tobytes(), tag
        assert (a[tag + "_lsi"].reshape(-1, 2) == np.stack([f.get("ls_idx"), f.get("ls_level")], 1)).all(), tag
        assert a[tag + "_pdesc"].tobytes() == f.get("pdesc").tobytes(), tag
        assert a[tag + "_ldesc"].tobytes() == f.get("ldesc").tobytes(), tag

    p0, p1 = a["f0_pdesc"].reshape(-1, 32), a["f1_pdesc"].reshape(-1, 32)
    l0, l1 = a["f0_ldesc"].reshape(-1, 32), a["f1_ldesc"].reshape(-1, 32)
    for name, q, t in (("pk12", p0, p1), ("pk21", p1, p0), ("lk12", l0, l1), ("lk21", l1, l0)):
        rc, idx, dist = O.knn2(q, t, 1)
        assert rc == 0
        off, ti, di = _rows(a, name)
        assert (np.diff(off) == 2).all() and (a[name + "_q"].reshape(-1, 2)[:, 0] == np.arange(len(q))).all(), name
        assert (ti.reshape(-1, 2) == idx).all() and di.reshape(-1, 2).tobytes() == dist.tobytes(), name
    for name, q, t, rad, cell in (("pr12", p0, p1, cfg.point_match_radius, 1), ("pr21", p1, p0, cfg.point_match_radius, 1),
                                  ("lr12", l0, l1, 80.0, 2)):
        off, idx, dist = O.radius_match(q, t, rad, cell)
        go, gt, gd = _rows(a, name)
        assert (go == off).all() and (gt == idx).all() and gd.tobytes() == dist.tobytes(), name
        assert off[-1] > 0, name
    _, _, pk = O.knn2(p0, p1, 1)
    _, _, lk = O.knn2(l0, l1, 1)
    ln = O.match_stats(1, lk[:, 0], lk[:, 1], cfg.max_line_match_num)
    pn = O.match_stats(0, pk[:, 0], pk[:, 1], cfg.max_point_match_num)
    want = [ln[0], ln[1], pn[0], pn[1], pn[2], ln[2]]
    assert a["stats"].tolist() == want, (a["stats"].tolist(), want)


@pytest.mark.gpu
def test_radius_and_stats_abi_edges():
    """gfpl_radius_hamming (device) / gfpl_radius_hamming_host / gfpl_match_stats_host vs the oracle:
    rows longer than a wave's chunk with many equal distances (a repeated train row), empty queries
    and trains, the capacity refusal (row_off filled, nothing else), HAMMING2; statistics with
    NaN ratios and n = 1."""
    import ctypes as C
    import torch
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    ctx = gfpl.Context(cam, cfg)
    L = ctx.L
    P = C.c_void_p
    L.gfpl_radius_hamming_host.argtypes = [P, P, C.c_int, P, C.c_int, C.c_int, C.c_float, P, C.c_int, P, P]
    L.gfpl_radius_hamming.argtypes = [P, P, C.c_int, P, C.c_int, C.c_int, C.c_float, P, C.c_int, P, P]
    L.gfpl_match_stats_host.argtypes = [P, C.c_int, P, P, C.c_int, C.c_int, P]
    rng = np.random.default_rng(3)
    t = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    t[100:230] = t[7]                      # 130 equal rows: equal distances span three 64-row chunks
    q = np.concatenate([t[:40] ^ (rng.random((40, 32)) < 0.05).astype(np.uint8), t[7:8]])
    for cell, rad in ((1, 50.0), (2, 30.0), (1, 256.0)):
        off_o, idx_o, dist_o = O.radius_match(q, t, rad, cell)
        tot = int(off_o[-1])
        off = np.zeros(len(q) + 1, np.int32)
        idx = np.zeros(max(tot, 1), np.int32)
        dist = np.zeros(max(tot, 1), np.float32)
        rc = L.gfpl_radius_hamming_host(ctx.h, q.ctypes.data, len(q), t.ctypes.data, len(t), cell, rad,
                                        off.ctypes.data, tot - 1, idx.ctypes.data, dist.ctypes.data)
        assert rc == -5 and (off == off_o).all()   # GFPL_E_CAPACITY, the sizes filled
        rc = L.gfpl_radius_hamming_host(ctx.h, q.ctypes.data, len(q), t.ctypes.data, len(t), cell, rad,
                                        off.ctypes.data, tot, idx.ctypes.data, dist.ctypes.data)
        assert rc == 0 and (off == off_o).all() and (idx[:tot] == idx_o).all() and (dist[:tot] == dist_o).all()
        # the device form on torch buffers
        dq, dt = torch.from_numpy(q).cuda(), torch.from_numpy(t).cuda()
        doff = torch.zeros(len(q) + 1, dtype=torch.int32, device="cuda")
        didx = torch.zeros(max(tot, 1), dtype=torch.int32, device="cuda")
        ddist = torch.zeros(max(tot, 1), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        rc = L.gfpl_radius_hamming(ctx.h, dq.data_ptr(), len(q), dt.data_ptr(), len(t), cell, rad, doff.data_ptr(),
                                   tot, didx.data_ptr(), ddist.data_ptr())
        assert rc == 0 and (doff.cpu().numpy() == off_o).all()
        assert (didx.cpu().numpy()[:tot] == idx_o).all() and (ddist.cpu().numpy()[:tot] == dist_o).all()
    off = np.zeros(5, np.int32)
    for nq, nt in ((0, 10), (4, 0)):
        rc = L.gfpl_radius_hamming_host(ctx.h, q.ctypes.data, nq, t.ctypes.data, nt, 1, 50.0, off.ctypes.data, 0, None,
                                        None)
        assert rc == 0 and (off[:nq + 1] == 0).all()
    for n in (1, 2, 7, 300):
        d0 = rng.integers(0, 60, n).astype(np.float32)
        d1 = (d0 + rng.integers(0, 30, n)).astype(np.float32)
        if n > 2:
            d0[1] = d1[1] = 0.0
        for kind in (0, 1):
            for mx in (1, 2, 500):
                out = np.zeros(3, np.float64)
                rc = L.gfpl_match_stats_host(ctx.h, kind, d0.ctypes.data, d1.ctypes.data, n, mx, out.ctypes.data)
                want = O.match_stats(kind, d0, d1, mx)
                assert rc == 0 and all(a == b or (a != a and b != b) for a, b in zip(out, want)), (n, kind, mx)
    out = np.zeros(3, np.float64)
    assert L.gfpl_match_stats_host(ctx.h, 1, d0.ctypes.data, d1.ctypes.data, 0, 5, out.ctypes.data) == -1
    ctx.close()
