"""The HIP path against the committed golden fixtures (tests/golden/oracle_golden.json).

Every case of tests/golden/make_golden.py — including BASELINE configs[0], the
EuRoC MH_01 stereo pair driven by the reference's own ground truth
(config/asl/gt-ass/mh_01/groundtruth.txt rows 1-2) through
StereoFrameHandler::initialize / insertStereoPair / optimizePose — runs on the
GPU through the C ABI and must reproduce the fixture's digests, matched lists,
cut ratios and pose bits exactly.  The fixtures are oracle outputs (parity is
pinned by the oracle's known answers)."""
import json
import os
import sys

import numpy as np
import pytest

import gfpl

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(HERE, "golden", "oracle_golden.json")))


def run_case_gpu(case):
    """make_golden.run_case with the HIP StereoFrameHandler in place of the oracle."""
    cfg, cam, H, keep = G.build_inputs(case)
    D = gfpl.DeviceFrames(H)
    ctx = gfpl.Context(cam, cfg)
    g = gfpl.StereoFrameHandler(ctx, case["n_seq"], case["kp"], case["kl"])
    out = {"inputs": G.digest(*H.arrays()), "frames": [[] for _ in range(case["n_seq"])]}
    g.initialize(D.frames(0))
    for b in range(case["n_seq"]):
        f = g.read_frame(gfpl.PREV, b)
        out["frames"][b].append({"n_pt": f.n_pt, "n_ls": f.n_ls, "core": G.digest(*[f.get(n) for n in G.CORE])})
    for k in range(1, case["n_frames"]):
        g.insertStereoPair(D.frames(k))
        tracks = [g.read_track(b) for b in range(case["n_seq"])]
        prevs = [g.read_frame(gfpl.PREV, b) for b in range(case["n_seq"])]
        g.optimizePose()
        for b in range(case["n_seq"]):
            tr, p = tracks[b], prevs[b]
            ml = tr["matched_ls"]
            c = g.read_frame(gfpl.CURR, b)
            tr2 = g.read_track(b)
            out["frames"][b].append({
                "n_pt": c.n_pt, "n_ls": c.n_ls, "core": G.digest(*[c.get(n) for n in G.CORE]),
                "matched_pt": tr["matched_pt"].tolist(), "matched_ls": ml.tolist(),
                "cut": [float(v).hex() for v in p.get("ls_cut")[ml].ravel()],
                "prev_matched": G.digest(p.get("ls_invcov")[ml], p.get("ls_sP")[ml], p.get("ls_eP")[ml],
                                         p.get("pt_pl_obs")[np.unique(tr["matched_pt"])]),
                "n_inliers": tr2["n_inliers"], "n_inliers_pt": tr2["n_inliers_pt"],
                "n_inliers_ls": tr2["n_inliers_ls"],
                "DT": [float(v).hex() for v in c.get("DT").ravel()],
                "Tfw": [float(v).hex() for v in c.get("Tfw").ravel()],
                "DT_cov_eig": [float(v).hex() for v in c.get("DT_cov_eig").ravel()],
                "err_norm": float(c.s.err_norm).hex(),
            })
        g.updateFrame()
    return out


@pytest.mark.parametrize("name", sorted(G.CASES))
def test_hip_path_matches_golden(name):
    got = run_case_gpu(G.CASES[name])
    exp = GOLD[name]
    assert got["inputs"] == exp["inputs"], "synthetic generator drifted"
    for b, (gs, es) in enumerate(zip(got["frames"], exp["frames"])):
        for k, (g, e) in enumerate(zip(gs, es)):
            for key in e:
                assert g[key] == e[key], f"{name} seq {b} frame {k}: {key}"


def test_euroc_mh01_pair_on_gpu_recovers_ground_truth():
    """BASELINE configs[0] on the HIP path: the pose is the fixture's, bit for bit,
    and it is the reference's ground-truth motion to the detection noise."""
    got = run_case_gpu(G.CASES["euroc_mh01_pair"])["frames"][0][1]
    exp = GOLD["euroc_mh01_pair"]["frames"][0][1]
    assert got["DT"] == exp["DT"] and got["Tfw"] == exp["Tfw"]
    DT = np.array([float.fromhex(v) for v in got["DT"]]).reshape(4, 4)
    T, _ = G.euroc_traj("mh_01", 2)
    T0 = np.vstack([T[0].reshape(3, 4), [0, 0, 0, 1]])
    T1 = np.vstack([T[1].reshape(3, 4), [0, 0, 0, 1]])
    gt = np.linalg.inv(T0) @ T1
    assert np.abs(DT[:3, 3] - gt[:3, 3]).max() < 5e-3
    assert np.abs(DT[:3, :3] - gt[:3, :3]).max() < 1e-3
