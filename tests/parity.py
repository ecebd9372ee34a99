"""Field-by-field comparison of frame states (GPU vs CPU oracle).

Which fields are defined at which point follows the reference: a feature
record's *_obs / cut / invCovPose fields are only written for matched
features (src/stereoFrameHandler.cpp:576-580, 666-673, 1644-1646, 1736-1762).
"""
from __future__ import annotations

import numpy as np

PT_CORE = ["pt_pl", "pt_disp", "pt_P", "pt_sigma2", "pt_idx", "pt_level", "pdesc"]
LS_CORE = ["ls_spl", "ls_epl", "ls_sdisp", "ls_edisp", "ls_angle", "ls_sigma2", "ls_sP", "ls_eP",
           "ls_le", "ls_idx", "ls_level", "ldesc"]
LS_MATCHED = ["ls_spl_obs", "ls_epl_obs", "ls_sdisp_obs", "ls_edisp_obs", "ls_le_obs", "ls_cut",
              "ls_invcov", "ls_spl", "ls_epl", "ls_sdisp", "ls_edisp", "ls_sP", "ls_eP", "ls_inlier"]
PT_MATCHED = ["pt_pl_obs", "pt_inlier"]
POSE = ["Tfw", "DT", "DT_cov", "Tfw_cov", "DT_cov_eig"]


def bitwise_equal(a: np.ndarray, b: np.ndarray) -> bool:
    a = np.ascontiguousarray(a); b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


def diff_fields(g, o, names, rows=None, what=""):
    """Return list of mismatching field descriptions (bit-exact)."""
    bad = []
    for n in names:
        ga, oa = g.get(n), o.get(n)
        if rows is not None:
            ga, oa = ga[rows], oa[rows]
        if not bitwise_equal(ga, oa):
            if ga.shape != oa.shape:
                bad.append(f"{what}{n}: shape {ga.shape} vs {oa.shape}")
                continue
            neq = np.argwhere(~((ga == oa) | (np.isnan(ga) & np.isnan(oa)) if ga.dtype.kind == "f" else ga == oa))
            first = neq[0] if len(neq) else None
            bad.append(f"{what}{n}: {len(neq)} elems differ, first at {first}: gpu={ga[tuple(first)] if first is not None else '?'} "
                       f"oracle={oa[tuple(first)] if first is not None else '?'}")
    return bad


def compare_core(g, o, what=""):
    bad = []
    if g.n_pt != o.n_pt:
        bad.append(f"{what}n_pt {g.n_pt} vs {o.n_pt}")
    if g.n_ls != o.n_ls:
        bad.append(f"{what}n_ls {g.n_ls} vs {o.n_ls}")
    if bad:
        return bad
    return diff_fields(g, o, PT_CORE, what=what) + diff_fields(g, o, LS_CORE, what=what)


def compare_track(tg: dict, to: dict, what=""):
    bad = []
    for k in ["matched_pt", "matched_ls"]:
        if not np.array_equal(tg[k], to[k]):
            bad.append(f"{what}{k}: len {len(tg[k])} vs {len(to[k])}")
    for k in ["n_inliers", "n_inliers_pt", "n_inliers_ls", "num_frame_loss"]:
        if tg[k] != to[k]:
            bad.append(f"{what}{k}: {tg[k]} vs {to[k]}")
    return bad


def compare_prev_matched(g, o, track: dict, what=""):
    pts = np.unique(track["matched_pt"]).astype(np.int64)
    lns = np.asarray(track["matched_ls"], np.int64)
    bad = diff_fields(g, o, PT_MATCHED, rows=pts, what=what)
    bad += diff_fields(g, o, LS_MATCHED, rows=lns, what=what)
    bad += diff_fields(g, o, ["ls_covS", "ls_covE"], what=what)
    return bad


def compare_pose(g, o, rtol=1e-6, atol=1e-12, what=""):
    """Return (tolerance failures, bitwise-equal flag)."""
    bad, exact = [], True
    for n in POSE:
        a, b = g.get(n), o.get(n)
        if not bitwise_equal(a, b):
            exact = False
        if not np.allclose(a, b, rtol=rtol, atol=atol, equal_nan=True):
            bad.append(f"{what}{n}: max abs diff {np.nanmax(np.abs(a - b))}")
    if not (g.s.err_norm == o.s.err_norm or np.isclose(g.s.err_norm, o.s.err_norm, rtol=rtol, atol=atol)):
        bad.append(f"{what}err_norm {g.s.err_norm} vs {o.s.err_norm}")
    if g.s.err_norm != o.s.err_norm:
        exact = False
    return bad, exact


def make_ragged(H):
    """Edge cases the reference guards (or would hit UB on): empty and tiny
    detection sets.  Needs >= 5 sequences and >= 3 frames."""
    assert H.B >= 5 and H.F >= 3
    H.n_kp_l[2, 1] = 0                       # no left keypoints -> no stereo points
    H.n_kl_r[1, 2] = 1                       # one right line (ledger U4) -> no stereo lines
    H.n_kp_l[2, 3] = 0; H.n_kp_r[2, 3] = 0   # nothing at all -> pose skipped
    H.n_kl_l[2, 3] = 0
    H.n_kp_l[1, 4] = 30; H.n_kl_l[1, 4] = 3  # tiny sets
    return H
