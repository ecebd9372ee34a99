"""ctypes binding of the CPU ORACLE (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker.  The product path never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "gf-pl-slam_amd"))
import gfpl  # noqa: E402  (struct definitions only)

_L = None


def lib() -> C.CDLL:
    global _L
    if _L is None:
        p = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(p):
            raise RuntimeError(f"{p} not built (make oracle)")
        L = C.CDLL(p)
        P = C.c_void_p
        L.gfplo_create.argtypes = [P, P]; L.gfplo_create.restype = P
        L.gfplo_destroy.argtypes = [P]; L.gfplo_destroy.restype = None
        for n in ["gfplo_initialize", "gfplo_insert_stereo_pair", "gfplo_begin_frame"]:
            getattr(L, n).argtypes = [P, P, C.c_int]; getattr(L, n).restype = C.c_int
        for n in ["gfplo_optimize_pose", "gfplo_update_frame", "gfplo_stereo_points",
                  "gfplo_stereo_lines", "gfplo_line_uncertainty", "gfplo_cross_points",
                  "gfplo_cross_lines", "gfplo_line_cut"]:
            getattr(L, n).argtypes = [P]; getattr(L, n).restype = C.c_int
        for n in ["gfplo_read_frame", "gfplo_write_frame"]:
            getattr(L, n).argtypes = [P, C.c_int, P]; getattr(L, n).restype = C.c_int
        for n in ["gfplo_read_track", "gfplo_write_track", "gfplo_need_new_kf", "gfplo_read_kf_state"]:
            getattr(L, n).argtypes = [P, P]; getattr(L, n).restype = C.c_int
        L.gfplo_curr_frame_is_kf.argtypes = [P]; L.gfplo_curr_frame_is_kf.restype = C.c_int
        L.gfplo_det6.argtypes = [P]; L.gfplo_det6.restype = C.c_double
        L.gfplo_optimize_pose_ini.argtypes = [P, P]; L.gfplo_optimize_pose_ini.restype = C.c_int
        L.gfplo_hamming.argtypes = [P, P, C.c_int]; L.gfplo_hamming.restype = C.c_int
        L.gfplo_knn2.argtypes = [P, C.c_int, P, C.c_int, C.c_int, P, P]; L.gfplo_knn2.restype = C.c_int
        L.gfplo_radius_match.argtypes = [P, C.c_int, P, C.c_int, C.c_int, C.c_float, P, C.c_int, P, P]
        L.gfplo_radius_match.restype = C.c_int
        L.gfplo_match_stats.argtypes = [C.c_int, P, P, C.c_int, C.c_int, P]; L.gfplo_match_stats.restype = C.c_int
        L.gfplo_kf_common_matches.argtypes = [P, P, P, P, P, P, P, P]
        L.gfplo_kf_common_matches.restype = C.c_int
        L.gfplo_kf_local_map_matches.argtypes = [P, P, P, P, C.c_double, C.c_double, P, P, P, P]
        L.gfplo_kf_local_map_matches.restype = C.c_int
        for n in ["gfplo_log", "gfplo_sin", "gfplo_cos"]:
            getattr(L, n).argtypes = [C.c_double]; getattr(L, n).restype = C.c_double
        L.gfplo_logdet6.argtypes = [P]; L.gfplo_logdet6.restype = C.c_double
        L.gfplo_ldlt_solve6.argtypes = [P, P, P]; L.gfplo_ldlt_solve6.restype = C.c_int
        for n in ["gfplo_inverse6", "gfplo_inverse4", "gfplo_expmap_se3", "gfplo_inverse_se3"]:
            getattr(L, n).argtypes = [P, P]; getattr(L, n).restype = C.c_int
        L.gfplo_eig_sym.argtypes = [P, C.c_int, P]; L.gfplo_eig_sym.restype = C.c_int
        L.gfplo_orb_extract.argtypes = [P, P, C.c_int, C.c_int, C.c_int, P, P, P, P, P, P]
        L.gfplo_orb_extract.restype = C.c_int
        L.gfplo_orb_resize.argtypes = [P, C.c_int, C.c_int, P, C.c_int, C.c_int]; L.gfplo_orb_resize.restype = C.c_int
        L.gfplo_orb_blur.argtypes = [P, C.c_int, C.c_int, P]; L.gfplo_orb_blur.restype = C.c_int
        L.gfplo_orb_fast.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, P]; L.gfplo_orb_fast.restype = C.c_int
        L.gfplo_fast_atan2.argtypes = [C.c_float, C.c_float]; L.gfplo_fast_atan2.restype = C.c_float
        L.gfplo_lbd_compute.argtypes = [P, C.c_int, C.c_int, P, C.c_int, P, P]; L.gfplo_lbd_compute.restype = C.c_int
        L.gfplo_lbd_gradients.argtypes = [P, C.c_int, C.c_int, P, P, P]; L.gfplo_lbd_gradients.restype = C.c_int
        L.gfplo_lbd_coefs.argtypes = [P, P]; L.gfplo_lbd_coefs.restype = C.c_int
        L.gfplo_lbd_num_pixels.argtypes = [P, C.c_int, C.c_int]; L.gfplo_lbd_num_pixels.restype = C.c_int
        L.gfplo_lsd_detect.argtypes = [P, P, C.c_int, C.c_int, C.c_int, P, P, P, P, C.c_int, P]
        L.gfplo_lsd_detect.restype = C.c_int
        L.gfplo_lsd_constants.argtypes = [P, C.c_int, C.c_int, P, P, P]; L.gfplo_lsd_constants.restype = C.c_int
        L.gfplo_atan2.argtypes = [C.c_double, C.c_double]; L.gfplo_atan2.restype = C.c_double
        L.gfplo_sort_desc.argtypes = [P, C.c_int]; L.gfplo_sort_desc.restype = C.c_int
        _L = L
    return _L


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


class OracleHandler:
    """One reference StereoFrameHandler restated on the CPU."""

    def __init__(self, cam: gfpl.Camera, cfg: gfpl.Config, kp_cap: int, kl_cap: int):
        self.L = lib()
        self.h = self.L.gfplo_create(C.byref(cam), C.byref(cfg))
        if not self.h:
            raise RuntimeError("gfplo_create failed (camera tables disagree with the oracle's?)")
        self.kp_cap, self.kl_cap = kp_cap, kl_cap

    def _c(self, code, what):
        if code != 0:
            raise RuntimeError(f"oracle {what}: {code}")

    def initialize(self, fr: gfpl.Frames, seq: int):
        self._c(self.L.gfplo_initialize(self.h, C.byref(fr), seq), "initialize")

    def insertStereoPair(self, fr: gfpl.Frames, seq: int):
        self._c(self.L.gfplo_insert_stereo_pair(self.h, C.byref(fr), seq), "insert")

    def optimizePose(self, DT_ini=None):
        """optimizePose(prev_frame->DT) (Q2), or optimizePose(Matrix4d DT_ini)."""
        if DT_ini is None:
            self._c(self.L.gfplo_optimize_pose(self.h), "optimize_pose")
        else:
            d = np.ascontiguousarray(DT_ini, dtype=np.float64).reshape(16)
            self._c(self.L.gfplo_optimize_pose_ini(self.h, d.ctypes.data), "optimize_pose_ini")

    def updateFrame(self):
        self._c(self.L.gfplo_update_frame(self.h), "update_frame")

    def begin_frame(self, fr: gfpl.Frames, seq: int):
        self._c(self.L.gfplo_begin_frame(self.h, C.byref(fr), seq), "begin_frame")

    def stereoPoints(self):
        self._c(self.L.gfplo_stereo_points(self.h), "stereo_points")

    def stereoLines(self):
        self._c(self.L.gfplo_stereo_lines(self.h), "stereo_lines")

    def estimateStereoUncertainty(self):
        self._c(self.L.gfplo_line_uncertainty(self.h), "line_uncertainty")

    def crossFrameMatchingPoints(self):
        self._c(self.L.gfplo_cross_points(self.h), "cross_points")

    def crossFrameMatchingLines(self):
        self._c(self.L.gfplo_cross_lines(self.h), "cross_lines")

    def estimateProjUncertainty_submodular(self):
        self._c(self.L.gfplo_line_cut(self.h), "line_cut")

    def read_frame(self, which: int) -> gfpl.FrameHost:
        fh = gfpl.FrameHost(self.kp_cap, self.kl_cap)
        self._c(self.L.gfplo_read_frame(self.h, which, fh.ptr()), "read_frame")
        return fh

    def write_frame(self, which: int, fh: gfpl.FrameHost):
        self._c(self.L.gfplo_write_frame(self.h, which, fh.ptr()), "write_frame")

    def read_track(self) -> dict:
        t = gfpl.TrackHost()
        self._c(self.L.gfplo_read_track(self.h, C.byref(t)), "read_track")
        return t.as_dict()

    def write_track(self, tr: gfpl.TrackHost):
        self._c(self.L.gfplo_write_track(self.h, C.byref(tr)), "write_track")

    def needNewKF(self) -> bool:
        f = C.c_int(0)
        self._c(self.L.gfplo_need_new_kf(self.h, C.byref(f)), "need_new_kf")
        return bool(f.value)

    def currFrameIsKF(self):
        self._c(self.L.gfplo_curr_frame_is_kf(self.h), "curr_frame_is_kf")

    def read_kf_state(self) -> dict:
        st = gfpl.KFState()
        self._c(self.L.gfplo_read_kf_state(self.h, C.byref(st)), "read_kf_state")
        return st.as_dict()

    def __del__(self):
        try:
            if self.h:
                self.L.gfplo_destroy(self.h)
                self.h = None
        except Exception:
            pass


# ---- primitives
def kf_common_matches(cam, cfg, kf0: "gfpl.KeyFrameView", kf1: "gfpl.KeyFrameView"):
    """MapHandler::lookForCommonMatches keyframe-pair stage on host views (device=None)."""
    pp = np.zeros((max(kf0.s.n_pt, 1), 2), np.int32)
    lp = np.zeros((max(kf0.s.n_ls, 1), 2), np.int32)
    npt, nls = C.c_int(0), C.c_int(0)
    rc = lib().gfplo_kf_common_matches(C.byref(cam), C.byref(cfg), C.byref(kf0.s), C.byref(kf1.s),
                                       _p(pp), C.byref(npt), _p(lp), C.byref(nls))
    if rc != 0:
        raise RuntimeError(f"gfplo_kf_common_matches -> {rc}")
    return pp[: npt.value].copy(), lp[: nls.value].copy()


def kf_local_map_matches(cam, cfg, local_map: "gfpl.MapView", kf1: "gfpl.KeyFrameView",
                         max_kf_epip_p: float = 1.0, max_kf_epip_l: float = 1.0):
    """lookForCommonMatches local-map stage on host views (device=None)."""
    pp = np.zeros((max(local_map.s.n_pt, 1), 2), np.int32)
    lp = np.zeros((max(local_map.s.n_ls, 1), 2), np.int32)
    npt, nls = C.c_int(0), C.c_int(0)
    rc = lib().gfplo_kf_local_map_matches(C.byref(cam), C.byref(cfg), C.byref(local_map.s), C.byref(kf1.s),
                                          max_kf_epip_p, max_kf_epip_l, _p(pp), C.byref(npt), _p(lp), C.byref(nls))
    if rc != 0:
        raise RuntimeError(f"gfplo_kf_local_map_matches -> {rc}")
    return pp[: npt.value].copy(), lp[: nls.value].copy()


def hamming(a: np.ndarray, b: np.ndarray, cell: int = 1) -> int:
    a = np.ascontiguousarray(a, np.uint8); b = np.ascontiguousarray(b, np.uint8)
    return lib().gfplo_hamming(_p(a), _p(b), cell)


def knn2(q: np.ndarray, t: np.ndarray, cell: int = 1):
    q = np.ascontiguousarray(q, np.uint8); t = np.ascontiguousarray(t, np.uint8)
    idx = np.zeros((len(q), 2), np.int32); dist = np.zeros((len(q), 2), np.float32)
    rc = lib().gfplo_knn2(_p(q), len(q), _p(t), len(t), cell, _p(idx), _p(dist))
    return rc, idx, dist


def radius_match(q, t, max_dist: float, cell: int = 1):
    """BFMatcher::radiusMatch rows: (row_off[nq + 1], train idx, dist) (ledger T1 / T2)."""
    q = np.ascontiguousarray(q, np.uint8).reshape(-1, 32); t = np.ascontiguousarray(t, np.uint8).reshape(-1, 32)
    off = np.zeros(len(q) + 1, np.int32)
    cap = len(q) * len(t)
    idx = np.zeros(max(cap, 1), np.int32); dist = np.zeros(max(cap, 1), np.float32)
    rc = lib().gfplo_radius_match(_p(q), len(q), _p(t), len(t), cell, max_dist, _p(off), cap, _p(idx), _p(dist))
    if rc:
        raise RuntimeError(f"gfplo_radius_match: {rc}")
    return off, idx[: off[-1]], dist[: off[-1]]


def match_stats(kind: int, d0, d1, max_num: int):
    """(nn_mad, nn12_mad, thres_budget) of a knn-2 list: kind 0 point, 1 line."""
    d0 = np.ascontiguousarray(d0, np.float32); d1 = np.ascontiguousarray(d1, np.float32)
    out = np.zeros(3, np.float64)
    rc = lib().gfplo_match_stats(kind, _p(d0), _p(d1), len(d0), max_num, _p(out))
    if rc:
        raise RuntimeError(f"gfplo_match_stats: {rc}")
    return tuple(float(x) for x in out)


def log(x: float) -> float: return lib().gfplo_log(x)
def sin(x: float) -> float: return lib().gfplo_sin(x)
def cos(x: float) -> float: return lib().gfplo_cos(x)


def logdet6(M: np.ndarray) -> float:
    return lib().gfplo_logdet6(_p(np.ascontiguousarray(M, np.float64)))


def ldlt_solve6(H: np.ndarray, g: np.ndarray) -> np.ndarray:
    x = np.zeros(6); H = np.ascontiguousarray(H, np.float64); g = np.ascontiguousarray(g, np.float64)
    lib().gfplo_ldlt_solve6(_p(H), _p(g), _p(x)); return x


def det6(A) -> float:
    return lib().gfplo_det6(_p(np.ascontiguousarray(A, np.float64)))


def inverse6(A):
    o = np.zeros((6, 6)); A = np.ascontiguousarray(A, np.float64); lib().gfplo_inverse6(_p(A), _p(o)); return o


def inverse4(A):
    o = np.zeros((4, 4)); A = np.ascontiguousarray(A, np.float64); lib().gfplo_inverse4(_p(A), _p(o)); return o


def eig_sym(A):
    A = np.ascontiguousarray(A, np.float64); n = A.shape[0]; w = np.zeros(n)
    lib().gfplo_eig_sym(_p(A), n, _p(w)); return w


def expmap_se3(x):
    x = np.ascontiguousarray(x, np.float64); T = np.zeros((4, 4)); lib().gfplo_expmap_se3(_p(x), _p(T)); return T


def inverse_se3(T):
    T = np.ascontiguousarray(T, np.float64); o = np.zeros((4, 4)); lib().gfplo_inverse_se3(_p(T), _p(o)); return o


# ---- ORB extraction (gfpl_orb_oracle.cpp, ledger O1-O7)
def orb_extract(image: np.ndarray, nfeatures: int = 2000, scale_factor: float = 1.2, nlevels: int = 4,
                ini_th: int = 20, min_th: int = 7, kp_cap: int = 0):
    """ORBextractor::operator() on one grey image: dict of keypoints (KEYPOINT_DT), angle,
    response, desc [n][32] and the packed level images."""
    image = np.ascontiguousarray(image, np.uint8)
    h, w = image.shape
    prm = gfpl.OrbParams(nfeatures, scale_factor, nlevels, ini_th, min_th)
    kp_cap = kp_cap or nfeatures + 64 * nlevels + 64
    kps = np.zeros(kp_cap, gfpl.KEYPOINT_DT)
    ang = np.zeros(kp_cap, np.float32); rsp = np.zeros(kp_cap, np.float32)
    desc = np.zeros((kp_cap, 32), np.uint8)
    pyr = np.zeros(w * h * 4, np.uint8)   # sum of 1/scale^2 < 1 / (1 - 1/1.2^2) < 4
    n = C.c_int(0)
    rc = lib().gfplo_orb_extract(C.byref(prm), _p(image), w, h, kp_cap, _p(kps), _p(ang), _p(rsp), _p(desc),
                                 C.byref(n), _p(pyr))
    if rc != 0:
        raise RuntimeError(f"gfplo_orb_extract -> {rc}")
    k = n.value
    return {"kps": kps[:k].copy(), "angle": ang[:k].copy(), "response": rsp[:k].copy(), "desc": desc[:k].copy(),
            "pyramid": pyr}


def orb_resize(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8); d = np.zeros((dh, dw), np.uint8)
    lib().gfplo_orb_resize(_p(src), src.shape[1], src.shape[0], _p(d), dw, dh); return d


def orb_blur(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8); d = np.zeros_like(src)
    lib().gfplo_orb_blur(_p(src), src.shape[1], src.shape[0], _p(d)); return d


def orb_fast(img: np.ndarray, threshold: int, cap: int = 1 << 16) -> np.ndarray:
    """cv::FAST(img, kps, threshold, true): [n][3] (x, y, response) in row-major order."""
    img = np.ascontiguousarray(img, np.uint8); o = np.zeros((cap, 3), np.float32)
    n = lib().gfplo_orb_fast(_p(img), img.shape[1], img.shape[0], threshold, cap, _p(o))
    return o[:min(n, cap)].copy()


def fast_atan2(y: float, x: float) -> float:
    return lib().gfplo_fast_atan2(y, x)


# ---- LBD descriptors (gfpl_lbd_oracle.cpp, ledger L1-L5)
def lbd_compute(image: np.ndarray, keylines: np.ndarray):
    """BinaryDescriptor::compute on one grey image: (desc [n][32] u8, the float LBD [n][72])."""
    image = np.ascontiguousarray(image, np.uint8)
    kl = np.ascontiguousarray(keylines, gfpl.KEYLINE_DT)
    n = len(kl)
    d = np.zeros((max(n, 1), 32), np.uint8)
    f = np.zeros((max(n, 1), 72), np.float32)
    rc = lib().gfplo_lbd_compute(_p(image), image.shape[1], image.shape[0], _p(kl) if n else None, n, _p(d), _p(f))
    if rc != 0:
        raise RuntimeError(f"gfplo_lbd_compute -> {rc}")
    return d[:n].copy(), f[:n].copy()


def lbd_gradients(image: np.ndarray):
    image = np.ascontiguousarray(image, np.uint8)
    h, w = image.shape
    b = np.zeros_like(image); dx = np.zeros((h, w), np.int16); dy = np.zeros((h, w), np.int16)
    lib().gfplo_lbd_gradients(_p(image), w, h, _p(b), _p(dx), _p(dy))
    return b, dx, dy


def lbd_coefs():
    cl = np.zeros(21, np.float32); cg = np.zeros(63, np.float32)
    lib().gfplo_lbd_coefs(_p(cl), _p(cg))
    return cl, cg


def lbd_num_pixels(kl) -> int:
    k = np.ascontiguousarray(np.asarray(kl, gfpl.KEYLINE_DT).reshape(1))
    return lib().gfplo_lbd_num_pixels(_p(k), 0, 0)


# ---- LSD line detection (gfpl_lsd_oracle.cpp, ledger S1-S7)
def lsd_detect(image: np.ndarray, params=None, kl_cap: int = 0, seg_cap: int = 8192):
    """LSDDetectorC::detect + StereoFrame's response filter on one grey image:
    (keylines KEYLINE_DT, response f32, raw segments [n_seg][4] f32)."""
    image = np.ascontiguousarray(image, np.uint8)
    h, w = image.shape
    prm = params if params is not None else gfpl.LsdParams.reference(w, h)
    kl_cap = kl_cap or max(seg_cap, 1)
    kl = np.zeros(kl_cap, gfpl.KEYLINE_DT)
    rsp = np.zeros(kl_cap, np.float32)
    segs = np.zeros((seg_cap, 4), np.float32)
    n = C.c_int(0); ns = C.c_int(0)
    rc = lib().gfplo_lsd_detect(C.byref(prm), _p(image), w, h, kl_cap, _p(kl), _p(rsp), C.byref(n), _p(segs),
                                seg_cap, C.byref(ns))
    if rc != 0:
        raise RuntimeError(f"gfplo_lsd_detect -> {rc}")
    return kl[:n.value].copy(), rsp[:n.value].copy(), segs[:min(ns.value, seg_cap)].copy()


def lsd_constants(width: int, height: int, params=None):
    prm = params if params is not None else gfpl.LsdParams.reference(width, height)
    pr = C.c_double(0); rho = C.c_double(0); mrs = C.c_int(0)
    lib().gfplo_lsd_constants(C.byref(prm), width, height, C.byref(pr), C.byref(rho), C.byref(mrs))
    return pr.value, rho.value, mrs.value


def lsd_defined_count(image: np.ndarray, params=None) -> int:
    """Pixels with a defined level-line angle (ledger S1: norm = sqrt((gx^2 + gy^2) / 4) > rho,
    the last row and column NOTDEF)."""
    im = np.asarray(image, np.int64)
    h, w = im.shape
    _, rho, _ = lsd_constants(w, h, params)
    da = im[1:, 1:] - im[:-1, :-1]
    bc = im[:-1, 1:] - im[1:, :-1]
    gx, gy = da + bc, da - bc
    return int((np.sqrt((gx * gx + gy * gy) / 4.0) > rho).sum())


def atan2(y: float, x: float) -> float:
    return lib().gfplo_atan2(y, x)


def sort_desc(a: np.ndarray) -> np.ndarray:
    """std::sort of u64 elements by descending high 32 bits (ledger S2)."""
    a = np.ascontiguousarray(a, np.uint64).copy()
    lib().gfplo_sort_desc(_p(a), len(a))
    return a
