"""gfpl — Python host side of the MI355X-native GF-PL-SLAM tracking path.

Thin ctypes mirror of ``include/gfpl.h``.  The compute path is the HIP library
``gf-pl-slam_amd/lib/libgfpl_hip.so`` (hand-written gfx950 kernels); this module
only marshals structs and (optionally) torch device buffers.  There is no CPU
fallback: the product classes raise if the HIP library is missing.

The class names mirror the reference's operator interface
(``StVO::StereoFrameHandler`` — include/stereoFrameHandler.h:38-174) so the parity
tests read like the reference's own call sequence (app/plslam_mod.cpp:375-477):
``initialize`` -> ``insertStereoPair`` -> ``optimizePose`` -> ``updateFrame``.
"""
from __future__ import annotations

import ctypes as C
import json
import os
from typing import Optional

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_DIR, "lib")
REPO_DIR = os.path.dirname(PKG_DIR)

DESC = 32
MAX_LEVELS = 8
MAX_MATCHED_PT = 2048
MAX_MATCHED_LS = 1024
PREV, CURR = 0, 1
HAMMING, HAMMING2 = 1, 2

ERRORS = {0: "ok", -1: "invalid argument", -2: "HIP runtime error", -3: "no HIP device",
          -4: "knn-2 needs at least 2 train descriptors", -5: "capacity exceeded",
          -6: "call order violated", -7: "unsupported config"}


class GfplError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        super().__init__(f"{what}: gfpl error {code} ({ERRORS.get(code, '?')})")
        self.code = code


# --------------------------------------------------------------- structs --
class Camera(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int),
                ("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
                ("b", C.c_double), ("n_levels", C.c_int),
                ("scale", C.c_float * MAX_LEVELS), ("inv_scale", C.c_float * MAX_LEVELS),
                ("lvl_cols", C.c_int * MAX_LEVELS), ("lvl_rows", C.c_int * MAX_LEVELS),
                ("lvl_offset", C.c_int64 * MAX_LEVELS), ("pyr_bytes", C.c_int64),
                ("sigma2_pt", C.c_double * MAX_LEVELS), ("sigma2_ln", C.c_double * MAX_LEVELS)]


class Config(C.Structure):
    _fields_ = [("best_lr_matches", C.c_int), ("lr_in_parallel", C.c_int),
                ("use_line_conf_cut", C.c_int), ("cut_with_max_vol", C.c_int),
                ("ratio_disp_std", C.c_double), ("ratio_disp_std_hor", C.c_double),
                ("max_line_match_num", C.c_int), ("max_point_match_num", C.c_int),
                ("max_dist_epip", C.c_double), ("min_disp", C.c_double),
                ("max_ratio_12_p", C.c_double), ("point_match_radius", C.c_double),
                ("stereo_overlap_th", C.c_double), ("line_horiz_th", C.c_double),
                ("desc_th_l", C.c_double), ("line_cov_th", C.c_double),
                ("homog_th", C.c_double), ("min_features", C.c_int),
                ("max_iters", C.c_int), ("max_iters_ref", C.c_int),
                ("min_error", C.c_double), ("min_error_change", C.c_double),
                ("inlier_k", C.c_double), ("motion_step_th", C.c_double),
                ("orb_scale_factor", C.c_double), ("orb_n_levels", C.c_int),
                ("lsd_scale", C.c_double), ("cut_step", C.c_double),
                ("cut_rng", C.c_double * 2), ("proj_gate_px", C.c_double),
                ("min_entropy_ratio", C.c_double), ("max_kf_num_frames", C.c_int),
                ("cut_certify", C.c_double), ("cut_proof", C.c_int)]


KEYPOINT_DT = np.dtype([("x", "<f4"), ("y", "<f4"), ("octave", "<i4")])
# cv::KeyPoint fields ORBextractor::operator() fills (src/ORBextractor.cc:1085-1101)
CV_KEYPOINT_DT = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4")])
KEYLINE_DT = np.dtype([("sx", "<f4"), ("sy", "<f4"), ("ex", "<f4"), ("ey", "<f4"),
                       ("angle", "<f4"), ("octave", "<i4")])

_vp = C.c_void_p


class Frames(C.Structure):
    _fields_ = [("batch", C.c_int), ("kp_cap", C.c_int), ("kl_cap", C.c_int),
                ("n_kp_l", _vp), ("n_kp_r", _vp), ("kp_l", _vp), ("kp_r", _vp),
                ("pdesc_l", _vp), ("pdesc_r", _vp),
                ("n_kl_l", _vp), ("n_kl_r", _vp), ("kl_l", _vp), ("kl_r", _vp),
                ("ldesc_l", _vp), ("ldesc_r", _vp), ("pyr_r", _vp), ("time_stamp", _vp),
                ("ready", _vp), ("consumed", _vp)]


# (name, dtype, per-feature shape) of gfpl_frame_host arrays, in struct order
PT_FIELDS = [("pt_pl", np.float64, (2,)), ("pt_pl_obs", np.float64, (2,)),
             ("pt_disp", np.float64, ()), ("pt_P", np.float64, (3,)),
             ("pt_sigma2", np.float64, ()), ("pt_idx", np.int32, ()),
             ("pt_level", np.int32, ()), ("pt_inlier", np.uint8, ()),
             ("pdesc", np.uint8, (DESC,))]
LS_FIELDS = [("ls_spl", np.float64, (2,)), ("ls_epl", np.float64, (2,)),
             ("ls_spl_obs", np.float64, (2,)), ("ls_epl_obs", np.float64, (2,)),
             ("ls_sdisp", np.float64, ()), ("ls_edisp", np.float64, ()),
             ("ls_sdisp_obs", np.float64, ()), ("ls_edisp_obs", np.float64, ()),
             ("ls_angle", np.float64, ()), ("ls_sigma2", np.float64, ()),
             ("ls_sP", np.float64, (3,)), ("ls_eP", np.float64, (3,)),
             ("ls_le", np.float64, (3,)), ("ls_le_obs", np.float64, (3,)),
             ("ls_covS", np.float64, (9,)), ("ls_covE", np.float64, (9,)),
             ("ls_cut", np.float64, (2,)), ("ls_invcov", np.float64, (36,)),
             ("ls_idx", np.int32, ()), ("ls_level", np.int32, ()),
             ("ls_inlier", np.uint8, ()), ("ldesc", np.uint8, (DESC,))]
POSE_FIELDS = [("Tfw", 16), ("DT", 16), ("DT_cov", 36), ("Tfw_cov", 36), ("DT_cov_eig", 6)]


class FrameHostStruct(C.Structure):
    _fields_ = ([("n_pt", C.c_int), ("n_ls", C.c_int)]
                + [(n, _vp) for n, _, _ in PT_FIELDS]
                + [(n, _vp) for n, _, _ in LS_FIELDS]
                + [(n, C.c_double * k) for n, k in POSE_FIELDS]
                + [("err_norm", C.c_double), ("time_stamp", C.c_double)])


class TrackHost(C.Structure):
    _fields_ = [("n_matched_pt", C.c_int), ("n_matched_ls", C.c_int),
                ("matched_pt", C.c_int32 * MAX_MATCHED_PT),
                ("matched_ls", C.c_int32 * MAX_MATCHED_LS),
                ("n_inliers", C.c_int), ("n_inliers_pt", C.c_int), ("n_inliers_ls", C.c_int),
                ("num_frame_loss", C.c_int)]

    def as_dict(self) -> dict:
        return {"matched_pt": np.array(self.matched_pt[: self.n_matched_pt], dtype=np.int32),
                "matched_ls": np.array(self.matched_ls[: self.n_matched_ls], dtype=np.int32),
                "n_inliers": self.n_inliers, "n_inliers_pt": self.n_inliers_pt,
                "n_inliers_ls": self.n_inliers_ls, "num_frame_loss": self.num_frame_loss}


class KFState(C.Structure):
    """gfpl_kf_state: keyframe-decision state (include/stereoFrameHandler.h:147-153)."""
    _fields_ = [("T_prevKF", C.c_double * 16), ("cov_prevKF_currF", C.c_double * 36),
                ("entropy_first_prevKF", C.c_double), ("entropy_ratio", C.c_double),
                ("prev_f_iskf", C.c_int), ("num_frame_since_kf", C.c_int), ("need_new_kf", C.c_int)]

    def as_dict(self) -> dict:
        return {"T_prevKF": np.array(self.T_prevKF[:]).reshape(4, 4),
                "cov_prevKF_currF": np.array(self.cov_prevKF_currF[:]).reshape(6, 6),
                "entropy_first_prevKF": self.entropy_first_prevKF, "entropy_ratio": self.entropy_ratio,
                "prev_f_iskf": self.prev_f_iskf, "num_frame_since_kf": self.num_frame_since_kf,
                "need_new_kf": self.need_new_kf}


class KFViewStruct(C.Structure):
    """gfpl_kf_view: one keyframe's stereo features (KeyFrame::stereo_frame)."""
    _fields_ = [("n_pt", C.c_int), ("pdesc", _vp), ("P", _vp), ("pl", _vp), ("pt_sigma2", _vp),
                ("n_ls", C.c_int), ("ldesc", _vp), ("sP", _vp), ("eP", _vp), ("le", _vp), ("ls_sigma2", _vp),
                ("T_kf_w", C.c_double * 16)]


KF_PT = [("pdesc", "pdesc"), ("P", "pt_P"), ("pl", "pt_pl"), ("pt_sigma2", "pt_sigma2")]
KF_LS = [("ldesc", "ldesc"), ("sP", "ls_sP"), ("eP", "ls_eP"), ("le", "ls_le"), ("ls_sigma2", "ls_sigma2")]


class KeyFrameView:
    """The arrays of one KeyFrame (src/keyFrame.cpp:26-58) that the keyframe
    consumers read: stereo_pt / stereo_ls rows of a FrameHost and T_kf_w.
    device=None keeps host arrays (oracle); otherwise they are copied to that
    torch device once and stay resident."""

    def __init__(self, fh: "FrameHost", T_kf_w, device=None):
        self.s = KFViewStruct()
        self.s.n_pt, self.s.n_ls = fh.n_pt, fh.n_ls
        self.s.T_kf_w[:] = [float(x) for x in np.asarray(T_kf_w, np.float64).reshape(16)]
        self.keep = {}
        for cf, fn in KF_PT + KF_LS:
            n = fh.n_pt if cf in dict(KF_PT) else fh.n_ls
            a = np.ascontiguousarray(fh.arr[fn][:max(n, 1)])
            if device is not None:
                import torch
                a = torch.from_numpy(a.copy()).to(device)
            self.keep[cf] = a
            setattr(self.s, cf, _ptr(a))


class MapViewStruct(C.Structure):
    """gfpl_map_view: the local map rows lookForCommonMatches' second stage reads."""
    _fields_ = [("n_pt", C.c_int), ("pdesc", _vp), ("P", _vp), ("n_ls", C.c_int), ("ldesc", _vp), ("L", _vp)]


class MapView:
    """Local map points / lines (med_desc row 0, point3D, line3D) as numpy arrays,
    copied to `device` (torch) when given."""

    def __init__(self, pdesc, P, ldesc, L, device=None):
        self.s = MapViewStruct()
        arrs = {"pdesc": np.ascontiguousarray(pdesc, np.uint8).reshape(-1, 32),
                "P": np.ascontiguousarray(P, np.float64).reshape(-1, 3),
                "ldesc": np.ascontiguousarray(ldesc, np.uint8).reshape(-1, 32),
                "L": np.ascontiguousarray(L, np.float64).reshape(-1, 6)}
        self.s.n_pt, self.s.n_ls = len(arrs["pdesc"]), len(arrs["ldesc"])
        self.keep = {}
        for k, a in arrs.items():
            if device is not None:
                import torch
                a = torch.from_numpy(a.copy()).to(device) if a.size else torch.zeros(1, device=device)
            self.keep[k] = a
            setattr(self.s, k, _ptr(a) if (device is not None or a.size) else 0)


class OrbParams(C.Structure):
    """gfpl_orb_params: ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)."""
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int)]


class LsdParams(C.Structure):
    """gfpl_lsd_params: LSDDetectorC::LSDOptions + Config::lsdNFeatures as StereoFrame builds
    them (src/stereoFrame.cpp:1163-1172; defaults src/config.cpp:143-152, min_length =
    Config::minLineLength 0.025 * min(W, H), src/stereoFrame.cpp:151)."""
    _fields_ = [("refine", C.c_int), ("scale", C.c_double), ("quant", C.c_double), ("ang_th", C.c_double),
                ("density_th", C.c_double), ("n_bins", C.c_int), ("min_length", C.c_double),
                ("n_features", C.c_int)]

    @classmethod
    def reference(cls, width: int, height: int, n_features: int = 300, min_line_length: float = 0.025):
        return cls(1, 1.0, 2.0, 22.5, 0.6, 1024, min_line_length * min(width, height), n_features)


class DetectorParams(C.Structure):
    """gfpl_detector_params: the ORB + LSD options StereoFrame's detection runs with
    (src/stereoFrame.cpp:33-36, 1160-1172) and the raw LSD segment capacity."""
    _fields_ = [("orb", OrbParams), ("lsd", LsdParams), ("seg_cap", C.c_int)]

    @classmethod
    def reference(cls, cam: "Camera", cfg: Optional["Config"] = None, nfeatures: Optional[int] = None):
        p = cls()
        check(hiplib().gfpl_detector_params_default(C.byref(cam), C.byref(cfg) if cfg is not None else None,
                                                    C.byref(p)), "detector_params_default")
        if nfeatures is not None:
            p.orb.nfeatures = nfeatures
        return p


class DetectionsHost(C.Structure):
    _fields_ = [("n_kp_l", C.c_int), ("n_kp_r", C.c_int), ("n_kl_l", C.c_int), ("n_kl_r", C.c_int),
                ("kp_l", _vp), ("kp_r", _vp), ("pdesc_l", _vp), ("pdesc_r", _vp),
                ("kl_l", _vp), ("kl_r", _vp), ("ldesc_l", _vp), ("ldesc_r", _vp)]


class SynthParams(C.Structure):
    _fields_ = [("n_kp", C.c_int), ("n_kl", C.c_int), ("n_world_pts", C.c_int),
                ("n_world_lines", C.c_int), ("dt", C.c_double), ("v_fwd", C.c_double),
                ("yaw_rate", C.c_double), ("z_min", C.c_double), ("z_max", C.c_double),
                ("px_noise", C.c_double), ("distractor_frac", C.c_double),
                ("margin", C.c_int), ("seed", C.c_uint64),
                ("traj", _vp), ("n_traj", C.c_int), ("traj_t", _vp), ("respawn", C.c_int),
                ("outlier_frac", C.c_double), ("pyr_from_l0", C.c_int)]


# ------------------------------------------------------------- libraries --
_LIBS: dict = {}


def lib_path(name: str) -> str:
    # GFPL_LIB_DIR: load an alternative in-tree build (kernel experiments in tools/)
    return os.path.join(os.environ.get("GFPL_LIB_DIR", LIB_DIR), name)


def _load(name: str) -> C.CDLL:
    if name not in _LIBS:
        p = lib_path(name)
        if not os.path.exists(p):
            raise GfplError(-3, f"{p} is not built (run __graft_entry__.build())")
        _LIBS[name] = C.CDLL(p)
    return _LIBS[name]


def hiplib() -> C.CDLL:
    """The product library (HIP kernels + C ABI).  Raises if not built.

    torch (when importable) is imported first so the process has ONE HIP
    runtime: torch's libamdhip64 is then what libgfpl_hip.so's NEEDED
    libamdhip64.so.7 resolves to (a second copy loaded under another file name
    would see no devices)."""
    if "libgfpl_hip.so" not in _LIBS:
        try:
            import torch  # noqa: F401
        except Exception:
            pass
    L = _load("libgfpl_hip.so")
    if not getattr(L, "_gfpl_typed", False):
        P = C.c_void_p
        sigs = {
            "gfpl_abi_version": ([], C.c_int),
            "gfpl_config_default": ([P], C.c_int),
            "gfpl_camera_init": ([P, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                  C.c_double, C.c_double, P], C.c_int),
            "gfpl_create": ([C.c_int, P, C.POINTER(P)], C.c_int),
            "gfpl_create_async": ([C.c_int, C.POINTER(P)], C.c_int),
            "gfpl_get_stream": ([P], C.c_void_p),
            "gfpl_event_create": ([P, C.POINTER(P)], C.c_int),
            "gfpl_event_destroy": ([P], C.c_int),
            "gfpl_event_record": ([P, P], C.c_int),
            "gfpl_event_wait": ([P, P], C.c_int),
            "gfpl_event_synchronize": ([P], C.c_int),
            "gfpl_event_record_count": ([P, P], C.c_int),
            "gfpl_orb_extract_async": ([P, P, C.c_int, P, P, P, P, P, P, C.c_int64], C.c_int),
            "gfpl_orb_status": ([P], C.c_int),
            "gfpl_lsd_detect_async": ([P, P, C.c_int, P, P, P], C.c_int),
            "gfpl_lsd_status": ([P], C.c_int),
            "gfpl_lbd_compute_async": ([P, P, C.c_int, P, P, P], C.c_int),
            "gfpl_lbd_status": ([P], C.c_int),
            "gfpl_destroy": ([P], C.c_int),
            "gfpl_set_camera": ([P, P], C.c_int),
            "gfpl_set_config": ([P, P], C.c_int),
            "gfpl_get_camera": ([P, P], C.c_int),
            "gfpl_get_config": ([P, P], C.c_int),
            "gfpl_synchronize": ([P], C.c_int),
            "gfpl_copy_to_host": ([P, P, P, C.c_size_t], C.c_int),
            "gfpl_seqbatch_create": ([P, C.c_int, C.c_int, C.c_int, C.POINTER(P)], C.c_int),
            "gfpl_seqbatch_destroy": ([P], C.c_int),
            "gfpl_seqbatch_bytes": ([P], C.c_int64),
            "gfpl_initialize": ([P, P], C.c_int),
            "gfpl_insert_stereo_pair": ([P, P], C.c_int),
            "gfpl_optimize_pose": ([P], C.c_int),
            "gfpl_optimize_pose_ini": ([P, P], C.c_int),
            "gfpl_update_frame": ([P], C.c_int),
            "gfpl_frame_step": ([P, P], C.c_int),
            "gfpl_upload_frames": ([P, P, P], C.c_int),
            "gfpl_upload_frames_async": ([P, P, C.c_int, C.c_int, P], C.c_int),
            "gfpl_upload_wait": ([P, C.c_int64], C.c_int),
            "gfpl_upload_frames_l0_async": ([P, P, C.c_int, C.c_int, C.c_int64, P], C.c_int),
            "gfpl_staged_frames": ([P, C.c_int, P], C.c_int),
            "gfpl_stereo_points": ([P, P], C.c_int),
            "gfpl_stereo_lines": ([P, P], C.c_int),
            "gfpl_line_uncertainty": ([P], C.c_int),
            "gfpl_cross_points": ([P], C.c_int),
            "gfpl_cross_lines": ([P], C.c_int),
            "gfpl_line_cut": ([P], C.c_int),
            "gfpl_knn2_hamming": ([P, P, C.c_int, P, C.c_int, C.c_int, P, P], C.c_int),
            "gfpl_kf_common_matches": ([P, P, P, P, P, P, P], C.c_int),
            "gfpl_kf_local_map_matches": ([P, P, P, C.c_double, C.c_double, P, P, P, P], C.c_int),
            "gfpl_read_frame": ([P, C.c_int, C.c_int, P], C.c_int),
            "gfpl_write_frame": ([P, C.c_int, C.c_int, P], C.c_int),
            "gfpl_read_track": ([P, C.c_int, P], C.c_int),
            "gfpl_read_last_track": ([P, C.c_int, P], C.c_int),
            "gfpl_need_new_kf": ([P, P], C.c_int),
            "gfpl_curr_frame_is_kf": ([P, P], C.c_int),
            "gfpl_read_kf_state": ([P, C.c_int, P], C.c_int),
            "gfpl_write_track": ([P, C.c_int, P], C.c_int),
            "gfpl_set_timing": ([P, C.c_int], C.c_int),
            "gfpl_get_stage_times": ([P, P], C.c_int),
            "gfpl_get_kernel_times": ([P, P], C.c_int),
            "gfpl_last_step_kernel_bytes": ([P, P], C.c_int),
            "gfpl_last_step_bytes": ([P, P], C.c_int),
            "gfpl_last_step_stage_bytes": ([P, P], C.c_int),
            "gfpl_last_step_counts": ([P, P], C.c_int),
            "gfpl_last_step_track_counts": ([P, P], C.c_int),
            "gfpl_last_step_cut_proof": ([P, P], C.c_int),
            "gfpl_debug_cut_records": ([P, C.c_int, P, C.c_int], C.c_int),
            "gfpl_debug_step_records": ([P, P], C.c_int),
            "gfpl_debug_clocks": ([P, P], C.c_int),
            "gfpl_lsd_create": ([P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(P)], C.c_int),
            "gfpl_lsd_destroy": ([P], C.c_int),
            "gfpl_lsd_detect": ([P, P, C.c_int, P, P, P], C.c_int),
            "gfpl_lsd_sort_desc": ([P, P, C.c_int], C.c_int),
            "gfpl_strerror": ([C.c_int], C.c_char_p),
            "gfpl_orb_create": ([P, C.c_int, C.c_int, P, C.c_int, C.c_int, C.POINTER(P)], C.c_int),
            "gfpl_orb_destroy": ([P], C.c_int),
            "gfpl_orb_pyramid_bytes": ([P, P], C.c_int),
            "gfpl_orb_extract": ([P, P, C.c_int, P, P, P, P, P, P, C.c_int64], C.c_int),
            "gfpl_lbd_create": ([P, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(P)], C.c_int),
            "gfpl_lbd_destroy": ([P], C.c_int),
            "gfpl_lbd_compute": ([P, P, C.c_int, P, P, P], C.c_int),
            "gfpl_lbd_gradients": ([P, P, P], C.c_int),
            "gfpl_detector_params_default": ([P, P, P], C.c_int),
            "gfpl_detector_create": ([P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(P)], C.c_int),
            "gfpl_detector_destroy": ([P], C.c_int),
            "gfpl_detect_stereo_async": ([P, P, P, C.c_int, P, P], C.c_int),
            "gfpl_detect_stereo_host": ([P, P, P, C.c_int, P, P], C.c_int),
            "gfpl_detect_stereo": ([P, P, P, C.c_int, P, C.c_int, P], C.c_int),
            "gfpl_detector_status": ([P], C.c_int),
            "gfpl_detector_discard": ([P, P], C.c_int),
            "gfpl_read_detections": ([P, P, C.c_int, P], C.c_int),
        }
        for n, (a, r) in sigs.items():
            try:
                f = getattr(L, n)
            except AttributeError:   # partial builds: the missing entry point fails when called
                continue
            f.argtypes = a
            f.restype = r
        L._gfpl_typed = True
    return L


def synthlib() -> C.CDLL:
    L = _load("libgfpl_synth.so")
    if not getattr(L, "_gfpl_typed", False):
        P = C.c_void_p
        L.gfpl_synth_default.argtypes = [P]
        L.gfpl_synth_default.restype = None
        L.gfpl_synth_batch.argtypes = ([P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
                                       + [P] * 14 + [C.c_int])
        L.gfpl_synth_batch.restype = C.c_int
        L.gfpl_synth_image.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, P]
        L.gfpl_synth_image.restype = C.c_int
        L.gfpl_synth_frame_ex.argtypes = [P, P, C.c_int, C.c_int, C.c_int, C.c_int] + [P] * 16
        L.gfpl_synth_frame_ex.restype = C.c_int
        L._gfpl_typed = True
    return L


def check(code: int, what: str = "") -> None:
    if code != 0:
        raise GfplError(code, what)


# ------------------------------------------------------------ parameters --
def default_config(**over) -> Config:
    cfg = Config()
    check(hiplib().gfpl_config_default(C.byref(cfg)), "config_default")
    for k, v in over.items():
        setattr(cfg, k, v)
    return cfg


# Cameras of the BASELINE configs (intrinsics from the reference's YAMLs).
CAMERAS = {
    # config/gazebo_params.yaml:2,8-11 — the reference's synthetic VGA rig (cfg 2)
    "vga": dict(width=640, height=480, fx=554.25626, fy=554.25626, cx=320.0, cy=240.0, b=0.1),
    # config/euroc_params.yaml:2,8-11 (raw left K; cfg 1 and 4)
    "euroc": dict(width=752, height=480, fx=458.654, fy=457.296, cx=367.215, cy=248.375, b=0.110077842),
    # config/kitti/kitti00-02.yaml:2-13 (cfg 3)
    "kitti": dict(width=1241, height=376, fx=718.856, fy=718.856, cx=607.1928, cy=185.2157, b=0.537165719),
    # gazebo x3 (cfg 5 stress)
    "stress": dict(width=1920, height=1080, fx=1662.76878, fy=1662.76878, cx=960.0, cy=540.0, b=0.1),
}


EUROC_SEQS = ["mh_01", "mh_02", "mh_03", "mh_04", "mh_05", "v1_01", "v1_02", "v1_03"]


EUROC_MAX_POSES = 512


def euroc_traj(seq: str = "mh_01", n: int = 64):
    """First n ground-truth camera poses (3x4 row-major T_w<-c) and timestamps [s] of a
    EuRoC sequence, from the reference's config/asl/gt-ass/<seq> files (data/euroc_gt.npz,
    the first 512 poses of each; tests/golden/make_euroc_fixture.py).  n beyond the stored
    poses raises: the generator never wraps a trajectory around."""
    if n > EUROC_MAX_POSES:
        raise ValueError(f"euroc_traj: {n} poses requested, {EUROC_MAX_POSES} stored for {seq}")
    with np.load(os.path.join(os.path.dirname(LIB_DIR), "data", "euroc_gt.npz")) as d:
        T = np.ascontiguousarray(d[seq + "_T"][:n])
        t = np.ascontiguousarray(d[seq + "_t"][:n])
    return T, t


def make_camera(name: str = "vga", cfg: Optional[Config] = None, **over) -> Camera:
    p = dict(CAMERAS[name])
    p.update(over)
    cfg = cfg or default_config()
    cam = Camera()
    check(hiplib().gfpl_camera_init(C.byref(cam), p["width"], p["height"], p["fx"], p["fy"],
                                    p["cx"], p["cy"], p["b"], C.byref(cfg)), "camera_init")
    return cam


def synth_image(seq: int, frame: int, width: int, height: int, seed: int = 0x6A09E667) -> np.ndarray:
    """A synthetic grey image [height][width] u8 (gfpl_synth_image: shapes on a gradient +
    noise), deterministic in (seed, seq, frame)."""
    out = np.zeros((height, width), np.uint8)
    check(synthlib().gfpl_synth_image(seed, seq, frame, width, height, out.ctypes.data), "synth_image")
    return out


def synth_keylines(n: int, w: int, h: int, seed: int, min_len: float = 2.0, max_len: float = 200.0,
                   border: bool = False) -> np.ndarray:
    """n synthetic octave-0 keylines (KEYLINE_DT) inside a w x h image: fractional endpoints,
    the LSD wrapper's angle = atan2(ey - sy, ex - sx) in float (src/LSDDetector_custom.cpp:285);
    border=True clamps the far endpoint onto the image edge."""
    rng = np.random.default_rng(seed)
    kl = np.zeros(n, KEYLINE_DT)
    for i in range(n):
        while True:
            sx, sy = rng.uniform(0, w - 1), rng.uniform(0, h - 1)
            a = rng.uniform(-np.pi, np.pi)
            ln = rng.uniform(min_len, max_len)
            ex, ey = sx + ln * np.cos(a), sy + ln * np.sin(a)
            if border:
                ex, ey = min(max(ex, 0.0), w - 1.0), min(max(ey, 0.0), h - 1.0)
            if 0 <= ex <= w - 1 and 0 <= ey <= h - 1:
                break
        fs, fe = np.float32(sx), np.float32(sy)
        gx, gy = np.float32(ex), np.float32(ey)
        kl[i] = (fs, fe, gx, gy, np.arctan2(gy - fe, gx - fs).astype(np.float32), 0)
    return kl


def synth_true_counts(cam: Camera, sp: SynthParams, seq: int, frame: int, kp_cap: int = 0, kl_cap: int = 0):
    """(true keypoints, true keylines) per side in frame `frame` of sequence `seq`: the
    detections that observe a landmark / 3-D segment (the rest are distractors)."""
    kp_cap, kl_cap = kp_cap or sp.n_kp, kl_cap or sp.n_kl
    n = np.zeros(6, np.int32)
    kp = np.zeros((2, kp_cap), KEYPOINT_DT)
    kl = np.zeros((2, kl_cap), KEYLINE_DT)
    pd = np.zeros((2, kp_cap, DESC), np.uint8)
    ld = np.zeros((2, kl_cap, DESC), np.uint8)
    pyr = np.zeros(cam.pyr_bytes, np.uint8)
    ts = np.zeros(1, np.float64)
    nt = np.zeros(2, np.int32)
    a = n.ctypes.data
    check(synthlib().gfpl_synth_frame_ex(C.byref(sp), C.byref(cam), seq, frame, kp_cap, kl_cap, a, a + 4,
                                         kp[0].ctypes.data, kp[1].ctypes.data, pd[0].ctypes.data, pd[1].ctypes.data,
                                         a + 8, a + 12, kl[0].ctypes.data, kl[1].ctypes.data, ld[0].ctypes.data,
                                         ld[1].ctypes.data, pyr.ctypes.data, ts.ctypes.data, None, nt.ctypes.data),
          "synth_frame_ex")
    return int(nt[0]), int(nt[1])


def synth_params(**over) -> SynthParams:
    sp = SynthParams()
    synthlib().gfpl_synth_default(C.byref(sp))
    for k, v in over.items():
        setattr(sp, k, v)
    return sp


def _ptr(a) -> int:
    if a is None:
        return 0
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())   # torch tensor


# ----------------------------------------------------- synthetic batches --
class HostFrames:
    """Synthetic input frames on the host: arrays [F][B][cap] (numpy)."""

    def __init__(self, cam: Camera, sp: SynthParams, n_seq: int, n_frames: int,
                 kp_cap: int, kl_cap: int, seq0: int = 0, frame0: int = 0, threads: int = 0):
        self.cam, self.sp = cam, sp
        self.B, self.F, self.kp_cap, self.kl_cap = n_seq, n_frames, kp_cap, kl_cap
        F, B = n_frames, n_seq
        self.n_kp_l = np.zeros((F, B), np.int32)
        self.n_kp_r = np.zeros((F, B), np.int32)
        self.kp_l = np.zeros((F, B, kp_cap), KEYPOINT_DT)
        self.kp_r = np.zeros((F, B, kp_cap), KEYPOINT_DT)
        self.pdesc_l = np.zeros((F, B, kp_cap, DESC), np.uint8)
        self.pdesc_r = np.zeros((F, B, kp_cap, DESC), np.uint8)
        self.n_kl_l = np.zeros((F, B), np.int32)
        self.n_kl_r = np.zeros((F, B), np.int32)
        self.kl_l = np.zeros((F, B, kl_cap), KEYLINE_DT)
        self.kl_r = np.zeros((F, B, kl_cap), KEYLINE_DT)
        self.ldesc_l = np.zeros((F, B, kl_cap, DESC), np.uint8)
        self.ldesc_r = np.zeros((F, B, kl_cap, DESC), np.uint8)
        self.pyr_r = np.zeros((F, B, cam.pyr_bytes), np.uint8)
        self.time_stamp = np.zeros((F, B), np.float64)
        threads = threads or min(16, os.cpu_count() or 1)
        check(synthlib().gfpl_synth_batch(
            C.byref(sp), C.byref(cam), seq0, B, frame0, F, kp_cap, kl_cap,
            *[_ptr(a) for a in self.arrays()], threads), "synth_batch")

    def arrays(self):
        return [self.n_kp_l, self.n_kp_r, self.kp_l, self.kp_r, self.pdesc_l, self.pdesc_r,
                self.n_kl_l, self.n_kl_r, self.kl_l, self.kl_r, self.ldesc_l, self.ldesc_r,
                self.pyr_r, self.time_stamp]

    def frames(self, f: int) -> Frames:
        """gfpl_frames with HOST pointers for frame f (what the oracle reads)."""
        a = [x[f] for x in self.arrays()]
        return make_frames(self.B, self.kp_cap, self.kl_cap, a)


class HostBatch:
    """One input frame of B sequences in host memory, refilled in place frame by frame
    (the bench's input ring: generate on the host, upload with gfpl_upload_frames).
    pinned=True page-locks the buffers (torch pinned memory) so the upload runs at the
    PCIe DMA rate."""

    def __init__(self, cam: Camera, sp: SynthParams, n_seq: int, kp_cap: int, kl_cap: int,
                 seq0: int = 0, pinned: bool = False):
        self.cam, self.sp, self.B, self.kp_cap, self.kl_cap, self.seq0 = cam, sp, n_seq, kp_cap, kl_cap, seq0
        B = n_seq
        spec = [((B,), np.int32), ((B,), np.int32), ((B, kp_cap), KEYPOINT_DT), ((B, kp_cap), KEYPOINT_DT),
                ((B, kp_cap, DESC), np.uint8), ((B, kp_cap, DESC), np.uint8),
                ((B,), np.int32), ((B,), np.int32), ((B, kl_cap), KEYLINE_DT), ((B, kl_cap), KEYLINE_DT),
                ((B, kl_cap, DESC), np.uint8), ((B, kl_cap, DESC), np.uint8),
                ((B, cam.pyr_bytes), np.uint8), ((B,), np.float64)]
        self._keep, self._arrs = [], []
        for shape, dt in spec:
            dt = np.dtype(dt)
            n = int(np.prod(shape)) * dt.itemsize
            if pinned:
                import torch
                t = torch.empty(n, dtype=torch.uint8, pin_memory=True)
                self._keep.append(t)
                a = t.numpy().view(dt).reshape(shape)
            else:
                a = np.zeros(shape, dt)
            self._arrs.append(a)
        self.frame_idx = -1

    def arrays(self):
        return self._arrs

    def fill(self, frame_idx: int, threads: int = 0, seq0: Optional[int] = None, n: Optional[int] = None):
        """Generate frame `frame_idx` of sequences [seq0, seq0 + n) (gfpl_synth_batch) into
        the first n rows (default: the batch's own seq0 and all B rows)."""
        threads = threads or min(16, os.cpu_count() or 1)
        seq0 = self.seq0 if seq0 is None else seq0
        n = self.B if n is None else n
        if not 0 < n <= self.B:
            raise ValueError(f"fill: {n} sequences into a batch of {self.B}")
        check(synthlib().gfpl_synth_batch(
            C.byref(self.sp), C.byref(self.cam), seq0, n, frame_idx, 1, self.kp_cap, self.kl_cap,
            *[_ptr(a) for a in self._arrs], threads), "synth_batch")
        self.frame_idx, self.n = frame_idx, n

    def frames(self, n: Optional[int] = None) -> Frames:
        """gfpl_frames (HOST pointers) of the first n rows (default all B)."""
        n = self.B if n is None else n
        return make_frames(n, self.kp_cap, self.kl_cap, [a[:n] for a in self._arrs])

    def nbytes(self) -> int:
        return sum(a.nbytes for a in self._arrs)


def make_frames(B: int, kp_cap: int, kl_cap: int, arrs) -> Frames:
    fr = Frames()
    fr.batch, fr.kp_cap, fr.kl_cap = B, kp_cap, kl_cap
    names = ["n_kp_l", "n_kp_r", "kp_l", "kp_r", "pdesc_l", "pdesc_r", "n_kl_l", "n_kl_r",
             "kl_l", "kl_r", "ldesc_l", "ldesc_r", "pyr_r", "time_stamp"]
    for n, a in zip(names, arrs):
        setattr(fr, n, _ptr(a))
    fr._keep = list(arrs)   # keep buffers alive
    return fr


def input_bytes_per_frame(cam: Camera, kp_cap: int, kl_cap: int) -> int:
    """Bytes of one sequence's input frame in the [B][cap] layout."""
    return (2 * 4 + 2 * kp_cap * (KEYPOINT_DT.itemsize + DESC) + 2 * 4 + 2 * kl_cap * (KEYLINE_DT.itemsize + DESC)
            + cam.pyr_bytes + 8)


class DeviceFrames:
    """Input frames resident in HBM (torch uint8 buffers), one gfpl_frames per frame."""

    def __init__(self, host: HostFrames = None, device: str = "cuda"):
        self.bufs = []
        if host is None:
            return
        import torch
        self.B, self.kp_cap, self.kl_cap = host.B, host.kp_cap, host.kl_cap
        for a in host.arrays():
            t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(a.shape[0], -1))
            self.bufs.append(t.to(device))

    @classmethod
    def generate(cls, cam: Camera, sp: SynthParams, n_seq: int, n_frames: int, kp_cap: int, kl_cap: int,
                 seq0: int = 0, device="cuda", threads: int = 0) -> "DeviceFrames":
        """Generate frame by frame on the host and stage each into HBM, so host memory
        holds one frame of the batch at a time (frames are independent given the
        sequence seed, gfpl_synth)."""
        import torch
        d = cls(None)
        d.B, d.kp_cap, d.kl_cap = n_seq, kp_cap, kl_cap
        for f in range(n_frames):
            h = HostFrames(cam, sp, n_seq, 1, kp_cap, kl_cap, seq0=seq0, frame0=f, threads=threads)
            arrs = h.arrays()
            if not d.bufs:
                d.bufs = [torch.empty((n_frames, a[0].nbytes), dtype=torch.uint8, device=device) for a in arrs]
            for buf, a in zip(d.bufs, arrs):
                buf[f].copy_(torch.from_numpy(np.ascontiguousarray(a[0]).view(np.uint8).reshape(-1)))
            del h
        return d

    def frames(self, f: int) -> Frames:
        arrs = [b[f] for b in self.bufs]
        return make_frames(self.B, self.kp_cap, self.kl_cap, arrs)

    def frames_slice(self, f: int, s0: int, n: int) -> Frames:
        """Frame f of sequences [s0, s0 + n) (a view: every field is [B][...] row-major)."""
        if s0 < 0 or n <= 0 or s0 + n > self.B:
            raise ValueError(f"sequence slice [{s0}, {s0 + n}) outside [0, {self.B})")
        arrs = [b[f].view(self.B, -1)[s0:s0 + n] for b in self.bufs]
        return make_frames(n, self.kp_cap, self.kl_cap, arrs)

    def nbytes(self) -> int:
        return sum(b.numel() for b in self.bufs)


# ----------------------------------------------------------- frame state --
class FrameHost:
    """numpy-backed gfpl_frame_host (one sequence's frame state)."""

    def __init__(self, kp_cap: int, kl_cap: int):
        self.kp_cap, self.kl_cap = kp_cap, kl_cap
        self.s = FrameHostStruct()
        self.arr = {}
        for n, dt, sh in PT_FIELDS:
            self.arr[n] = np.zeros((kp_cap,) + sh, dt)
            setattr(self.s, n, self.arr[n].ctypes.data)
        for n, dt, sh in LS_FIELDS:
            self.arr[n] = np.zeros((kl_cap,) + sh, dt)
            setattr(self.s, n, self.arr[n].ctypes.data)

    @property
    def n_pt(self) -> int:
        return self.s.n_pt

    @property
    def n_ls(self) -> int:
        return self.s.n_ls

    def get(self, name: str) -> np.ndarray:
        if name in self.arr:
            n = self.s.n_pt if name.startswith("pt_") or name == "pdesc" else self.s.n_ls
            return self.arr[name][:n]
        if name in ("err_norm", "time_stamp"):
            return np.array(getattr(self.s, name))
        k = dict(POSE_FIELDS)[name]
        v = np.ctypeslib.as_array(getattr(self.s, name))[:k].copy()
        return v.reshape(4, 4) if k == 16 else v.reshape(6, 6) if k == 36 else v

    def pose(self) -> dict:
        return {n: self.get(n) for n, _ in POSE_FIELDS} | {"err_norm": float(self.s.err_norm)}

    def ptr(self):
        return C.byref(self.s)


# ---------------------------------------------------------- GPU handles --
class Context:
    """gfpl_ctx: one HIP device + stream + camera + config.  stream: a hipStream_t handle
    (0 = the default stream); own_stream=True gives the context its own non-blocking stream
    (gfpl_create_async), e.g. for detection beside a tracking context."""

    def __init__(self, cam: Camera, cfg: Config, device: int = 0, stream: int = 0, own_stream: bool = False):
        self.L = hiplib()
        h = C.c_void_p()
        if own_stream:
            check(self.L.gfpl_create_async(device, C.byref(h)), "gfpl_create_async")
        else:
            check(self.L.gfpl_create(device, C.c_void_p(stream), C.byref(h)), "gfpl_create")
        self.h = h
        self.device = device
        check(self.L.gfpl_set_camera(h, C.byref(cam)), "set_camera")
        check(self.L.gfpl_set_config(h, C.byref(cfg)), "set_config")
        self.cam, self.cfg = cam, cfg

    def synchronize(self):
        check(self.L.gfpl_synchronize(self.h), "synchronize")

    @property
    def stream(self) -> int:
        """the hipStream_t handle the context enqueues on (0: the default stream)"""
        return int(self.L.gfpl_get_stream(self.h) or 0)

    def torch_stream(self):
        """the context's stream as a torch stream (torch work ordered with the gfpl calls)"""
        import torch
        dev = torch.device("cuda", self.device)
        return torch.cuda.ExternalStream(self.stream, device=dev) if self.stream else torch.cuda.default_stream(dev)

    def set_config(self, cfg: Config):
        """gfpl_set_config between steps (e.g. the line cut's proof mode); the context keeps a copy."""
        check(self.L.gfpl_set_config(self.h, C.byref(cfg)), "set_config")
        self.cfg = cfg

    def set_timing(self, on: bool):
        check(self.L.gfpl_set_timing(self.h, int(on)), "set_timing")

    def stage_times(self) -> np.ndarray:
        out = np.zeros(7, np.float32)
        check(self.L.gfpl_get_stage_times(self.h, out.ctypes.data), "stage_times")
        return out

    def kernel_times(self) -> np.ndarray:
        """[k_cut_prep, k_cut_search, k_cut_finish, k_pose] device ms of the last step."""
        out = np.zeros(4, np.float32)
        check(self.L.gfpl_get_kernel_times(self.h, out.ctypes.data), "kernel_times")
        return out

    def knn2(self, q_dev, nq: int, t_dev, nt: int, cell: int, idx_dev, dist_dev) -> int:
        return self.L.gfpl_knn2_hamming(self.h, _ptr(q_dev), nq, _ptr(t_dev), nt, cell,
                                        _ptr(idx_dev), _ptr(dist_dev))

    def lookForCommonMatches(self, kf0: KeyFrameView, kf1: KeyFrameView):
        """MapHandler::lookForCommonMatches keyframe-pair stage (src/mapHandler.cpp:199-470):
        the accepted (kf0 row, kf1 row) point and line pairs, in the order the reference's
        loops visit them; the map bookkeeping stays with the caller."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        pp = torch.zeros(2 * max(kf0.s.n_pt, 1), dtype=torch.int32, device=dev)
        lp = torch.zeros(2 * max(kf0.s.n_ls, 1), dtype=torch.int32, device=dev)
        npt, nls = C.c_int(0), C.c_int(0)
        torch.cuda.synchronize()
        check(self.L.gfpl_kf_common_matches(self.h, C.byref(kf0.s), C.byref(kf1.s), _ptr(pp), C.byref(npt),
                                            _ptr(lp), C.byref(nls)), "kf_common_matches")
        return (pp[: 2 * npt.value].cpu().numpy().reshape(-1, 2),
                lp[: 2 * nls.value].cpu().numpy().reshape(-1, 2))

    def lookForLocalMapMatches(self, local_map: MapView, kf1_unmatched: KeyFrameView,
                               max_kf_epip_p: float = 1.0, max_kf_epip_l: float = 1.0):
        """lookForCommonMatches local-map stage (src/mapHandler.cpp:472-772): (map row,
        kf1 unmatched row) point and line pairs in the reference's loop order."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        pp = torch.zeros(2 * max(local_map.s.n_pt, 1), dtype=torch.int32, device=dev)
        lp = torch.zeros(2 * max(local_map.s.n_ls, 1), dtype=torch.int32, device=dev)
        npt, nls = C.c_int(0), C.c_int(0)
        torch.cuda.synchronize()
        check(self.L.gfpl_kf_local_map_matches(self.h, C.byref(local_map.s), C.byref(kf1_unmatched.s),
                                               max_kf_epip_p, max_kf_epip_l, _ptr(pp), C.byref(npt),
                                               _ptr(lp), C.byref(nls)), "kf_local_map_matches")
        return (pp[: 2 * npt.value].cpu().numpy().reshape(-1, 2),
                lp[: 2 * nls.value].cpu().numpy().reshape(-1, 2))

    def close(self):
        """gfpl_destroy.  Refused (GfplError, the handle kept) while a StereoFrameHandler
        created on this context is still open: close those first."""
        if getattr(self, "h", None):
            check(self.L.gfpl_destroy(self.h), "gfpl_destroy (close the StereoFrameHandlers of this context first)")
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Event:
    """gfpl_event: record on one context's stream, make another context's stream wait."""

    def __init__(self, ctx: Context):
        self.L = ctx.L
        h = C.c_void_p()
        check(self.L.gfpl_event_create(ctx.h, C.byref(h)), "gfpl_event_create")
        self.h = h

    def record(self, ctx: Context):
        check(self.L.gfpl_event_record(self.h, ctx.h), "gfpl_event_record")

    def wait(self, ctx: Context):
        """ctx's stream waits for the last record"""
        check(self.L.gfpl_event_wait(ctx.h, self.h), "gfpl_event_wait")

    def synchronize(self):
        check(self.L.gfpl_event_synchronize(self.h), "gfpl_event_synchronize")

    @property
    def record_count(self) -> int:
        """records so far (gfpl_event_record, or a tracker call's gfpl_frames.consumed mark)"""
        n = C.c_int64(0)
        check(self.L.gfpl_event_record_count(self.h, C.byref(n)), "gfpl_event_record_count")
        return n.value

    def close(self):
        if getattr(self, "h", None):
            self.L.gfpl_event_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class StereoFrameHandler:
    """B independent StVO::StereoFrameHandler objects resident on one GPU.

    Method names follow include/stereoFrameHandler.h:38-174."""

    def __init__(self, ctx: Context, batch: int, kp_cap: int, kl_cap: int):
        self.ctx, self.L = ctx, ctx.L
        h = C.c_void_p()
        check(self.L.gfpl_seqbatch_create(ctx.h, batch, kp_cap, kl_cap, C.byref(h)), "seqbatch_create")
        self.h = h
        self.B, self.kp_cap, self.kl_cap = batch, kp_cap, kl_cap

    def initialize(self, fr: Frames):
        check(self.L.gfpl_initialize(self.h, C.byref(fr)), "initialize")

    def insertStereoPair(self, fr: Frames):
        check(self.L.gfpl_insert_stereo_pair(self.h, C.byref(fr)), "insert_stereo_pair")

    def optimizePose(self, DT_ini=None):
        """optimizePose(prev_frame->DT) (the app's call, Q2), or optimizePose(Matrix4d DT_ini)
        with DT_ini a 4x4 (all sequences) or [B,4,4] host array."""
        if DT_ini is None:
            check(self.L.gfpl_optimize_pose(self.h), "optimize_pose")
            return
        d = np.asarray(DT_ini, dtype=np.float64)
        d = np.ascontiguousarray(np.broadcast_to(d.reshape(-1, 4, 4), (self.B, 4, 4)))
        check(self.L.gfpl_optimize_pose_ini(self.h, d.ctypes.data), "optimize_pose_ini")

    def updateFrame(self):
        check(self.L.gfpl_update_frame(self.h), "update_frame")

    def frameStep(self, fr: Frames):
        check(self.L.gfpl_frame_step(self.h, C.byref(fr)), "frame_step")

    # stage entry points
    def stereoPoints(self, fr: Frames):
        check(self.L.gfpl_stereo_points(self.h, C.byref(fr)), "stereo_points")

    def stereoLines(self, fr: Frames):
        check(self.L.gfpl_stereo_lines(self.h, C.byref(fr)), "stereo_lines")

    def estimateStereoUncertainty(self):
        check(self.L.gfpl_line_uncertainty(self.h), "line_uncertainty")

    def crossFrameMatchingPoints(self):
        check(self.L.gfpl_cross_points(self.h), "cross_points")

    def crossFrameMatchingLines(self):
        check(self.L.gfpl_cross_lines(self.h), "cross_lines")

    def estimateProjUncertainty_submodular(self):
        check(self.L.gfpl_line_cut(self.h), "line_cut")

    # state transfer
    def upload_frames(self, host: Frames) -> Frames:
        """gfpl_upload_frames: copy one batch of HOST input frames into the seqbatch's
        device staging area (synchronous, PCIe) and return its device view."""
        dev = Frames()
        check(self.L.gfpl_upload_frames(self.h, C.byref(host), C.byref(dev)), "upload_frames")
        dev._keep = [host]
        return dev

    def upload_async(self, host: Frames, s0: int, slot: int, l0_stride: int = 0) -> int:
        """gfpl_upload_frames_async: enqueue the copy of host.batch sequences of HOST frames
        into sequences [s0, s0 + host.batch) of staging buffer `slot` on the seqbatch's copy
        stream; returns the ticket for upload_wait (host memory untouched until then).
        l0_stride > 0 (gfpl_upload_frames_l0_async): only level 0 of each right pyramid is
        copied (rows l0_stride bytes apart) and the device builds levels 1.. from it."""
        t = C.c_int64()
        if l0_stride > 0:
            check(self.L.gfpl_upload_frames_l0_async(self.h, C.byref(host), s0, slot, l0_stride, C.byref(t)),
                  "upload_frames_l0_async")
        else:
            check(self.L.gfpl_upload_frames_async(self.h, C.byref(host), s0, slot, C.byref(t)), "upload_frames_async")
        return t.value

    def upload_wait(self, ticket: int):
        check(self.L.gfpl_upload_wait(self.h, ticket), "upload_wait")

    def staged_frames(self, slot: int) -> Frames:
        """Device view of staging buffer `slot` (every tracker call reading it waits for its copies)."""
        dev = Frames()
        check(self.L.gfpl_staged_frames(self.h, slot, C.byref(dev)), "staged_frames")
        return dev

    def read_frame(self, which: int, seq: int) -> FrameHost:
        fh = FrameHost(self.kp_cap, self.kl_cap)
        check(self.L.gfpl_read_frame(self.h, which, seq, fh.ptr()), "read_frame")
        return fh

    def write_frame(self, which: int, seq: int, fh: FrameHost):
        check(self.L.gfpl_write_frame(self.h, which, seq, fh.ptr()), "write_frame")

    def read_track(self, seq: int) -> dict:
        t = TrackHost()
        check(self.L.gfpl_read_track(self.h, seq, C.byref(t)), "read_track")
        return t.as_dict()

    def read_last_track(self, seq: int) -> dict:
        """The track of the step before the last updateFrame / frameStep: the matched lists
        it cleared and the inlier counters (gfpl_read_last_track)."""
        t = TrackHost()
        check(self.L.gfpl_read_last_track(self.h, seq, C.byref(t)), "read_last_track")
        return t.as_dict()

    # keyframe decision (src/stereoFrameHandler.cpp:2309-2379)
    def needNewKF(self) -> np.ndarray:
        """needNewKF() of every sequence; returns the [B] decisions (bool)."""
        flags = np.zeros(self.B, np.int32)
        check(self.L.gfpl_need_new_kf(self.h, flags.ctypes.data), "need_new_kf")
        return flags.astype(bool)

    def currFrameIsKF(self, mask=None):
        """currFrameIsKF() for the sequences where mask is true (None: the last
        needNewKF decisions)."""
        if mask is None:
            check(self.L.gfpl_curr_frame_is_kf(self.h, None), "curr_frame_is_kf")
            return
        m = np.ascontiguousarray(np.broadcast_to(np.asarray(mask), (self.B,)), dtype=np.int32)
        check(self.L.gfpl_curr_frame_is_kf(self.h, m.ctypes.data), "curr_frame_is_kf")

    def read_kf_state(self, seq: int) -> dict:
        st = KFState()
        check(self.L.gfpl_read_kf_state(self.h, seq, C.byref(st)), "read_kf_state")
        return st.as_dict()

    def write_track(self, seq: int, tr: TrackHost):
        check(self.L.gfpl_write_track(self.h, seq, C.byref(tr)), "write_track")

    def last_step_bytes(self) -> int:
        v = C.c_int64()
        check(self.L.gfpl_last_step_bytes(self.h, C.byref(v)), "last_step_bytes")
        return v.value

    def last_step_stage_bytes(self) -> np.ndarray:
        v = np.zeros(7, np.int64)
        check(self.L.gfpl_last_step_stage_bytes(self.h, v.ctypes.data), "last_step_stage_bytes")
        return v

    STEP_COUNTS = ["N_o", "N_k", "M_o", "S_p", "S_l", "M_p", "M_l", "n_inliers"]

    def last_step_counts(self) -> dict:
        """Per-sequence means of the counts the last step's bytes are priced on
        (gfpl_last_step_counts): keypoints / keylines (both sides), SAD keypoints,
        stereo points / lines of the new frame, matched points / lines, inliers."""
        v = np.zeros(8, np.int64)
        check(self.L.gfpl_last_step_counts(self.h, v.ctypes.data), "last_step_counts")
        return {n: float(x) / self.B for n, x in zip(self.STEP_COUNTS, v)}

    def last_step_track_counts(self) -> dict:
        """The last step, summed over the batch (gfpl_last_step_track_counts): line-cut greedy
        steps, those the certified search evaluated exactly, and the inliers
        left after optimize_pose."""
        v = np.zeros(4, np.int64)
        check(self.L.gfpl_last_step_track_counts(self.h, v.ctypes.data), "last_step_track_counts")
        return {"steps": int(v[0]), "exact_steps": int(v[1]), "inliers_after_pose": int(v[2]),
                "lines_unbounded": int(v[3])}

    def last_step_cut_proof(self) -> dict:
        """Proven line cut (cut_proof 1) of the last step, summed over the batch
        (gfpl_last_step_cut_proof): sequences redone by the eager-proven search because the
        recorded search could not be proven, margined steps proven, reference variances
        evaluated, lines with margined steps."""
        v = np.zeros(4, np.int64)
        check(self.L.gfpl_last_step_cut_proof(self.h, v.ctypes.data), "last_step_cut_proof")
        return {"redone": int(v[0]), "steps_proven": int(v[1]), "vref_evals": int(v[2]), "lines": int(v[3])}

    def debug_cut_records(self, b: int, n_lines: int) -> np.ndarray:
        """gfpl_debug_cut_records: sequence b's line-cut records [n_lines][80] (float64)."""
        out = np.zeros((n_lines, 80), np.float64)
        check(self.L.gfpl_debug_cut_records(self.h, b, out.ctypes.data, n_lines), "debug_cut_records")
        return out

    def debug_step_records(self) -> np.ndarray:
        """gfpl_debug_step_records: every sequence's record of the last step [B][24] (int64)."""
        out = np.zeros((self.B, 24), np.int64)
        check(self.L.gfpl_debug_step_records(self.h, out.ctypes.data), "debug_step_records")
        return out

    def debug_clocks(self) -> np.ndarray:
        """gfpl_debug_clocks: per-sequence debug slots [B][8] (int64): the instrumented builds' clocks;
        in the product build slots 6 / 7 hold the measured-mode line-cut wave's HW_ID / XCC_ID."""
        out = np.zeros((self.B, 8), np.int64)
        check(self.L.gfpl_debug_clocks(self.h, out.ctypes.data), "debug_clocks")
        return out

    def last_step_kernel_bytes(self) -> np.ndarray:
        v = np.zeros(4, np.int64)
        check(self.L.gfpl_last_step_kernel_bytes(self.h, v.ctypes.data), "last_step_kernel_bytes")
        return v

    def nbytes(self) -> int:
        return int(self.L.gfpl_seqbatch_bytes(self.h))

    def close(self):
        if getattr(self, "h", None):
            self.L.gfpl_seqbatch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def track_from_dict(d: dict) -> TrackHost:
    t = TrackHost()
    t.n_matched_pt = len(d["matched_pt"])
    t.n_matched_ls = len(d["matched_ls"])
    for i, v in enumerate(d["matched_pt"]):
        t.matched_pt[i] = int(v)
    for i, v in enumerate(d["matched_ls"]):
        t.matched_ls[i] = int(v)
    t.n_inliers, t.n_inliers_pt, t.n_inliers_ls = d["n_inliers"], d["n_inliers_pt"], d["n_inliers_ls"]
    t.num_frame_loss = d["num_frame_loss"]
    return t


class ORBextractor:
    """ORB_SLAM2::ORBextractor on the GPU (include/ORBextractor.h:49-106; constructor
    src/ORBextractor.cc:410-470, operator() :1043-1105), as StereoFrame builds it
    (src/stereoFrame.cpp:33-36).  One extractor serves images of one size; __call__
    takes one host image like the reference's operator(), extract() a batch of images
    already on the device (the product path's form).

    ctx: a Context (its device and stream), or None for a bare context on `device`."""

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                 width: int, height: int, max_images: int = 1, kp_cap: Optional[int] = None,
                 ctx: Optional[Context] = None, device: int = 0):
        self.L = hiplib()
        self.prm = OrbParams(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        self.width, self.height, self.max_images = width, height, max_images
        self.kp_cap = kp_cap or nfeatures + 64 * nlevels + 64
        self._own = None
        if ctx is None:
            h = C.c_void_p()
            check(self.L.gfpl_create(device, None, C.byref(h)), "gfpl_create")
            self._own = h
            ch = h
        else:
            ch = ctx.h
        self._ctx = ctx
        o = C.c_void_p()
        check(self.L.gfpl_orb_create(ch, width, height, C.byref(self.prm), max_images, self.kp_cap, C.byref(o)),
              "orb_create")
        self.h = o
        b = C.c_int64()
        check(self.L.gfpl_orb_pyramid_bytes(o, C.byref(b)), "orb_pyramid_bytes")
        self.pyramid_bytes = b.value
        # ORBextractor tables (:414-431)
        sc = [1.0]
        for _ in range(1, nlevels):
            sc.append(float(np.float32(sc[-1]) * np.float32(scaleFactor)))
        self.mvScaleFactor = np.array(sc, np.float32)
        self.mvLevelSigma2 = self.mvScaleFactor * self.mvScaleFactor
        self.mvInvScaleFactor = np.float32(1.0) / self.mvScaleFactor
        self.mvInvLevelSigma2 = np.float32(1.0) / self.mvLevelSigma2
        self.mvImagePyramid = []

    # the reference's accessors (include/ORBextractor.h:65-88)
    def GetLevels(self) -> int: return self.prm.nlevels
    def GetScaleFactor(self) -> float: return float(np.float32(self.prm.scale_factor))
    def GetScaleFactors(self): return self.mvScaleFactor.copy()
    def GetInverseScaleFactors(self): return self.mvInvScaleFactor.copy()
    def GetScaleSigmaSquares(self): return self.mvLevelSigma2.copy()
    def GetInverseScaleSigmaSquares(self): return self.mvInvLevelSigma2.copy()

    def level_sizes(self):
        """(cols, rows) of every level: cvRound(W / scale), cvRound(H / scale) (:1111-1112)."""
        return [(int(np.rint(np.float32(self.width) * self.mvInvScaleFactor[l])),
                 int(np.rint(np.float32(self.height) * self.mvInvScaleFactor[l]))) for l in range(self.prm.nlevels)]

    def extract(self, images_dev, n: int, kps_dev, desc_dev, n_kp_dev, angle_dev=None, response_dev=None,
                pyramid_dev=None, pyr_stride: int = 0) -> None:
        """gfpl_orb_extract on device buffers: images [n][H][W] u8; per image i the rows
        [i*kp_cap, i*kp_cap + n_kp[i]) of kps (KEYPOINT_DT) / desc (32 B) / angle / response."""
        check(self.L.gfpl_orb_extract(self.h, _ptr(images_dev), n, _ptr(kps_dev), _ptr(desc_dev), _ptr(n_kp_dev),
                                      _ptr(angle_dev), _ptr(response_dev), _ptr(pyramid_dev), pyr_stride),
              "orb_extract")

    def extract_async(self, images_dev, n: int, kps_dev, desc_dev, n_kp_dev, angle_dev=None, response_dev=None,
                      pyramid_dev=None, pyr_stride: int = 0) -> None:
        """gfpl_orb_extract_async: enqueued on the context's stream; status() reports capacity errors."""
        check(self.L.gfpl_orb_extract_async(self.h, _ptr(images_dev), n, _ptr(kps_dev), _ptr(desc_dev),
                                            _ptr(n_kp_dev), _ptr(angle_dev), _ptr(response_dev), _ptr(pyramid_dev),
                                            pyr_stride), "orb_extract_async")

    def status(self) -> None:
        check(self.L.gfpl_orb_status(self.h), "orb_status")

    def __call__(self, image: np.ndarray):
        """operator()(image, noArray(), keypoints, descriptors) on one HOST grey image:
        returns (keypoints [CV_KEYPOINT_DT], descriptors [n][32] u8); mvImagePyramid holds
        the level images afterwards."""
        import torch
        image = np.ascontiguousarray(image, np.uint8)
        if image.shape != (self.height, self.width):
            raise ValueError(f"image {image.shape} != ({self.height}, {self.width})")
        dev = torch.device("cuda", torch.cuda.current_device())
        img = torch.from_numpy(image).to(dev)
        kc = self.kp_cap
        kps = torch.zeros(kc * KEYPOINT_DT.itemsize, dtype=torch.uint8, device=dev)
        desc = torch.zeros(kc * DESC, dtype=torch.uint8, device=dev)
        nkp = torch.zeros(1, dtype=torch.int32, device=dev)
        ang = torch.zeros(kc, dtype=torch.float32, device=dev)
        rsp = torch.zeros(kc, dtype=torch.float32, device=dev)
        pyr = torch.zeros(self.pyramid_bytes, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        self.extract(img, 1, kps, desc, nkp, ang, rsp, pyr, self.pyramid_bytes)
        n = int(nkp.item())
        k = kps.cpu().numpy().view(KEYPOINT_DT)[:n]
        out = np.zeros(n, CV_KEYPOINT_DT)
        out["x"], out["y"], out["octave"] = k["x"], k["y"], k["octave"]
        out["size"] = np.float32(31) * self.mvScaleFactor[k["octave"]]   # scaledPatchSize (:1090)
        out["angle"] = ang[:n].cpu().numpy()
        out["response"] = rsp[:n].cpu().numpy()
        p = pyr.cpu().numpy()
        self.mvImagePyramid, off = [], 0
        for (w, h) in self.level_sizes():
            self.mvImagePyramid.append(p[off:off + w * h].reshape(h, w).copy())
            off += w * h
        return out, desc.cpu().numpy().reshape(kc, DESC)[:n].copy()

    def close(self):
        if getattr(self, "h", None):
            self.L.gfpl_orb_destroy(self.h)
            self.h = None
        if getattr(self, "_own", None):
            self.L.gfpl_destroy(self._own)
            self._own = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LSDDetector:
    """line_descriptor::LSDDetectorC on the GPU, the detect(image, keylines, scale, numOctaves,
    opts) path StereoFrame uses (3rdparty/line_descriptor/src/LSDDetector_custom.cpp:218-316,
    src/stereoFrame.cpp:1160-1186: LSD_REFINE_STD at scale 1, one octave, the min-length
    filter, the response sort + resize to Config::lsdNFeatures) for images of one size.
    detect() takes one host image like the reference; detect_batch() device buffers (the
    product path's form, writing keylines where gfpl_lbd_compute / gfpl_frames read them)."""

    def __init__(self, width: int, height: int, params: Optional["LsdParams"] = None, max_images: int = 1,
                 kl_cap: int = 512, seg_cap: int = 4096, ctx: Optional[Context] = None, device: int = 0):
        self.L = hiplib()
        self.width, self.height, self.max_images, self.kl_cap, self.seg_cap = width, height, max_images, kl_cap, seg_cap
        self.params = params if params is not None else LsdParams.reference(width, height)
        self._own = None
        if ctx is None:
            h = C.c_void_p()
            check(self.L.gfpl_create(device, None, C.byref(h)), "gfpl_create")
            self._own = h
            ch = h
        else:
            ch = ctx.h
        self._ctx = ctx
        o = C.c_void_p()
        check(self.L.gfpl_lsd_create(ch, C.byref(self.params), width, height, max_images, kl_cap, seg_cap,
                                     C.byref(o)), "lsd_create")
        self.h = o

    def detect_batch(self, images_dev, n: int, keylines_dev, n_kl_dev, response_dev=None) -> None:
        check(self.L.gfpl_lsd_detect(self.h, _ptr(images_dev), n, _ptr(keylines_dev), _ptr(n_kl_dev),
                                     _ptr(response_dev) if response_dev is not None else None), "lsd_detect")

    def detect_async(self, images_dev, n: int, keylines_dev, n_kl_dev, response_dev=None) -> None:
        """gfpl_lsd_detect_async: enqueued on the context's stream; status() reports capacity errors."""
        check(self.L.gfpl_lsd_detect_async(self.h, _ptr(images_dev), n, _ptr(keylines_dev), _ptr(n_kl_dev),
                                           _ptr(response_dev) if response_dev is not None else None), "lsd_detect_async")

    def status(self) -> None:
        check(self.L.gfpl_lsd_status(self.h), "lsd_status")

    def sort_desc(self, a_dev, n: int) -> None:
        """ledger S2 test hook: std::sort by descending high 32 bits of a device u64 array."""
        check(self.L.gfpl_lsd_sort_desc(self.h, _ptr(a_dev), n), "lsd_sort_desc")

    def detect(self, image: np.ndarray):
        """detect(image, keylines, ...) on one HOST image: (keylines KEYLINE_DT, response f32)."""
        import torch
        image = np.ascontiguousarray(image, np.uint8)
        if image.shape != (self.height, self.width):
            raise ValueError(f"image {image.shape} != ({self.height}, {self.width})")
        dev = torch.device("cuda", torch.cuda.current_device())
        d_img = torch.from_numpy(image).to(dev)
        d_kl = torch.zeros(self.kl_cap * KEYLINE_DT.itemsize, dtype=torch.uint8, device=dev)
        d_n = torch.zeros(1, dtype=torch.int32, device=dev)
        d_r = torch.zeros(self.kl_cap, dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        self.detect_batch(d_img, 1, d_kl, d_n, d_r)
        n = int(d_n.cpu()[0])
        kl = d_kl.cpu().numpy().view(KEYLINE_DT)[:n].copy()
        return kl, d_r.cpu().numpy()[:n].copy()

    def close(self):
        if getattr(self, "h", None):
            self.L.gfpl_lsd_destroy(self.h)
            self.h = None
        if getattr(self, "_own", None):
            self.L.gfpl_destroy(self._own)
            self._own = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BinaryDescriptor:
    """line_descriptor::BinaryDescriptor on the GPU, the compute() path StereoFrame uses
    (3rdparty/line_descriptor/src/binary_descriptor_custom.cpp:539-687; computeLBD
    :1026-1372): 32-byte LBD descriptors of octave-0 keylines (Config::lsdOctaveNum = 1)
    for images of one size.  compute() takes one host image like the reference;
    compute_batch() device buffers (the product path's form)."""

    def __init__(self, width: int, height: int, max_images: int = 1, kl_cap: int = 512,
                 ctx: Optional[Context] = None, device: int = 0):
        self.L = hiplib()
        self.width, self.height, self.max_images, self.kl_cap = width, height, max_images, kl_cap
        self._own = None
        if ctx is None:
            h = C.c_void_p()
            check(self.L.gfpl_create(device, None, C.byref(h)), "gfpl_create")
            self._own = h
            ch = h
        else:
            ch = ctx.h
        self._ctx = ctx
        o = C.c_void_p()
        check(self.L.gfpl_lbd_create(ch, width, height, max_images, kl_cap, C.byref(o)), "lbd_create")
        self.h = o

    def compute_batch(self, images_dev, n: int, keylines_dev, n_kl_dev, desc_dev) -> None:
        check(self.L.gfpl_lbd_compute(self.h, _ptr(images_dev), n, _ptr(keylines_dev), _ptr(n_kl_dev),
                                      _ptr(desc_dev)), "lbd_compute")

    def compute_async(self, images_dev, n: int, keylines_dev, n_kl_dev, desc_dev) -> None:
        """gfpl_lbd_compute_async: enqueued on the context's stream; status() reports errors."""
        check(self.L.gfpl_lbd_compute_async(self.h, _ptr(images_dev), n, _ptr(keylines_dev), _ptr(n_kl_dev),
                                            _ptr(desc_dev)), "lbd_compute_async")

    def status(self) -> None:
        check(self.L.gfpl_lbd_status(self.h), "lbd_status")

    def compute(self, image: np.ndarray, keylines: np.ndarray) -> np.ndarray:
        """compute(image, keylines, descriptors) on one HOST image; keylines: KEYLINE_DT rows.
        Returns [n][32] u8."""
        import torch
        image = np.ascontiguousarray(image, np.uint8)
        if image.shape != (self.height, self.width):
            raise ValueError(f"image {image.shape} != ({self.height}, {self.width})")
        n = len(keylines)
        if n > self.kl_cap:
            raise ValueError(f"{n} keylines > kl_cap {self.kl_cap}")
        dev = torch.device("cuda", torch.cuda.current_device())
        kl = np.zeros(self.kl_cap, KEYLINE_DT)
        kl[:n] = keylines
        d_img = torch.from_numpy(image).to(dev)
        d_kl = torch.from_numpy(kl.view(np.uint8)).to(dev)
        d_n = torch.tensor([n], dtype=torch.int32, device=dev)
        d_desc = torch.zeros(self.kl_cap * DESC, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        self.compute_batch(d_img, 1, d_kl, d_n, d_desc)
        return d_desc.cpu().numpy().reshape(self.kl_cap, DESC)[:n].copy()

    def close(self):
        if getattr(self, "h", None):
            self.L.gfpl_lbd_destroy(self.h)
            self.h = None
        if getattr(self, "_own", None):
            self.L.gfpl_destroy(self._own)
            self._own = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class StereoDetector:
    """gfpl_detector: StereoFrame's detection from a stereo pair of images on the device —
    ORB of both images (the right pyramid kept for the sub-pixel refinement), LSD with the
    lsdNFeatures cut and LBD of both (src/stereoFrame.cpp:148-172, 411-450, 1128-1227), for
    up to `batch` stereo frames per call, on two streams of the detector's own.  detect()
    returns the gfpl_frames view the tracker (StereoFrameHandler.initialize / insertStereoPair
    / frameStep) reads with no copy, ordered by the view's ready / consumed events: at most
    `sets` views may be outstanding (a tracker call reading a view, or discard(), frees it)."""

    def __init__(self, ctx: Context, batch: int, kp_cap: int, kl_cap: int, params: Optional[DetectorParams] = None,
                 sets: int = 2):
        self.L = ctx.L
        self.ctx, self.B, self.kp_cap, self.kl_cap = ctx, batch, kp_cap, kl_cap
        self.params = params if params is not None else DetectorParams.reference(ctx.cam, ctx.cfg)
        h = C.c_void_p()
        check(self.L.gfpl_detector_create(ctx.h, C.byref(self.params), batch, kp_cap, kl_cap, sets, C.byref(h)),
              "detector_create")
        self.h = h

    def detect(self, left, right, time_stamp, n: Optional[int] = None) -> Frames:
        """left / right: device u8 [n][H][W] (torch), time_stamp: device f64 [n]; produced on
        the context's stream.  Asynchronous (status() reports capacity errors)."""
        n = self.B if n is None else n
        fr = Frames()
        check(self.L.gfpl_detect_stereo_async(self.h, _ptr(left), _ptr(right), n, _ptr(time_stamp), C.byref(fr)),
              "detect_stereo_async")
        fr._keep = [left, right, time_stamp]
        return fr

    def detect_host(self, left: np.ndarray, right: np.ndarray, time_stamp) -> Frames:
        """HOST images [n][H][W] u8 (or one [H][W] image) and time stamps [n]."""
        left = np.ascontiguousarray(left, np.uint8)
        right = np.ascontiguousarray(right, np.uint8)
        ts = np.ascontiguousarray(np.atleast_1d(time_stamp), np.float64)
        n = 1 if left.ndim == 2 else left.shape[0]
        if right.shape != left.shape or len(ts) != n:
            raise ValueError("detect_host: left / right / time stamps disagree")
        fr = Frames()
        check(self.L.gfpl_detect_stereo_host(self.h, left.ctypes.data, right.ctypes.data, n, ts.ctypes.data,
                                             C.byref(fr)), "detect_stereo_host")
        return fr

    def status(self) -> None:
        check(self.L.gfpl_detector_status(self.h), "detector_status")

    def discard(self, fr: Frames) -> None:
        check(self.L.gfpl_detector_discard(self.h, C.byref(fr)), "detector_discard")

    def read(self, fr: Frames, seq: int) -> dict:
        """one sequence's detections of a view, on the host: kp_l / kp_r (KEYPOINT_DT),
        pdesc_l / pdesc_r, kl_l / kl_r (KEYLINE_DT), ldesc_l / ldesc_r"""
        out = {"kp_l": np.zeros(fr.kp_cap, KEYPOINT_DT), "kp_r": np.zeros(fr.kp_cap, KEYPOINT_DT),
               "pdesc_l": np.zeros((fr.kp_cap, DESC), np.uint8), "pdesc_r": np.zeros((fr.kp_cap, DESC), np.uint8),
               "kl_l": np.zeros(fr.kl_cap, KEYLINE_DT), "kl_r": np.zeros(fr.kl_cap, KEYLINE_DT),
               "ldesc_l": np.zeros((fr.kl_cap, DESC), np.uint8), "ldesc_r": np.zeros((fr.kl_cap, DESC), np.uint8)}
        d = DetectionsHost()
        for k, a in out.items():
            setattr(d, k, a.ctypes.data)
        check(self.L.gfpl_read_detections(self.ctx.h, C.byref(fr), seq, C.byref(d)), "read_detections")
        n = {"kp": (d.n_kp_l, d.n_kp_r), "pdesc": (d.n_kp_l, d.n_kp_r), "kl": (d.n_kl_l, d.n_kl_r),
             "ldesc": (d.n_kl_l, d.n_kl_r)}
        return {k: a[:n[k.split("_")[0]][0 if k.endswith("_l") else 1]].copy() for k, a in out.items()}

    def close(self):
        if getattr(self, "h", None):
            self.L.gfpl_detector_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
