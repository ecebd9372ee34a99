"""The C-ABI library (the drop-in boundary) loads without a GPU, exports every
entry point include/gfpl.h declares, and its host-side setup matches the
reference's Config / ORBextractor tables.  No compute calls here."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import gfpl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gfpl.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gfpl_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_survey_boundary():
    names = declared_symbols()
    # what the C-ABI replacement must export
    for n in ["gfpl_create", "gfpl_destroy", "gfpl_set_camera", "gfpl_set_config", "gfpl_knn2_hamming",
              "gfpl_stereo_points", "gfpl_stereo_lines", "gfpl_line_uncertainty", "gfpl_cross_points",
              "gfpl_cross_lines", "gfpl_line_cut", "gfpl_optimize_pose", "gfpl_frame_step"]:
        assert n in names, n


def test_library_exports_every_declared_symbol():
    L = gfpl.hiplib()
    missing = [n for n in declared_symbols() if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", gfpl.lib_path("libgfpl_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (gfpl_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_abi_version_and_strerror():
    L = gfpl.hiplib()
    assert L.gfpl_abi_version() == 6   # 6: STEP_REC 24, cut_proof 0-3; 5: gfpl_config.cut_proof; 4: gfpl_detector (image input), event record counts
    assert L.gfpl_strerror(-4) == b"knn-2 needs at least 2 train descriptors"


def test_config_defaults_match_reference():
    c = gfpl.default_config()
    # src/config.cpp:77-153
    assert (c.max_line_match_num, c.max_point_match_num) == (300, 500)
    assert (c.max_dist_epip, c.min_disp, c.max_ratio_12_p, c.point_match_radius) == (2.0, 1.0, 0.9, 50.0)
    assert (c.stereo_overlap_th, c.line_horiz_th, c.desc_th_l, c.line_cov_th) == (0.5, 0.1, 0.1, 10.0)
    assert (c.homog_th, c.min_features, c.max_iters, c.max_iters_ref) == (1e-7, 10, 5, 10)
    assert (c.min_error, c.min_error_change, c.inlier_k, c.motion_step_th) == (1e-7, 1e-7, 2.0, 10.0)
    assert (c.ratio_disp_std, c.ratio_disp_std_hor, c.orb_scale_factor, c.orb_n_levels) == (0.15, 0.9, 1.2, 4)
    assert (c.cut_step, list(c.cut_rng), c.proj_gate_px) == (0.05, [0.0, 1.0], 10.0)
    assert c.cut_certify == 1e-9   # (new) certified line-cut margin; 0 = exact steps only


def test_camera_tables_match_orbextractor():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    # ORBextractor ctor: float scale factor stored in a double member (src/ORBextractor.cc:410-431)
    s = [np.float32(1.0)]
    for i in range(1, 4):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(1.2))))
    assert [np.float32(v) for v in list(cam.scale)[:4]] == s
    assert [np.float32(v) for v in list(cam.inv_scale)[:4]] == [np.float32(1.0) / v for v in s]
    assert list(cam.lvl_cols)[:4] == [640, 533, 444, 370]
    assert list(cam.lvl_rows)[:4] == [480, 400, 333, 278]
    # PointFeature sigma2 = 1/(1.2^(l+1))^2 (src/stereoFeatures.cpp:41-47)
    for l in range(4):
        assert cam.sigma2_pt[l] == 1.0 / (1.2 ** (l + 1)) ** 2 or abs(cam.sigma2_pt[l] * (1.2 ** (l + 1)) ** 2 - 1) < 1e-15
    assert cam.pyr_bytes % 256 == 0


def test_unsupported_config_rejected_without_device():
    # config validation happens before any device work
    L = gfpl.hiplib()
    c = gfpl.default_config(best_lr_matches=0)
    # no context possible without a GPU: set_config on a NULL ctx is an argument error
    assert L.gfpl_set_config(None, C.byref(c)) == -1


@pytest.mark.skipif(os.environ.get("GFPL_EXPECT_GPU") == "1", reason="GPU present")
def test_create_fails_loudly_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    with pytest.raises(gfpl.GfplError) as e:
        gfpl.Context(gfpl.make_camera("vga"), gfpl.default_config())
    assert e.value.code == -3
