"""Generate the oracle golden fixtures (tests/golden/oracle_golden.json).

The reference cannot be compiled here, so these vectors come
from the CPU restatement (oracle/) on deterministic synthetic inputs
(gf-pl-slam_amd/synth); they pin the oracle against drift and are what the GPU
parity tests and smoke compare against on the box.  Re-run after an
intentional oracle change:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gfpl  # noqa: E402
import oracle as O  # noqa: E402

CORE = ["pt_pl", "pt_disp", "pt_P", "pt_idx", "pt_level", "pdesc", "ls_spl", "ls_epl", "ls_sdisp",
        "ls_edisp", "ls_sP", "ls_eP", "ls_le", "ls_idx", "ldesc"]


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:32]


def euroc_traj(seq="mh_01", n=2):
    return gfpl.euroc_traj(seq, n)


CASES = {
    # BASELINE configs[0]: single EuRoC MH_01 pair through optimizePose (plumbing)
    "euroc_mh01_pair": dict(cam="euroc", cfg={}, n_seq=1, n_frames=2, kp=2048, kl=512,
                            synth=dict(z_min=2.0, z_max=12.0), traj=("mh_01", 2)),
    "vga_small": dict(cam="vga", cfg={}, n_seq=2, n_frames=4, kp=1024, kl=256,
                      synth=dict(n_kp=800, n_kl=200, n_world_pts=1100, n_world_lines=280, seed=5)),
    # BASELINE configs[1] workload (bench overrides), one sequence
    "vga_cfg2": dict(cam="vga", cfg=dict(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0),
                     n_seq=1, n_frames=3, kp=2048, kl=512, synth=dict(seed=9)),
}


def build_inputs(case):
    cfg = gfpl.default_config(**case["cfg"])
    cam = gfpl.make_camera(case["cam"], cfg)
    keep = []
    over = dict(case["synth"])
    if "traj" in case:
        T, t = euroc_traj(*case["traj"])
        keep += [T, t]
        over.update(traj=T.ctypes.data, n_traj=len(t), traj_t=t.ctypes.data)
    sp = gfpl.synth_params(**over)
    H = gfpl.HostFrames(cam, sp, case["n_seq"], case["n_frames"], case["kp"], case["kl"], threads=1)
    return cfg, cam, H, keep


def run_case(case):
    cfg, cam, H, keep = build_inputs(case)
    out = {"inputs": digest(*H.arrays()), "frames": []}
    for b in range(case["n_seq"]):
        h = O.OracleHandler(cam, cfg, case["kp"], case["kl"])
        h.initialize(H.frames(0), b)
        f = h.read_frame(gfpl.PREV)
        seq = [{"n_pt": f.n_pt, "n_ls": f.n_ls, "core": digest(*[f.get(n) for n in CORE])}]
        for k in range(1, case["n_frames"]):
            h.insertStereoPair(H.frames(k), b)
            tr = h.read_track()
            p = h.read_frame(gfpl.PREV)
            ml = tr["matched_ls"]
            h.optimizePose()
            c = h.read_frame(gfpl.CURR)
            tr2 = h.read_track()
            seq.append({
                "n_pt": c.n_pt, "n_ls": c.n_ls, "core": digest(*[c.get(n) for n in CORE]),
                "matched_pt": tr["matched_pt"].tolist(), "matched_ls": ml.tolist(),
                "cut": [float(v).hex() for v in p.get("ls_cut")[ml].ravel()],
                "prev_matched": digest(p.get("ls_invcov")[ml], p.get("ls_sP")[ml], p.get("ls_eP")[ml],
                                       p.get("pt_pl_obs")[np.unique(tr["matched_pt"])]),
                "n_inliers": tr2["n_inliers"], "n_inliers_pt": tr2["n_inliers_pt"],
                "n_inliers_ls": tr2["n_inliers_ls"],
                "DT": [float(v).hex() for v in c.get("DT").ravel()],
                "Tfw": [float(v).hex() for v in c.get("Tfw").ravel()],
                "DT_cov_eig": [float(v).hex() for v in c.get("DT_cov_eig").ravel()],
                "err_norm": float(c.s.err_norm).hex(),
            })
            h.updateFrame()
        out["frames"].append(seq)
    return out


def main():
    res = {name: run_case(c) for name, c in CASES.items()}
    with open(os.path.join(HERE, "oracle_golden.json"), "w") as f:
        json.dump(res, f, indent=0)
    print("wrote", os.path.join(HERE, "oracle_golden.json"))


if __name__ == "__main__":
    main()
