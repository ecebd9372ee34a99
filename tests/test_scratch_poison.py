"""Read-before-write audit of the tracking step (round-5 review, item 1).

Every byte of a seqbatch — frame slots, track lists, all scratch — and of its staging buffers
is filled with 0xFF at creation (GFPL_DEBUG_FILL: NaN doubles, -1 ints) in one run and with
zeros in the other; both runs track the same 2048 sequences of the bench workload (cfg2:
VGA, 2000 ORB + 500 LBD per side, 10+10 GN) through the uploaded staging path.  Every
sequence's step record (greedy line-cut steps, exact steps, counts, bytes) and its whole
frame state (features, matched lists, cut ratios, invCovPose, pose) must be identical: a
kernel that read memory no step wrote would see NaN / -1 in one run and 0 in the other.  Compared
are the fields the reference defines at that point (tests/parity.py): a feature record's obs /
cut / invCovPose fields are written for matched features only, in the reference as here.
"""
import hashlib

import numpy as np
import pytest

import gfpl
from parity import LS_CORE, LS_MATCHED, POSE, PT_CORE, PT_MATCHED

pytestmark = pytest.mark.gpu


def _h(h, a):
    h.update(np.ascontiguousarray(a).tobytes())


def new_frame_digest(fh) -> bytes:
    """The new frame's defined fields (the ones bench.py's parity sampler compares)."""
    h = hashlib.sha256()
    _h(h, np.array([fh.n_pt, fh.n_ls], np.int64))
    for name in PT_CORE + LS_CORE + POSE:
        _h(h, fh.get(name))
    _h(h, np.array([fh.s.err_norm, fh.s.time_stamp], np.float64))
    return h.digest()


def old_frame_digest(fh, tr: dict) -> bytes:
    """The previous frame's fields written for matched features only (obs, cut ratios,
    invCovPose, inlier flags), at the matched rows (tests/parity.py: compare_prev_matched)."""
    h = hashlib.sha256()
    pts = np.unique(tr["matched_pt"]).astype(np.int64)
    lns = np.asarray(tr["matched_ls"], np.int64)
    for name in PT_MATCHED:
        _h(h, fh.get(name)[pts])
    for name in LS_MATCHED:
        _h(h, fh.get(name)[lns])
    for name in ("ls_covS", "ls_covE"):
        _h(h, fh.get(name))
    return h.digest()


def track_digest(tr: dict) -> bytes:
    h = hashlib.sha256()
    for k in sorted(tr):
        _h(h, np.asarray(tr[k]).astype(np.int64))
    return h.digest()


def _run(monkeypatch, fill, cam, cfg, H, n, F, KP, KL):
    monkeypatch.setenv("GFPL_DEBUG_FILL", fill)
    ctx = gfpl.Context(cam, cfg)
    h = gfpl.StereoFrameHandler(ctx, n, KP, KL)

    def staged(k):
        h.upload_wait(h.upload_async(H.frames(k), 0, k % 2))
        return h.staged_frames(k % 2)
    h.initialize(staged(0))
    recs, digests = [], []
    for k in range(1, F):
        h.frameStep(staged(k))
        recs.append(h.debug_step_records().copy())
        dk = []
        for b in range(n):
            tr = h.read_last_track(b)
            dk.append((new_frame_digest(h.read_frame(gfpl.PREV, b)), old_frame_digest(h.read_frame(gfpl.CURR, b), tr),
                       track_digest(tr)))
        digests.append(dk)
    h.close()
    ctx.close()
    monkeypatch.delenv("GFPL_DEBUG_FILL")
    return recs, digests


@pytest.mark.parametrize("layout", ["bench", "small"])
def test_poisoned_scratch_matches_zeroed(monkeypatch, layout):
    if layout == "bench":   # the B = 16384 kernels: 8 sequences per search wave, one pose wave per sequence
        monkeypatch.setenv("GFPL_CUT_WAVE_MAX_B", "0")
        monkeypatch.setenv("GFPL_POSE_MULTI_MAX_B", "0")
        monkeypatch.setenv("GFPL_POSE_W8_MAX_B", "0")
        monkeypatch.setenv("GFPL_CUT_PREP_W8_MAX_B", "0")
    n, F, KP, KL = 2048 if layout == "bench" else 64, 4, 2048, 512
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0)
    cam = gfpl.make_camera("vga", cfg)
    H = gfpl.HostFrames(cam, gfpl.synth_params(respawn=16, seed=5), n, F, KP, KL, threads=8)
    r0, d0 = _run(monkeypatch, "0x00", cam, cfg, H, n, F, KP, KL)
    r1, d1 = _run(monkeypatch, "0xFF", cam, cfg, H, n, F, KP, KL)
    for k in range(F - 1):
        diff = np.nonzero((r0[k] != r1[k]).any(axis=1))[0]
        cols = np.nonzero((r0[k] != r1[k]).any(axis=0))[0]
        assert len(diff) == 0, (f"step {k + 1}: step records differ for {len(diff)} sequences {diff[:8]}, record "
                                f"slots {cols}: {r0[k][diff[0], cols]} vs {r1[k][diff[0], cols]}")
        bad = [b for b in range(n) if d0[k][b] != d1[k][b]]
        parts = sorted({i for b in bad for i in range(3) if d0[k][b][i] != d1[k][b][i]})
        assert not bad, (f"step {k + 1}: state differs for {len(bad)} sequences {bad[:8]} in "
                         f"{[['new frame', 'previous frame (matched rows)', 'track'][i] for i in parts]}")
    steps = int(sum(r[:, 16].sum() for r in r0))
    assert steps > 0   # the line cut ran (greedy steps recorded)
