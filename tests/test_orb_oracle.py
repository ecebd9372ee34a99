"""Known-answer tests of the CPU ORB oracle (oracle/gfpl_orb_oracle.cpp).

The reference's ORB arithmetic lives in OpenCV 3.4.1 (absent from this image), so the
oracle is PARITY UNPINNED against the reference binary (DESIGN.md ledger O1-O7).  These
tests pin each piece against an independent numpy / pure-Python statement of the same
published algorithm, and the whole extractor against the ORBextractor invariants
(per-level quotas, borders, output order)."""
import math

import numpy as np
import pytest

import gfpl
import oracle as O

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def test_fast_atan2_known_answers():
    # cv::fastAtan2: degrees in [0, 360), exact on the axes
    assert O.fast_atan2(0.0, 1.0) == 0.0
    assert O.fast_atan2(1.0, 0.0) == 90.0
    assert O.fast_atan2(0.0, -1.0) == 180.0
    assert O.fast_atan2(-1.0, 0.0) == 270.0
    rng = np.random.default_rng(3)
    for y, x in rng.uniform(-500, 500, (400, 2)):
        ref = math.degrees(math.atan2(y, x)) % 360.0
        d = abs(O.fast_atan2(float(y), float(x)) - ref)
        assert min(d, 360 - d) < 0.01   # the polynomial's documented accuracy


def _bilinear_float(src, dw, dh):
    sh, sw = src.shape
    out = np.zeros((dh, dw))
    for y in range(dh):
        fy = (y + 0.5) * sh / dh - 0.5
        y0 = math.floor(fy); ay = fy - y0
        r0, r1 = min(max(y0, 0), sh - 1), min(max(y0 + 1, 0), sh - 1)
        for x in range(dw):
            fx = (x + 0.5) * sw / dw - 0.5
            x0 = math.floor(fx); ax = fx - x0
            if x0 < 0:
                x0, ax = 0, 0.0
            x1 = min(x0 + 1, sw - 1)
            if x0 >= sw - 1:
                x0, ax = sw - 1, 0.0
            top = src[r0, x0] * (1 - ax) + src[r0, x1] * ax
            bot = src[r1, x0] * (1 - ax) + src[r1, x1] * ax
            out[y, x] = top * (1 - ay) + bot * ay
    return out


@pytest.mark.parametrize("sw,sh", [(64, 48), (77, 31), (640, 480)])
def test_resize_is_fixed_point_bilinear(sw, sh):
    """O1: INTER_LINEAR with 11-bit coefficients = float bilinear (half-pixel centres,
    clamped borders) to within one grey level; constants stay constant."""
    rng = np.random.default_rng(sw)
    src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
    dw, dh = round(sw / 1.2), round(sh / 1.2)
    got = O.orb_resize(src, dw, dh).astype(int)
    if sw * sh <= 4096:
        ref = _bilinear_float(src.astype(float), dw, dh)
        assert np.abs(got - ref).max() <= 1.0
    c = np.full((sh, sw), 173, np.uint8)
    assert (O.orb_resize(c, dw, dh) == 173).all()


def _gauss_taps():
    cf = np.array([np.float32(math.exp(-0.125 * (i - 3) ** 2)) for i in range(7)], np.float32)
    s = 1.0 / float(sum(float(v) for v in cf))
    return np.array([int(np.rint(np.float32(float(v) * s) * np.float32(256))) for v in cf])


def test_blur_taps_and_formula():
    """O2: 8-bit taps of getGaussianKernel(7, 2) (they sum to 257, so a constant image
    brightens by 1/257 before rounding), rows exact, columns (s + 2^15) >> 16, REFLECT_101."""
    k = _gauss_taps()
    assert k.tolist() == [18, 34, 49, 55, 49, 34, 18]
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, (41, 57), dtype=np.uint8)
    h, w = src.shape
    xi = np.abs(np.arange(-3, w + 3)); xi = np.where(xi >= w, 2 * w - 2 - xi, xi)
    yi = np.abs(np.arange(-3, h + 3)); yi = np.where(yi >= h, 2 * h - 2 - yi, yi)
    pad = src.astype(np.int64)[yi][:, xi]
    rows = sum(k[t] * pad[:, t:t + w] for t in range(7))
    cols = sum(k[t] * rows[t:t + h, :] for t in range(7))
    ref = np.clip((cols + (1 << 15)) >> 16, 0, 255)
    assert (O.orb_blur(src) == ref).all()
    assert (O.orb_blur(np.full((20, 20), 100, np.uint8)) == 101).all()


def _fast_py(img, t):
    """cv::FAST(img, kps, t, true) restated directly from its definition: a corner has
    >= 9 contiguous circle pixels all darker than v - t or all brighter than v + t; its
    score is the largest such arc minimum |v - p| minus 1; strict 3x3 maxima survive."""
    h, w = img.shape
    im = img.astype(int)
    score = np.zeros((h, w), int)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            v = im[y, x]
            d = [v - im[y + dy, x + dx] for dx, dy in CIRCLE]
            best = None
            for s in range(16):
                arc = [d[(s + i) % 16] for i in range(9)]
                for sign in (1, -1):
                    m = min(sign * a for a in arc)
                    if m > t:
                        best = m if best is None else max(best, m)
            if best is not None:
                # cornerScore: max(threshold, best arc minimum over ALL arcs) - 1
                arcs = [min(sign * d[(s + i) % 16] for i in range(9)) for s in range(16) for sign in (1, -1)]
                score[y, x] = max(t, max(arcs)) - 1
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            s = score[y, x]
            if s and all(s > score[y + dy, x + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dx or dy):
                out.append((x, y, s))
    return out


@pytest.mark.parametrize("t", [7, 20])
def test_fast_matches_definition(t):
    img = gfpl.synth_image(11, 0, 96, 72)
    rng = np.random.default_rng(t)
    img = np.clip(img.astype(int) + rng.integers(-25, 26, img.shape), 0, 255).astype(np.uint8)
    got = [tuple(int(v) for v in r) for r in O.orb_fast(img, t)]
    ref = _fast_py(img, t)
    assert len(ref) > 20
    assert got == ref


def _n_per_level(nf, sf, nl):
    f = np.float32(1.0) / np.float32(sf)
    nd = np.float32(nf * (1 - f) / (1 - np.float32(math.pow(float(f), nl))))
    out, s = [], 0
    for _ in range(nl - 1):
        out.append(int(np.rint(nd))); s += out[-1]; nd = np.float32(nd * f)
    out.append(max(nf - s, 0))
    return out


@pytest.mark.parametrize("cam,seq", [("vga", 3), ("kitti", 5), ("euroc", 7)])
def test_extractor_invariants(cam, seq):
    """ORBextractor::operator() structure: keypoints level by level, per-level counts
    within the quota + 3 nodes (DistributeOctTree stops at >= N), inside the EDGE_THRESHOLD
    borders, coordinates on the level grid scaled by the level factor, responses = FAST
    scores (integers), angles in [0, 360)."""
    c = gfpl.CAMERAS[cam]
    img = gfpl.synth_image(seq, 0, c["width"], c["height"])
    r = O.orb_extract(img)
    k = r["kps"]
    assert len(k) > 300
    oc = k["octave"]
    assert (np.diff(oc) >= 0).all()
    quota = _n_per_level(2000, 1.2, 4)
    assert quota == [644, 537, 447, 372]
    sc = [1.0]
    for _ in range(3):
        sc.append(float(np.float32(sc[-1]) * np.float32(1.2)))
    for l in range(4):
        m = oc == l
        assert m.sum() <= quota[l] + 3
        lw, lh = round(c["width"] / sc[l]), round(c["height"] / sc[l])
        xs = k["x"][m] / np.float32(sc[l]) if l else k["x"][m]
        ys = k["y"][m] / np.float32(sc[l]) if l else k["y"][m]
        assert (np.abs(xs - np.rint(xs)) < 1e-3).all() and (np.abs(ys - np.rint(ys)) < 1e-3).all()
        assert (np.rint(xs) >= 19).all() and (np.rint(xs) < lw - 19).all()
        assert (np.rint(ys) >= 19).all() and (np.rint(ys) < lh - 19).all()
    assert (r["response"] == np.rint(r["response"])).all() and (r["response"] >= 6).all()
    assert (r["angle"] >= 0).all() and (r["angle"] < 360).all()
    # deterministic
    r2 = O.orb_extract(img)
    assert (r2["desc"] == r["desc"]).all() and (r2["kps"] == k).all()


def test_extractor_flat_image_has_no_keypoints():
    r = O.orb_extract(np.full((120, 160), 90, np.uint8))
    assert len(r["kps"]) == 0


def test_extractor_pyramid_levels_are_resizes():
    img = gfpl.synth_image(2, 1, 320, 240)
    r = O.orb_extract(img, nlevels=3)
    p = r["pyramid"]
    l1 = O.orb_resize(img, round(320 / 1.2), round(240 / 1.2))
    off = 320 * 240
    assert (p[:off] == img.reshape(-1)).all()
    assert (p[off:off + l1.size] == l1.reshape(-1)).all()
