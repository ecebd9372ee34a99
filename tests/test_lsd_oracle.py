"""CPU oracle of the LSD row (oracle/gfpl_lsd_oracle.cpp, ledger S1-S7), SURVEY.md §8(f)2.

Pins: fdlibm atan2 against libm (S4), flsd's constants (S5), an independent pure-Python
statement of libstdc++'s introsort (S2) against the library's std::sort on tie-heavy keys
(the algorithm the GPU restates in parallel), known answers on drawn rectangles / lines
(segment endpoints on the true edges), and LSDDetector_custom.cpp's keyline fields."""
import math
import os
import struct
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "gf-pl-slam_amd"))
import gfpl  # noqa: E402
import oracle as O  # noqa: E402


def _ulps(a, b):
    ia = struct.unpack("<q", struct.pack("<d", a))[0]
    ib = struct.unpack("<q", struct.pack("<d", b))[0]
    return abs(ia - ib)


def test_atan2_matches_libm():
    rng = np.random.default_rng(1)
    worst = 0
    for y, x in rng.uniform(-2000, 2000, (20000, 2)):
        worst = max(worst, _ulps(O.atan2(float(y), float(x)), math.atan2(y, x)))
    for y, x in ((0.0, 1.0), (0.0, -1.0), (-0.0, -1.0), (1.0, 0.0), (-1.0, 0.0), (3.0, 1.0), (1e-30, 1e30),
                 (5.0, -1e-300), (-7.5, 7.5), (0.4375, 1.0), (2.4375, 1.0)):
        worst = max(worst, _ulps(O.atan2(y, x), math.atan2(y, x)))
    assert worst <= 1


def test_lsd_constants():
    prec, rho, mrs = O.lsd_constants(640, 480)
    assert prec == math.pi * 22.5 / 180
    assert rho == 2.0 / math.sin(prec)
    log_nt = 5 * (math.log10(640) + math.log10(480)) / 2 + math.log10(11.0)
    assert mrs == int(-log_nt / math.log10(22.5 / 180)) == 16


# ---- libstdc++ std::sort, stated serially (bits/stl_algo.h, GCC >= 4.9) -------------------
def _introsort(a, comp):
    def med3(res, x, y, z):
        if comp(a[x], a[y]):
            if comp(a[y], a[z]):
                a[res], a[y] = a[y], a[res]
            elif comp(a[x], a[z]):
                a[res], a[z] = a[z], a[res]
            else:
                a[res], a[x] = a[x], a[res]
        elif comp(a[x], a[z]):
            a[res], a[x] = a[x], a[res]
        elif comp(a[y], a[z]):
            a[res], a[z] = a[z], a[res]
        else:
            a[res], a[y] = a[y], a[res]

    def upart(first, last, piv):
        while True:
            while comp(a[first], a[piv]):
                first += 1
            last -= 1
            while comp(a[piv], a[last]):
                last -= 1
            if not first < last:
                return first
            a[first], a[last] = a[last], a[first]
            first += 1

    def adjust(first, hole, ln, value):
        top = hole
        second = hole
        while second < (ln - 1) // 2:
            second = 2 * (second + 1)
            if comp(a[first + second], a[first + second - 1]):
                second -= 1
            a[first + hole] = a[first + second]
            hole = second
        if (ln & 1) == 0 and second == (ln - 2) // 2:
            second = 2 * (second + 1)
            a[first + hole] = a[first + second - 1]
            hole = second - 1
        parent = (hole - 1) // 2
        while hole > top and comp(a[first + parent], value):
            a[first + hole] = a[first + parent]
            hole = parent
            parent = (hole - 1) // 2
        a[first + hole] = value

    def heapsort(first, last):
        ln = last - first
        if ln >= 2:
            parent = (ln - 2) // 2
            while True:
                adjust(first, parent, ln, a[first + parent])
                if parent == 0:
                    break
                parent -= 1
        while ln > 1:
            ln -= 1
            v = a[first + ln]
            a[first + ln] = a[first]
            adjust(first, 0, ln, v)

    def loop(first, last, depth):
        while last - first > 16:
            if depth == 0:
                heapsort(first, last)
                return
            depth -= 1
            mid = first + (last - first) // 2
            med3(first, first + 1, mid, last - 1)
            cut = upart(first + 1, last, first)
            loop(cut, last, depth)
            last = cut

    def ins(first, last):
        for i in range(first + 1, last):
            v = a[i]
            if comp(v, a[first]):
                a[first + 1:i + 1] = a[first:i]
                a[first] = v
            else:
                j = i
                while comp(v, a[j - 1]):
                    a[j] = a[j - 1]
                    j -= 1
                a[j] = v

    n = len(a)
    if n < 2:
        return a
    loop(0, n, 2 * (n.bit_length() - 1))
    if n > 16:
        ins(0, 16)
        for i in range(16, n):   # __unguarded_insertion_sort
            v = a[i]
            j = i
            while comp(v, a[j - 1]):
                a[j] = a[j - 1]
                j -= 1
            a[j] = v
    else:
        ins(0, n)
    return a


@pytest.mark.parametrize("n,nkeys,seed", [(17, 3, 0), (100, 2, 1), (1000, 5, 2), (5000, 1024, 3), (20000, 40, 4),
                                          (3000, 1, 5)])
def test_std_sort_permutation_restated(n, nkeys, seed):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, nkeys, n).astype(np.uint64)
    a = (keys << np.uint64(32)) | np.arange(n, dtype=np.uint64)
    ref = O.sort_desc(a)
    got = _introsort([int(v) for v in a], lambda x, y: (x >> 32) > (y >> 32))
    assert [int(v) for v in ref] == got


def test_std_sort_presorted_and_reversed():
    n = 4000
    for keys in (np.arange(n)[::-1] % 700, np.arange(n) % 700, np.zeros(n, int)):
        a = (keys.astype(np.uint64) << np.uint64(32)) | np.arange(n, dtype=np.uint64)
        ref = O.sort_desc(a)
        got = _introsort([int(v) for v in a], lambda x, y: (x >> 32) > (y >> 32))
        assert [int(v) for v in ref] == got


# ---- known answers -------------------------------------------------------------------
def _rect_image(w=160, h=120, x0=40, y0=30, x1=120, y1=90, lo=40, hi=200):
    img = np.full((h, w), lo, np.uint8)
    img[y0:y1, x0:x1] = hi
    return img


def test_rectangle_edges_found():
    img = _rect_image()
    prm = gfpl.LsdParams.reference(160, 120, n_features=0)
    kl, rsp, segs = O.lsd_detect(img, prm)
    assert len(kl) == 4
    # each keyline lies on one of the four edges (the step between pixel rows 29|30 etc. sits
    # at coordinate 30 in LSD's pixel-centre + 0.5 convention) and spans most of it
    edges = {"top": 0, "bottom": 0, "left": 0, "right": 0}
    for k in kl:
        sx, sy, ex, ey = float(k["sx"]), float(k["sy"]), float(k["ex"]), float(k["ey"])
        if abs(sy - ey) < 1.0:
            y = (sy + ey) / 2
            assert abs(y - 30) < 1.0 or abs(y - 90) < 1.0, (sx, sy, ex, ey)
            assert abs(abs(ex - sx) - 80) < 4
            edges["top" if y < 60 else "bottom"] += 1
        else:
            assert abs(sx - ex) < 1.0, (sx, sy, ex, ey)
            x = (sx + ex) / 2
            assert abs(x - 40) < 1.0 or abs(x - 120) < 1.0
            assert abs(abs(ey - sy) - 60) < 4
            edges["left" if x < 80 else "right"] += 1
    assert edges == {"top": 1, "bottom": 1, "left": 1, "right": 1}
    # KeyLine fields (LSDDetector_custom.cpp:281-299)
    for k, r in zip(kl, rsp):
        dx, dy = np.float32(k["ex"] - k["sx"]), np.float32(k["ey"] - k["sy"])
        ln = np.float32(math.sqrt(float(dx) ** 2 + float(dy) ** 2))
        assert r == np.float32(ln / np.float32(160))
        assert abs(float(k["angle"]) - math.atan2(float(dy), float(dx))) < 1e-6
        assert k["octave"] == 0


def test_flat_and_tiny_images():
    for w, h in ((8, 8), (64, 48)):
        kl, rsp, segs = O.lsd_detect(np.full((h, w), 77, np.uint8))
        assert len(kl) == 0 and len(segs) == 0


def test_min_length_and_nfeatures():
    w, h = 320, 240
    img = gfpl.synth_image(3, 0, w, h)
    all_kl, all_r, segs = O.lsd_detect(img, gfpl.LsdParams.reference(w, h, n_features=0))
    assert len(segs) >= len(all_kl) > 10
    min_len = 0.025 * 240
    lens = np.hypot(all_kl["ex"] - all_kl["sx"], all_kl["ey"] - all_kl["sy"])
    assert (lens > min_len - 1e-4).all()
    k = 7
    top, top_r, _ = O.lsd_detect(img, gfpl.LsdParams.reference(w, h, n_features=k))
    assert len(top) == k
    assert (np.diff(top_r) <= 0).all()
    assert np.isclose(top_r[0], all_r.max())
    # the kept set is the k largest responses (ties broken by std::sort's permutation)
    assert top_r[-1] >= np.sort(all_r)[::-1][k - 1]


def test_lines_of_the_staircase_scene():
    from gfpl import pipeline as P
    left, right, _, _ = P.synth_stereo_steps(0, 0, 640, 480)
    for img in (left, right):
        kl, rsp, segs = O.lsd_detect(img)
        assert 20 <= len(kl) <= 300
        assert (np.diff(rsp) <= 0).all() or len(kl) < 300


def test_lsd_params_match_reference_config():
    """gfpl.LsdParams.reference = StereoFrame's LSDOptions from Config (src/config.cpp:107,
    143-152; src/stereoFrame.cpp:151, 1163-1172)."""
    p = gfpl.LsdParams.reference(640, 480)
    assert (p.refine, p.scale, p.quant, p.ang_th, p.density_th, p.n_bins) == (1, 1.0, 2.0, 22.5, 0.6, 1024)
    assert p.n_features == 300 and p.min_length == 0.025 * 480


def test_unsupported_lsd_options_refused():
    img = np.zeros((16, 16), np.uint8)
    for f, v in (("refine", 2), ("scale", 0.8)):
        prm = gfpl.LsdParams.reference(16, 16)
        setattr(prm, f, v)
        with pytest.raises(RuntimeError):
            O.lsd_detect(img, prm)
