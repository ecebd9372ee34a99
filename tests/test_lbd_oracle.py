"""Known-answer tests of the CPU LBD oracle (oracle/gfpl_lbd_oracle.cpp).

The descriptor's arithmetic lives in OpenCV 3.4.1 (GaussianBlur, Sobel) and libm, absent here:
PARITY UNPINNED against the reference binary (DESIGN.md ledger L1-L5).  The pieces are
checked against independent numpy / pure-Python statements of the same algorithms; the
float LBD vector of a few lines is recomputed step by step in numpy float32 from the
reference's computeLBD (binary_descriptor_custom.cpp:1026-1372)."""
import math

import numpy as np
import pytest

import gfpl
import oracle as O
from lbd_common import synth_keylines


def _refl(i, n):
    i = np.abs(i)
    return np.where(i >= n, 2 * n - 2 - i, i)


def test_blur_taps_and_sobel_are_exact():
    cf = [np.float32(math.exp(-0.5 * (i - 2) ** 2)) for i in range(5)]
    s = 1.0 / float(sum(float(v) for v in cf))
    k = np.array([int(np.rint(np.float32(float(v) * s) * np.float32(256))) for v in cf])
    assert k.tolist() == [14, 63, 103, 63, 14]   # L1: sum 257
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    h, w = img.shape
    pad = img.astype(np.int64)[_refl(np.arange(-2, h + 2), h)][:, _refl(np.arange(-2, w + 2), w)]
    rows = sum(k[t] * pad[:, t:t + w] for t in range(5))
    ref = np.clip((sum(k[t] * rows[t:t + h] for t in range(5)) + (1 << 15)) >> 16, 0, 255)
    b, dx, dy = O.lbd_gradients(img)
    assert (b == ref).all()
    bp = ref[_refl(np.arange(-1, h + 1), h)][:, _refl(np.arange(-1, w + 1), w)]
    gx = (bp[:-2, 2:] - bp[:-2, :-2]) + 2 * (bp[1:-1, 2:] - bp[1:-1, :-2]) + (bp[2:, 2:] - bp[2:, :-2])
    gy = (bp[2:, :-2] - bp[:-2, :-2]) + 2 * (bp[2:, 1:-1] - bp[:-2, 1:-1]) + (bp[2:, 2:] - bp[:-2, 2:])
    assert (dx == gx).all() and (dy == gy).all()


def test_coefficients_and_pixels():
    cl, cg = O.lbd_coefs()
    assert cl.argmax() == 10 and cl[10] == 1.0 and np.allclose(cl, np.exp(-((np.arange(21) - 10.0) ** 2) / (2 * 7.0 ** 2)))
    assert cg.argmax() == 31 and np.allclose(cg, np.exp(-((np.arange(63) - 31.0) ** 2) / (2 * 31.0 ** 2)))
    k = np.zeros(1, gfpl.KEYLINE_DT)
    k[0] = (10.4, 20.6, 30.5, 21.5, 0.0, 0)   # rounded (10, 21) -> (30, 22): dx 20, dy 1
    assert O.lbd_num_pixels(k[0]) == 21
    k[0] = (5.0, 5.0, 5.0, 5.0, 0.0, 0)
    assert O.lbd_num_pixels(k[0]) == 1


def test_flat_image_gives_zero_descriptors():
    kl = synth_keylines(5, 120, 90, 3)
    d, f = O.lbd_compute(np.full((90, 120), 77, np.uint8), kl)
    assert (d == 0).all() and np.isnan(f).all()   # 0 / 0 normalisations: NaN, no comparison holds


def _lbd_py(img, kl):
    """computeLBD for one line in numpy float32, statement by statement."""
    f32 = np.float32
    _, gx, gy = O.lbd_gradients(img)
    h, w = img.shape
    cl, cg = O.lbd_coefs()
    L = O.lbd_num_pixels(kl)
    hw, hh = (L - 1) // 2, 31
    mx = f32(0.5 * float(f32(kl["sx"]) + f32(kl["ex"])))
    my = f32(0.5 * float(f32(kl["sy"]) + f32(kl["ey"])))
    d0, d1 = f32(O.cos(float(kl["angle"]))), f32(O.sin(float(kl["angle"])))
    o0, o1 = -d1, d0
    sx0 = f32(f32(f32(-d0) * f32(hw)) + f32(d1 * f32(hh))) + mx
    sy0 = f32(f32(f32(-d1) * f32(hw)) - f32(d0 * f32(hh))) + my
    band = np.zeros((9, 8), np.float32)   # pL nL pL2 nL2 pO nO pO2 nO2
    rnd = lambda v: int(math.copysign(math.floor(abs(float(v)) + 0.5), float(v)))
    for r in range(63):
        sx, sy = sx0, sy0
        acc = [f32(0)] * 4
        for _ in range(L):
            xc = min(max(rnd(sx), 0), w - 1)
            yc = min(max(rnd(sy), 0), h - 1)
            dx, dy = f32(gx[yc, xc]), f32(gy[yc, xc])
            gdl = f32(dx * d0) + f32(dy * d1)
            gdo = f32(dx * o0) + f32(dy * o1)
            if gdl > 0: acc[0] = f32(acc[0] + gdl)
            else: acc[1] = f32(acc[1] - gdl)
            if gdo > 0: acc[2] = f32(acc[2] + gdo)
            else: acc[3] = f32(acc[3] - gdo)
            sx, sy = f32(sx + d0), f32(sy + d1)
        sx0, sy0 = f32(sx0 - d1), f32(sy0 + d0)
        pl, nl, po, no = (f32(cg[r] * a) for a in acc)
        row = [pl, nl, f32(pl * pl), f32(nl * nl), po, no, f32(po * po), f32(no * no)]
        b = r // 7
        for bb, c in ((b, cl[r % 7 + 7]), (b - 1, cl[r % 7 + 14]), (b + 1, cl[r % 7])):
            if 0 <= bb < 9:
                for s in range(8):
                    t = f32(f32(c * c) * row[s]) if s in (2, 3, 6, 7) else f32(c * row[s])
                    band[bb, s] = f32(band[bb, s] + t)
    dv = np.zeros(72, np.float32)
    for b in range(9):
        inv = f32(1.0 / 14.0) if b in (0, 8) else f32(1.0 / 21.0)
        for k, (m, q) in enumerate(((0, 2), (1, 3), (4, 6), (5, 7))):
            t = f32(band[b, m] * inv)
            dv[8 * b + k] = t
            with np.errstate(invalid="ignore"):
                dv[8 * b + 4 + k] = np.sqrt(f32(f32(band[b, q] * inv) - f32(t * t)))
    tm = ts = f32(0)
    for b in range(9):
        for k in range(4): tm = f32(tm + f32(dv[8 * b + k] * dv[8 * b + k]))
        for k in range(4, 8): ts = f32(ts + f32(dv[8 * b + k] * dv[8 * b + k]))
    tm, ts = f32(f32(1) / np.sqrt(tm)), f32(f32(1) / np.sqrt(ts))
    for i in range(72):
        dv[i] = f32(dv[i] * (tm if i % 8 < 4 else ts))
        if float(dv[i]) > 0.4: dv[i] = f32(0.4)
    t = f32(0)
    for i in range(72): t = f32(t + f32(dv[i] * dv[i]))
    t = f32(f32(1) / np.sqrt(t))
    return np.array([f32(v * t) for v in dv], np.float32)


def test_lbd_vector_matches_statement_by_statement_numpy():
    img = gfpl.synth_image(9, 1, 160, 120)
    kl = synth_keylines(3, 160, 120, 11, max_len=60.0)
    d, f = O.lbd_compute(img, kl)
    for i in range(3):
        ref = _lbd_py(img, kl[i])
        assert (f[i].view(np.uint32) == ref.view(np.uint32)).all(), i
    # binarisation: byte c compares bands of pair c bit by bit (combinations :74-106)
    pairs = [(i, j) for i in range(9) for j in range(i + 1, 9) if not (i <= 1 and j >= 7)]
    assert len(pairs) == 32 and pairs[0] == (0, 1) and pairs[15] == (2, 7) and pairs[-1] == (7, 8)
    for i in range(3):
        for c, (a, b) in enumerate(pairs):
            byte = sum(1 << k for k in range(8) if f[i, 8 * a + k] > f[i, 8 * b + k])
            assert d[i, c] == byte


def test_descriptor_properties_and_order():
    img = gfpl.synth_image(4, 0, 320, 240)
    kl = synth_keylines(40, 320, 240, 5, border=True)
    d, f = O.lbd_compute(img, kl)
    ok = ~np.isnan(f).any(axis=1)
    assert ok.sum() >= 38
    assert np.allclose(np.linalg.norm(f[ok], axis=1), 1.0, atol=1e-5)
    # descriptors are per line: a permutation of the keylines permutes the rows
    perm = np.random.default_rng(1).permutation(40)
    d2, _ = O.lbd_compute(img, kl[perm])
    assert (d2 == d[perm]).all()
    with pytest.raises(RuntimeError):
        k2 = kl.copy(); k2["octave"][3] = 1
        O.lbd_compute(img, k2)
