"""GPU LSD line detection (gfpl_lsd_detect, k_lsd.hip) vs the CPU oracle (gfplo_lsd_detect),
SURVEY.md §8(f)2 (detector part).  Bar: bit-exact keylines (sx sy ex ey angle octave),
responses and counts for every image of a batch; the std::sort restatement (S2) equal to the
library's permutation on tie-heavy keys."""
import numpy as np
import pytest

import gfpl
import oracle as O
from gfpl import pipeline as P

pytestmark = pytest.mark.gpu


def _detect(det, imgs):
    import torch
    n, h, w = imgs.shape
    dev = torch.device("cuda", 0)
    cap = det.kl_cap
    d_img = torch.from_numpy(np.ascontiguousarray(imgs)).to(dev)
    d_kl = torch.zeros(n * cap * gfpl.KEYLINE_DT.itemsize, dtype=torch.uint8, device=dev)
    d_n = torch.zeros(n, dtype=torch.int32, device=dev)
    d_r = torch.zeros(n * cap, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    det.detect_batch(d_img, n, d_kl, d_n, d_r)
    kl = d_kl.cpu().numpy().view(gfpl.KEYLINE_DT).reshape(n, cap)
    return kl, d_n.cpu().numpy(), d_r.cpu().numpy().reshape(n, cap)


def _check(imgs, params=None, kl_cap=512):
    n, h, w = imgs.shape
    prm = params if params is not None else gfpl.LsdParams.reference(w, h)
    det = gfpl.LSDDetector(w, h, prm, max_images=n, kl_cap=kl_cap)
    kl, cnt, rsp = _detect(det, imgs)
    tot = 0
    for i in range(n):
        rk, rr, _ = O.lsd_detect(imgs[i], prm)
        assert cnt[i] == len(rk), (i, cnt[i], len(rk))
        g = kl[i, :cnt[i]]
        bad = np.argwhere(g.view(np.uint8).reshape(-1, 24) != rk.view(np.uint8).reshape(-1, 24))
        assert len(bad) == 0, (i, bad[:5], g[bad[0, 0]], rk[bad[0, 0]])
        assert (rsp[i, :cnt[i]].view(np.uint32) == rr.view(np.uint32)).all()
        tot += cnt[i]
    det.close()
    return tot


def test_lsd_parity_vga_batch():
    imgs = [gfpl.synth_image(20 + i, i, 640, 480) for i in range(2)]
    left, right, _, _ = P.synth_stereo_steps(1, 0, 640, 480)
    l2, r2, _, _ = P.synth_stereo_scene(2, 3, 640, 480)
    tot = _check(np.stack(imgs + [left, right, l2, r2]))
    assert tot > 100


@pytest.mark.parametrize("cam", ["euroc", "kitti"])
def test_lsd_parity_cameras(cam):
    c = gfpl.CAMERAS[cam]
    w, h = c["width"], c["height"]
    left, right, _, _ = P.synth_stereo_steps(3, 1, w, h)
    _check(np.stack([left, right, gfpl.synth_image(5, 0, w, h)]))


def test_lsd_parity_large_image():
    """1280 x 720: a 28.8 KB compact used map (a quarter of the pixels)."""
    w, h = 1280, 720
    left, _, _, _ = P.synth_stereo_steps(4, 0, w, h)
    _check(np.stack([left]), kl_cap=600)


def test_lsd_parity_mixed_used_maps():
    """One batch whose noise images define more than a quarter of their pixels (HBM byte map,
    k_lsd_grow_glb) between scene images (compact LDS bitmap, k_lsd_grow_lds)."""
    w, h = 320, 240
    rng = np.random.default_rng(11)
    noise = rng.integers(0, 256, (h, w)).astype(np.uint8)
    blocks = np.clip(noise.astype(np.int32) // 4 + np.kron(rng.integers(0, 4, (h // 40, w // 40)) * 60,
                                                           np.ones((40, 40), np.int32)), 0, 255).astype(np.uint8)
    left, right, _, _ = P.synth_stereo_steps(4, 0, w, h)
    ndef = [O.lsd_defined_count(im) for im in (noise, blocks, left)]
    assert ndef[0] > w * h // 4 and ndef[1] > w * h // 4 and ndef[2] < w * h // 4, ndef
    _check(np.stack([left, noise, right, blocks]), gfpl.LsdParams.reference(w, h, n_features=0), kl_cap=4096)


def test_lsd_keep_all_and_small_budget():
    w, h = 640, 480
    left, right, _, _ = P.synth_stereo_steps(5, 2, w, h)
    imgs = np.stack([left, gfpl.synth_image(6, 0, w, h)])
    _check(imgs, gfpl.LsdParams.reference(w, h, n_features=0), kl_cap=2048)
    _check(imgs, gfpl.LsdParams.reference(w, h, n_features=5), kl_cap=8)


def test_lsd_edge_images():
    w, h = 64, 48
    img = np.full((h, w), 90, np.uint8)
    img2 = img.copy()
    img2[10:40, 20:50] = 200
    _check(np.stack([img, img2, np.zeros((h, w), np.uint8)]), kl_cap=16)
    _check(np.stack([np.full((8, 8), 3, np.uint8)]), kl_cap=4)


@pytest.mark.parametrize("n,nkeys", [(17, 2), (700, 3), (2048, 1024), (2049, 7), (30000, 40), (150000, 1024),
                                     (100000, 1)])
def test_lsd_sort_matches_std_sort(n, nkeys):
    import torch
    rng = np.random.default_rng(n + nkeys)
    keys = rng.integers(0, nkeys, n).astype(np.uint64)
    a = (keys << np.uint64(32)) | np.arange(n, dtype=np.uint64)
    det = gfpl.LSDDetector(640, 480, max_images=1)
    d = torch.from_numpy(a.view(np.int64).copy()).to("cuda")
    det.sort_desc(d, n)
    got = d.cpu().numpy().view(np.uint64)
    assert (got == O.sort_desc(a)).all()
    det.close()


def test_lsd_feeds_lbd_on_device():
    """LSD keylines written straight where gfpl_lbd_compute reads them, bit-exact against the
    oracle LSD -> oracle LBD chain (StereoFrame::detectLineFeatures, src/stereoFrame.cpp:1175-1194)."""
    import torch
    w, h = 640, 480
    left, right, _, _ = P.synth_stereo_steps(7, 0, w, h)
    imgs = np.stack([left, right])
    n, cap = 2, 320
    det = gfpl.LSDDetector(w, h, max_images=n, kl_cap=cap)
    lbd = gfpl.BinaryDescriptor(w, h, max_images=n, kl_cap=cap)
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(imgs).to(dev)
    d_kl = torch.zeros(n * cap * gfpl.KEYLINE_DT.itemsize, dtype=torch.uint8, device=dev)
    d_n = torch.zeros(n, dtype=torch.int32, device=dev)
    d_desc = torch.zeros(n * cap * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    det.detect_batch(d_img, n, d_kl, d_n)
    lbd.compute_batch(d_img, n, d_kl, d_n, d_desc)
    desc = d_desc.cpu().numpy().reshape(n, cap, 32)
    cnt = d_n.cpu().numpy()
    for i in range(n):
        rk, _, _ = O.lsd_detect(imgs[i])
        rd, _ = O.lbd_compute(imgs[i], rk)
        assert cnt[i] == len(rk)
        assert (desc[i, :cnt[i]] == rd).all()


def _dense_image(seed, w, h):
    """Random rectangles, discs and ramps over noise: many regions, refinements and
    radius reductions."""
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 12, (h, w)).astype(np.int32) + 40
    yy, xx = np.mgrid[0:h, 0:w]
    for _ in range(40):
        x0, y0 = rng.integers(0, w), rng.integers(0, h)
        a, b = rng.integers(4, w // 3), rng.integers(4, h // 3)
        v = int(rng.integers(0, 200))
        k = rng.integers(0, 3)
        if k == 0:
            img[y0:y0 + b, x0:x0 + a] += v // 2
        elif k == 1:
            img[(xx - x0) ** 2 + (yy - y0) ** 2 < a * a] = v
        else:
            img += ((xx * int(rng.integers(-3, 4)) + yy * int(rng.integers(-3, 4))) // 7 % 3)
    return np.clip(img, 0, 255).astype(np.uint8)


def test_lsd_parity_dense_scenes():
    w, h = 640, 480
    _check(np.stack([_dense_image(s, w, h) for s in range(3)]), gfpl.LsdParams.reference(w, h, n_features=0),
           kl_cap=4096)


def test_lsd_parity_large_batch_small_lds_sort():
    """More than 4 images per CU: the sort runs with the 512-element LDS capacity (k_lsd_sort<512>)."""
    w, h = 96, 72
    n = 1100
    imgs = np.stack([_dense_image(1000 + i, w, h) if i % 50 == 0 else gfpl.synth_image(i, 0, w, h)
                     for i in range(n)])
    assert _check(imgs, kl_cap=64) > 0


def test_lsd_parity_dense_bar_scene():
    """The images -> poses bench scene at the north-star load (gfpl.pipeline: 600 anti-aliased bars
    per Mpx over the staircase): several hundred segments per image, the 300-keyline response cut
    (S7) deciding among them, and the keep-all budget — bit-exact against the oracle."""
    w, h = 640, 480
    imgs = []
    for seq, fr in ((0, 0), (9, 3), (31, 7)):
        left, right, _, _ = P.synth_stereo_steps(seq, fr, w, h, bars=600)
        imgs += [left, right]
    imgs = np.stack(imgs)
    tot = _check(imgs)
    assert tot == 300 * len(imgs), tot   # every image fills lsdNFeatures
    _check(imgs[:2], gfpl.LsdParams.reference(w, h, n_features=0), kl_cap=2048)
