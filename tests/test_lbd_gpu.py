"""GPU LBD descriptors (gfpl_lbd_compute, k_lbd.hip) vs the CPU oracle (gfplo_lbd_compute),
SURVEY.md §8(f)2 (descriptor part).  Bar: bit-exact 32-byte descriptors for every keyline
of every image of a batch."""
import numpy as np
import pytest

import gfpl
import oracle as O
from lbd_common import synth_keylines

pytestmark = pytest.mark.gpu


def _run(lbd, imgs, kls, counts):
    import torch
    n, h, w = imgs.shape
    cap = lbd.kl_cap
    dev = torch.device("cuda", 0)
    kl = np.zeros((n, cap), gfpl.KEYLINE_DT)
    for i in range(n):
        kl[i, :counts[i]] = kls[i][:counts[i]]
    d_img = torch.from_numpy(imgs).to(dev)
    d_kl = torch.from_numpy(kl.view(np.uint8).reshape(-1)).to(dev)
    d_n = torch.tensor(counts, dtype=torch.int32, device=dev)
    d_desc = torch.zeros(n * cap * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    lbd.compute_batch(d_img, n, d_kl, d_n, d_desc)
    return d_desc.cpu().numpy().reshape(n, cap, 32)


@pytest.mark.parametrize("cam", ["vga", "euroc", "kitti"])
def test_lbd_parity_batch(cam):
    c = gfpl.CAMERAS[cam]
    w, h = c["width"], c["height"]
    n = 3
    imgs = np.stack([gfpl.synth_image(20 + i, i, w, h) for i in range(n)])
    kls = [synth_keylines(300, w, h, 100 + i, border=(i == 2)) for i in range(n)]
    counts = [300, 217, 300]
    lbd = gfpl.BinaryDescriptor(w, h, max_images=n, kl_cap=320)
    got = _run(lbd, imgs, kls, counts)
    for i in range(n):
        ref, _ = O.lbd_compute(imgs[i], kls[i][:counts[i]])
        assert (got[i, :counts[i]] == ref).all(), (i, np.argwhere((got[i, :counts[i]] != ref).any(axis=1))[:5].ravel())


def test_lbd_edge_cases():
    """Points (1 pixel), segments on the image border (clamped samples), very long
    segments, an empty image of the batch, a flat image."""
    w, h = 200, 150
    k = np.zeros(6, gfpl.KEYLINE_DT)
    k[0] = (50.0, 50.0, 50.0, 50.0, 0.0, 0)
    k[1] = (0.0, 0.0, 199.0, 0.0, 0.0, 0)
    k[2] = (199.0, 149.0, 0.0, 0.0, np.arctan2(np.float32(-149), np.float32(-199)), 0)
    k[3] = (0.0, 75.5, 0.0, 10.25, np.float32(-np.pi / 2), 0)
    k[4] = (10.5, 10.5, 11.5, 12.5, np.arctan2(np.float32(2), np.float32(1)), 0)
    k[5] = (199.0, 0.0, 0.0, 149.0, np.arctan2(np.float32(149), np.float32(-199)), 0)
    imgs = np.stack([gfpl.synth_image(3, 0, w, h), gfpl.synth_image(4, 0, w, h), np.full((h, w), 60, np.uint8)])
    lbd = gfpl.BinaryDescriptor(w, h, max_images=3, kl_cap=8)
    got = _run(lbd, imgs, [k, k, k], [6, 0, 6])
    for i, cnt in ((0, 6), (2, 6)):
        ref, _ = O.lbd_compute(imgs[i], k[:cnt])
        assert (got[i, :cnt] == ref).all(), i
    assert (got[2, :6] == 0).all()


def test_lbd_host_call_and_octave_refusal():
    w, h = 320, 240
    img = gfpl.synth_image(7, 2, w, h)
    kl = synth_keylines(50, w, h, 8)
    lbd = gfpl.BinaryDescriptor(w, h, kl_cap=64)
    ref, _ = O.lbd_compute(img, kl)
    assert (lbd.compute(img, kl) == ref).all()
    kl["octave"][10] = 1
    with pytest.raises(gfpl.GfplError):
        lbd.compute(img, kl)


def test_lbd_more_keylines_than_capacity_is_an_error():
    """The reference describes every keyline: n_kl > kl_cap is GFPL_E_CAPACITY (the first kl_cap
    rows are still described), like LSD's and ORB's capacity errors; the asynchronous form
    reports it through gfpl_lbd_status, and the status clears after it is read."""
    import torch
    w, h = 320, 240
    img = gfpl.synth_image(7, 0, w, h)
    kl = synth_keylines(40, w, h, 3)
    lbd = gfpl.BinaryDescriptor(w, h, max_images=1, kl_cap=40)
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(img).to(dev)
    d_kl = torch.from_numpy(kl.view(np.uint8).reshape(-1)).to(dev)
    d_desc = torch.zeros(40 * 32, dtype=torch.uint8, device=dev)
    over = torch.tensor([41], dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    with pytest.raises(gfpl.GfplError) as e:
        lbd.compute_batch(d_img, 1, d_kl, over, d_desc)
    assert e.value.code == -5
    assert (d_desc.cpu().numpy().reshape(40, 32) == O.lbd_compute(img, kl)[0]).all()
    lbd.compute_async(d_img, 1, d_kl, over, d_desc)
    with pytest.raises(gfpl.GfplError):
        lbd.status()
    lbd.status()   # cleared
    lbd.compute_batch(d_img, 1, d_kl, torch.tensor([40], dtype=torch.int32, device=dev), d_desc)
