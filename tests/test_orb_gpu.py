"""GPU ORB extraction (gfpl_orb_extract, k_orb.hip) vs the CPU oracle
(gfplo_orb_extract), SURVEY.md §8(f)1.  Bar: bit-exact — keypoint coordinates,
octaves, angles, responses, descriptors and the pyramid bytes, in the reference's
output order, for every image of a batch."""
import numpy as np
import pytest

import gfpl
import oracle as O

pytestmark = pytest.mark.gpu


def _images(n, w, h, seq0, noise=0):
    imgs = np.stack([gfpl.synth_image(seq0 + i, i, w, h) for i in range(n)])
    if noise:
        rng = np.random.default_rng(seq0)
        imgs = np.clip(imgs.astype(int) + rng.integers(-noise, noise + 1, imgs.shape), 0, 255).astype(np.uint8)
    return imgs


def _run_gpu(orb, imgs):
    import torch
    n, h, w = imgs.shape
    kc = orb.kp_cap
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(imgs).to(dev)
    kps = torch.zeros(n * kc * gfpl.KEYPOINT_DT.itemsize, dtype=torch.uint8, device=dev)
    desc = torch.zeros(n * kc * 32, dtype=torch.uint8, device=dev)
    nkp = torch.zeros(n, dtype=torch.int32, device=dev)
    ang = torch.zeros(n * kc, dtype=torch.float32, device=dev)
    rsp = torch.zeros(n * kc, dtype=torch.float32, device=dev)
    stride = (orb.pyramid_bytes + 255) // 256 * 256
    pyr = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    orb.extract(d_img, n, kps, desc, nkp, ang, rsp, pyr, stride)
    return (kps.cpu().numpy().view(gfpl.KEYPOINT_DT).reshape(n, kc), desc.cpu().numpy().reshape(n, kc, 32),
            nkp.cpu().numpy(), ang.cpu().numpy().reshape(n, kc), rsp.cpu().numpy().reshape(n, kc),
            pyr.cpu().numpy().reshape(n, stride))


def _compare(orb, imgs, nfeatures, nlevels, scale=1.2):
    k, d, nk, a, r, p = _run_gpu(orb, imgs)
    total = 0
    for i, img in enumerate(imgs):
        o = O.orb_extract(img, nfeatures=nfeatures, scale_factor=scale, nlevels=nlevels, kp_cap=orb.kp_cap)
        n = len(o["kps"])
        assert nk[i] == n, (i, nk[i], n)
        assert (k[i, :n] == o["kps"]).all(), i
        assert (a[i, :n].view(np.uint32) == o["angle"].view(np.uint32)).all(), i
        assert (r[i, :n] == o["response"]).all(), i
        assert (d[i, :n] == o["desc"]).all(), i
        pb = orb.pyramid_bytes
        assert (p[i, :pb] == o["pyramid"][:pb]).all(), i
        total += n
    return total


@pytest.mark.parametrize("cam", ["vga", "euroc", "kitti"])
def test_orb_parity_batch(cam):
    c = gfpl.CAMERAS[cam]
    orb = gfpl.ORBextractor(2000, 1.2, 4, 20, 7, c["width"], c["height"], max_images=3)
    n = _compare(orb, _images(3, c["width"], c["height"], 40), 2000, 4)
    assert n > 900


def test_orb_parity_textured_many_corners():
    """Heavy texture: far more FAST corners than the quotas, so DistributeOctTree runs its
    second (sorted-expansion) phase on every level."""
    orb = gfpl.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_images=2)
    n = _compare(orb, _images(2, 640, 480, 7, noise=40), 1000, 8)
    assert n >= 990


@pytest.mark.parametrize("nf,nl,sf", [(500, 3, 1.3), (150, 5, 1.2), (8000, 4, 1.2)])
def test_orb_parity_params(nf, nl, sf):
    orb = gfpl.ORBextractor(nf, sf, nl, 20, 7, 752, 480, max_images=2)
    _compare(orb, _images(2, 752, 480, 91, noise=10), nf, nl, sf)


def test_orb_edge_images():
    """Flat (no corners), small (one or two 30-px cells per level) and a single bright
    square; and the sizes the reference cannot handle (a level without a cell) refused."""
    orb = gfpl.ORBextractor(2000, 1.2, 3, 20, 7, 128, 112, max_images=3)
    sq = np.full((112, 128), 40, np.uint8)
    sq[40:70, 45:90] = 220
    imgs = np.stack([np.full((112, 128), 90, np.uint8), _images(1, 128, 112, 5, noise=30)[0], sq])
    _compare(orb, imgs, 2000, 3)
    _, _, nk, _, _, _ = _run_gpu(orb, imgs[:1])
    assert nk[0] == 0
    with pytest.raises(gfpl.GfplError):
        gfpl.ORBextractor(2000, 1.2, 5, 20, 7, 128, 112)      # level 4 has no 30-px cell row
    with pytest.raises(RuntimeError):
        O.orb_extract(imgs[0], nlevels=5)


def test_orb_host_call_matches_oracle():
    """operator()(image) on a host image: keypoints as cv::KeyPoint fields, mvImagePyramid."""
    c = gfpl.CAMERAS["vga"]
    orb = gfpl.ORBextractor(2000, 1.2, 4, 20, 7, c["width"], c["height"])
    img = _images(1, c["width"], c["height"], 77)[0]
    kps, desc = orb(img)
    o = O.orb_extract(img)
    assert (kps["x"] == o["kps"]["x"]).all() and (kps["octave"] == o["kps"]["octave"]).all()
    assert (kps["size"] == np.float32(31) * orb.GetScaleFactors()[kps["octave"]]).all()
    assert (desc == o["desc"]).all()
    assert orb.mvImagePyramid[0].shape == (480, 640) and (orb.mvImagePyramid[0] == img).all()
    assert [p.shape for p in orb.mvImagePyramid] == [(h, w) for (w, h) in orb.level_sizes()]


def test_orb_rejects_bad_arguments():
    with pytest.raises(gfpl.GfplError):
        gfpl.ORBextractor(2000, 1.2, 9, 20, 7, 640, 480)       # > GFPL_MAX_LEVELS
    with pytest.raises(gfpl.GfplError):
        gfpl.ORBextractor(2000, 1.0, 4, 20, 7, 640, 480)       # scale factor must be > 1
    orb = gfpl.ORBextractor(2000, 1.2, 4, 20, 7, 640, 480, max_images=1)
    with pytest.raises(gfpl.GfplError):
        orb.extract(None, 2, None, None, None)                # n > max_images


def test_orb_pyramid_is_the_trackers_right_pyramid():
    """The right pyramid the tracker's sub-pixel SAD reads (gfpl_frames.pyr_r) written by
    gfpl_orb_extract straight into the device frame buffers (no PCIe): the GPU pyramid of
    each right image equals the oracle's, and tracking on it stays bit-exact with the oracle
    tracking on the oracle's pyramid."""
    import torch
    from test_gpu_parity import _check, _run_sequence
    seen = {}

    def host_pyr(H):
        cam = H.cam
        for f in range(H.F):
            for b in range(H.B):
                img = gfpl.synth_image(500 + b, f, cam.width, cam.height)
                o = O.orb_extract(img, nfeatures=2000, scale_factor=1.2, nlevels=cam.n_levels)
                pb = int(sum(cam.lvl_cols[l] * cam.lvl_rows[l] for l in range(cam.n_levels)))
                H.pyr_r[f, b, :pb] = o["pyramid"][:pb]
        return H

    def dev_hook(cam, H, D):
        orb = gfpl.ORBextractor(2000, 1.2, cam.n_levels, 20, 7, cam.width, cam.height, max_images=H.B)
        assert [int(cam.lvl_offset[l]) for l in range(cam.n_levels)] == list(
            np.cumsum([0] + [cam.lvl_cols[l] * cam.lvl_rows[l] for l in range(cam.n_levels - 1)]))
        kc = orb.kp_cap
        dev = torch.device("cuda", 0)
        kps = torch.zeros(H.B * kc * gfpl.KEYPOINT_DT.itemsize, dtype=torch.uint8, device=dev)
        desc = torch.zeros(H.B * kc * 32, dtype=torch.uint8, device=dev)
        nkp = torch.zeros(H.B, dtype=torch.int32, device=dev)
        pb = orb.pyramid_bytes
        for f in range(H.F):
            imgs = np.stack([gfpl.synth_image(500 + b, f, cam.width, cam.height) for b in range(H.B)])
            pyr = D.bufs[12][f]                       # [B * cam.pyr_bytes] device bytes
            view = pyr.view(H.B, int(cam.pyr_bytes))
            view[:, :pb] = 0                          # the ORB launch must write every level byte
            torch.cuda.synchronize()
            orb.extract(torch.from_numpy(imgs).to(dev), H.B, kps, desc, nkp, None, None, pyr, int(cam.pyr_bytes))
            got = view[:, :pb].cpu().numpy()
            assert (got == H.pyr_r[f, :, :pb]).all(), f
        seen["ok"] = True

    rep = _run_sequence("vga", {}, n_seq=2, n_frames=3, kp_cap=2048, kl_cap=512, mutate=host_pyr, dev_hook=dev_hook)
    assert seen.get("ok")
    _check(rep)


def test_orb_pyramid_for_the_tracker_must_match_the_camera():
    """gfpl_orb_extract refuses to write the tracker's right pyramid (a context camera of the
    image size, stride = its pyr_bytes) with other level geometry (e.g. another scale factor):
    the sub-pixel SAD would silently read other pixels (GFPL_E_INVALID)."""
    import torch
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    ctx = gfpl.Context(cam, cfg)
    W, H = int(cam.width), int(cam.height)
    dev = torch.device("cuda", 0)
    img = torch.from_numpy(gfpl.synth_image(1, 0, W, H)).to(dev)
    for scale, ok in ((1.2, True), (1.3, False)):
        orb = gfpl.ORBextractor(1000, scale, int(cam.n_levels), 20, 7, W, H, ctx=ctx)
        kc = orb.kp_cap
        kps = torch.zeros(kc * gfpl.KEYPOINT_DT.itemsize, dtype=torch.uint8, device=dev)
        desc = torch.zeros(kc * 32, dtype=torch.uint8, device=dev)
        nkp = torch.zeros(1, dtype=torch.int32, device=dev)
        pyr = torch.zeros(int(cam.pyr_bytes), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        if ok:
            orb.extract(img, 1, kps, desc, nkp, None, None, pyr, int(cam.pyr_bytes))
        else:
            with pytest.raises(gfpl.GfplError) as e:
                orb.extract(img, 1, kps, desc, nkp, None, None, pyr, int(cam.pyr_bytes))
            assert e.value.code == -1
            # any other stride is a pyramid for some other consumer: not checked
            orb.extract(img, 1, kps, desc, nkp, None, None, torch.zeros(orb.pyramid_bytes + 256, dtype=torch.uint8,
                                                                          device=dev), orb.pyramid_bytes + 256)
        orb.close()


def test_orb_async_on_own_stream_context_with_events():
    """The FFI form of stream ordering: a context with its own stream (gfpl_create_async),
    ORB extraction enqueued there (gfpl_orb_extract_async), an event recorded on it and
    waited for by a second context's stream; the host waits on the event only."""
    import torch
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    det = gfpl.Context(cam, cfg, own_stream=True)
    trk = gfpl.Context(cam, cfg)
    assert det.stream != 0 and det.stream != trk.stream
    W, H = int(cam.width), int(cam.height)
    img_np = gfpl.synth_image(4, 2, W, H)
    dev = torch.device("cuda", 0)
    img = torch.from_numpy(img_np).to(dev)
    orb = gfpl.ORBextractor(2000, 1.2, 4, 20, 7, W, H, ctx=det)
    kc = orb.kp_cap
    kps = torch.zeros(kc * gfpl.KEYPOINT_DT.itemsize, dtype=torch.uint8, device=dev)
    desc = torch.zeros(kc * 32, dtype=torch.uint8, device=dev)
    nkp = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ev = gfpl.Event(det)
    orb.extract_async(img, 1, kps, desc, nkp)
    ev.record(det)
    ev.wait(trk)
    ev.synchronize()
    orb.status()
    o = O.orb_extract(img_np, kp_cap=kc)
    n = int(nkp.cpu()[0])
    assert n == len(o["kps"])
    assert (kps.cpu().numpy().view(gfpl.KEYPOINT_DT)[:n] == o["kps"]).all()
    assert (desc.cpu().numpy().reshape(kc, 32)[:n] == o["desc"]).all()
    orb.close()
    ev.close()
    det.close()
