"""Images -> detection -> tracking on one device (SURVEY.md §8(f)1-2 feeding rows a-e).

StereoFrame's detectFeatures (src/stereoFrame.cpp:1145-1200) runs ORB_SLAM2::ORBextractor on
both images, LSDDetectorC::detect and BinaryDescriptor::compute on both; here all three run on
the GPU (gfpl_orb_extract_async, gfpl_lsd_detect_async, gfpl_lbd_compute_async) straight into
the device buffers a gfpl_frames view points at — keypoints, descriptors, keylines, the right
pyramid for the sub-pixel SAD — so the tracker (StereoFrameHandler) reads them without a copy,
on a detection stream of its own, ordered with the tracker by events (no host synchronisation).
detect_images() is that whole path; detect() takes the keylines as an input instead.

The synthetic scene helper renders what a calibrated rig would see while translating along
x over a fronto-parallel textured plane: every pixel has the same disparity, the right image is
the left one shifted by it, and each frame shifts the view by a fixed number of pixels.
"""
from __future__ import annotations

import functools

import numpy as np

from . import (DESC, KEYLINE_DT, KEYPOINT_DT, BinaryDescriptor, Context, Event, LSDDetector, LsdParams,
               ORBextractor, make_frames, synth_image, synth_keylines)


def _draw_bars(img: np.ndarray, n: int, seed: int) -> np.ndarray:
    """n anti-aliased bars (rotated rectangles 30-110 px long, 8-24 px wide, dark or bright, none
    within 20 degrees of horizontal) over img: straight high-contrast edges LSD finds as segments
    (an aliased staircase edge breaks its level-line regions) and corners for FAST."""
    rng = np.random.default_rng(seed)
    h, w = img.shape
    out = img.astype(np.float32)
    for _ in range(n):
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        ln, wd = rng.uniform(30, 110), rng.uniform(8, 24)
        a = rng.uniform(0.35, np.pi - 0.35)
        ca, sa = np.float32(np.cos(a)), np.float32(np.sin(a))
        r = ln / 2 + wd / 2 + 2
        x0, x1 = int(max(0, cx - r)), int(min(w, cx + r + 1))
        y0, y1 = int(max(0, cy - r)), int(min(h, cy + r + 1))
        if x0 >= x1 or y0 >= y1:
            continue
        yy, xx = np.mgrid[y0:y1, x0:x1].astype(np.float32)
        X, Y = xx - np.float32(cx), yy - np.float32(cy)
        d = np.maximum(np.abs(X * ca + Y * sa) - np.float32(ln / 2), np.abs(Y * ca - X * sa) - np.float32(wd / 2))
        cov = np.clip(0.5 - d, 0.0, 1.0)
        val = np.float32(rng.integers(0, 2) * 190 + rng.integers(15, 50))
        blk = out[y0:y1, x0:x1]
        out[y0:y1, x0:x1] = blk + (val - blk) * cov
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


@functools.lru_cache(maxsize=4096)
def _plane(seq: int, base_w: int, height: int, n_segs: int, bars: int = 0, flat: bool = False):
    base = synth_image(0xB45E + seq, 0, base_w, height)
    if flat:   # a plain grey plane with mild noise (only the bars give features)
        rng = np.random.default_rng(0xF1A7 + seq)
        base = (118 + rng.integers(0, 21, base.shape)).astype(np.uint8)
    if bars:
        base = _draw_bars(base, bars, 0xBA25 + seq)
    base.setflags(write=False)
    segs = synth_keylines(n_segs, base_w, height, 0x5E65 + seq, min_len=8.0, max_len=120.0)
    segs.setflags(write=False)
    return base, segs


def synth_stereo_scene(seq: int, frame: int, width: int, height: int, disparity: int = 12, step_px: int = 2,
                       n_lines: int = 300, frames: int = 64):
    """Left / right grey images of a textured plane seen from a camera translating along x
    (every frame `step_px` pixels), and the plane's line segments as keylines in both images
    (those leaving the view dropped).  Returns (left, right, kl_left, kl_right)."""
    base_w = width + disparity + step_px * frames + 8
    base, segs = _plane(seq, base_w, height, n_lines * 3)
    off = step_px * frame
    left = np.ascontiguousarray(base[:, off:off + width])
    right = np.ascontiguousarray(base[:, off + disparity:off + disparity + width])
    def view(shift):
        k = segs.copy()
        k["sx"] -= shift
        k["ex"] -= shift
        inside = (k["sx"] >= 0) & (k["ex"] >= 0) & (k["sx"] <= width - 1) & (k["ex"] <= width - 1)
        return k[inside]

    kl_l, kl_r = view(off), view(off + disparity)
    # the same plane segments on both sides, LSD's cap (Config::lsdNFeatures) on the left count
    return left, right, kl_l[:n_lines], kl_r[:n_lines]


def synth_stereo_steps(seq: int, frame: int, width: int, height: int, disparities=(2, 12, 20, 8), band: int = 96,
                       n_lines: int = 300, frames: int = 64, bars: int = 0, bar_min_disp: int = 0):
    """A staircase of fronto-parallel textured bands (world columns [band i, band (i+1)) at
    disparity disparities[i % len]) seen from a camera translating along x by half a baseline
    per frame: band b moves d_b / 2 px per frame in the left image and sits d_b px further
    left in the right one; nearer bands occlude farther ones, and columns no band covers show
    the farthest band's texture.  Unlike the single plane, the depth spread keeps the pose
    information of the lines well conditioned (the single plane couples rotation and
    translation, and the line cut then takes the reference's exact step at every step).
    Keylines are the plane segments lying inside one band, shifted per view and kept when both
    endpoints stay in the image.  bars: anti-aliased bars drawn over the plane's texture per
    `bars` per 1000 x 1000 px of it (the north-star load: ~2000 ORB keypoints and >= 300 LSD
    keylines per VGA image at 500; 0 keeps the plain texture, ~50 keylines per image).
    Returns (left, right, kl_left, kl_right)."""
    ds = [int(d) for d in disparities]
    assert all(d % 2 == 0 and d > 0 for d in ds)
    dmax = max(ds)
    base_w = width + dmax * (frames // 2 + 1) + band
    nb = int(round(bars * base_w * height / 1e6))
    base, segs = _plane(seq, base_w, height, n_lines * 6, nb)
    # bar_min_disp > 0: bands at that disparity or more show bars on a plain plane instead (their
    # features are then the bars' edges and corners; the textured near-field bands carry the points)
    base_b = _plane(seq, base_w, height, n_lines * 6, nb, True)[0] if bar_min_disp else base
    n_band = (base_w + band - 1) // band
    disp = [ds[i % len(ds)] for i in range(n_band)]
    far = min(ds)
    views = []
    for side in range(2):
        shift = lambda d: (frame * d) // 2 + (d if side else 0)
        img = np.ascontiguousarray(base[:, shift(far):shift(far) + width])   # the far layer
        for i in sorted(range(n_band), key=lambda i: disp[i]):   # far to near: near bands occlude
            u0, u1 = i * band, min((i + 1) * band, base_w)
            x0, x1 = u0 - shift(disp[i]), u1 - shift(disp[i])
            c0, c1 = max(x0, 0), min(x1, width)
            if c0 < c1:
                src = base_b if bar_min_disp and disp[i] >= bar_min_disp else base
                img[:, c0:c1] = src[:, u0 + (c0 - x0):u0 + (c1 - x0)]
        views.append(img)
    bi = np.floor(segs["sx"] / band).astype(np.int64)
    same = (bi == np.floor(segs["ex"] / band).astype(np.int64))
    inner = (np.minimum(segs["sx"], segs["ex"]) >= bi * band + 2) & (np.maximum(segs["sx"], segs["ex"]) <= (bi + 1) * band - 3)
    pool = segs[same & inner]
    d_of = np.array(disp, np.int64)[np.floor(pool["sx"] / band).astype(np.int64)]
    kls = []
    for side in range(2):
        k = pool.copy()
        sh = ((frame * d_of) // 2 + (d_of if side else 0)).astype(np.float32)
        k["sx"] -= sh
        k["ex"] -= sh
        kls.append(k)
    inside = np.ones(len(pool), bool)
    for k in kls:
        inside &= (k["sx"] >= 0) & (k["ex"] >= 0) & (k["sx"] <= width - 1) & (k["ex"] <= width - 1)
    return views[0], views[1], kls[0][inside][:n_lines], kls[1][inside][:n_lines]


class ImagePipeline:
    """Detection for B sequences on the device, as gfpl_frames for StereoFrameHandler:
    ORB (nfeatures, Config::orbScaleFactor / orbNLevels of the configuration, FAST 20 / 7),
    LSD (lsd=True: the reference's LSDOptions, Config::lsdNFeatures = 300, min length
    0.025 * min(W, H)) and LBD.

    Detection runs on two contexts of its own (two streams: ORB on one, LSD then LBD on the
    other, so ORB of a batch overlaps its latency-bound LSD; the two join before `ready`) into
    `sets` buffer sets in turn, through the stream-ordered detector calls (gfpl_*_async).  Every
    gfpl_frames it returns carries two events: `ready` (its detection is done) and
    `consumed` (recorded by the tracker call that reads it, gfpl_frames.ready / consumed),
    so a tracker call on another context waits for exactly that detection and the next
    detection into the same set waits for exactly that read: detecting frame k + 1 while
    frame k is tracked needs no host synchronisation.  At most `sets` views may be
    outstanding: detecting into a set whose last view no tracker call has read yet raises
    (discard() releases a view that will not be tracked).  Capacity / octave errors of the
    asynchronous detectors are reported by status(); device outputs are complete after
    synchronize() (status() waits for the detectors' own status words only)."""

    def __init__(self, ctx: Context, cam, batch: int, kl_cap: int, nfeatures: int = 2000, lsd: bool = False,
                 cfg=None, sets: int = 2):
        import torch
        cfg = cfg if cfg is not None else ctx.cfg
        self.ctx, self.cam, self.B, self.kl_cap, self.sets = ctx, cam, batch, kl_cap, sets
        W, H = int(cam.width), int(cam.height)
        # the detection stream is a torch stream (pooled by torch, never destroyed), so torch's
        # allocator may record the inputs' use on it (Tensor.record_stream)
        self._tstream = torch.cuda.Stream(device=torch.device("cuda", ctx.device))
        self._ostream = torch.cuda.Stream(device=torch.device("cuda", ctx.device))
        self.det = Context(cam, cfg, device=ctx.device, stream=self._tstream.cuda_stream)
        self.det_orb = Context(cam, cfg, device=ctx.device, stream=self._ostream.cuda_stream)
        self.orb = ORBextractor(nfeatures, float(cfg.orb_scale_factor), int(cfg.orb_n_levels), 20, 7, W, H,
                                max_images=batch, ctx=self.det_orb)
        # the extractor writes the tracker's right pyramid (gfpl_frames.pyr_r): its levels must
        # be the camera's (gfpl_orb_extract checks it as well)
        geo = [(int(cam.lvl_cols[l]), int(cam.lvl_rows[l])) for l in range(int(cam.n_levels))]
        if self.orb.level_sizes() != geo or self.orb.pyramid_bytes > int(cam.pyr_bytes):
            raise ValueError(f"ORB pyramid {self.orb.level_sizes()} ({self.orb.pyramid_bytes} B) does not match the "
                             f"camera's {geo} ({int(cam.pyr_bytes)} B): build both from the same config")
        self.lbd = BinaryDescriptor(W, H, max_images=batch, kl_cap=kl_cap, ctx=self.det)
        # both images of the B stereo frames go through LSD in one call (2B images in flight)
        self.lsd = LSDDetector(W, H, LsdParams.reference(W, H), max_images=2 * batch, kl_cap=kl_cap,
                               ctx=self.det) if lsd else None
        self.kp_cap = self.orb.kp_cap
        dev = torch.device("cuda", ctx.device)
        B, kc = batch, self.kp_cap
        z = lambda n, dt=torch.uint8: torch.zeros(n, dtype=dt, device=dev)
        kls = B * kl_cap * KEYLINE_DT.itemsize
        self.bufs = []
        for _ in range(sets):
            n_kl_lr, kl_lr = z(2 * B, torch.int32), z(2 * kls)
            self.bufs.append({
                "n_kp": [z(B, torch.int32), z(B, torch.int32)],
                "kps": [z(B * kc * KEYPOINT_DT.itemsize), z(B * kc * KEYPOINT_DT.itemsize)],
                "pdesc": [z(B * kc * DESC), z(B * kc * DESC)],
                "n_kl_lr": n_kl_lr, "kl_lr": kl_lr,
                "n_kl": [n_kl_lr[:B], n_kl_lr[B:]], "kl": [kl_lr[:kls], kl_lr[kls:]],
                "img_lr": z(2 * B * W * H) if lsd else None,
                "ldesc": [z(B * kl_cap * DESC), z(B * kl_cap * DESC)],
                "pyr_l": z(B * int(cam.pyr_bytes)),   # the left pyramid (not read by the tracker)
                "pyr_r": z(B * int(cam.pyr_bytes)),
                "ts": torch.zeros(B, dtype=torch.float64, device=dev)})
        self.ready = [Event(self.det) for _ in range(sets)]
        self.orb_done = [Event(self.det_orb) for _ in range(sets)]
        self.consumed = [Event(ctx) for _ in range(sets)]
        self.k = 0
        self._handed = [None] * sets   # consumed[s].record_count when set s's view was returned
        torch.cuda.synchronize(dev)   # the buffers' zero fills (default stream) before any detection

    def _begin(self, inputs):
        """next buffer set; the detection stream waits for the tracker's last read of it and for
        the caller's stream (which produced the inputs); so does the ORB stream"""
        import torch
        s = self.k % self.sets
        if self._handed[s] is not None and self.consumed[s].record_count <= self._handed[s]:
            raise RuntimeError(f"ImagePipeline: buffer set {s} still holds a view no tracker call has read "
                               f"(at most {self.sets} detections may be outstanding; discard() releases one)")
        self.k += 1
        self.consumed[s].wait(self.det)
        self.consumed[s].wait(self.det_orb)
        ts = self._tstream
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(ts.device))
        for st in (ts, self._ostream):
            st.wait_event(ev)
            for t in inputs:
                t.record_stream(st)   # the caching allocator keeps them until the detection ran
        return s, ts

    def detect(self, left, right, kl_left, n_kl_left, kl_right, n_kl_right, time_stamp):
        """left / right: device u8 [B][H][W]; kl_*: device KEYLINE_DT rows [B][kl_cap];
        n_kl_*: device int32 [B]; time_stamp: device f64 [B].  Returns the gfpl_frames
        (asynchronous: a tracker call on it waits for its `ready` event)."""
        import torch
        s, ts = self._begin([left, right, kl_left, n_kl_left, kl_right, n_kl_right, time_stamp])
        b = self.bufs[s]
        with torch.cuda.stream(ts):
            for side, (kl, n) in enumerate(((kl_left, n_kl_left), (kl_right, n_kl_right))):
                b["kl"][side].copy_(kl.view(-1))
                b["n_kl"][side].copy_(n)
        return self._describe(s, ts, left, right, time_stamp)

    def detect_images(self, left, right, time_stamp):
        """StereoFrame::detectFeatures with every detector on the device: LSD keylines of both
        images (detectLineFeatures, src/stereoFrame.cpp:1160-1186) written where LBD and the
        tracker read them, then ORB and LBD.  Needs lsd=True."""
        import torch
        if self.lsd is None:
            raise RuntimeError("ImagePipeline(lsd=True) runs LSD on the device")
        s, ts = self._begin([left, right, time_stamp])
        b = self.bufs[s]
        n = self.B * int(self.cam.width) * int(self.cam.height)
        with torch.cuda.stream(ts):
            b["img_lr"][:n].copy_(left.reshape(-1))
            b["img_lr"][n:].copy_(right.reshape(-1))
        self.lsd.detect_async(b["img_lr"], 2 * self.B, b["kl_lr"], b["n_kl_lr"])
        return self._describe(s, ts, left, right, time_stamp)

    def _describe(self, s, ts, left, right, time_stamp):
        import torch
        B, pb, b = self.B, int(self.cam.pyr_bytes), self.bufs[s]
        for side, img in ((0, left), (1, right)):
            pyr = b["pyr_l"] if side == 0 else b["pyr_r"]
            self.orb.extract_async(img, B, b["kps"][side], b["pdesc"][side], b["n_kp"][side], None, None, pyr, pb)
        self.orb_done[s].record(self.det_orb)
        for side in range(2):
            self.lbd.compute_async(left if side == 0 else right, B, b["kl"][side], b["n_kl"][side], b["ldesc"][side])
        with torch.cuda.stream(ts):
            b["ts"].copy_(time_stamp)
        self.orb_done[s].wait(self.det)
        self.ready[s].record(self.det)
        arrs = [b["n_kp"][0], b["n_kp"][1], b["kps"][0], b["kps"][1], b["pdesc"][0], b["pdesc"][1],
                b["n_kl"][0], b["n_kl"][1], b["kl"][0], b["kl"][1], b["ldesc"][0], b["ldesc"][1], b["pyr_r"], b["ts"]]
        fr = make_frames(B, self.kp_cap, self.kl_cap, arrs)
        fr.ready, fr.consumed = self.ready[s].h, self.consumed[s].h
        fr._events = (self.ready[s], self.consumed[s])
        self._handed[s] = self.consumed[s].record_count
        return fr

    def discard(self, fr):
        """release a view no tracker call will read (its set may be detected into again)"""
        for s in range(self.sets):
            if fr.consumed == self.consumed[s].h.value:
                self.consumed[s].record(self.det)
                return
        raise ValueError("discard: not a view of this pipeline")

    def status(self):
        """capacity / octave errors of the detections since the last status (waits for them)"""
        self.orb.status()
        self.lbd.status()
        if self.lsd is not None:
            self.lsd.status()

    def synchronize(self):
        self.det_orb.synchronize()
        self.det.synchronize()

    def close(self):
        self.det_orb.synchronize()
        self.det.synchronize()
        self.orb.close()
        self.lbd.close()
        if self.lsd is not None:
            self.lsd.close()
        for e in self.ready + self.orb_done + self.consumed:
            e.close()
        self.det.close()
        self.det_orb.close()
