"""The synthetic input generator: deterministic, within capacity, detections
inside the margins the sub-pixel SAD needs, descriptors with the intended
Hamming statistics."""
import numpy as np

import gfpl


def test_counts_margins_and_octaves():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(seed=1)
    H = gfpl.HostFrames(cam, sp, 2, 2, 2048, 512)
    assert (H.n_kp_l == 2000).all() and (H.n_kp_r == 2000).all()
    assert (H.n_kl_l == 500).all() and (H.n_kl_r == 500).all()
    kp = H.kp_l[0, 0, :2000]
    assert kp["x"].min() >= 40 - 1.5 and kp["x"].max() <= 640 - 41 + 1.5
    assert set(np.unique(kp["octave"])) <= {0, 1, 2, 3}
    assert np.all(H.time_stamp[1] - H.time_stamp[0] > 0.049)


def test_descriptor_statistics():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    H = gfpl.HostFrames(cam, gfpl.synth_params(seed=2), 1, 1, 2048, 512)
    dl, dr = H.pdesc_l[0, 0, :2000], H.pdesc_r[0, 0, :2000]
    # random pairs ~128 bits apart
    x = np.unpackbits(np.bitwise_xor(dl[:500], dr[500:1000]), axis=1).sum(1)
    assert 110 < x.mean() < 146


def test_seq_offset_equals_global_id():
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(n_kp=300, n_kl=60, n_world_pts=400, n_world_lines=90, seed=4)
    A = gfpl.HostFrames(cam, sp, 3, 2, 512, 128)
    B = gfpl.HostFrames(cam, sp, 1, 2, 512, 128, seq0=2)
    for a, b in zip(A.arrays(), B.arrays()):
        assert np.array_equal(a[:, 2], b[:, 0])


def test_frames_independent_of_chunking():
    """bench.py stages inputs frame by frame (DeviceFrames.generate): a frame must
    not depend on which other frames were generated with it."""
    cfg = gfpl.default_config()
    cam = gfpl.make_camera("vga", cfg)
    sp = gfpl.synth_params(seed=3, n_kp=300, n_kl=60, n_world_pts=400, n_world_lines=90)
    whole = gfpl.HostFrames(cam, sp, 3, 4, 512, 128, seq0=5)
    one = gfpl.HostFrames(cam, sp, 3, 1, 512, 128, seq0=5, frame0=2)
    for a, b in zip(whole.arrays(), one.arrays()):
        assert np.array_equal(a[2], b[0])
    assert gfpl.input_bytes_per_frame(cam, 512, 128) == sum(a[0].nbytes for a in one.arrays()) // 3
