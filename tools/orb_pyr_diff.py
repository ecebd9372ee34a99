"""Per-level pyramid differences, GPU ORB vs the oracle, on one synthetic VGA image (diagnostic)."""
import sys, numpy as np
sys.path[:0] = ["gf-pl-slam_amd", "oracle", "tests"]
import gfpl, oracle as O
from test_orb_gpu import _run_gpu, _images
orb = gfpl.ORBextractor(2000, 1.2, 4, 20, 7, 640, 480, max_images=1)
imgs = _images(1, 640, 480, 40)
k, d, nk, a, r, p = _run_gpu(orb, imgs)
o = O.orb_extract(imgs[0], nfeatures=2000, scale_factor=1.2, nlevels=4, kp_cap=orb.kp_cap)
off = 0
for l, (w, h) in enumerate(orb.level_sizes()):
    g = p[0, off:off + w * h].reshape(h, w); c = o["pyramid"][off:off + w * h].reshape(h, w)
    bad = np.argwhere(g != c)
    print(l, w, h, off, len(bad), bad[:5].tolist(), [ (int(g[y,x]), int(c[y,x])) for y,x in bad[:5]])
    off += w * h
