"""Probe: B sequences as S independent handlers on S HIP streams, phase-shifted so
the latency-bound line-cut search of one handler overlaps the throughput-bound
stages of another.  Prints frames/s per S."""
import sys, os, time, json
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))
import gfpl

B = int(sys.argv[1]); K = int(sys.argv[2]); Ss = [int(x) for x in sys.argv[3].split(",")]
KP, KL = 2048, 512
cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0)
cam = gfpl.make_camera("vga", cfg)
sp = gfpl.synth_params()
F = K + 2
D = gfpl.DeviceFrames.generate(cam, sp, B, F, KP, KL, seq0=0, device=0, threads=16)
for S in Ss:
    n = B // S
    streams = [torch.cuda.Stream() for _ in range(S)]
    ctxs = [gfpl.Context(cam, cfg, device=0, stream=s.cuda_stream) for s in streams]
    hs = [gfpl.StereoFrameHandler(c, n, KP, KL) for c in ctxs]
    def fr(k, i):
        return D.frames_slice(k, i * n, n)
    for i, h in enumerate(hs):
        h.initialize(fr(0, i)); h.frameStep(fr(1, i))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prev_ev = None
    # staggered first step
    for i, h in enumerate(hs):
        with torch.cuda.stream(streams[i]):
            if prev_ev is not None:
                streams[i].wait_event(prev_ev)
            f = fr(2, i)
            h.stereoPoints(f); h.stereoLines(f); h.estimateStereoUncertainty()
            h.crossFrameMatchingPoints(); h.crossFrameMatchingLines()
            ev = torch.cuda.Event(); ev.record(streams[i]); prev_ev = ev
            h.estimateProjUncertainty_submodular(); h.optimizePose(); h.updateFrame()
    for k in range(3, K + 2):
        for i, h in enumerate(hs):
            h.frameStep(fr(k, i))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"S": S, "B": B, "K": K, "frames_s": B * K / dt, "ms_step": dt / K * 1e3}), flush=True)
    del hs, ctxs
