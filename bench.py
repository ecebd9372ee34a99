#!/usr/bin/env python3
"""bench.py — stereo frames/s of the GF-PL-SLAM tracking hot path on MI355X.

Metric (BASELINE.json): stereo frames/sec (2k ORB + 500 LBD, 10 GN iters) at
1/2/4/8 GPU; % HBM peak.  Workload (BASELINE configs[1], SURVEY.md §8(d)
config 2): synthetic VGA stereo (the reference's gazebo rig,
config/gazebo_params.yaml), 2000 ORB + 500 LBD per side, harness overrides
maxIters = maxItersRef = 10 and minError = minErrorChange = 0.

A "step" = one StereoFrameHandler step (insertStereoPair + optimizePose +
updateFrame, app/plslam_mod.cpp:387-477) for every one of the B independent
sequences resident on a GPU.  Input detections for all frames are generated on
the host (splitmix64, deterministic) and copied to HBM before the timed region.

Multi-GPU: one process per GPU (torch.distributed.run); rank r owns sequences
[r*B, (r+1)*B) — no data-path collective (weak scaling); the camera/config
block is RCCL-broadcast from rank 0 over xGMI at start-up, the elapsed times
are MAX-reduced.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))
import gfpl  # noqa: E402

STAGES = ["stereo_points", "stereo_lines", "cross_points", "cross_lines", "line_cut", "pose"]
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)

WORKLOADS = {
    # name: (camera, synth overrides, description)
    "cfg2": ("vga", {}, "cfg2: synthetic VGA 640x480 stereo (gazebo rig), 2000 ORB + 500 LBD per side, 10+10 GN iters"),
    "cfg3": ("kitti", dict(dt=0.1, v_fwd=8.0, z_min=4.0, z_max=40.0),
             "cfg3: KITTI-00 1241x376 stream (synthetic detections), 2000 ORB + 500 LBD, 10+10 GN iters"),
    # BASELINE configs[3]: the EuRoC rig following the ground-truth motion of the 8 EuRoC
    # sequences (config/asl/gt-ass/*), sequence (rank mod 8) on rank r
    # BASELINE configs[4]: stress, 8000 ORB + 2000 LBD per 1920x1080 frame, line cut on
    "cfg5": ("stress", dict(n_kp=8000, n_kl=2000, n_world_pts=10400, n_world_lines=2800, z_max=12.0),
             "cfg5: stress 1920x1080 stereo (gazebo x3), 8000 ORB + 2000 LBD per side, good-line-cut on, "
             "10+10 GN iters"),
    "cfg4": ("euroc", dict(z_min=2.0, z_max=12.0),
             "cfg4: EuRoC 752x480 rig on the MH_01..V1_03 ground-truth trajectories (rank mod 8), "
             "2000 ORB + 500 LBD, 10+10 GN iters"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16384, help="sequences per GPU (reduced to fit HBM if needed)")
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seqs", type=int, default=16)
    ap.add_argument("--cpu-frames", type=int, default=128)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--diag-every-step", action="store_true",
                    help="read the per-stage / per-kernel HIP-event times after every timed step "
                         "(one host sync per step); default: after the last timed step only")
    ap.add_argument("--input-mem-frac", type=float, default=0.7,
                    help="max fraction of free HBM used by the staged input frames")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="PMC traffic summary written by tools/pmc_summary.py (optional)")
    return ap.parse_args()


def cpu_baseline(cam, cfg, sp, n_threads, n_seqs, n_frames, kp_cap, kl_cap):
    """The CPU oracle (C++ restatement of the reference path, oracle/) timed on this
    host: n_seqs sequences x n_frames steps, one sequence per worker thread at a
    time (ctypes releases the GIL), initialisation and input generation excluded."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    H = gfpl.HostFrames(cam, sp, n_seqs, n_frames + 1, kp_cap, kl_cap, seq0=100000)
    hs = [O.OracleHandler(cam, cfg, kp_cap, kl_cap) for _ in range(n_seqs)]
    frames = [H.frames(f) for f in range(n_frames + 1)]
    for b, h in enumerate(hs):
        h.initialize(frames[0], b)
    todo = list(range(n_seqs))
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                if not todo:
                    return
                b = todo.pop()
            h = hs[b]
            for k in range(1, n_frames + 1):
                h.insertStereoPair(frames[k], b)
                h.optimizePose()
                h.updateFrame()

    nt = max(1, min(n_threads, n_seqs))
    th = [threading.Thread(target=worker) for _ in range(nt)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    return {"value": n_seqs * n_frames / dt, "unit": "stereo frames/s", "cores": nt, "kind": "port",
            "sample": f"{n_seqs} sequences x {n_frames} frames of the same workload on {nt} host threads "
                      f"({dt:.1f} s wall, {os.cpu_count()} CPUs visible)"}


def shard_first_seq(rank: int, batch: int) -> int:
    """Sequences are partitioned across ranks: rank r owns [r*B, (r+1)*B)."""
    return rank * batch


def broadcast_setup(cam, cfg, dist, device):
    """Broadcast rank 0's camera + config block to every rank (RCCL over xGMI
    with the nccl backend; gloo on CPU in the tests) and load it in place."""
    blob = bytes(cam) + bytes(cfg)
    import torch
    t = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device)
    dist.broadcast(t, src=0)
    raw = t.cpu().numpy().tobytes()
    C.memmove(C.addressof(cam), raw[: C.sizeof(cam)], C.sizeof(cam))
    C.memmove(C.addressof(cfg), raw[C.sizeof(cam):], C.sizeof(cfg))


def reduce_job(elapsed: float, frames: int, dist, device):
    """MAX over ranks of the timed region, SUM of processed frames."""
    import torch
    el = torch.tensor([elapsed], dtype=torch.float64, device=device)
    cnt = torch.tensor([frames], dtype=torch.int64, device=device)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    dist.all_reduce(cnt)
    return float(el.item()), int(cnt.item())


def load_pmc(path, kernel_name, batch, workload):
    """HBM bytes per launch of a kernel from the PMC summary (tools/pmc_summary.py),
    only when it was collected on this workload and batch size."""
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("batch") != batch or d.get("workload", "cfg2") != workload:
            return None
        return float(d["kernels"][kernel_name]["hbm_bytes_per_launch"])
    except Exception:
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cam_name, synth_over, desc = WORKLOADS[args.workload]
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0)
    cam = gfpl.make_camera(cam_name, cfg)
    if world > 1:
        # RCCL broadcast of the camera + config block; every rank
        # then runs with rank 0's bytes.
        broadcast_setup(cam, cfg, dist, dev)

    B, W, K = args.batch, args.warmup, args.steps
    KP, KL = (8192, 2048) if args.workload == "cfg5" else (2048, 512)
    F = 1 + W + K
    keep = []
    if args.workload == "cfg4":
        T, t = gfpl.euroc_traj(gfpl.EUROC_SEQS[rank % len(gfpl.EUROC_SEQS)], 64)
        keep += [T, t]   # the generator reads them through raw pointers
        if F > len(t):
            print(f"note: {F} frames > {len(t)} ground-truth poses; the trajectory wraps", file=sys.stderr)
        synth_over = dict(synth_over, traj=T.ctypes.data, n_traj=len(t), traj_t=t.ctypes.data)
        desc = desc + f" [this rank: {gfpl.EUROC_SEQS[rank % len(gfpl.EUROC_SEQS)]}]"
    sp = gfpl.synth_params(**synth_over)
    # all F input frames of the B sequences are staged in HBM before timing; bound
    # them to a fraction of device memory (inputs resident)
    free, total = torch.cuda.mem_get_info(dev)
    per_seq_frame = gfpl.input_bytes_per_frame(cam, KP, KL)
    b_fit = int(args.input_mem_frac * free // (per_seq_frame * F)) // 64 * 64
    if b_fit < B:
        print(f"note: --batch {B} x {F} frames does not fit; using {b_fit} sequences", file=sys.stderr)
        B = max(64, b_fit)
    t0 = time.perf_counter()
    D = gfpl.DeviceFrames.generate(cam, sp, B, F, KP, KL, seq0=shard_first_seq(rank, B), device=dev, threads=16)
    t_gen = time.perf_counter() - t0
    in_bytes = D.nbytes()
    stream = torch.cuda.current_stream(dev).cuda_stream
    ctx = gfpl.Context(cam, cfg, device=local, stream=stream)
    h = gfpl.StereoFrameHandler(ctx, B, KP, KL)
    h.initialize(D.frames(0))
    for w in range(W):
        h.frameStep(D.frames(1 + w))
    torch.cuda.synchronize(dev)
    ctx.set_timing(True)
    stage_ms, stage_bytes, kern_ms, kern_bytes = [], [], [], []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(K):
        h.frameStep(D.frames(1 + W + k))
        if args.diag_every_step or k == K - 1:
            # HIP events on the context stream; reading them synchronises, so by default
            # only the last timed step is sampled (the steps are statistically identical)
            stage_ms.append(ctx.stage_times())
            stage_bytes.append(h.last_step_stage_bytes())
            kern_ms.append(ctx.kernel_times())
            kern_bytes.append(h.last_step_kernel_bytes())
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t_max, frames_total = reduce_job(elapsed, B * K, dist, dev)
    else:
        t_max, frames_total = elapsed, B * K
    # tracking health: fraction of sequences still tracked
    lost = sum(h.read_track(b)["num_frame_loss"] > 0 for b in range(0, B, max(1, B // 16)))

    if rank == 0:
        sm = np.mean(np.array(stage_ms, dtype=np.float64)[:, :6], axis=0)
        sb = np.mean(np.array(stage_bytes)[:, :6], axis=0).astype(np.float64)
        km = np.mean(np.array(kern_ms, dtype=np.float64), axis=0)
        kb = np.mean(np.array(kern_bytes), axis=0).astype(np.float64)
        # candidate kernels for the roofline line: the single-kernel stages and the
        # two kernels that dominate the line-cut and pose stages
        cands = {"k_stereo_points": (sm[0], sb[0]), "k_stereo_lines": (sm[1], sb[1]),
                 "k_cross_points": (sm[2], sb[2]), "k_cross_lines": (sm[3], sb[3]),
                 "k_cut_search": (km[1], kb[1]), "k_pose": (km[3], kb[3])}
        kname = max(cands, key=lambda k: cands[k][0])
        k_ms, k_bytes = cands[kname]
        achieved = k_bytes / (k_ms * 1e-3) / 1e9
        step_bytes = float(np.mean(np.array(stage_bytes)[:, 6]))
        ms_step = t_max / K * 1e3
        value = frames_total / t_max
        traffic = load_pmc(args.pmc, kname, B, args.workload)
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(cam, cfg, sp, args.cpu_threads, args.cpu_seqs, args.cpu_frames, KP, KL)
        out = {
            "metric": "stereo frames/sec (2k ORB + 500 LBD, 10 GN iters)",
            "value": value,
            "unit": "stereo frames/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (deterministic splitmix64 stereo detections + right ORB pyramid, gfpl_synth)",
            "config": {"workload": desc, "sequences_per_gpu": B, "kp_per_side": int(sp.n_kp), "kl_per_side": int(sp.n_kl),
                       "gn_iters": "10+10", "parallelism": f"sequences sharded 1/{world} per GPU"},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": float(achieved), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": float(achieved / HBM_PEAK_GBS), "traffic": traffic,
                         "algorithmic_bytes_per_launch": float(k_bytes), "avg_launch_ms": float(k_ms)},
            "hbm_frac_step": float(step_bytes / (t_max / K) / 1e9 / HBM_PEAK_GBS),
            "stage_ms": {n: round(float(v), 4) for n, v in zip(STAGES, sm)},
            "kernel_ms": {n: round(float(v), 4) for n, v in zip(["k_cut_prep", "k_cut_search", "k_cut_finish", "k_pose"], km)},
            "stage_bytes_per_step": {n: int(v) for n, v in zip(STAGES, sb)},
            "cpu_baseline": cpu,
            "gen_s": round(t_gen, 2),
            "input_hbm_bytes": in_bytes,
            "lost_sampled": int(lost),
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
