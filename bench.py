#!/usr/bin/env python3
"""bench.py — stereo frames/s of the GF-PL-SLAM tracking hot path on MI355X.

Metric (BASELINE.json): stereo frames/sec (2k ORB + 500 LBD, 10 GN iters) at
1/2/4/8 GPU; % HBM peak.  Workload (BASELINE configs[1], SURVEY.md §8(d)
config 2): synthetic VGA stereo (the reference's gazebo rig,
config/gazebo_params.yaml), 2000 ORB + 500 LBD per side, harness overrides
maxIters = maxItersRef = 10 and minError = minErrorChange = 0.

A "step" = one StereoFrameHandler step (insertStereoPair + optimizePose +
updateFrame, app/plslam_mod.cpp:387-477) for every one of the B independent
sequences resident on a GPU (B = 65536 by default, independent of --steps; ~140 GB of the
288 GB HBM with both staging buffers: every kernel's grid tail is amortised over more waves —
DESIGN.md §5g, 741.6k / 759.9k / 774.4k frames/s at 32768 / 49152 / 65536 on one box).

Input ring: before each step the host generates the next input frame of all B
sequences (splitmix64, deterministic; gfpl_synth) chunk by chunk into a ring of
two pinned chunks and uploads each chunk with gfpl_upload_frames_async into the
seqbatch's device staging buffer (the next chunk is generated while the last one
is copied), all outside the timed brackets.  Each step is timed on its own,
bracketed by barrier + device synchronize on both sides with the inputs resident
in HBM; the reported time is the sum over the K timed steps (MAX over ranks).
The synthetic scene is stationary (landmarks re-spawn in the frustum, gfpl_synth
`respawn`), so per-step work does not drift with --steps; the bench line carries
the per-step mean feature counts.  `host_fed` is measured after the timed steps:
two frames held in pinned host memory are uploaded on the copy stream into the
two staging buffers while the step on the other one runs (PCIe-inclusive rate).

Parity at the operating point: `parity_sampled` replays a sample of the timed
sequences (same ids, same frames) on the CPU oracle after every step and
compares matched lists, stereo features, cut ratios / invCovPose and poses bit
for bit.  The oracle is the checker here, never the thing measured.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` without a
torch.distributed environment launches `torch.distributed.run` with N workers
(before any GPU call) and exits with its code; rank r owns sequences
[r*B, (r+1)*B) — no data-path collective (weak scaling); the camera/config
block is RCCL-broadcast from rank 0 over xGMI at start-up, B is MIN-reduced,
times MAX-reduced and frame / mismatch counts SUM-reduced.  `--dry-run` runs
the launcher, broadcast, sharding, input generation and reductions on CPU
(gloo) without any tracking step (value null).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gf-pl-slam_amd"))

STAGES = ["stereo_points", "stereo_lines", "cross_points", "cross_lines", "line_cut", "pose"]
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
# VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz, one wave64 VALU instruction per 2 cycles
# per SIMD (MI355X_MICROARCH.md §Wave scheduling) = 1228.8 G wave-instructions/s
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 2

CUT_MODES = {0: "measured", 1: "proven", 2: "proven-eager", 3: "proven-redo-all"}

# Every workload re-spawns its landmarks (gfpl_synth `respawn`: each pool slot is re-sampled in
# the current frustum every `respawn` frames, phases spread), so 90 % of the detections observe a
# landmark at every frame (10 % distractors) and the per-step work is stationary.
WORKLOADS = {
    # name: (camera, synth overrides, description)
    "cfg2": ("vga", dict(respawn=16),
             "cfg2: synthetic VGA 640x480 stereo (gazebo rig), 2000 ORB + 500 LBD per side, 10+10 GN iters"),
    # KITTI moves 0.8 m per frame: landmarks live 4 frames, from a larger pool
    "cfg3": ("kitti", dict(dt=0.1, v_fwd=8.0, z_min=4.0, z_max=40.0, respawn=4, n_world_pts=3200, n_world_lines=900),
             "cfg3: KITTI-00 1241x376 stream (synthetic detections), 2000 ORB + 500 LBD, 10+10 GN iters"),
    # BASELINE configs[3]: the EuRoC rig following the ground-truth motion of the 8 EuRoC
    # sequences (config/asl/gt-ass/*), sequence (rank mod 8) on rank r
    "cfg4": ("euroc", dict(z_min=2.0, z_max=12.0, respawn=16),
             "cfg4: EuRoC 752x480 rig on the MH_01..V1_03 ground-truth trajectories (rank mod 8), "
             "2000 ORB + 500 LBD, 10+10 GN iters"),
    # cfg2 with 10% of the true observations displaced 3-8 px per frame: the pose optimisation's
    # outlier branch (removeOutliers) and the MAD path run on a non-empty outlier set
    "cfg2o": ("vga", dict(respawn=16, outlier_frac=0.1),
              "cfg2o: cfg2 with 10% outlier observations (3-8 px displacements), 2000 ORB + 500 LBD per side, "
              "10+10 GN iters"),
    # BASELINE configs[4]: stress, 8000 ORB + 2000 LBD per 1920x1080 frame, line cut on
    "cfg5": ("stress", dict(n_kp=8000, n_kl=2000, n_world_pts=10400, n_world_lines=3200, z_max=12.0, respawn=16),
             "cfg5: stress 1920x1080 stereo (gazebo x3), 8000 ORB + 2000 LBD per side, good-line-cut on, "
             "10+10 GN iters"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536, help="sequences per GPU (reduced only if HBM is short)")
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-detect", action="store_true", help="skip the ORB / LBD detection rates")
    ap.add_argument("--gen-threads", type=int, default=16,
                    help="host threads generating the input frames (capped by this rank's share of the cores)")
    ap.add_argument("--distinct", type=int, default=0,
                    help="distinct synthetic sequences per rank: 0 = all B with >= 8 generator threads, else one chunk's "
                         "worth (8 ranks sharing a host; each uploaded to every chunk of the batch) — a fixed rule "
                         "of (B, threads), never a timing, so one command always tracks the same inputs")
    ap.add_argument("--chunk", type=int, default=0,
                    help="sequences per pinned host chunk of the input ring (0: B/8 within [256, 2048])")
    ap.add_argument("--no-host-fed", action="store_true", help="skip the pipelined host-fed (PCIe) measurement")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline work (timed seconds)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU-baseline threads (0 = the cores this process may use)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--cpu-sweep-seconds", type=float, default=2.5,
                    help="timed seconds per point of the CPU baseline's 1/2/4/8 thread sweep (0: no sweep)")
    ap.add_argument("--no-b1", action="store_true", help="skip the one-sequence latency leg (B = 1)")
    ap.add_argument("--proven-steps", type=int, default=5,
                    help="N = 1, measured mode: after the timed window, this many further steps (one more untimed) "
                         "in proven mode (cut_proof 1), reported as cut_search.proven_leg (0: skip)")
    ap.add_argument("--dump-records", default=None,
                    help="save every sequence's record of the last timed step (gfpl_debug_step_records, .npy) "
                         "and the instrumented builds' clocks (gfpl_debug_clocks, *_clk.npy)")
    ap.add_argument("--cut-certify", type=float, default=None,
                    help="gfpl_config.cut_certify (the certified line-cut margin; default: the library's)")
    ap.add_argument("--cut-proof", type=int, nargs="?", const=1, default=None,
                    help="gfpl_config.cut_proof: 0 measured, 1 proven (the recorded search proven after the fact, "
                         "unproven sequences redone eagerly), 2 eager-proven search (DESIGN.md §3); default: the "
                         "library's")
    ap.add_argument("--b1-steps", type=int, default=40, help="timed steps of the B = 1 latency leg")
    ap.add_argument("--parity-seqs", type=int, default=16,
                    help="sampled sequences replayed on the oracle per rank (-1: every sequence of the batch)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only (gloo): launcher, broadcast, sharding, input generation and reductions; "
                         "no tracking step is run and value is null")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="PMC summary written by tools/pmc_summary.py (HBM traffic, SQ counters)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher --
def launch_workers(args) -> int:
    """--gpus N > 1 without a torch.distributed environment: run N workers through
    torch.distributed.run as a child process (nothing here touches the GPU)."""
    port = args.master_port or (29500 + os.getpid() % 2000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def host_cores():
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = int(q) / int(per)
    except Exception:
        pass
    eff = max(1, min(n, int(quota))) if quota else n
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except Exception:
        pass
    return eff, {"affinity_cpus": n, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count(), "model": model}


# ------------------------------------------------------- collectives (RCCL) --
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


def reduce_min_int(v: int, dist, device) -> int:
    import torch
    t = torch.tensor([v], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def reduce_sum_ints(vals, dist, device):
    import torch
    t = torch.tensor(list(vals), dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return [int(x) for x in t.tolist()]


def load_pmc(path, kernel_name, batch, workload, steps, warmup):
    """Per-launch PMC summary of a kernel (tools/pmc_summary.py) over the same window of
    launches as this run's timed steps: only when it was collected on this workload,
    batch size, --steps and --warmup (else None, and the line says why)."""
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception as e:
        return None, f"no PMC summary ({type(e).__name__})"
    want = {"batch": batch, "workload": workload, "steps": steps, "warmup": warmup}
    got = {k: d.get(k) for k in want}
    if got != want:
        return None, f"PMC summary window {got} != this run {want}"
    k = d["kernels"].get(kernel_name)
    return k, None if k else f"{kernel_name} not in the PMC summary"


def kernel_traffic(path, batch, workload, steps, warmup, km, kb, sp_ms, sp_bytes):
    """Per-kernel algorithmic bytes per launch (gfpl_last_step_kernel_bytes; k_stereo_points: its
    stage's) beside the PMC-counted traffic of the same launches when the PMC summary covers this
    window (tools/pmc_summary.py: FETCH_SIZE / 0.95 + WRITE_SIZE, the gather calibration)."""
    names = ["k_cut_prep", "k_cut_search", "k_cut_finish", "k_pose"]
    rows = {n: (float(ms), float(by)) for n, ms, by in zip(names, km, kb)}
    rows["k_stereo_points"] = (float(sp_ms), float(sp_bytes))
    out = {}
    for n, (ms, by) in rows.items():
        pmc, _ = load_pmc(path, n, batch, workload, steps, warmup)
        cnt = (pmc or {}).get("hbm_bytes_per_launch_gather_cal")
        out[n] = {"algorithmic_bytes": int(by), "avg_launch_ms": round(ms, 4),
                  "algorithmic_GBps": round(by / (ms * 1e-3) / 1e9, 1) if ms > 0 else None,
                  "counted_bytes_gather_cal": int(cnt) if cnt else None,
                  "counted_over_algorithmic": round(cnt / by, 2) if cnt and by > 0 else None}
    return out


def rank_share(cores: int, world: int) -> int:
    """Host threads one rank may use: the process's cores (cgroup quota) split over the
    ranks of this node (the quota is shared by every rank's process)."""
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world) or world)
    return max(1, cores // max(1, local))


# ------------------------------------------------------- parity at the bench --
class ParitySampler:
    """Replays sampled sequences of the timed batch on the CPU oracle (the checker)
    and compares them with the GPU state after every step, bit for bit."""

    def __init__(self, cam, cfg, sp, kp_cap, kl_cap, seq0, seqs, threads, seq_of=None):
        self.cam, self.sp, self.kp_cap, self.kl_cap, self.seq0 = cam, sp, kp_cap, kl_cap, seq0
        self.seq_of = seq_of or (lambda b: b)   # tracked sequence b runs generator sequence seq0 + seq_of(b)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle as O
        import parity as PT
        self.PT = PT
        self.seqs = list(seqs)
        self.orc = [O.OracleHandler(cam, cfg, kp_cap, kl_cap) for _ in self.seqs]
        self.threads = max(1, min(threads, len(self.seqs)))
        self.frames = self.mismatch_frames = 0
        self.msgs = []

    def _par(self, fn):
        todo = list(range(len(self.seqs)))
        lock = threading.Lock()
        done = [0]

        def work():
            while True:
                with lock:
                    if not todo:
                        return
                    i = todo.pop()
                fn(i)
                with lock:   # progress of long (full-batch) replays: a watchdog sees output
                    done[0] += 1
                    if done[0] % 4096 == 0:
                        print(f"[parity] {done[0]} / {len(self.seqs)} sequences", file=sys.stderr, flush=True)
        th = [threading.Thread(target=work) for _ in range(self.threads)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    def _frame(self, k, i):
        """Frame k of sampled sequence i, generated again on the host (the generator is a pure
        function of (seed, sequence, frame), so these are the bytes the GPU step read)."""
        import gfpl
        return gfpl.HostFrames(self.cam, self.sp, 1, 1, self.kp_cap, self.kl_cap,
                               seq0=self.seq0 + self.seq_of(self.seqs[i]), frame0=k, threads=1)

    def initialize(self, h):
        res = [None] * len(self.seqs)

        def run(i):
            H = self._frame(0, i)
            self.orc[i].initialize(H.frames(0), 0)
            res[i] = self.PT.compare_core(h.read_frame(0, self.seqs[i]), self.orc[i].read_frame(0),
                                          f"init s{self.seqs[i]} ")
        self._par(run)
        for bad in res:
            self._record(bad)

    def step(self, h, k):
        """Per sampled sequence, on the worker threads (the ABI reads synchronise on the step's
        stream and release the GIL, as do the generator and the oracle): the GPU state after the
        step, frame k regenerated, the oracle's step, the bitwise comparison."""
        PT = self.PT
        res = [None] * len(self.seqs)

        def run(i):
            b = self.seqs[i]
            g_new = h.read_frame(0, b)      # PREV after update = the new frame
            g_old = h.read_frame(1, b)      # CURR slot = the old prev (cut results)
            g_tr = h.read_last_track(b)
            H = self._frame(k, i)
            o = self.orc[i]
            o.insertStereoPair(H.frames(0), 0)
            o.optimizePose()
            o_new, o_old, o_tr = o.read_frame(1), o.read_frame(0), o.read_track()   # before the update: CURR, PREV
            o.updateFrame()
            tag = f"f{k} s{b} "
            bad = PT.compare_core(g_new, o_new, tag) + PT.compare_track(g_tr, o_tr, tag)
            pb, exact = PT.compare_pose(g_new, o_new, what=tag)
            bad += pb if pb else ([] if exact else [tag + "pose not bit-identical"])
            if not PT.compare_track(g_tr, o_tr):
                bad += PT.compare_prev_matched(g_old, o_old, o_tr, tag)
            res[i] = bad
        self._par(run)
        for bad in res:
            self._record(bad)

    def _record(self, bad):
        self.frames += 1
        if bad:
            self.mismatch_frames += 1
            self.msgs += bad[:3]


def cpu_baseline(cam, cfg, sp, kp_cap, kl_cap, n_threads, target_s, cores_info, gen_threads, n_frames):
    """The CPU oracle (C++ restatement of the reference path, oracle/) timed on this
    host on the bench's own workload: rounds of n_threads fresh sequences (one per
    worker thread), each initialised untimed and then tracked over frames 1..n_frames
    (the frames the GPU bench steps through), until about target_s seconds of timed
    work.  Input generation and initialisation are excluded, as on the GPU."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import gfpl
    import oracle as O
    n_seqs = n_threads
    timed, frames, rounds = 0.0, 0, 0
    while timed < target_s and rounds < 200:
        seq0 = (1 << 20) + rounds * n_seqs
        H = gfpl.HostFrames(cam, sp, n_seqs, n_frames + 1, kp_cap, kl_cap, seq0=seq0, threads=gen_threads)
        hs = [O.OracleHandler(cam, cfg, kp_cap, kl_cap) for _ in range(n_seqs)]
        for b, h in enumerate(hs):
            h.initialize(H.frames(0), b)

        def worker(b):
            h = hs[b]
            for k in range(1, n_frames + 1):
                h.insertStereoPair(H.frames(k), b)
                h.optimizePose()
                h.updateFrame()
        th = [threading.Thread(target=worker, args=(b,)) for b in range(n_seqs)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        timed += time.perf_counter() - t0
        frames += n_seqs * n_frames
        rounds += 1
        del H, hs
    return {"value": frames / timed, "unit": "stereo frames/s", "cores": n_threads, "kind": "port",
            "sample": f"{rounds} rounds x {n_seqs} sequences x frames 1..{n_frames} of the bench workload, one "
                      f"sequence per host thread ({timed:.1f} s timed; oracle/ C++ -O3 restatement; input "
                      f"generation and initialisation excluded)",
            "host": cores_info}


def cpu_thread_sweep(cam, cfg, sp, kp_cap, kl_cap, n_threads, seconds, gen_threads, n_frames, full, b1_ms):
    """The CPU baseline at 1, 2, 4, 8 threads (and the full count from `full`), a few seconds of
    timed work each: per-thread ms/frame shows whether the n-thread rate is n x the 1-thread rate
    (efficiency) or loses to a shared resource (cgroup quota, memory, frequency)."""
    pts = {}
    for t in sorted({t for t in (1, 2, 4, 8) if t < n_threads}):
        r = cpu_baseline(cam, cfg, sp, kp_cap, kl_cap, t, seconds, None, gen_threads, n_frames)
        pts[str(t)] = r["value"]
    pts[str(n_threads)] = full["value"]
    one = pts["1"] if "1" in pts else full["value"] / n_threads
    return {"frames_per_s": {k: round(v, 1) for k, v in pts.items()},
            "ms_per_frame_per_thread": {k: round(1e3 * int(k) / v, 2) for k, v in pts.items()},
            "efficiency_vs_1thread": {k: round(v / (int(k) * one), 3) for k, v in pts.items()},
            "b1_leg_cpu_1thread_ms_per_frame": b1_ms,
            "note": f"{seconds:.1f} s timed per point; same frames and workload as the baseline"}


def latency_b1(ctx, cam, cfg, sp, kp_cap, kl_cap, seq, warmup, steps):
    """Per-frame latency of ONE sequence (B = 1, rank 0 at N = 1, after the timed batch; not
    part of `value`): the same workload's sequence `seq` stepped alone — wall clock per
    frameStep bracketed by device syncs (inputs resident in HBM, uploaded before), HIP-event
    stage / kernel times of every timed step — beside the CPU oracle's single-thread time per
    frame on the same frames of the same sequence (the reference runs one sequence on one
    core: app/plslam_mod.cpp:387-411)."""
    import torch
    import gfpl
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    n_fr = warmup + steps + 1
    H = gfpl.HostFrames(cam, sp, 1, n_fr, kp_cap, kl_cap, seq0=seq, threads=1)
    h = gfpl.StereoFrameHandler(ctx, 1, kp_cap, kl_cap)

    def staged(k):
        h.upload_wait(h.upload_async(H.frames(k), 0, k % 2))
        return h.staged_frames(k % 2)
    h.initialize(staged(0))
    wall, st, kt = [], [], []
    for k in range(1, n_fr):
        dv = staged(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h.frameStep(dv)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if k > warmup:
            wall.append(t1 - t0)
            st.append(ctx.stage_times())
            kt.append(ctx.kernel_times())
    h.close()
    o = O.OracleHandler(cam, cfg, kp_cap, kl_cap)
    o.initialize(H.frames(0), 0)
    cpu = []
    for k in range(1, n_fr):
        t0 = time.perf_counter()
        o.insertStereoPair(H.frames(k), 0)
        o.optimizePose()
        o.updateFrame()
        if k > warmup:
            cpu.append(time.perf_counter() - t0)
    sm = np.mean(np.array(st, dtype=np.float64)[:, :6], axis=0)
    km = np.mean(np.array(kt, dtype=np.float64), axis=0)
    lat = 1e3 * float(np.mean(wall))
    cpu_ms = 1e3 * float(np.mean(cpu))
    return {"latency_b1_ms": lat, "latency_b1_p50_ms": 1e3 * float(np.median(wall)),
            "latency_b1_max_ms": 1e3 * float(np.max(wall)),
            "stage_ms_b1": {n: round(float(v), 4) for n, v in zip(STAGES, sm)},
            "kernel_ms_b1": {n: round(float(v), 4) for n, v in
                             zip(["k_cut_prep", "k_cut_search", "k_cut_finish", "k_pose"], km)},
            "b1_slowest_stage": STAGES[int(np.argmax(sm))],
            "stage_sum_b1_ms": float(np.sum(sm)),
            "cpu_1thread_ms_per_frame": cpu_ms,
            "gpu_b1_vs_one_core": cpu_ms / lat,
            "sample": f"sequence {seq}, frames {warmup + 1}..{n_fr - 1} ({steps} steps) after {warmup} warm-up steps; "
                      f"CPU: oracle/ C++ on one host thread, the same frames"}


# ----------------------------------------------------------------------- main --
def detection_rates(cam, upload_Bps, n_img=256, n_lines=300, steps=5):
    """SURVEY §8(f)1-2 on the bench camera, measured after the timed tracking steps (not part of
    `value`): ORB extraction (gfpl_orb_extract, nfeatures 2000 / 1.2 / 4 levels / FAST 20-7) and
    LBD descriptors (gfpl_lbd_compute, 300 octave-0 keylines) over n_img synthetic images resident
    in HBM, each call synchronised; one image of each checked bit-exact against the oracle."""
    import torch
    import gfpl
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    W, H = int(cam.width), int(cam.height)
    dev = torch.device("cuda", torch.cuda.current_device())
    imgs = np.stack([gfpl.synth_image(i, i % 7, W, H) for i in range(n_img)])
    d_img = torch.from_numpy(imgs).to(dev)
    out = {"images_per_call": n_img, "image": f"{W}x{H}", "data": "synthetic (gfpl_synth_image)"}
    # ORB
    orb = gfpl.ORBextractor(2000, 1.2, 4, 20, 7, W, H, max_images=n_img)
    kc = orb.kp_cap
    kps = torch.zeros(n_img * kc * gfpl.KEYPOINT_DT.itemsize, dtype=torch.uint8, device=dev)
    desc = torch.zeros(n_img * kc * 32, dtype=torch.uint8, device=dev)
    nkp = torch.zeros(n_img, dtype=torch.int32, device=dev)
    stride = (orb.pyramid_bytes + 255) // 256 * 256
    pyr = torch.zeros(n_img * stride, dtype=torch.uint8, device=dev)
    orb.extract(d_img, n_img, kps, desc, nkp, None, None, pyr, stride)
    t = []
    for _ in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        orb.extract(d_img, n_img, kps, desc, nkp, None, None, pyr, stride)
        t.append(time.perf_counter() - t0)
    o = O.orb_extract(imgs[0], kp_cap=kc)
    n0 = len(o["kps"])
    k0 = kps.cpu().numpy().view(gfpl.KEYPOINT_DT)[:n0]
    d0 = desc.cpu().numpy().reshape(n_img, kc, 32)[0, :n0]
    out["orb"] = {"images_per_s": n_img / float(np.mean(t)), "ms_per_call": 1e3 * float(np.mean(t)),
                  "kp_per_image": float(nkp.float().mean().item()),
                  "parity_vs_oracle_image0": bool(int(nkp[0].item()) == n0 and (k0 == o["kps"]).all() and (d0 == o["desc"]).all())}
    orb.close()
    # LBD
    kls = np.stack([gfpl.synth_keylines(n_lines, W, H, 1000 + i, max_len=150.0) for i in range(n_img)])
    lbd = gfpl.BinaryDescriptor(W, H, max_images=n_img, kl_cap=n_lines)
    d_kl = torch.from_numpy(np.ascontiguousarray(kls).view(np.uint8).reshape(-1)).to(dev)
    d_n = torch.full((n_img,), n_lines, dtype=torch.int32, device=dev)
    d_desc = torch.zeros(n_img * n_lines * 32, dtype=torch.uint8, device=dev)
    lbd.compute_batch(d_img, n_img, d_kl, d_n, d_desc)
    t = []
    for _ in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lbd.compute_batch(d_img, n_img, d_kl, d_n, d_desc)
        t.append(time.perf_counter() - t0)
    ref, _ = O.lbd_compute(imgs[0], kls[0])
    out["lbd"] = {"images_per_s": n_img / float(np.mean(t)), "ms_per_call": 1e3 * float(np.mean(t)),
                  "keylines_per_image": n_lines,
                  "parity_vs_oracle_image0": bool((d_desc.cpu().numpy().reshape(n_img, n_lines, 32)[0] == ref).all())}
    lbd.close()
    # LSD (gfpl_lsd_detect, the reference's LSDOptions, 300 keylines kept): its per-image chain
    # (sort + region growing, one workgroup per image) is latency-bound and needs images in
    # flight: measured at 3072 images per call (the left and right images of
    # images_to_poses_lsd's 1536-frame step; 4096 measured 60.9k, profiles/r04_n), 2048 and 1024
    from gfpl.pipeline import synth_stereo_steps
    n_max = 3072
    li = np.stack([synth_stereo_steps(i // 2, 0, W, H)[i % 2] for i in range(8)]
                  + [imgs[i % n_img] for i in range(n_max - 8)])
    d_li = torch.from_numpy(li).to(dev)
    lsd = gfpl.LSDDetector(W, H, max_images=n_max, kl_cap=320)
    d_kl = torch.zeros(n_max * 320 * gfpl.KEYLINE_DT.itemsize, dtype=torch.uint8, device=dev)
    d_n = torch.zeros(n_max, dtype=torch.int32, device=dev)
    for n_lsd, key in ((3072, "lsd"), (2048, "lsd_2048"), (1024, "lsd_1024")):
        lsd.detect_batch(d_li, n_lsd, d_kl, d_n)
        t = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lsd.detect_batch(d_li, n_lsd, d_kl, d_n)
            t.append(time.perf_counter() - t0)
        kl_all = d_kl.cpu().numpy().view(gfpl.KEYLINE_DT).reshape(n_max, 320)
        cnt = d_n.cpu().numpy()[:n_lsd]
        par = True
        for i in (0, 1, 8):
            rk, _, _ = O.lsd_detect(li[i])
            par = par and int(cnt[i]) == len(rk) and kl_all[i, :cnt[i]].tobytes() == rk.tobytes()
        out[key] = {"images_per_s": n_lsd / float(np.mean(t)), "ms_per_call": 1e3 * float(np.mean(t)),
                    "images_per_call": n_lsd, "keylines_per_image": float(cnt.mean()),
                    "parity_vs_oracle_images_0_1_8": bool(par),
                    "data": "8 staircase stereo images + gfpl_synth_image textures"}
    lsd.close()
    # with detection on the GPU a host-fed pipeline uploads the two grey images of a stereo
    # frame instead of the pyramid + features: the PCIe ceiling derived from the measured rate
    out["host_fed_images_ceiling"] = {"value": upload_Bps / (2.0 * W * H), "unit": "stereo frames/s",
                                      "note": "derived: measured upload GB/s / (2 x W x H bytes); every detector on the GPU"}
    return out


PIPE_BARS = 600         # bars per Mpx of scene plane: ~2000 ORB + 300 LSD keylines per VGA image (north-star load)
PIPE_SCENES = 128       # distinct scenes of the images -> poses legs (sequence b shows scene b % PIPE_SCENES)


def pipeline_rate(cam, cfg, B=1024, steps=3, lsd=False, progress=False, bars=PIPE_BARS):
    """Images in HBM to poses on one device (gfpl.pipeline), measured after the
    timed tracking steps (not part of `value`): per step ORB on both images of B stereo frames,
    LBD (and LSD when lsd) on the pipeline's detection stream, one StereoFrameHandler step on
    the tracking stream; staircase scene (gfpl.pipeline.synth_stereo_steps), two untimed
    warm-up steps.  `serial`: each step's detection then its tracking, synchronised in
    between (the split); `value`: the overlapped order — detection of frame k + 1 enqueued
    before the tracking of frame k, ordered only by the gfpl_frames ready / consumed events.
    Parity is the -m gpu tests' (tests/test_pipeline_gpu.py)."""
    import torch
    import gfpl
    from gfpl.pipeline import ImagePipeline, synth_stereo_steps
    W, H, KL = int(cam.width), int(cam.height), 320
    dev = torch.device("cuda", torch.cuda.current_device())
    ctx = gfpl.Context(cam, cfg)
    pipe = ImagePipeline(ctx, cam, B, KL, lsd=lsd)
    g = gfpl.StereoFrameHandler(ctx, B, pipe.kp_cap, KL)
    det = (lambda f: pipe.detect_images(f[0], f[1], f[6])) if lsd else (lambda f: pipe.detect(*f))
    frames = []
    for k in range(2 + 2 * steps):
        sc = [synth_stereo_steps(b % PIPE_SCENES, k, W, H, bars=bars) for b in range(B)]
        if progress:
            print(f"[pipeline_rate] frame {k} of {2 + 2 * steps} generated", file=sys.stderr, flush=True)
        kl = [np.zeros((B, KL), gfpl.KEYLINE_DT) for _ in range(2)]
        n = [np.zeros(B, np.int32) for _ in range(2)]
        for b, x in enumerate(sc):
            for side in range(2):
                n[side][b] = len(x[2 + side])
                kl[side][b, :n[side][b]] = x[2 + side]
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        frames.append((to(np.stack([x[0] for x in sc])), to(np.stack([x[1] for x in sc])),
                       to(kl[0].view(np.uint8).reshape(-1)), to(n[0]), to(kl[1].view(np.uint8).reshape(-1)), to(n[1]),
                       torch.full((B,), 0.05 * k, dtype=torch.float64, device=dev)))
    g.initialize(det(frames[0]))
    g.frameStep(det(frames[1]))
    torch.cuda.synchronize()
    t_det = t_trk = 0.0
    for k in range(2, steps + 2):
        t0 = time.perf_counter()
        fr = det(frames[k])
        pipe.synchronize()
        t1 = time.perf_counter()
        g.frameStep(fr)
        ctx.synchronize()
        t_det += t1 - t0
        t_trk += time.perf_counter() - t1
    pipe.status()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fr_next = det(frames[steps + 2])
    for k in range(steps + 2, 2 * steps + 2):
        cur = fr_next
        if k + 1 < 2 * steps + 2:
            fr_next = det(frames[k + 1])
        g.frameStep(cur)
    ctx.synchronize()
    pipe.synchronize()
    t_ovl = time.perf_counter() - t0
    pipe.status()
    tr = g.read_last_track(0)
    sc_counts = g.last_step_counts()   # per-sequence means of the last step: S_p', S_l', M_p, M_l
    g.close()
    pipe.close()
    ctx.close()
    return {"value": B * steps / t_ovl, "unit": "stereo frames/s", "sequences": B, "steps": steps,
            "ms_per_step": 1e3 * t_ovl / steps,
            "serial": {"value": B * steps / (t_det + t_trk), "detect_ms_per_step": 1e3 * t_det / steps,
                       "track_ms_per_step": 1e3 * t_trk / steps},
            "matched_pt_seq0": len(tr["matched_pt"]), "matched_ls_seq0": len(tr["matched_ls"]),
            "per_frame_mean": {"stereo_pt": round(sc_counts["S_p"], 1), "stereo_ls": round(sc_counts["S_l"], 1),
                               "matched_pt": round(sc_counts["M_p"], 1), "matched_ls": round(sc_counts["M_l"], 1),
                               "keypoints_both_sides": round(sc_counts["N_o"], 1),
                               "keylines_both_sides": round(sc_counts["N_k"], 1)},
            "scene": f"staircase bands at disparity 2/12/20/8 px, {bars} anti-aliased bars per Mpx of plane "
                     f"({PIPE_SCENES} distinct scenes), 2000 ORB, " +
                     ("LSD on the device (<= 300 keylines per side)" if lsd else "300 given keylines per side"),
            "overlap": "detection of frame k+1 (detection stream) beside the tracking of frame k (tracking stream)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if args.gpus > 1 and world == 0:
        sys.exit(launch_workers(args))
    world = world or 1
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    import gfpl

    dry = args.dry_run
    if dry:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        if not torch.cuda.is_available():
            print("error: no GPU visible (bench.py measures the HIP path; --dry-run rehearses the launcher on CPU)",
                  file=sys.stderr)
            sys.exit(3)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)

    cam_name, synth_over, desc = WORKLOADS[args.workload]
    cfg = gfpl.default_config(max_iters=10, max_iters_ref=10, min_error=0.0, min_error_change=0.0)
    if args.cut_certify is not None:
        cfg.cut_certify = args.cut_certify
    if args.cut_proof is not None:
        cfg.cut_proof = args.cut_proof
    cam = gfpl.make_camera(cam_name, cfg)
    if world > 1:
        # RCCL broadcast of the camera + config block; every rank
        # then runs with rank 0's bytes
        broadcast_setup(cam, cfg, dist, dev)

    B, W, K = args.batch, args.warmup, args.steps
    KP, KL = (8192, 2048) if args.workload == "cfg5" else (2048, 512)
    keep = []
    # init + warmup + timed + the proven leg's (one untimed + --proven-steps) + the two host-fed frames
    n_frames_needed = W + K + 3 + (args.proven_steps + 1 if args.proven_steps > 0 else 0)
    if args.workload == "cfg4":
        if n_frames_needed > gfpl.EUROC_MAX_POSES:
            print(f"error: cfg4 needs {n_frames_needed} ground-truth poses, {gfpl.EUROC_MAX_POSES} stored",
                  file=sys.stderr)
            sys.exit(2)
        T, t = gfpl.euroc_traj(gfpl.EUROC_SEQS[rank % len(gfpl.EUROC_SEQS)], n_frames_needed)
        keep += [T, t]   # the generator reads them through raw pointers
        synth_over = dict(synth_over, traj=T.ctypes.data, n_traj=len(t), traj_t=t.ctypes.data)
        desc = desc + f" [rank 0: {gfpl.EUROC_SEQS[0]}]"
    # the right pyramid's levels 1.. are resized from level 0 (ComputePyramid): the host
    # generates and uploads level 0 only (gfpl_upload_frames_l0_async builds the rest on the
    # device); the oracle's frames (parity sampler, CPU baseline) carry the host-resized levels
    sp = gfpl.synth_params(**synth_over, pyr_from_l0=1)
    sp_up = gfpl.synth_params(**synth_over, pyr_from_l0=2)
    per_in = gfpl.input_bytes_per_frame(cam, KP, KL)
    l0_bytes = int(cam.lvl_cols[0]) * int(cam.lvl_rows[0])
    per_up = per_in - int(cam.pyr_bytes) + l0_bytes   # bytes per sequence-frame over PCIe

    if not dry:
        # device footprint per sequence: resident state + one staged input frame
        ctx = gfpl.Context(cam, cfg, device=local, stream=torch.cuda.current_stream(dev).cuda_stream)
        probe = gfpl.StereoFrameHandler(ctx, 64, KP, KL)
        per_state = probe.nbytes() / 64
        probe.close()
        free, _ = torch.cuda.mem_get_info(dev)
        b_fit = int(0.85 * free // (per_state + per_in)) // 64 * 64
        if b_fit < B:
            print(f"note: --batch {B} does not fit in HBM; using {b_fit} sequences", file=sys.stderr)
            B = max(64, b_fit)
    if world > 1:
        B = reduce_min_int(B, dist, dev)   # one B on every rank: shards [r*B, (r+1)*B)
    seq0 = shard_first_seq(rank, B)

    # host resources of this rank: its share of the process cores, a ring of two pinned
    # chunks of the input batch (not a whole batch: 8 ranks share one host)
    cores, cores_info = host_cores()
    share = rank_share(cores, world)
    gen_threads = max(1, min(args.gen_threads, share))
    chunk = args.chunk or min(2048, max(256, (B // 8 + 63) // 64 * 64))   # (<= 4.2 GB pinned per rank)
    chunk = min(chunk, B)
    ring = [gfpl.HostBatch(cam, sp_up, chunk, KP, KL, seq0=seq0, pinned=not dry) for _ in range(2)]
    pinned_bytes = 0 if dry else sum(r.nbytes() for r in ring)
    t_gen = 0.0
    # input generation per rank: the generator costs ~1 ms per sequence-frame and core, the
    # GPU step ~2 us per sequence-frame, so overlapping the two gains < 3%; with several ranks
    # sharing one host's cores (8 ranks: 2 cores each) one chunk of distinct sequences is
    # generated per frame and uploaded into every chunk of the batch — every sequence is still
    # tracked on the GPU from its own state.  The rule depends on (B, threads) only: a timing-based
    # choice once gave two runs of one command different inputs (round-5 review, item 1); the
    # thread count is this rank's share of the host's cores (cgroup quota / ranks per node)
    n_proven = args.proven_steps + 1 if (world == 1 and args.proven_steps > 0 and not dry and
                                         int(cfg.cut_proof) == 0) else 0
    n_frames_gen = W + K + 1 + n_proven + (0 if (world > 1 or args.no_host_fed or dry) else 2)
    probe_n = min(chunk, 128)
    t0 = time.perf_counter()
    ring[1].fill(0, gen_threads, seq0=seq0, n=probe_n)
    per_seq_frame = (time.perf_counter() - t0) / probe_n
    gen_full_s = per_seq_frame * B * n_frames_gen
    if args.distinct > 0:
        distinct = min(args.distinct, B)
    else:
        distinct = B if gen_threads >= 8 else chunk   # 8 ranks on one 16-core share: 2 threads each
    if distinct < B:
        distinct = min(distinct, chunk)   # generated into one ring chunk, tiled, uploaded chunk-wise
    gen_projected_s = per_seq_frame * distinct * n_frames_gen
    replicate = distinct < B

    h = None if dry else gfpl.StereoFrameHandler(ctx, B, KP, KL)

    def stage_frame(k, slot=0):
        """Generate frame k of this rank's B sequences chunk by chunk into the pinned ring and
        copy each chunk into staging buffer `slot` (gfpl_upload_frames_async); the next chunk
        is generated while the previous one is copied.  Returns the staged device view."""
        tick = []
        if replicate:
            ring[0].fill(k, gen_threads, seq0=seq0, n=distinct)
            for d0 in range(distinct, chunk, distinct):   # tile the distinct rows over the chunk
                dn = min(distinct, chunk - d0)
                for a in ring[0].arrays():
                    a[d0:d0 + dn] = a[:dn]
        for ci, s0 in enumerate(range(0, B, chunk)):
            n = min(chunk, B - s0)
            hb = ring[0] if replicate else ring[ci % 2]
            if ci >= 2 and h is not None and not replicate:
                h.upload_wait(tick[ci - 2])   # the chunk's host buffer is free again
            if not replicate:
                hb.fill(k, gen_threads, seq0=seq0 + s0, n=n)
            if h is not None:
                tick.append(h.upload_async(hb.frames(n), s0, slot, l0_stride=int(cam.pyr_bytes)))
        if h is None:
            return None
        h.upload_wait(tick[-1])
        return h.staged_frames(slot)

    host_info = {"pinned_bytes_per_rank": int(pinned_bytes), "chunk_sequences": int(chunk),
                 "gen_threads_per_rank": int(gen_threads), "cores_share_per_rank": int(share),
                 "distinct_sequences_per_rank": int(distinct), "gen_ms_per_seq_frame": round(per_seq_frame * 1e3, 4),
                 "gen_projected_s_per_rank": round(gen_projected_s, 1),
                 "gen_all_distinct_s_per_rank": round(gen_full_s, 1)}
    if dry:
        t0 = time.perf_counter()
        stage_frame(0)
        t_gen += time.perf_counter() - t0
        frames_total = B * K
        if world > 1:
            _, frames_total = reduce_job(0.0, B * K, dist, dev)
        if rank == 0:
            print(json.dumps({"metric": "stereo frames/sec (2k ORB + 500 LBD, 10 GN iters)", "value": None,
                              "unit": "stereo frames/s", "n_gpus": world, "steps": K, "warmup": W,
                              "dry_run": True, "frames_sharded": frames_total,
                              "config": {"workload": desc, "sequences_per_gpu": B,
                                         "parallelism": f"sequences sharded 1/{world} per GPU"},
                              "input_bytes_per_step": int(per_in * B), "host": host_info,
                              "pinned_bytes_per_rank_if_gpu": int(sum(r.nbytes() for r in ring)),
                              "gen_s": round(t_gen, 2)}))
        if world > 1:
            dist.destroy_process_group()
        return

    sampler = None
    if args.parity_seqs != 0:
        seqs = list(range(B)) if args.parity_seqs < 0 else [int(x) for x in np.linspace(0, B - 1, min(args.parity_seqs, B))]
        sampler = ParitySampler(cam, cfg, sp, KP, KL, seq0, seqs, share,
                                seq_of=(lambda b: (b % chunk) % distinct) if replicate else None)

    def sync_all():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    t0 = time.perf_counter()
    dv = stage_frame(0)
    t_gen += time.perf_counter() - t0
    h.initialize(dv)
    if sampler:
        sampler.initialize(h)
    step_s = []
    stage_ms, stage_bytes, kern_ms, kern_bytes, counts, cutc, proofc = [], [], [], [], [], [], []
    ctx.set_timing(True)
    for k in range(1, 1 + W + K):
        t0 = time.perf_counter()
        dv = stage_frame(k)                           # host generation + upload (untimed)
        t_gen += time.perf_counter() - t0
        sync_all()
        ts0 = time.perf_counter()
        h.frameStep(dv)                               # the step: inputs resident in HBM
        sync_all()
        ts1 = time.perf_counter()
        if k > W:
            # the timed window: HIP-event stage / kernel times and the algorithmic bytes and
            # counts of every timed step (the PMC summary averages the same launches)
            step_s.append(ts1 - ts0)
            stage_ms.append(ctx.stage_times())
            stage_bytes.append(h.last_step_stage_bytes())
            kern_ms.append(ctx.kernel_times())
            kern_bytes.append(h.last_step_kernel_bytes())
            counts.append(h.last_step_counts())
            cutc.append(h.last_step_track_counts())
            proofc.append(h.last_step_cut_proof())
        if sampler:
            sampler.step(h, k)
        if rank == 0:   # progress (stderr): long runs under a watchdog keep writing
            print(f"[bench] step {k}/{W + K}: {1e3 * (ts1 - ts0):.2f} ms", file=sys.stderr, flush=True)
    elapsed = float(np.sum(step_s))
    if args.dump_records and rank == 0:
        np.save(args.dump_records, h.debug_step_records())
        try:
            np.save(args.dump_records.replace(".npy", "") + "_clk.npy", h.debug_clocks())
        except AttributeError:   # a library from before gfpl_debug_clocks
            pass
    lost = sum(h.read_track(b)["num_frame_loss"] > 0 for b in range(0, B, max(1, B // 16)))
    par = [sampler.frames, sampler.mismatch_frames] if sampler else [0, 0]
    if world > 1:
        t_max, frames_total = reduce_job(elapsed, B * K, dist, dev)
        par = reduce_sum_ints(par, dist, dev)
    else:
        t_max, frames_total = elapsed, B * K

    proven = None
    if n_proven:
        # the same sequences, tracked on in proven mode: one untimed step (the mode's first launches),
        # then timed steps bracketed like the window's; the mode is restored afterwards
        cfg1 = gfpl.Config()
        C.memmove(C.byref(cfg1), C.byref(cfg), C.sizeof(cfg))
        cfg1.cut_proof = 1
        ctx.set_config(cfg1)
        p_s, p_cut, p_redone = [], [], 0
        for i in range(n_proven):
            t0 = time.perf_counter()
            dv = stage_frame(W + K + 1 + i)
            t_gen += time.perf_counter() - t0
            sync_all()
            ts0 = time.perf_counter()
            h.frameStep(dv)
            sync_all()
            ts1 = time.perf_counter()
            if i > 0:
                p_s.append(ts1 - ts0)
                p_cut.append(float(ctx.stage_times()[4]))
                p_redone += int(h.last_step_cut_proof()["redone"])
        ctx.set_config(cfg)
        n_p = len(p_s)
        proven = {"value": B * n_p / float(np.sum(p_s)), "ms_per_step": 1e3 * float(np.mean(p_s)),
                  "line_cut_ms": float(np.mean(p_cut)), "steps": n_p, "redone_sequences": p_redone,
                  "note": "cut_proof 1 on the same sequences right after the timed window (frames "
                          f"{W + K + 2}..{W + K + n_proven}): the measured-mode line's decisions proven after the "
                          "fact, unproven sequences redone by the eager-proven search (DESIGN.md §3)"}
    host_fed = None
    if world == 1 and not args.no_host_fed:
        host_fed = host_fed_rate(h, cam, sp_up, B, KP, KL, seq0, W + K + 1 + n_proven, gen_threads, per_up, dev,
                                 distinct=distinct if replicate else B)

    if rank == 0:
        sm = np.mean(np.array(stage_ms, dtype=np.float64)[:, :6], axis=0)
        sb = np.mean(np.array(stage_bytes)[:, :6], axis=0).astype(np.float64)
        km = np.mean(np.array(kern_ms, dtype=np.float64), axis=0)
        kb = np.mean(np.array(kern_bytes), axis=0).astype(np.float64)
        # candidate kernels for the roofline line: the single-kernel stages and the
        # kernels that dominate the line-cut and pose stages
        cands = {"k_stereo_points": (sm[0], sb[0]), "k_stereo_lines": (sm[1], sb[1]),
                 "k_cross_points": (sm[2], sb[2]), "k_cross_lines": (sm[3], sb[3]),
                 "k_cut_search": (km[1], kb[1]), "k_pose": (km[3], kb[3])}
        kname = max(cands, key=lambda x: cands[x][0])
        k_ms, k_bytes = cands[kname]
        achieved = k_bytes / (k_ms * 1e-3) / 1e9
        step_bytes = float(np.mean(np.array(stage_bytes)[:, 6]))
        value = frames_total / t_max
        pmc, pmc_note = load_pmc(args.pmc, kname, B, args.workload, K, W)
        pmc = pmc or {}
        traffic = pmc.get("hbm_bytes_per_launch")
        roof_valu = None
        if pmc.get("SQ_INSTS_VALU"):
            gips = pmc["SQ_INSTS_VALU"] / (k_ms * 1e-3) / 1e9
            roof_valu = {"bound": "valu", "kernel": kname, "achieved": gips, "peak": VALU_PEAK_GIPS,
                         "unit": "G wave-VALU-instructions/s", "frac": gips / VALU_PEAK_GIPS,
                         "valu_insts_per_launch": pmc["SQ_INSTS_VALU"], "waves_per_launch": pmc.get("SQ_WAVES"),
                         "source": os.path.relpath(args.pmc, ROOT)}
        b1 = None
        if world == 1 and not args.no_b1:
            try:
                b1 = latency_b1(ctx, cam, cfg, sp, KP, KL, seq0, W, args.b1_steps)
            except Exception as e:   # reported, never fatal to the contract line
                b1 = {"error": f"{type(e).__name__}: {e}"}
        cpu = None
        if world == 1 and not args.no_cpu:
            nt = args.cpu_threads or cores
            cpu = cpu_baseline(cam, cfg, sp, KP, KL, nt, args.cpu_seconds, cores_info, gen_threads, W + K)
            if args.cpu_sweep_seconds > 0:
                cpu["thread_sweep"] = cpu_thread_sweep(cam, cfg, sp, KP, KL, nt, args.cpu_sweep_seconds,
                                                       gen_threads, W + K, cpu,
                                                       b1.get("cpu_1thread_ms_per_frame") if b1 else None)
        det = None
        if world == 1 and not args.no_detect:
            up_Bps = host_fed["upload_GBps"] * 1e9 if host_fed and host_fed.get("upload_GBps") else 0.0
            det = detection_rates(cam, up_Bps)
            try:
                det["images_to_poses"] = pipeline_rate(cam, cfg, bars=0)
                det["images_to_poses_lsd"] = pipeline_rate(cam, cfg, B=1536, lsd=True)
            except Exception as e:   # reported, never fatal to the contract line
                det["images_to_poses"] = {"error": f"{type(e).__name__}: {e}"}
        cmean = {n: round(float(np.mean([c[n] for c in counts])), 1) for n in gfpl.StereoFrameHandler.STEP_COUNTS}
        # matched entries the pose optimisation flagged as outliers (removeOutliers); n_inliers
        # above is the insert's (the list sizes), before optimize_pose
        cmean["outliers_after_pose"] = round(float(np.mean([c["M_p"] + c["M_l"] for c in counts]) -
                                                 np.mean([c["inliers_after_pose"] for c in cutc]) / B), 1)
        crange = {n: [round(float(min(c[n] for c in counts)), 1), round(float(max(c[n] for c in counts)), 1)]
                  for n in ("S_p", "S_l", "M_o", "M_p", "M_l")}
        out = {
            "metric": "stereo frames/sec (2k ORB + 500 LBD, 10 GN iters)",
            "value": value,
            "unit": "stereo frames/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": t_max / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (deterministic splitmix64 stereo detections + right ORB pyramid, gfpl_synth; "
                    "stationary scene: landmarks re-spawn in the frustum), generated per step on the host and "
                    "uploaded to HBM before each timed step" +
                    (f"; {distinct} distinct generated sequences per rank, each uploaded to {B // distinct} of "
                     f"the {B} tracked sequences (host generation budget)" if replicate else ""),
            "config": {"workload": desc, "sequences_per_gpu": B, "kp_per_side": int(sp.n_kp),
                       "kl_per_side": int(sp.n_kl), "gn_iters": "10+10",
                       "parallelism": f"sequences sharded 1/{world} per GPU",
                       "timing": "sum of K per-step brackets (barrier + device sync both sides), MAX over ranks"},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": float(achieved), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": float(achieved / HBM_PEAK_GBS), "traffic": traffic,
                         "traffic_gather_calibrated": pmc.get("hbm_bytes_per_launch_gather_cal"),
                         "traffic_calibration": "traffic = (2 FETCH_SIZE + WRITE_SIZE) KB as the microarch guide "
                                                "prescribes for 16-B streams; traffic_gather_calibrated = FETCH_SIZE / 0.95 "
                                                "+ WRITE_SIZE, the factor measured for dword gathers (profiles/r04_fcal)",
                         "traffic_note": pmc_note,
                         "algorithmic_bytes_per_launch": float(k_bytes), "avg_launch_ms": float(k_ms),
                         "occupancy": pmc.get("occupancy_waves_per_simd"),
                         "occupancy_unit": "mean resident waves per SIMD (4 x SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8) "
                                           "/ 1024 SIMDs, PMC over the same window)",
                         "cycles": {k: pmc.get(k) for k in ("frac_wait_any", "frac_wait_inst", "frac_active",
                                                             "cycle_closure")},
                         "window": f"the {K} timed steps (launches {W + 1}..{W + K} of each step kernel)"},
            "roofline_valu": roof_valu,
            "hbm_frac_step": float(step_bytes / (t_max / K) / 1e9 / HBM_PEAK_GBS),
            "counts_per_seq_step": cmean,
            "counts_range_over_steps": crange,
            "parity_sampled": {"sequences": len(sampler.seqs) * world if sampler else 0,
                               "frames": par[0], "mismatches": par[1],
                               "compared": "stereo features, matched lists, inlier counts, cut ratios, invCovPose, "
                                           "cut endpoints, pose (DT, Tfw, DT_cov, Tfw_cov, eig, err_norm) bitwise "
                                           "vs the CPU oracle (oracle/)",
                               "first": sampler.msgs[:3] if sampler else []},
            "cut_search": {"mode": CUT_MODES[int(cfg.cut_proof)], "cut_certify": float(cfg.cut_certify),
                           "proof": ({"redone_sequences": int(sum(c["redone"] for c in proofc)),
                                      "redone_frac": float(sum(c["redone"] for c in proofc) / (B * K)),
                                      "steps_proven_after_the_fact": int(sum(c["steps_proven"] for c in proofc)),
                                      "vref_evals_per_line": float(sum(c["vref_evals"] for c in proofc) /
                                                                   max(1, sum(c["lines"] for c in proofc))),
                                      "note": "k_cut_verify: every margined decision of the recorded search proven "
                                              "with the reference's own endpoint variances at the compared ratios "
                                              "and the two running invCov_sums; unproven sequences redone by the "
                                              "eager-proven search (DESIGN.md §3)"}
                                     if cfg.cut_proof == 1 else None),
                           "proven_leg": proven,
                           "steps": int(sum(c["steps"] for c in cutc)),
                           "exact_steps": int(sum(c["exact_steps"] for c in cutc)),
                           "exact_frac": float(sum(c["exact_steps"] for c in cutc) / max(1, sum(c["steps"] for c in cutc))),
                           "lines_unbounded_frac": float(sum(c["lines_unbounded"] for c in cutc) /
                                                         max(1.0, B * float(sum(c["M_l"] for c in counts)))),
                           "note": "greedy steps of the timed window; exact_steps: evaluated with the reference's own "
                                   "arithmetic because a margin or the proven agreement bound failed (DESIGN.md §3)"},
            "host_fed": host_fed,
            "stage_ms": {n: round(float(v), 4) for n, v in zip(STAGES, sm)},
            "kernel_ms": {n: round(float(v), 4) for n, v in zip(["k_cut_prep", "k_cut_search", "k_cut_finish", "k_pose"], km)},
            "kernel_bytes": kernel_traffic(args.pmc, B, args.workload, K, W, km, kb, sm[0], sb[0]),
            "stage_bytes_per_step": {n: int(v) for n, v in zip(STAGES, sb)},
            "cpu_baseline": cpu,
            "latency_b1_ms": b1.get("latency_b1_ms") if b1 else None,
            "latency_b1": b1,
            "detection": det,
            "host": host_info,
            "gen_s": round(t_gen, 2),
            "lost_sampled": int(lost),
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def host_fed_rate(h, cam, sp, B, KP, KL, seq0, f0, gen_threads, per_in, dev, steps=8, distinct=None):
    """PCIe-inclusive rate of a host-fed pipeline (rank 0 at N=1, after the timed steps):
    two input frames (f0, f0 + 1) of all B sequences held in pinned host memory are uploaded
    with gfpl_upload_frames_async into the two staging buffers in turn — the copy of step
    j + 1 on the seqbatch's copy stream, the step j on the context stream, ordered by the
    staging events — for `steps` steps (the frames alternate), wall clock from the first
    copy to the last step.  Generation excluded.  Needs two pinned input frames on the host
    and a second staging buffer in HBM; skipped (with the reason) when they do not fit."""
    import torch
    import gfpl
    in_bytes = per_in * B                                    # over PCIe per step
    row_bytes = gfpl.input_bytes_per_frame(cam, KP, KL) * B   # host rows (pyramid rows allocated whole)
    try:
        import psutil
        avail = psutil.virtual_memory().available
    except Exception:
        avail = None
    free, _ = torch.cuda.mem_get_info(dev)
    if (avail is not None and avail < 2.6 * row_bytes) or free < 1.1 * row_bytes:
        return {"skipped": f"needs 2 x {row_bytes / 1e9:.1f} GB pinned host memory and a second staging buffer"}
    hb = [gfpl.HostBatch(cam, sp, B, KP, KL, seq0=seq0, pinned=True) for _ in range(2)]   # sp: level 0 only
    D = distinct or B
    for i, x in enumerate(hb):
        x.fill(f0 + i, gen_threads, n=D)
        for s0 in range(D, B, D):   # replicated distinct sequences (see --distinct)
            n = min(D, B - s0)
            for a in x.arrays():
                a[s0:s0 + n] = a[:n]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    pb = int(cam.pyr_bytes)
    h.upload_async(hb[0].frames(), 0, 1, l0_stride=pb)
    for j in range(steps):
        if j + 1 < steps:
            h.upload_async(hb[(j + 1) % 2].frames(), 0, (j + 2) % 2, l0_stride=pb)
        h.frameStep(h.staged_frames((j + 1) % 2))
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    # the copy alone, for the upload rate
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    h.upload_wait(h.upload_async(hb[0].frames(), 0, 1, l0_stride=pb))
    up = time.perf_counter() - t1
    del hb
    return {"value": B * steps / wall, "unit": "stereo frames/s", "steps": steps,
            "ms_per_step": wall / steps * 1e3, "upload_ms_per_step": up * 1e3, "upload_GBps": in_bytes / up / 1e9,
            "input_bytes_per_step": int(in_bytes),
            "note": "frames f0, f0+1 of every sequence in pinned host memory, uploaded (gfpl_upload_frames_l0_async: "
                    "detections + level 0 of the right image; levels 1.. resized on the device, copy stream, two "
                    "staging buffers) while the step on the other buffer runs; the frames alternate; generation / "
                    "detection excluded"}


if __name__ == "__main__":
    main()
