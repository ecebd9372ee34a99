"""bench.py's multi-GPU launcher on CPU: `--gpus 2` without a torch.distributed
environment spawns two workers (torch.distributed.run, gloo in --dry-run), which
broadcast the camera/config block, shard the sequences, generate their inputs and
reduce the counters; rank 0 prints one JSON line with n_gpus == 2.  A world size
that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--dry-run", "--batch", "4", "--steps", "3", "--warmup", "0", "--no-cpu", "--gen-threads", "1"]


def _run(extra, env=None):
    e = dict(os.environ, MASTER_ADDR="127.0.0.1")
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + extra + ARGS,
                          capture_output=True, text=True, timeout=300, cwd=ROOT, env=e)


def test_launcher_spawns_two_ranks():
    r = _run(["--gpus", "2", "--master-port", str(29700 + os.getpid() % 200)])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] is True and d["value"] is None
    assert d["frames_sharded"] == 2 * 4 * 3           # SUM over ranks of B * K
    assert d["config"]["sequences_per_gpu"] == 4


def test_launcher_eight_ranks_fit_one_host():
    """The N=8 launch (the driver's scaling run) rehearsed on CPU: 8 gloo ranks, each with its
    share of the host cores and a ring of two pinned chunks of its batch (not the whole
    batch: 8 ranks x 16.5 GB pinned would not fit a host), stated in the line."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-run", "--batch", "1024",
                        "--steps", "2", "--warmup", "0", "--no-cpu", "--master-port", str(29900 + os.getpid() % 90)],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["frames_sharded"] == 8 * 1024 * 2
    h = d["host"]
    per_seq = d["input_bytes_per_step"] / 1024
    assert h["chunk_sequences"] == 256                       # B / 8, at least 256
    assert d["pinned_bytes_per_rank_if_gpu"] == 2 * 256 * per_seq   # two chunks, not the batch
    cores = len(os.sched_getaffinity(0))
    assert h["cores_share_per_rank"] == max(1, cores // 8) and h["gen_threads_per_rank"] <= h["cores_share_per_rank"]


def test_eight_rank_generation_fits_its_budget():
    """One rank's share of an 8-rank host (2 generator threads) at the headline batch (16384
    sequences, 20 + 5 steps): generating every sequence's frames would take minutes, so the
    rank generates one chunk of distinct sequences per frame and uploads it into every chunk
    (stated in the line), and its projected generation time stays within two minutes."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--batch", "16384",
                        "--steps", "20", "--warmup", "5", "--no-cpu", "--gen-threads", "2"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    h = d["host"]
    assert h["gen_threads_per_rank"] == 2
    assert h["gen_all_distinct_s_per_rank"] > 60.0          # all 16384 would not fit
    # a fixed rule (< 8 generator threads: one chunk), not a timing: the same command always
    # tracks the same inputs
    assert h["chunk_sequences"] == 2048 and h["distinct_sequences_per_rank"] == 2048
    assert h["gen_projected_s_per_rank"] <= 120.0   # (timed on this host: a bound, not a budget the rule follows)
    assert d["gen_s"] <= 0.2 * h["gen_projected_s_per_rank"] + 5.0   # the dry run generated one frame


def test_cfg4_refuses_frames_past_the_trajectory():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--workload", "cfg4",
                        "--steps", "600", "--batch", "4", "--no-cpu"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 2 and "ground-truth poses" in r.stderr


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "2"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_cfg4_trajectory_covers_the_proven_leg():
    """cfg4's ground-truth trajectory must hold every frame the run generates, the proven leg's
    (one untimed + --proven-steps) included: 505 timed steps + init + 2 host-fed frames fit the 512
    stored poses only without the leg (a run that passed the check once failed at its first proven step)."""
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--workload", "cfg4", "--steps", "505",
            "--warmup", "0", "--batch", "4", "--no-cpu", "--gen-threads", "1"]
    r = subprocess.run(base, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 2 and "ground-truth poses" in r.stderr
    r = subprocess.run(base + ["--proven-steps", "0"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
