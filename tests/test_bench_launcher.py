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


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "2"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
