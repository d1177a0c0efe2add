"""bench.py's multi-rank launcher and timing protocol on the CPU (gloo, --dry-run): `--gpus 2`
without a torch.distributed environment starts two ranks as child processes and rank 0 prints one
JSON line with n_gpus = 2 (the driver's N>1 runs use the same path under torch.distributed.run)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_launcher_two_ranks():
    line = _run("--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1")
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["scaling"] == "strong"
    assert line["value"] > 0 and line["ms_per_step"] > 0
    # BASELINE config 3: ONE 3M-impression set sharded over the ranks, contiguous and complete
    assert line["config"]["global_batch"] == 3_000_000
    assert [tuple(s) for s in line["config"]["shards"]] == [(0, 1_500_000), (1_500_000, 1_500_000)]


def test_single_rank_default():
    line = _run("--dry-run", "--steps", "2", "--warmup", "0")
    assert line["n_gpus"] == 1
    assert line["config"]["global_batch"] == 3_000_000
