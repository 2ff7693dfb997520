"""bench.py's multi-rank launch path on the CPU: `--gpus 2` without a torch.distributed
environment re-launches itself under torch.distributed.run (2 ranks, 127.0.0.1), and --dry-run
runs the process-group setup (gloo), barriers, max-over-ranks, batch slicing and the sharded
message exchange (WordExchange: all_gather_into_tensor + XOR) with no GPU work. The driver's
8-GPU scaling run is then not the first execution of this code."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""  # CPU rehearsal even on a GPU box
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout  # exactly one JSON line on stdout (rank 0)
    return json.loads(lines[0])


def test_bench_dry_run_world1():
    d = _run(["--dry-run"])
    assert d["dry_run"] and d["n_gpus"] == 1


def test_bench_dry_run_relaunch_world2():
    d = _run(["--gpus", "2", "--dry-run"])
    assert d["dry_run"] and d["n_gpus"] == 2
    assert d["rank_checks"] == {"xor_exchange_ok": True, "max_over_ranks": 1.0, "batch_slices_cover": True}
