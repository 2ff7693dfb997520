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


def test_valu_transform_budget(monkeypatch):
    """bench.py's transform-level VALU roofline: the sum of the passes'
    committed VALU counts per transform time against both ceilings, and the instruction budget the
    north star's 60 %-of-HBM target implies at the bitop3 ceiling."""
    sys.path.insert(0, ROOT)
    import bench

    counts = {"k0": 73.6e6, "k1": 85.9e6, "k2": 263.2e6}
    monkeypatch.setattr(bench, "kernel_counters", lambda name: ({"SQ_INSTS_VALU": counts[name]}, None))

    class Ntt:
        def pass_kernel_name(self, i):
            return "k%d" % i

    alg = 2 * 16 * (1 << 24)
    v = bench.valu_transform(Ntt(), 3, 0.70, alg)
    assert v["insts_per_transform"] == sum(counts.values())
    assert abs(v["achieved"] - 422.7e6 / 0.70e-3) < 1e3
    # at the bitop3 ceiling (0.34 of 0.5 per SIMD-cycle) 422.7M instructions take ~0.506 ms
    assert abs(v["floor_ms_at_ceiling"] - 0.5056) < 1e-3
    # the 60 % target: 537 MB in 0.1118 ms -> ~93.5M instructions, 4.5x fewer than now
    assert abs(v["target"]["ms"] - 0.11185) < 1e-4
    assert abs(v["target"]["insts_budget_at_ceiling"] / 1e6 - 93.5) < 0.5
    assert 4.4 < v["target"]["reduction_needed"] < 4.6
    assert 0.13 < v["hbm_frac_cap_at_ceiling"] < 0.14
    monkeypatch.setattr(bench, "kernel_counters", lambda name: (None, "profiled on another build"))
    v = bench.valu_transform(Ntt(), 3, 0.70, alg)
    assert v["insts_per_transform"] is None and "another build" in v["note"]
