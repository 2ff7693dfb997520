"""RCCL rehearsal on one GPU: the exact process-group call bench.py makes for N > 1
(`init_process_group("nccl", device_id=cuda:local)`), the device branch of
`distributed.WordExchange` (pinned host staging, `all_gather_into_tensor` on the GPU, one copy
back), the max-over-ranks `all_reduce` and a barrier, and ShardedSumcheck's device-resident round
exchange (the prover's message sink gathered directly) against an unsharded transcript, all over
the nccl (= RCCL) backend with world size 1. A single GPU cannot hold two RCCL ranks, so this is as far as the multi-GPU data path can
run before the driver's 8-GPU bench; its multi-rank logic is covered by the gloo tests
(tests/test_distributed.py, tests/test_bench_cli.py)."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(sys.argv[1], "binius-ntt_amd", "python"))
    from binius_ntt_amd import distributed as D
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    ex = D.WordExchange(24)
    assert ex.dev.type == "cuda"
    words = np.random.default_rng(7).integers(0, 2**32, size=24, dtype=np.uint64).astype(np.uint32)
    for _ in range(3):
        got = ex.gather(words)
        assert got.shape == (1, 24) and np.array_equal(got[0], words)
        assert np.array_equal(ex.xor(words), words)
    t = torch.tensor([1.5], device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    assert t.item() == 1.5 and ex.calls == 6

    # the sharded prover's device-resident exchange (message sink -> all_gather_into_tensor ->
    # one copy back, p(1) completed from the global claim), forced at world 1, against an
    # unsharded prover's transcript; and the host-staged path (WordExchange) beside it
    import json, time
    import binius_ntt_amd as B
    n, d = 18, 3
    rng = np.random.default_rng(1818)
    ev = rng.integers(0, 2**32, size=d * (4 << n), dtype=np.uint64).astype(np.uint32)
    ch = rng.integers(0, 2**32, size=(n, 4), dtype=np.uint64).astype(np.uint32)
    def transcript(sc):
        out = []
        for r in range(n + 1):
            s, p = sc.this_round_messages()
            out.append((s.copy(), p.copy()))
            if r < n:
                sc.move_to_next_round(ch[r])
        return out
    ref = B.Sumcheck(n, d, True, ev)
    want = transcript(ref)
    ref.close()
    # per-round cost of each path: whole transcripts (round kernels, waits and exchanges), the
    # modes alternated over several repetitions after one warm-up transcript each
    stats = {"device_round_ms": [], "host_round_ms": [], "device_exchange_ms": [], "host_exchange_ms": []}
    for rep in range(4):
        for mode in ("device", "host"):
            pr = B.Sumcheck(n, d, True, ev)
            sc = D.ShardedSumcheck(pr, device_exchange=(mode == "device"), exchange_at_world1=True)
            assert sc.device_exchange == (mode == "device")
            t0 = time.perf_counter()
            got = transcript(sc)
            dt = time.perf_counter() - t0
            for r, ((s1, p1), (s2, p2)) in enumerate(zip(got, want)):
                assert np.array_equal(s1, s2) and np.array_equal(p1, p2), (mode, r)
            assert sc.exchange_rounds == n + 1
            if rep:
                stats[mode + "_round_ms"].append(dt * 1e3 / (n + 1))
                stats[mode + "_exchange_ms"].append(sc.round_seconds * 1e3 / (n + 1))
            pr.close()
    stats = {k: float(np.median(v)) for k, v in stats.items()}
    dist.destroy_process_group()
    print("EXCHANGE " + json.dumps(dict(stats, n=n, d=d, world=1, backend="nccl",
                                        note="round_ms: transcript wall time per round; exchange_ms: "
                                             "this_round_messages per round (kernel wait included)")))
    print("rccl world1 ok")
""")


@pytest.mark.gpu
def test_rccl_process_group_and_word_exchange_world1():
    import socket
    with socket.socket() as so:  # a free port for the rendezvous
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl world1 ok" in r.stdout
    for line in r.stdout.splitlines():
        if line.startswith("EXCHANGE "):
            print(line)  # per-round exchange cost of both paths (pytest -s shows it)
