"""Multi-process (gloo, world size 2, CPU) coverage of the sharded paths' collective logic:
batch partitioning for the batched NTT, and the sharded sumcheck driver (partial round messages
all-gathered and XOR-ed, endgame gather of the last batches), against the oracle transcript.
The HIP prover implements the same shard interface; its single-process multi-shard parity is in
test_gpu_sumcheck.py."""
import os
import socket

import numpy as np
import pytest

import _oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, d, seed):
    import torch.distributed as dist

    from binius_ntt_amd.distributed import ShardedSumcheck
    from _shard_prover import OracleShardProver

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(seed)
        ev = rng.integers(0, 2**32, size=4 * (1 << n) * d, dtype=np.uint64).astype(np.uint32)
        ch = rng.integers(0, 2**32, size=(n, 4), dtype=np.uint64).astype(np.uint32)
        sums, pts = O.sumcheck_run(ev, n, d, 0, ch)
        prover = OracleShardProver(ev.reshape(d, 1 << n, 4), rank, world)
        sc = ShardedSumcheck(prover)
        for r in range(n + 1):
            s, p = sc.this_round_messages()
            assert np.array_equal(s, sums[r]), "round %d sum" % r
            assert np.array_equal(p, pts[r]), "round %d points" % r
            if r < n:
                sc.move_to_next_round(ch[r])
        assert sc.replicated
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,d", [(2, 7, 2), (2, 6, 3)])
def test_sharded_sumcheck_gloo(world, n, d):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), n, d, 100 + n + d), nprocs=world, join=True)


def test_batch_slices_partition():
    from binius_ntt_amd.distributed import batch_slice
    for total in (1, 7, 256):
        for world in (1, 2, 4, 8):
            got = [batch_slice(total, r, world) for r in range(world)]
            covered = [i for a, b in got for i in range(a, b)]
            assert covered == list(range(total))


def _xor_worker(rank, world, port):
    import torch.distributed as dist

    from binius_ntt_amd.distributed import xor_allreduce_words
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        mine = np.array([0xFFFFFFFF, rank, 1 << (31 - rank), 0xDEADBEEF], np.uint32)
        got = xor_allreduce_words(mine)
        want = np.bitwise_xor.reduce(
            np.stack([np.array([0xFFFFFFFF, r, 1 << (31 - r), 0xDEADBEEF], np.uint32) for r in range(world)]), axis=0)
        assert np.array_equal(got, want)
    finally:
        dist.destroy_process_group()


def test_xor_allreduce_gloo():
    import torch.multiprocessing as mp
    mp.spawn(_xor_worker, args=(2, _free_port()), nprocs=2, join=True)


def _gpu_worker(rank, world, port, n, d, seed, out_q, device_exchange=False, busy_stream=False):
    """One rank of the world-2 GPU rehearsal: the HIP shard prover (built from this rank's share
    only) driven by ShardedSumcheck over gloo, and this rank's slice of a batched GF(2^128) NTT.
    Both ranks use cuda:0 (the box has one GPU). busy_stream=True queues unrelated kernels on the
    prover's own stream between the protocol calls and, every other round, makes the host wait for
    them: the exchange (enqueued on that stream) and the last rounds' round server (resident on it)
    must neither deadlock nor reorder the transcript."""
    import torch
    import torch.distributed as dist

    import binius_ntt_amd as B
    from binius_ntt_amd.distributed import ShardedSumcheck, batch_slice

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        rng = np.random.default_rng(seed)
        ev = rng.integers(0, 2**32, size=d * (4 << n), dtype=np.uint32)  # bitsliced columns
        ch = rng.integers(0, 2**32, size=(n, 4), dtype=np.uint32)
        # this rank's batches b with b mod world == rank, column by column
        share = ev.reshape(d, (1 << n) // 32, 128)[:, rank::world, :]
        t = torch.from_numpy(np.ascontiguousarray(share).reshape(-1).view(np.int32)).to(dev)
        sc = ShardedSumcheck(B.Sumcheck.from_shard(n, d, t, rank, world), device_exchange=device_exchange)
        assert sc.device_exchange == device_exchange
        pstream = torch.cuda.ExternalStream(sc.prover.stream_handle(), device=dev)
        junk = torch.ones(1 << 20, device=dev)

        def churn(r):
            if busy_stream:
                with torch.cuda.stream(pstream):
                    junk.mul_(1.5).add_(-0.5)  # unrelated work on the prover's stream
                if r % 2:
                    pstream.synchronize()
        sums, pts = [], []
        for r in range(n + 1):
            churn(r)
            s, p = sc.this_round_messages()
            sums.append(s)
            pts.append(p)
            churn(r + 1)
            if r < n:
                sc.move_to_next_round(ch[r])
        assert sc.replicated
        # batched NTT: rank-contiguous slice of 6 transforms of 2^12 (no collective)
        total, log_h = 6, 12
        xs = np.stack([O.fill128(300 + b, 400 + b, 1 << log_h) for b in range(total)])
        lo, hi = batch_slice(total, rank, world)
        ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(7)))
        xin = torch.from_numpy(xs[lo:hi].reshape(-1).view(np.int32)).to(dev)
        yout = torch.empty_like(xin)
        ntt.forward_device(xin, yout, batch=hi - lo)
        torch.cuda.synchronize()
        y = yout.cpu().numpy().view(np.uint32).reshape(hi - lo, -1, 4)
        ntt_ok = bool(np.array_equal(y, O.antt128_batch(xs[lo:hi], log_h, 0)))
        out_q.put((rank, np.stack(sums), np.stack(pts), ntt_ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,device_exchange,busy", [(14, 3, False, False), (12, 2, False, False), (14, 3, True, False),
                                                      (13, 4, True, False), (14, 3, True, True), (12, 3, False, True)])
def test_sharded_hip_prover_world2_gloo(n, d, device_exchange, busy, dev):
    """World-2 gloo run of the HIP shard prover: the all-gathered + XOR-ed transcript equals the
    oracle's unsharded transcript, every rank sees the same messages, and each rank's slice of the
    batched NTT matches the oracle. device_exchange=True runs the RCCL path's protocol (message
    sink, flags, p(1) completed from the global claim) with the sink staged for gloo."""
    import torch.multiprocessing as mp
    seed = 700 + n + d
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_gpu_worker, args=(2, _free_port(), n, d, seed, q, device_exchange, busy), nprocs=2, join=True)
    got = dict()
    for _ in range(2):
        rank, s, p, ok = q.get(timeout=60)
        got[rank] = (s, p, ok)
    rng = np.random.default_rng(seed)
    ev = rng.integers(0, 2**32, size=d * (4 << n), dtype=np.uint32)
    ch = rng.integers(0, 2**32, size=(n, 4), dtype=np.uint32)
    want_s, want_p = O.sumcheck_run(ev, n, d, 1, ch)
    for rank in (0, 1):
        s, p, ok = got[rank]
        assert ok, "rank %d: batched NTT slice differs from the oracle" % rank
        assert np.array_equal(s, want_s), "rank %d: round sums" % rank
        assert np.array_equal(p, want_p), "rank %d: round points" % rank
