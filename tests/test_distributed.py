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
