"""Multi-GPU drivers (one process per GPU, torch.distributed over RCCL; gloo on CPU for tests).

The reference is single-GPU; the sharding below is this build's own:

* Batched additive NTT: transforms are independent, so rank g simply owns its slice of the
  batch (`batch_slice`) — no collective on the data path (weak scaling).
* Sumcheck (config 5): every column is sharded by 32-element batch index (rank g owns batches
  b with b mod world == g, bn_sumcheck_set_shard). Folds pair batch x with x + cur/64, which stay
  on one rank until each rank is down to one batch; round messages are XOR-sums, so each rank's
  partial (sum, points) is all-gathered and XOR-ed locally (RCCL has no XOR reduction). At the
  endgame every rank exports its last batch, the batches are all-gathered rank-major and every
  rank continues unsharded on the (tiny) gathered columns — the analogue of the reference's
  hand-over to the CPU at 32 evaluations (sumcheck.cuh:283-297).

`ShardedSumcheck` only needs a prover object with the `Sumcheck` shard methods
(this_round_messages, move_to_next_round, needs_gather, export_shard, import_gathered), so the
CPU tests drive the same collective logic with a test-side shard prover.
"""
import numpy as np


def batch_slice(total, rank, world):
    """Contiguous [start, stop) of `total` batched transforms owned by `rank`."""
    per = (total + world - 1) // world
    start = min(total, rank * per)
    return start, min(total, start + per)


def _device_for(dist, group):
    import torch
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def allgather_words(words, group=None):
    """All-gather a uint32 vector (same length on every rank); returns a (world, n) uint32 array."""
    import torch
    import torch.distributed as dist
    w = np.ascontiguousarray(words, dtype=np.uint32).reshape(-1)
    dev = _device_for(dist, group)
    t = torch.from_numpy(w.astype(np.int64)).to(dev)  # int64: every backend reduces/gathers it
    world = dist.get_world_size(group)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return np.stack([o.cpu().numpy().astype(np.uint32) for o in outs])


def xor_allreduce_words(words, group=None):
    """XOR-reduce a uint32 vector over all ranks (all-gather + local XOR)."""
    g = allgather_words(words, group)
    return np.bitwise_xor.reduce(g, axis=0)


class ShardedSumcheck:
    """Drives a sharded prover so that every rank sees the global round messages."""

    def __init__(self, prover, group=None):
        import torch.distributed as dist
        self.prover = prover
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.replicated = self.world == 1  # after the endgame gather every rank holds everything

    def _gather_if_needed(self):
        if not self.replicated and self.prover.needs_gather():
            mine = self.prover.export_shard()
            allw = allgather_words(mine, self.group)
            self.prover.import_gathered(allw.reshape(-1), self.world)
            self.replicated = True

    def this_round_messages(self):
        self._gather_if_needed()
        s, pts = self.prover.this_round_messages()
        d1 = pts.shape[0]
        flat = np.concatenate([np.asarray(s, np.uint32).reshape(-1), np.asarray(pts, np.uint32).reshape(-1)])
        if not self.replicated:
            flat = xor_allreduce_words(flat, self.group)
        return flat[:4].copy(), flat[4:].reshape(d1, 4).copy()

    def move_to_next_round(self, challenge):
        self._gather_if_needed()
        self.prover.move_to_next_round(challenge)
