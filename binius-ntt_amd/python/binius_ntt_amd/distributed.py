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


class WordExchange:
    """All-gather of a fixed-length uint32 vector over the group, on preallocated buffers: the
    words are staged into a (pinned, for RCCL) host tensor, copied once to the send buffer,
    `all_gather_into_tensor` fills a (world x n) receive buffer on the collective's device, and one
    copy brings it back to host. int32 carries the bits unchanged (no reduction is asked of the
    backend). RCCL has no XOR reduction, so XOR-reduce = this gather + a local XOR."""

    def __init__(self, n, group=None):
        import torch
        import torch.distributed as dist
        self.n, self.group = n, group
        self.world = dist.get_world_size(group)
        self.dev = _device_for(dist, group)
        pin = self.dev.type == "cuda"
        self.h_send = torch.empty(n, dtype=torch.int32, pin_memory=pin)
        self.h_recv = torch.empty(self.world * n, dtype=torch.int32, pin_memory=pin)
        self.d_send = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.d_recv = torch.empty(self.world * n, dtype=torch.int32, device=self.dev)
        self.seconds = 0.0  # wall time spent in exchanges (staging + collective + copy back)
        self.calls = 0

    def gather(self, words):
        import time
        import torch.distributed as dist
        t0 = time.perf_counter()
        w = np.ascontiguousarray(words, dtype=np.uint32).reshape(-1)
        if w.size != self.n:
            raise ValueError("WordExchange: %d words, built for %d" % (w.size, self.n))
        self.h_send.numpy()[:] = w.view(np.int32)
        if self.dev.type == "cuda":
            self.d_send.copy_(self.h_send, non_blocking=True)
            dist.all_gather_into_tensor(self.d_recv, self.d_send, group=self.group)
            self.h_recv.copy_(self.d_recv)  # synchronous: the host needs the words now
            out = self.h_recv.numpy()
        else:
            dist.all_gather_into_tensor(self.d_recv, self.h_send, group=self.group)
            out = self.d_recv.numpy()
        res = out.view(np.uint32).reshape(self.world, self.n).copy()
        self.seconds += time.perf_counter() - t0
        self.calls += 1
        return res

    def xor(self, words):
        return np.bitwise_xor.reduce(self.gather(words), axis=0)


def allgather_words(words, group=None):
    """All-gather a uint32 vector (same length on every rank); returns a (world, n) uint32 array."""
    w = np.ascontiguousarray(words, dtype=np.uint32).reshape(-1)
    return WordExchange(w.size, group).gather(w)


def xor_allreduce_words(words, group=None):
    """XOR-reduce a uint32 vector over all ranks (all-gather + local XOR)."""
    g = allgather_words(words, group)
    return np.bitwise_xor.reduce(g, axis=0)


SINK_WORDS = 40  # bn_sumcheck_set_message_sink: 4 * (8 + 1) point words, the p(1)-skipped flag at 36


class ShardedSumcheck:
    """Drives a sharded prover so that every rank sees the global round messages.

    Exchange paths for the per-round (sum, points) words:
      * device (default on an nccl group with a HIP prover): the prover's messages kernel also writes
        its raw partial points into a preallocated device sink (bn_sumcheck_set_message_sink) and
        the round is read with bn_sumcheck_round_messages_sink, which does not wait for the kernel.
        `all_gather_into_tensor` of the sink is enqueued on the PROVER's stream right behind the
        messages kernel, one copy on that stream brings the world x 40 words back, and the host
        waits only for that copy. The partial points are XOR-ed and p(1), sum are completed from the
        GLOBAL claim (p(1) = claim + p(0), sum = claim, the claim being the previous round's global
        points interpolated at its challenge);
      * host (gloo, or a prover without a sink): the prover's round_messages polls its posted
        points and the words are staged through WordExchange.
    device_exchange=True on a gloo group keeps the device path's protocol (sink, flags, p(1) from
    the global claim) and stages only the sink through host memory (a copy on the prover's stream)
    for the CPU collective: the world-2 gloo GPU test runs the multi-rank device path that way.
    exchange_at_world1=True runs the exchange even when the group has one rank (the RCCL rehearsal
    on a one-GPU box exercises the device path that way)."""

    def __init__(self, prover, group=None, device_exchange=None, exchange_at_world1=False):
        import torch.distributed as dist
        self.prover = prover
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.replicated = self.world == 1 and not exchange_at_world1  # after the endgame gather every rank holds everything
        self._msg = None  # WordExchange for the (d + 2) x 4 message words, built on first use
        self.exchange_seconds = 0.0  # per-round message exchanges + the endgame gather
        self.exchange_rounds = 0
        self.round_seconds = 0.0  # whole this_round_messages calls (the round's kernel wait included)
        if device_exchange is None:
            device_exchange = dist.is_initialized() and dist.get_backend(group) == "nccl"
        self.device_exchange = (bool(device_exchange) and hasattr(prover, "round_messages_sink")
                                and not self.replicated)
        self._claim = None     # global claim of the coming round (device path)
        self._last_pts = None  # previous round's global points (device path)
        if self.device_exchange:
            import torch
            pdev = torch.device("cuda", prover.device if getattr(prover, "device", None) is not None
                                else torch.cuda.current_device())
            cdev = _device_for(dist, group)
            self._stage = cdev.type != "cuda"  # a CPU collective (gloo)
            if not self._stage and cdev != pdev:
                raise ValueError("ShardedSumcheck: the prover runs on %s but the process group's device is %s"
                                 % (pdev, cdev))
            # the prover's own stream: the sink's consumers are enqueued behind its messages kernel
            self._pstream = torch.cuda.ExternalStream(prover.stream_handle(), device=pdev)
            self._sink = torch.zeros(SINK_WORDS, dtype=torch.int32, device=pdev)
            if self._stage:
                self._send = torch.empty(SINK_WORDS, dtype=torch.int32)
                self._recv = torch.empty(self.world * SINK_WORDS, dtype=torch.int32)
            else:
                self._recv = torch.empty(self.world * SINK_WORDS, dtype=torch.int32, device=pdev)
                self._h_recv = torch.empty(self.world * SINK_WORDS, dtype=torch.int32, pin_memory=True)
            prover.set_message_sink(self._sink)

    def _gather_if_needed(self):
        if not self.replicated and self.prover.needs_gather():
            mine = self.prover.export_shard()
            ex = WordExchange(mine.size, self.group)
            allw = ex.gather(mine)
            self.exchange_seconds += ex.seconds
            self.prover.import_gathered(allw.reshape(-1), self.world)
            self.replicated = True
            if self.device_exchange:
                self.prover.set_message_sink(None)

    def _device_round(self, d1):
        import time
        import torch
        import torch.distributed as dist
        t0 = time.perf_counter()
        self.prover.round_messages_sink()  # queued, not waited for
        # everything below runs on the prover's stream, behind its messages kernel (the documented
        # consumer contract of bn_sumcheck_set_message_sink); the host waits only for the last copy
        with torch.cuda.stream(self._pstream):
            if self._stage:
                self._send.copy_(self._sink)  # device -> pageable host: synchronous on this stream
                dist.all_gather_into_tensor(self._recv, self._send, group=self.group)
                g = self._recv.numpy().view(np.uint32).reshape(self.world, SINK_WORDS)
            else:
                dist.all_gather_into_tensor(self._recv, self._sink, group=self.group)
                self._h_recv.copy_(self._recv)  # after the collective on this stream; synchronous
                g = self._h_recv.numpy().view(np.uint32).reshape(self.world, SINK_WORDS)
        flag_words = g[:, 36]
        if not np.all(flag_words == flag_words[0]):
            raise RuntimeError("ShardedSumcheck: ranks disagree on the round's flags %s" % flag_words.tolist())
        raw = np.bitwise_xor.reduce(g[:, :4 * d1], axis=0).reshape(d1, 4).copy()
        flags = int(flag_words[0])
        if flags & 2:  # the last call (one evaluation left): words 0-3 are prod_j f_j(r)
            s = raw[0].copy()
            raw[:] = 0
        elif flags & 1:  # p(1) was not computed: complete it from the global claim
            if self._claim is None:
                raise RuntimeError("ShardedSumcheck: p(1) skipped without a global claim")
            raw[1] = self._claim ^ raw[0]
            s = self._claim.copy()
        else:
            s = raw[0] ^ raw[1]
        self.exchange_seconds += time.perf_counter() - t0
        self.exchange_rounds += 1
        return s, raw

    def this_round_messages(self):
        import time
        t0 = time.perf_counter()
        try:
            return self._round_messages()
        finally:
            self.round_seconds += time.perf_counter() - t0

    def _round_messages(self):
        self._gather_if_needed()
        if self.replicated:
            self._last_pts = None
            return self.prover.this_round_messages()
        if self.device_exchange:
            s, pts = self._device_round(self.prover.d + 1)
            self._last_pts = pts
            return s, pts
        s, pts = self.prover.this_round_messages()
        d1 = pts.shape[0]
        flat = np.concatenate([np.asarray(s, np.uint32).reshape(-1), np.asarray(pts, np.uint32).reshape(-1)])
        if self._msg is None:
            self._msg = WordExchange(flat.size, self.group)
        t = self._msg.seconds
        flat = self._msg.xor(flat)
        self.exchange_seconds += self._msg.seconds - t
        self.exchange_rounds += 1
        return flat[:4].copy(), flat[4:].reshape(d1, 4).copy()

    def move_to_next_round(self, challenge):
        self._gather_if_needed()
        self.prover.move_to_next_round(challenge)
        # the next round's global claim, computed while its messages kernel runs
        if self.device_exchange and self._last_pts is not None:
            from . import evaluate_univariate_given_points
            self._claim = np.asarray(evaluate_univariate_given_points(challenge, self._last_pts), np.uint32)
        else:
            self._claim = None
        self._last_pts = None
