"""Test-only CPU shard prover with the same semantics as the HIP prover's shard interface
(bn_sumcheck_set_shard / needs_gather / export_shard / import_gathered), built on the oracle's
GF(2^128) multiply. It lets the CPU (gloo) tests drive binius_ntt_amd.distributed.ShardedSumcheck
without a GPU. Small sizes only (one ctypes call per product)."""
import numpy as np

import _oracle as O


def _int(w):
    return int(w[0]) | (int(w[1]) << 32) | (int(w[2]) << 64) | (int(w[3]) << 96)


def _words(x):
    return np.array([(x >> (32 * i)) & 0xFFFFFFFF for i in range(4)], np.uint32)


class OracleShardProver:
    def __init__(self, compact_cols, rank, world):
        """compact_cols: (d, 2^n, 4) uint32 — the FULL columns; keeps batches b % world == rank."""
        cols = np.asarray(compact_cols, np.uint32)
        self.d, n = cols.shape[0], cols.shape[1]
        nb = n // 32
        keep = [b for b in range(nb) if b % world == rank]
        self.cols = [[_int(cols[j, 32 * b + e]) for b in keep for e in range(32)] for j in range(self.d)]
        self.world = world
        self.cur = len(self.cols[0])

    def needs_gather(self):
        return self.world > 1 and self.cur <= 32

    def this_round_messages(self):
        assert not self.needs_gather()
        d, cur = self.d, self.cur
        h = cur // 2
        pts = []
        if cur == 1:
            p = 1
            for j in range(d):
                p = O.mul128(p, self.cols[j][0])
            return _words(p), np.zeros((d + 1, 4), np.uint32)
        for k in range(d + 1):
            acc = 0
            for x in range(h):
                p = 1
                for j in range(d):
                    lo, hi = self.cols[j][x], self.cols[j][x + h]
                    p = O.mul128(p, lo ^ O.mul128(k, lo ^ hi))
                acc ^= p
            pts.append(acc)
        return _words(pts[0] ^ pts[1]), np.stack([_words(p) for p in pts])

    def move_to_next_round(self, challenge):
        assert not self.needs_gather() and self.cur >= 2
        r = _int(np.asarray(challenge, np.uint32))
        h = self.cur // 2
        for j in range(self.d):
            c = self.cols[j]
            self.cols[j] = [c[x] ^ O.mul128(r, c[x] ^ c[x + h]) for x in range(h)]
        self.cur = h

    def export_shard(self):
        # composition_size bitsliced 128-word batches, as bn_sumcheck_export_shard
        out = []
        for j in range(self.d):
            blk = np.zeros((32, 4), np.uint32)
            for e in range(self.cur):
                blk[e] = _words(self.cols[j][e])
            out.append(O.bitslice128(blk.reshape(-1)))
        return np.concatenate(out)

    def import_gathered(self, words, world):
        w = np.asarray(words, np.uint32).reshape(world, self.d, 128)
        self.cols = []
        for j in range(self.d):
            col = []
            for r in range(world):
                blk = O.unbitslice128(w[r, j]).reshape(32, 4)
                col += [_int(blk[e]) for e in range(32)]
            self.cols.append(col)
        self.world = 1
        self.cur = 32 * world
