"""BabyBear radix-2 NTT (the prime-field sibling path): CPU oracle pinned
to the reference's MD5 table bb31_ntt_hashes (src/ulvt/ntt/tests/test_ntt.cu:21-50, 126-152),
and the HIP engine (-m gpu) against the table, the oracle and the reference's 2^24 round trip
(test_ntt.cu:154-187)."""
import json
import os

import numpy as np
import pytest

import _oracle as O

P = O.BB31_P
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def bb_md5():
    with open(os.path.join(HERE, "golden", "bb31_ntt_md5.json")) as f:
        return json.load(f)["hashes"]


@pytest.mark.parametrize("log_n", range(1, 21))
def test_oracle_matches_reference_md5(bb_md5, log_n):
    # exactly the reference's "NTTBB31 all input lengths": BB31(mt19937(0xdeadbeef + log_len)())
    x = O.mt_fill(0xDEADBEEF + log_n, 1 << log_n)
    assert O.md5(O.bb31_ntt(x, log_n)) == bb_md5[log_n]


@pytest.mark.parametrize("log_n", [1, 2, 4, 7])
def test_oracle_is_the_natural_order_dft(log_n):
    n = 1 << log_n
    x = O.mt_fill(0x1234 + log_n, n)
    w = pow(137, 1 << (27 - log_n), P)
    xs = [int(v) % P for v in x]
    ref = [sum(xs[j] * pow(w, j * k, P) for j in range(n)) % P for k in range(n)]
    assert list(O.bb31_ntt(x, log_n)) == ref


def test_oracle_bit_reversed_input():
    log_n = 9
    x = O.mt_fill(7, 1 << log_n)
    rev = np.array([int(format(i, "09b")[::-1], 2) for i in range(1 << log_n)])
    assert np.array_equal(O.bb31_ntt(x[rev], log_n, bit_reversed=True), O.bb31_ntt(x, log_n))


def test_oracle_round_trip():
    log_n = 12
    x = O.mt_fill(0xAABBCCDD, 1 << log_n) % P
    y = O.bb31_ntt(x, log_n)
    z = O.bb31_ntt(y, log_n, gen=O.lib().orc_bb31_inv(137))
    inv_n = O.lib().orc_bb31_inv(1 << log_n)
    assert np.array_equal((z.astype(np.uint64) * inv_n % P).astype(np.uint32), x)


# ---------------------------------------------------------------------------- GPU
def _dev_run(B, ntt, x, dev, batch=1, bit_reversed=False):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint32).view(np.int32)).to(dev)
    y = torch.empty_like(t)
    ntt.forward_device(t, y, batch=batch, bit_reversed=bit_reversed)
    torch.cuda.synchronize()
    return y.cpu().numpy().view(np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", list(range(1, 25)) + [pytest.param(h, marks=pytest.mark.slow) for h in (25, 26, 27)])
def test_gpu_reference_md5(bb_md5, log_n, dev):
    import binius_ntt_amd as B
    x = O.mt_fill(0xDEADBEEF + log_n, 1 << log_n)
    ntt = B.NTT(B.NTTConfRad2(B.BB31(137), 27, log_n))
    out = B.NTTData(1 << log_n)
    ntt.apply(B.NTTData(1 << log_n, B.DataOrder.IN_ORDER, 32, x), out)
    assert out.order == B.DataOrder.IN_ORDER
    assert O.md5(out.data) == bb_md5[log_n]


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", [3, 13, 14, 17, 19, 21])
def test_gpu_bit_reversed_batched_vs_oracle(log_n, dev):
    import binius_ntt_amd as B
    batch = 3
    xs = np.stack([O.mt_fill(50 + b + log_n, 1 << log_n) for b in range(batch)])
    ntt = B.NTT(B.NTTConfRad2(B.BB31(137), 27, log_n))
    got = _dev_run(B, ntt, xs.reshape(-1), dev, batch=batch, bit_reversed=True).reshape(batch, -1)
    for b in range(batch):
        assert np.array_equal(got[b], O.bb31_ntt(xs[b], log_n, bit_reversed=True))


@pytest.mark.gpu
def test_gpu_round_trip_2_24(dev):
    # the reference's "NTTBB31 round trip" (test_ntt.cu:154-187)
    import binius_ntt_amd as B
    log_n = 24
    x = O.mt_fill(0xAABBCCDD, 1 << log_n)
    g = B.BB31(137)
    fwd = B.NTT(B.NTTConfRad2(g, 27, log_n))
    inv = B.NTT(B.NTTConfRad2(B.BB31.inv(g), 27, log_n))
    y = _dev_run(B, fwd, x, dev)
    assert not np.array_equal(y, x % P)
    z = _dev_run(B, inv, y, dev)
    inv_n = B.BB31.inv(B.BB31(1 << log_n)).asUInt32()
    assert np.array_equal((z.astype(np.uint64) * inv_n % P).astype(np.uint32), x % P)


@pytest.mark.gpu
def test_gpu_rejects_bad_sizes(dev):
    import binius_ntt_amd as B
    with pytest.raises(ValueError):
        B.NTTConfRad2(B.BB31(137), 27, 28)
    ntt = B.NTT(B.NTTConfRad2(B.BB31(137), 27, 10))
    with pytest.raises(ValueError):
        ntt.apply(B.NTTData(1 << 9, B.DataOrder.IN_ORDER, 32), B.NTTData(1 << 10))


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", [5, 13, 17, 22])
def test_gpu_montgomery_words_in_montgomery_words_out(log_n, dev):
    # risc0 Fp (risc0_baby_bear.h:60-66) keeps val = x * 2^32 mod p in memory, so a raw-buffer
    # caller passing NTTData<BB31>'s bytes hands over Montgomery words. The transform is linear
    # and multiplies only by twiddles stored in Montgomery form (one Montgomery product each), so
    # Montgomery words in give Montgomery words out: the result's bytes equal the reference's.
    import binius_ntt_amd as B
    R = (1 << 32) % P
    x = (O.mt_fill(0x3031 + log_n, 1 << log_n).astype(np.uint64) % P)
    mont = (x * R % P).astype(np.uint32)
    ntt = B.NTT(B.NTTConfRad2(B.BB31(137), 27, log_n))
    got = _dev_run(B, ntt, mont, dev)
    want = (O.bb31_ntt(x.astype(np.uint32), log_n).astype(np.uint64) * R % P).astype(np.uint32)
    assert np.array_equal(got, want)
