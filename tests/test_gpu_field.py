"""GPU parity for the tower-field kernels: compact and bitsliced products vs the reference KATs
(test_fanpaartower.cu, tests.cu) and the oracle; bitslice transposes vs BitsliceUtils."""
import numpy as np
import pytest

import _oracle as O
import binius_ntt_amd as B

pytestmark = pytest.mark.gpu


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(dev)


def _np(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


def _rand(n, seed):
    return np.random.default_rng(seed).integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)


def test_gf32_kats(field_kats, dev):
    import torch
    k = np.array(field_kats["mul32"], dtype=np.uint64).astype(np.uint32)
    a, b = _t(k[:, 0], dev), _t(k[:, 1], dev)
    o = torch.empty_like(a)
    B.gf32_mul(a, b, o)
    assert np.array_equal(_np(o), k[:, 2])


def test_gf128_compact_kats_and_random(field_kats, dev):
    import torch
    pairs = [(a, b, c) for a, b, c in field_kats["mul128"]]
    blk = field_kats["mul128_block"]
    for e in range(4):
        a = sum(blk["a"][4 * e + i] << (32 * i) for i in range(4))
        b = sum(blk["b"][4 * e + i] << (32 * i) for i in range(4))
        pairs.append((a, b, O.mul128(a, b)))
    rng = np.random.default_rng(11)
    for _ in range(200):
        a = int.from_bytes(rng.bytes(16), "little")
        b = int.from_bytes(rng.bytes(16), "little")
        pairs.append((a, b, O.mul128(a, b)))
    w = lambda x: [(x >> (32 * i)) & 0xFFFFFFFF for i in range(4)]
    A = np.array([w(p[0]) for p in pairs], dtype=np.uint64).astype(np.uint32)
    Bm = np.array([w(p[1]) for p in pairs], dtype=np.uint64).astype(np.uint32)
    C = np.array([w(p[2]) for p in pairs], dtype=np.uint64).astype(np.uint32)
    ta, tb = _t(A.reshape(-1), dev), _t(Bm.reshape(-1), dev)
    to = torch.empty_like(ta)
    B.gf128_mul(ta, tb, to)
    assert np.array_equal(_np(to).reshape(-1, 4), C)


def test_bitslice_roundtrip_matches_oracle(dev):
    x = _rand(128 * 300, 5)
    t = _t(x, dev)
    B.bitslice(t)
    bs = _np(t)
    assert np.array_equal(bs, O.bitslice128(x))
    B.bitslice(t, untranspose=True)
    assert np.array_equal(_np(t), x)


@pytest.mark.parametrize("nblk", [1, 15, 16, 17, 63, 64, 65, 1000])
def test_bitslice_sizes_both_directions(nblk, dev):
    """bn_bitslice_device runs 16 blocks per wave and 64 per work-group: every ragged tail, in both
    directions, against BitsliceUtils (the oracle), and nothing written past the last block."""
    import torch
    x = _rand(128 * nblk, 600 + nblk)
    buf = torch.full((128 * (nblk + 16),), 0x3C3C3C3C, dtype=torch.int32, device=dev)
    buf[:128 * nblk] = _t(x, dev)
    B.bitslice(buf[:128 * nblk])
    got = _np(buf)
    assert np.array_equal(got[:128 * nblk], O.bitslice128(x))
    assert np.all(got[128 * nblk:] == 0x3C3C3C3C)
    y = _rand(128 * nblk, 700 + nblk)
    buf[:128 * nblk] = _t(y, dev)
    B.bitslice(buf[:128 * nblk], untranspose=True)
    got = _np(buf)
    assert np.array_equal(got[:128 * nblk], O.unbitslice128(y))
    assert np.all(got[128 * nblk:] == 0x3C3C3C3C)


def test_bitslice_round_trip_at_size(dev):
    """2^20 blocks (512 MiB): untranspose(transpose(x)) == x, and a sampled block against the oracle."""
    import torch
    g = torch.Generator(device="cpu").manual_seed(9)
    x = torch.randint(-2**31, 2**31, (128 << 20,), dtype=torch.int32, generator=g).to(dev)
    y = x.clone()
    B.bitslice(y)
    blk = 777777
    want = O.bitslice128(x[128 * blk:128 * (blk + 1)].cpu().numpy().view(np.uint32))
    assert np.array_equal(_np(y[128 * blk:128 * (blk + 1)]), want)
    B.bitslice(y, untranspose=True)
    torch.cuda.synchronize()
    assert torch.equal(x, y)


def test_bitsliced_gf128_mul_kat_and_random(field_kats, dev):
    import torch
    # reference KAT block (test_fanpaartower.cu:199-273) padded with random elements
    blk = field_kats["mul128_block"]
    a = _rand(128 * 64, 21)
    b = _rand(128 * 64, 22)
    a[:16] = blk["a"]
    b[:16] = blk["b"]
    ta, tb = _t(O.bitslice128(a), dev), _t(O.bitslice128(b), dev)
    to = torch.empty_like(ta)
    B.gf128_mul_bitsliced(ta, tb, to)
    out = O.unbitslice128(_np(to))
    assert list(out[:16]) == blk["out"]
    exp = np.array([[(O.mul128(sum(int(a[4 * e + i]) << (32 * i) for i in range(4)),
                                sum(int(b[4 * e + i]) << (32 * i) for i in range(4))) >> (32 * i)) & 0xFFFFFFFF
                     for i in range(4)] for e in range(256)], dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(out[:1024].reshape(-1, 4), exp)
    # alias-safe: out == a
    B.gf128_mul_bitsliced(ta, tb, ta)
    assert np.array_equal(O.unbitslice128(_np(ta))[:16], np.array(blk["out"], dtype=np.uint32))


@pytest.mark.parametrize("kind,threads", [(0, 64), (1, 64), (2, 64), (2, 70)])
def test_repeat_microbench_kernels_match_oracle(kind, threads, dev):
    iters = 3
    words = 4 if kind == 0 else 128
    s0 = _rand(threads * words, 31 + kind)
    op = _rand(threads * words, 41 + kind)
    ts, top = _t(s0, dev), _t(op, dev)
    B.gf128_mul_repeat(kind, ts, top, threads, iters)
    got = _np(ts)
    if kind >= 1:
        got, s_c, o_c = O.unbitslice128(got), O.unbitslice128(s0), O.unbitslice128(op)
    else:
        s_c, o_c = s0, op
    to_int = lambda v, e: sum(int(v[4 * e + i]) << (32 * i) for i in range(4))
    for e in range(0, len(s_c) // 4, 7):
        x = to_int(s_c, e)
        for _ in range(iters):
            x = O.mul128(x, to_int(o_c, e))
        assert x == to_int(got, e), e


def _mul128_rows(A, Bm):
    w = lambda x: [(x >> (32 * i)) & 0xFFFFFFFF for i in range(4)]
    v = lambda r: sum(int(r[i]) << (32 * i) for i in range(4))
    return np.array([w(O.mul128(v(a), v(b))) for a, b in zip(A, Bm)], dtype=np.uint64).astype(np.uint32)


@pytest.mark.parametrize("n", [1, 31, 32, 33, 511, 512, 513, 2047, 2048, 2049, 4100])
def test_gf128_compact_ragged_sizes(n, dev):
    """bn_gf128_mul_device runs 512 elements per wave and 2048 per work-group: every ragged tail
    (partial quad, partial wave, partial work-group) against the oracle, and nothing written past n."""
    import torch
    A = _rand(4 * n, 100 + n).reshape(-1, 4)
    Bm = _rand(4 * n, 200 + n).reshape(-1, 4)
    ta, tb = _t(A.reshape(-1), dev), _t(Bm.reshape(-1), dev)
    guard = torch.full((4 * (n + 64),), 0x5A5A5A5A, dtype=torch.int32, device=dev)
    B.gf128_mul(ta, tb, guard[:4 * n])
    got = _np(guard)
    idx = np.arange(0, n, max(1, n // 300))  # every element for small n, a spread for the rest
    assert np.array_equal(got[:4 * n].reshape(-1, 4)[idx], _mul128_rows(A[idx], Bm[idx]))
    assert np.all(got[4 * n:] == 0x5A5A5A5A)


def test_gf128_compact_alias_safe(dev):
    n = 3000
    A = _rand(4 * n, 7).reshape(-1, 4)
    Bm = _rand(4 * n, 8).reshape(-1, 4)
    exp = _mul128_rows(A[::97], Bm[::97])
    ta, tb = _t(A.reshape(-1), dev), _t(Bm.reshape(-1), dev)
    B.gf128_mul(ta, tb, ta)  # out == a
    assert np.array_equal(_np(ta).reshape(-1, 4)[::97], exp)
    ta = _t(A.reshape(-1), dev)
    B.gf128_mul(ta, tb, tb)  # out == b
    assert np.array_equal(_np(tb).reshape(-1, 4)[::97], exp)


def test_gf128_compact_matches_bitsliced_path_at_size(dev):
    """2^22 compact products against the bitsliced product (itself oracle- and KAT-checked above)
    on the same operands: bitslice -> multiply_unrolled<7> -> unbitslice."""
    import torch
    n = 1 << 22
    g = torch.Generator(device="cpu").manual_seed(5)
    a = torch.randint(-2**31, 2**31, (4 * n,), dtype=torch.int32, generator=g).to(dev)
    b = torch.randint(-2**31, 2**31, (4 * n,), dtype=torch.int32, generator=g).to(dev)
    o = torch.empty_like(a)
    B.gf128_mul(a, b, o)
    abs_, bbs = a.clone(), b.clone()
    B.bitslice(abs_)
    B.bitslice(bbs)
    B.gf128_mul_bitsliced(abs_, bbs, abs_)
    B.bitslice(abs_, untranspose=True)
    torch.cuda.synchronize()
    assert torch.equal(o, abs_)


@pytest.mark.parametrize("n", [1, 255, 4097])
def test_gf32_random_and_zero_operands(n, dev):
    """bn_gf32_mul_device on random words with zero bytes planted (the GF(2^8) leaves index the
    exp table at log(0) = 512 and above, where it holds 0), against the oracle's tower product."""
    import torch
    a = _rand(n, 300 + n)
    b = _rand(n, 400 + n)
    a[::3] &= 0xFFFF00FF  # a zero byte in a leaf operand
    b[::5] &= 0x00FFFFFF
    a[::7] = 0
    b[1::11] = 0
    ta, tb = _t(a, dev), _t(b, dev)
    o = torch.empty_like(ta)
    B.gf32_mul(ta, tb, o)
    exp = np.array([O.mul(int(x), int(y), 5) for x, y in zip(a, b)], dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(_np(o), exp)
