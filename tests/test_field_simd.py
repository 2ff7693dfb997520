"""Field primitives beside the hot path: multiply_unrolled<H> (binary_tower_unrolled.cuh:4-5),
mul_binary_tower_32b_simd<H>, interleave_32b<H>, xor_adjacent_32b<H> (binary_tower_simd.cuh:77-150)
against the reference's KATs (test_fanpaartower.cu:10-52, tests.cu:17-95) and the oracle.

The host forms (library host functions, no GPU) run in the CPU suite; the device batches are
`-m gpu`."""
import numpy as np
import pytest

import _oracle as O
import binius_ntt_amd as B


def _rand(n, seed):
    return np.random.default_rng(seed).integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)


def _elements(words, h):
    """Bitsliced block of 2^h words -> the 32 compact elements (python ints)."""
    return [sum(((int(words[i]) >> e) & 1) << i for i in range(1 << h)) for e in range(32)]


def _bitslice(elems, h):
    return np.array([sum(((x >> i) & 1) << e for e, x in enumerate(elems)) for i in range(1 << h)], dtype=np.uint64).astype(
        np.uint32)


def _oracle_mul(a, b, h):
    return O.mul128(a, b) if h == 7 else O.mul(a, b, h)


def _expected(a, b, h):
    ea, eb = _elements(a, h), _elements(b, h)
    return _bitslice([_oracle_mul(x, y, h) for x, y in zip(ea, eb)], h)


# ---------------------------------------------------------------- host forms (CPU suite)
@pytest.mark.parametrize("h", [2, 3, 4, 5, 6, 7])
def test_multiply_unrolled_host_matches_oracle(h):
    a, b = _rand(1 << h, 10 + h), _rand(1 << h, 20 + h)
    want = _expected(a, b, h)
    assert np.array_equal(B.multiply_unrolled(h, a, b), want)
    # alias-safe: destination == first operand (core.cu:21 multiplies in place)
    x = a.copy()
    B.multiply_unrolled(h, x, b, x)
    assert np.array_equal(x, want)


def test_multiply_unrolled7_reference_kat(field_kats):
    # tests.cu:115-201 (multiply_unrolled<7> on the bitsliced 128-bit KAT) via the KAT block of
    # test_fanpaartower.cu:199-273: 4 elements, padded with zeros to one 32-element block
    blk = field_kats["mul128_block"]
    a = np.zeros(128, np.uint32)
    b = np.zeros(128, np.uint32)
    a[:16], b[:16] = blk["a"], blk["b"]
    out = O.unbitslice128(B.multiply_unrolled(7, O.bitslice128(a), O.bitslice128(b)))
    assert list(out[:16]) == blk["out"]
    sa, sb, sc = field_kats["mul128"][0]
    w = lambda x: [(x >> (32 * i)) & 0xFFFFFFFF for i in range(4)]
    a[:4], b[:4] = w(sa), w(sb)
    out = O.unbitslice128(B.multiply_unrolled(7, O.bitslice128(a), O.bitslice128(b)))
    assert list(out[:4]) == w(sc)


@pytest.mark.parametrize("key,h", [("simd_h0", 0), ("simd_h2", 2), ("simd8", 3), ("simd16", 4), ("simd_h5", 5)])
def test_mul_binary_tower_32b_simd_kats(field_kats, key, h):
    for a, b, c in field_kats[key]:
        assert B.mul_binary_tower_32b_simd(h, a, b) == c, (h, hex(a), hex(b))


def test_mul_binary_tower_32b_simd_matches_oracle():
    rng = np.random.default_rng(3)
    for h in range(6):
        w = 1 << h
        for _ in range(20):
            a, b = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
            want = 0
            for s in range(0, 32, w):
                m = (1 << w) - 1
                want |= O.mul((a >> s) & m, (b >> s) & m, h) << s
            assert B.mul_binary_tower_32b_simd(h, a, b) == want


def test_interleave_and_xor_adjacent_kats(field_kats):
    for h, a, b, c, d in field_kats["interleave32"]:
        assert B.interleave_32b(h, a, b) == (c, d), (h, hex(a), hex(b))
    # xor_adjacent: each pair of adjacent 2^h-bit blocks replaced by their sum in both places
    rng = np.random.default_rng(4)
    for h in range(5):
        w = 1 << h
        for _ in range(10):
            a = int(rng.integers(0, 2**32))
            want = 0
            for s in range(0, 32, 2 * w):
                m = (1 << w) - 1
                x = ((a >> s) & m) ^ ((a >> (s + w)) & m)
                want |= (x << s) | (x << (s + w))
            assert B.xor_adjacent_32b(h, a) == want


def test_field_simd_rejects_bad_heights():
    with pytest.raises(B.BnError):
        B.mul_binary_tower_32b_simd(6, 1, 1)
    with pytest.raises(B.BnError):
        B.interleave_32b(5, 1, 1)
    with pytest.raises(ValueError):
        B.multiply_unrolled(5, np.zeros(16, np.uint32), np.zeros(32, np.uint32))
    with pytest.raises(B.BnError):
        B._check(B.lib().bn_multiply_unrolled(8, B._u32p(np.zeros(256, np.uint32)), B._u32p(np.zeros(256, np.uint32)),
                                              B._u32p(np.zeros(256, np.uint32))))


# ---------------------------------------------------------------- device batches
def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(dev)


def _np(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("h", [2, 3, 4, 5, 6, 7])
def test_multiply_unrolled_device_matches_oracle(h, dev):
    import torch
    nblk = 37
    a, b = _rand(nblk << h, 30 + h), _rand(nblk << h, 40 + h)
    ta, tb = _t(a, dev), _t(b, dev)
    to = torch.empty_like(ta)
    B.multiply_unrolled_device(h, ta, tb, to)
    got = _np(to).reshape(nblk, -1)
    for k in (0, 1, nblk - 1):
        assert np.array_equal(got[k], _expected(a.reshape(nblk, -1)[k], b.reshape(nblk, -1)[k], h)), k
    host = np.stack([B.multiply_unrolled(h, a.reshape(nblk, -1)[k], b.reshape(nblk, -1)[k]) for k in range(nblk)])
    assert np.array_equal(got, host)
    B.multiply_unrolled_device(h, ta, tb, ta)  # alias-safe on the device too
    assert np.array_equal(_np(ta).reshape(nblk, -1), host)


@pytest.mark.gpu
def test_multiply_unrolled7_device_quad_path_large(dev):
    # multiply_unrolled<7> on the device runs on the quad-lane product, a persistent grid of 64-block
    # work-groups whose quads walk their blocks with the next operands prefetched: a batch of many grid
    # rounds (and a ragged last one), with the product written over the SECOND operand (alias-safe,
    # core.cu:21), sampled against the host
    import torch
    nblk = 262144 + 77
    g = np.random.default_rng(77)
    a = torch.randint(-2**31, 2**31 - 1, (128 * nblk,), dtype=torch.int32, device=dev, generator=None)
    b = torch.from_numpy(g.integers(0, 2**32, size=128 * nblk, dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
    a_np, b_np = _np(a).reshape(nblk, 128), _np(b).reshape(nblk, 128)
    B.multiply_unrolled_device(7, a, b, b)
    got = _np(b).reshape(nblk, 128)
    for k in (0, 1, 63, 64, 4095, 262143, 262144, nblk - 1) + tuple(g.integers(0, nblk, size=24)):
        assert np.array_equal(got[k], B.multiply_unrolled(7, a_np[k], b_np[k])), k


@pytest.mark.gpu
def test_packed32_device_kats(field_kats, dev):
    import torch
    for key, h in (("simd_h0", 0), ("simd_h2", 2), ("simd8", 3), ("simd16", 4), ("simd_h5", 5)):
        k = np.array(field_kats[key], dtype=np.uint64).astype(np.uint32)
        a, b = _t(k[:, 0], dev), _t(k[:, 1], dev)
        c = torch.empty_like(a)
        B.packed32_device(0, h, a, b, c)
        assert np.array_equal(_np(c), k[:, 2]), key
    for h in range(5):
        rows = [r for r in field_kats["interleave32"] if r[0] == h]
        k = np.array([r[1:] for r in rows], dtype=np.uint64).astype(np.uint32)
        a, b = _t(k[:, 0], dev), _t(k[:, 1], dev)
        c, d = torch.empty_like(a), torch.empty_like(a)
        B.packed32_device(1, h, a, b, c, d)
        assert np.array_equal(_np(c), k[:, 2]) and np.array_equal(_np(d), k[:, 3]), h
        x = _rand(1000, 50 + h)
        tx = _t(x, dev)
        ty = torch.empty_like(tx)
        B.packed32_device(2, h, tx, None, ty)
        assert all(int(v) == B.xor_adjacent_32b(h, int(u)) for u, v in zip(x[:64], _np(ty)[:64]))
