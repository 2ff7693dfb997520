"""CPU: pin the oracle (oracle/) against the reference's own golden vectors and KATs.

additive_ntt_hashes: src/ulvt/ntt/tests/test_ntt.cu:52-124 (input std::mt19937(0xdeadbeef+log_h+r),
MD5 over output u32s). Field KATs: src/ulvt/finite_fields/tests/test_fanpaartower.cu, tests.cu.
"""
import numpy as np
import pytest

import _oracle as O


@pytest.mark.parametrize("log_h", list(range(1, 21)))
def test_antt32_r0_matches_reference_md5(ntt_md5, log_h):
    x = O.mt_fill(0xDEADBEEF + log_h, 1 << log_h)
    assert O.md5(O.antt32(x, log_h, 0)) == ntt_md5["0"][log_h]


@pytest.mark.parametrize("log_h", list(range(1, 17)))
def test_antt32_r2_matches_reference_md5(ntt_md5, log_h):
    x = O.mt_fill(0xDEADBEEF + log_h + 2, 1 << log_h)
    assert O.md5(O.antt32(x, log_h, 2)) == ntt_md5["2"][log_h]


@pytest.mark.parametrize("log_h,r", [(1, 0), (3, 1), (6, 0), (9, 2), (10, 3), (7, 4), (11, 0)])
def test_antt128_full_multiply_equals_limbwise(log_h, r):
    # GF(2^128) transform with full 128-bit multiplies == four GF(2^32) limb transforms
    x = O.fill128(0xDEADBEEF + log_h + r, 0x5EED0000, 1 << log_h)
    assert np.array_equal(O.antt128(x, log_h, r, limbwise=False), O.antt128(x, log_h, r, limbwise=True))


@pytest.mark.parametrize("log_h", [12, 16, 18])
def test_antt128_limb_planes_match_reference_md5(ntt_md5, log_h):
    # put the reference's own input stream in every limb: every output limb plane hashes to the table
    x = O.mt_fill(0xDEADBEEF + log_h, 1 << log_h)
    X = np.stack([x, x, x, x], axis=1)
    y = O.antt128(X, log_h, 0)
    for limb in range(4):
        assert O.md5_limb(y, limb) == ntt_md5["0"][log_h]


def test_subspace_table_same_in_gf32_and_gf128():
    s32 = O.subspace_evals(12, 3, 32)
    s128 = O.subspace_evals(12, 3, 128)
    assert np.array_equal(s128[:, :, 0], s32) and not s128[:, :, 1:].any()


def test_field_kats(field_kats):
    for a, b, c in field_kats["mul32"]:
        assert O.mul(a, b, 5) == c
    for a, c in field_kats["sqr32"]:
        assert O.square(a, 5) == c
    for a, c in field_kats["inv32"]:
        assert O.inv(a, 5) == c
    for a, b, c in field_kats["simd16"]:
        assert O.mul(a, b, 4) == c
    for a, b, c in field_kats["simd8"]:
        assert O.mul(a, b, 3) == c
    for a, b, c in field_kats["mul128"]:
        assert O.mul128(a, b) == c
    blk = field_kats["mul128_block"]
    for e in range(4):
        a = sum(blk["a"][4 * e + i] << (32 * i) for i in range(4))
        b = sum(blk["b"][4 * e + i] << (32 * i) for i in range(4))
        c = sum(blk["out"][4 * e + i] << (32 * i) for i in range(4))
        assert O.mul128(a, b) == c


def test_inverse128_roundtrip():
    rng = np.random.default_rng(7)
    for _ in range(20):
        a = int(rng.integers(1, 2**63)) | (int(rng.integers(0, 2**63)) << 64)
        assert O.mul128(a, O.inv128(a)) == 1


def test_bitslice_layout():
    # word 32*l + i, bit e  ==  bit i of limb l of element e   (bitslicing.cuh:32-47)
    rng = np.random.default_rng(3)
    blk = rng.integers(0, 2**32, size=128, dtype=np.uint64).astype(np.uint32)
    bs = O.bitslice128(blk)
    for l in range(4):
        for i in range(32):
            w = int(bs[32 * l + i])
            for e in range(32):
                assert ((w >> e) & 1) == ((int(blk[4 * e + l]) >> i) & 1)
    assert np.array_equal(O.unbitslice128(bs), blk)


@pytest.mark.parametrize("n,d,bs", [(6, 2, 0), (7, 3, 1), (8, 4, 0), (6, 3, 1)])
def test_sumcheck_oracle_invariants(n, d, bs):
    # the reference's protocol checks (src/ulvt/sumcheck/test/test.cu:41,49,77,100)
    rng = np.random.default_rng(n * 10 + d)
    ev = rng.integers(0, 2**32, size=4 * (1 << n) * d, dtype=np.uint64).astype(np.uint32)
    ch = rng.integers(0, 2**32, size=(n, 4), dtype=np.uint64).astype(np.uint32)
    sums, pts = O.sumcheck_run(ev, n, d, bs, ch)
    claim = None
    for r in range(n + 1):
        if r > 0:
            assert np.array_equal(sums[r], claim)
        if r < n:
            assert np.array_equal(sums[r], pts[r, 0] ^ pts[r, 1])
            claim = O.interpolate(pts[r], ch[r])
    comp = O.unbitslice128(ev) if bs else ev
    assert np.array_equal(O.multilinear_composition(comp, n, d, ch), claim)


@pytest.mark.parametrize("n,d", [(1, 1), (5, 2), (8, 3), (11, 4)])
def test_fold_multilinear_matches_lagrange_sum(n, d):
    # the large-size final-claim checker (fold form, multithreaded) vs the direct Lagrange-basis
    # restatement of evaluate_multilinear_composition (verifier.cu:88-107), compact and bitsliced
    rng = np.random.default_rng(40 + n + d)
    ev = rng.integers(0, 2**32, size=d * (4 << n), dtype=np.uint32)
    ch = rng.integers(0, 2**32, size=(n, 4), dtype=np.uint32)
    want = O.multilinear_composition(ev, n, d, ch)
    assert np.array_equal(O.multilinear_composition_fold(ev, n, d, False, ch), want)
    if n >= 5:
        bs = np.concatenate([O.bitslice128(c) for c in ev.reshape(d, -1)])
        assert np.array_equal(O.multilinear_composition_fold(bs, n, d, True, ch), want)


def test_multithreaded_ntt_matches_serial():
    L = O.lib()
    # at most one thread per 4096 butterflies of a stage (a small transform runs on one thread)
    assert L.orc_antt_mt_threads(10, 16) == 1
    assert L.orc_antt_mt_threads(15, 3) == 3 and L.orc_antt_mt_threads(15, 8) == 4
    assert L.orc_antt_mt_threads(24, 16) == 16 and L.orc_antt_mt_threads(24, 0) == 1
    for log_h, r in ((1, 0), (6, 0), (13, 0), (15, 0), (16, 1)):
        x = O.fill128(11 + log_h, 12, 1 << log_h)
        want = O.antt128(x, log_h, r)
        for nt in (1, 3, 8, 2):  # the persistent pool grows, then serves a smaller count
            out = np.zeros_like(want)
            L.orc_antt128_limbwise_mt(x.reshape(-1), out.reshape(-1), log_h, r, nt)
            assert np.array_equal(out, want), (log_h, r, nt)
