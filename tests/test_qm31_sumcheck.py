"""QM31 sumcheck (the prime-field sibling). There are no golden vectors for
this path: parity is pinned by the reference test's protocol invariants
(src/ulvt/prime_field_sumcheck/test_sumcheck.cu:9-99: claim = p0 + p1, next claim =
interpolate_at(r, points)), the final brute-force check, and the CPU oracle's transcripts."""
import numpy as np
import pytest

import _oracle as O

REF_CHALLENGE = [32482843, 85864538, 8348234, 9544334]  # test_sumcheck.cu:68


def _ref_evals(n):
    # test_sumcheck.cu:18-24: both columns hold QM31(i)
    e = np.zeros((2, 1 << n, 4), np.uint32)
    e[0, :, 0] = np.arange(1 << n)
    e[1, :, 0] = np.arange(1 << n)
    return e


def _random_evals(n, seed):
    return np.random.default_rng(seed).integers(0, O.M31_P, size=(2, 1 << n, 4), dtype=np.uint64).astype(np.uint32)


def _check_protocol(points, evals, challenges, finals=None):
    """The reference test's invariants plus the final claim f0(r) f1(r)."""
    n = len(points)
    claim = np.zeros(4, np.uint32)
    for x in range(evals.shape[1]):
        claim = (claim.astype(np.uint64) + O.qm31_mul(evals[0, x], evals[1, x])) % O.M31_P
    claim = claim.astype(np.uint32)
    for i in range(n):
        s = ((points[i][0].astype(np.uint64) + points[i][1]) % O.M31_P).astype(np.uint32)
        assert np.array_equal(s, claim), "round %d: p0 + p1 != claim" % i
        claim = O.qm31_interpolate(points[i], challenges[i])
    if finals is not None:
        assert np.array_equal(O.qm31_mul(finals[0], finals[1]), claim)


@pytest.mark.parametrize("n,seed", [(1, 1), (6, 2), (10, 3)])
def test_oracle_protocol_invariants(n, seed):
    ev = _random_evals(n, seed)
    ch = np.random.default_rng(seed + 100).integers(0, O.M31_P, size=(n, 4), dtype=np.uint64).astype(np.uint32)
    pts = O.qm31_sumcheck_run(ev, n, ch)
    _check_protocol(pts, ev, ch)


def test_python_qm31_matches_oracle():
    import binius_ntt_amd.prime_field as PF
    g = np.random.default_rng(5)
    for _ in range(50):
        a = g.integers(0, O.M31_P, size=4)
        b = g.integers(0, O.M31_P, size=4)
        assert (PF.QM31(list(a)) * PF.QM31(list(b))).c == list(O.qm31_mul(a, b))
    pts = [PF.QM31(list(g.integers(0, O.M31_P, size=4))) for _ in range(3)]
    r = PF.QM31(REF_CHALLENGE)
    assert PF.interpolate_at(r, pts).c == list(O.qm31_interpolate(np.stack([p.words() for p in pts]), r.words()))


# ---------------------------------------------------------------------------- GPU
def _gpu_run(n, ev, ch):
    import binius_ntt_amd.prime_field as PF
    sc = PF.Sumcheck(n, ev.reshape(-1, 4))
    pts = []
    for i in range(n):
        p = sc.this_round_messages()
        pts.append(np.stack([q.words() for q in p]))
        sc.fold(PF.QM31(list(ch[i])))
    f0, f1 = sc.final_values()
    return np.stack(pts), (f0.words(), f1.words())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 5, 9, 12, 15])
def test_gpu_transcript_matches_oracle(n, dev):
    ev = _random_evals(n, 40 + n)
    ch = np.random.default_rng(7 + n).integers(0, O.M31_P, size=(n, 4), dtype=np.uint64).astype(np.uint32)
    pts, finals = _gpu_run(n, ev, ch)
    assert np.array_equal(pts, O.qm31_sumcheck_run(ev, n, ch))
    _check_protocol(pts, ev, ch, finals)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [20, pytest.param(24, marks=pytest.mark.slow)])
def test_gpu_reference_test_flow(n, dev):
    # "Prime Field Sumcheck Test" (test_sumcheck.cu:9-99): evals QM31(i), fixed challenge
    import binius_ntt_amd.prime_field as PF
    ev = _ref_evals(n)
    expected = PF.QM31(sum(i * i for i in range(1 << n)))
    sc = PF.Sumcheck(n, ev.reshape(-1, 4))
    r = PF.QM31(REF_CHALLENGE)
    for _ in range(n):
        pts = sc.this_round_messages()
        assert pts[0] + pts[1] == expected
        expected = PF.interpolate_at(r, pts)
        sc.fold(r)
    f0, f1 = sc.final_values()
    assert f0 * f1 == expected


@pytest.mark.gpu
def test_gpu_rejects_bad_arguments(dev):
    import binius_ntt_amd as B
    import binius_ntt_amd.prime_field as PF
    with pytest.raises(ValueError):
        PF.Sumcheck(3, np.zeros((7, 4), np.uint32))
    sc = PF.Sumcheck(1, np.zeros((4, 4), np.uint32))
    sc.this_round_messages()
    sc.fold(PF.QM31(3))
    with pytest.raises(B.BnError):
        sc.this_round_messages()


@pytest.mark.gpu
def test_gpu_folds_without_messages(dev):
    # fold is deferred and fused into the next round's messages; consecutive folds and a final
    # fold must still apply in order
    import binius_ntt_amd.prime_field as PF
    n = 11
    ev = _random_evals(n, 77)
    ch = np.random.default_rng(78).integers(0, O.M31_P, size=(n, 4), dtype=np.uint64).astype(np.uint32)
    want = O.qm31_sumcheck_run(ev, n, ch)
    sc = PF.Sumcheck(n, ev.reshape(-1, 4))
    for i in range(n):
        if i % 3 == 1:
            got = np.stack([q.words() for q in sc.this_round_messages()])
            assert np.array_equal(got, want[i]), i
        sc.fold(PF.QM31(list(ch[i])))
    f0, f1 = sc.final_values()
    _, finals = _gpu_run(n, ev, ch)
    assert (f0.words().tolist(), f1.words().tolist()) == (finals[0].tolist(), finals[1].tolist())
