"""Host-side verifier helper of the library (bn_sumcheck_interpolate, the reference's
evaluate_univariate_given_points, verifier.cu:9-31) against the oracle; runs on CPU."""
import numpy as np
import pytest

import _oracle as O
import binius_ntt_amd as B


@pytest.mark.parametrize("npts", [1, 2, 3, 4, 5, 9, 16])
def test_interpolate_matches_oracle(npts):
    g = np.random.default_rng(npts)
    for _ in range(20):
        p = g.integers(0, 2**32, size=(npts, 4), dtype=np.uint64).astype(np.uint32)
        c = g.integers(0, 2**32, size=4, dtype=np.uint64).astype(np.uint32)
        assert np.array_equal(B.evaluate_univariate_given_points(c, p), O.interpolate(p, c))


def test_interpolate_reproduces_the_points():
    # the interpolant through (k, p_k) evaluates to p_k at k
    g = np.random.default_rng(5)
    p = g.integers(0, 2**32, size=(4, 4), dtype=np.uint64).astype(np.uint32)
    for k in range(4):
        assert np.array_equal(B.evaluate_univariate_given_points(np.array([k, 0, 0, 0], np.uint32), p), p[k])


def test_interpolate_rejects_bad_sizes():
    with pytest.raises(B.BnError):
        B.evaluate_univariate_given_points(np.zeros(4, np.uint32), np.zeros((17, 4), np.uint32))
