"""The reference's sumcheck test matrix at size (src/ulvt/sumcheck/test/test.cu:103-142:
N in {20, 24, 28} x d in {2, 3, 4} x DATA_IS_TRANSPOSED in {true, false}) on the GPU, with the
reference test's verifier loop (test.cu:31-100): every round sum == p(0) + p(1), every later sum
== the previous round polynomial interpolated at the challenge (verifier.cu:9-31), and the final
claim == prod_j f_j(r) computed on the CPU by the ORACLE (a fold-based restatement of
evaluate_multilinear_composition, verifier.cu:88-107; oracle/sumcheck.c), not by this library.

N = 28 runs one case (d = 3, bitsliced: configs 4-5's layout), generated on the device.
"""
import numpy as np
import pytest

import _oracle as O
import binius_ntt_amd as B

pytestmark = pytest.mark.gpu


def _verifier_loop(sc, n, ch):
    claim = None
    for r in range(n):
        s, p = sc.this_round_messages()
        if r > 0:
            assert np.array_equal(s, claim), "round %d: sum != previous claim" % r
        assert np.array_equal(s, p[0] ^ p[1]), "round %d: sum != p(0) + p(1)" % r
        claim = O.interpolate(p, ch[r])
        sc.move_to_next_round(ch[r])
    s, _ = sc.this_round_messages()
    assert np.array_equal(s, claim), "final round: prod_j f_j(r) != last claim"
    return claim


@pytest.mark.parametrize("transposed", [True, False])
@pytest.mark.parametrize("d", [2, 3, 4])
@pytest.mark.parametrize("n", [20, 24])
def test_reference_matrix(n, d, transposed, dev):
    rng = np.random.default_rng(0x5C00 + 100 * n + 10 * d + transposed)
    # any words are a valid bitsliced input; compact input is random elements
    ev = rng.integers(0, 2**32, size=d * (4 << n), dtype=np.uint32)
    ch = rng.integers(0, 2**32, size=(n, 4), dtype=np.uint32)
    sc = B.Sumcheck(n, d, transposed, ev)
    claim = _verifier_loop(sc, n, ch)
    sc.close()
    assert np.array_equal(O.multilinear_composition_fold(ev, n, d, transposed, ch), claim)


def test_2p28_d3_bitsliced(dev):
    import torch
    n, d = 28, 3
    g = torch.Generator(device=dev)
    g.manual_seed(0x28D3)
    ev_dev = torch.randint(-2**31, 2**31 - 1, (d * (4 << n),), dtype=torch.int32, device=dev, generator=g)
    ch = np.random.default_rng(0xC4A1).integers(0, 2**32, size=(n, 4), dtype=np.uint32)
    sc = B.Sumcheck(n, d, True, ev_dev)  # copies the columns (2 x 12 GiB on the device)
    ev = ev_dev.cpu().numpy().view(np.uint32)
    del ev_dev
    torch.cuda.empty_cache()
    claim = _verifier_loop(sc, n, ch)
    sc.close()
    assert np.array_equal(O.multilinear_composition_fold(ev, n, d, True, ch), claim)
