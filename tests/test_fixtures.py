"""The committed oracle fixtures (tests/golden/oracle_fixtures.json, made by
tests/golden/make_fixtures.py; SURVEY.md §8c "fixtures to commit"):

* CPU: the oracle reproduces them, and the GF(2^128) NTT fixtures are tied to the reference's own
  MD5 table (limb 0 of each input is the reference's mt19937 stream, so that limb plane of the
  output must hash to additive_ntt_hashes[r][log_h], src/ulvt/ntt/tests/test_ntt.cu:52-124);
* GPU: the HIP NTT, sumcheck and compact multiply reproduce them through the C-ABI (including the
  2^24 headline transform, whose oracle run is too slow for the CPU suite)."""
import json
import os

import numpy as np
import pytest

import _oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
FX = json.load(open(os.path.join(HERE, "golden", "oracle_fixtures.json")))
REF_MD5 = json.load(open(os.path.join(HERE, "golden", "additive_ntt_md5.json")))["hashes"]

import sys  # noqa: E402
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_fixtures as M  # noqa: E402


def _ntt_ids(e):
    return "log_h%d_r%d" % (e["log_h"], e["log_rate"])


def _sc_ids(c):
    return "n%d_d%d_t%d" % (c["n"], c["d"], c["transposed"])


def _ref_md5(r, log_h):
    t = REF_MD5[str(r)]
    return t[str(log_h)] if isinstance(t, dict) else t[log_h]


def _check_ntt(out, e):
    assert O.md5(out) == e["md5"]
    assert [O.md5_limb(out, j) for j in range(4)] == e["md5_limbs"]
    assert M.words(out[:16]) == e["head"] and M.words(out[-16:]) == e["tail"]


def _check_transcript(sums, pts, c):
    assert M.words(sums) == c["sums"]
    assert M.words(pts) == c["points"]


@pytest.mark.parametrize("e", FX["ntt128"], ids=_ntt_ids)
def test_ntt_fixture_limb0_is_the_reference_md5(e):
    assert e["md5_limbs"][0] == _ref_md5(e["log_rate"], e["log_h"])


@pytest.mark.parametrize("e", [e for e in FX["ntt128"] if e["log_h"] <= 20], ids=_ntt_ids)
def test_oracle_reproduces_ntt_fixture(e):
    x = O.fill128(e["seed0"], e["seed64"], 1 << e["log_h"])
    _check_ntt(O.antt128(x, e["log_h"], e["log_rate"]), e)


@pytest.mark.parametrize("c", FX["sumcheck"], ids=_sc_ids)
def test_oracle_reproduces_sumcheck_fixture(c):
    cols, ch = M.sc_inputs(c["n"], c["d"])
    inp = O.bitslice128(cols) if c["transposed"] else cols
    sums, pts = O.sumcheck_run(inp, c["n"], c["d"], c["transposed"], ch)
    _check_transcript(sums, pts, c)
    assert M.words(sums[-1]) == c["final_claim"]


def test_oracle_reproduces_mul_fixture():
    a, b = M.mul_inputs()
    p = M.mul_rows(a, b)
    assert O.md5(p) == FX["mul128"]["md5"] and M.words(p[:16]) == FX["mul128"]["head"]


# ---------------------------------------------------------------- GPU: the HIP path vs the fixtures
@pytest.mark.gpu
@pytest.mark.parametrize("e", FX["ntt128"], ids=_ntt_ids)
def test_hip_ntt_matches_fixture(e, dev):
    import torch
    import binius_ntt_amd as B
    log_h, r = e["log_h"], e["log_rate"]
    x = O.fill128(e["seed0"], e["seed64"], 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, r, B.FanPaarTowerField(7), device=dev.index or 0))
    d_in = torch.from_numpy(x.reshape(-1).view(np.int32)).to(dev)
    d_out = torch.empty(x.size << r, dtype=torch.int32, device=dev)
    ntt.forward_device(d_in, d_out)
    torch.cuda.synchronize()
    _check_ntt(d_out.cpu().numpy().view(np.uint32).reshape(-1, 4), e)


@pytest.mark.gpu
@pytest.mark.parametrize("c", FX["sumcheck"], ids=_sc_ids)
def test_hip_sumcheck_matches_fixture(c, dev):
    import binius_ntt_amd as B
    n, d, t = c["n"], c["d"], c["transposed"]
    cols, ch = M.sc_inputs(n, d)
    sc = B.Sumcheck(n, d, t, O.bitslice128(cols) if t else cols)
    sums, pts = [], []
    for i in range(n + 1):
        s, p = sc.this_round_messages()
        sums.append(s)
        pts.append(p)
        if i < n:
            sc.move_to_next_round(ch[i])
    sc.close()
    _check_transcript(np.stack(sums), np.stack(pts), c)


@pytest.mark.gpu
def test_hip_compact_mul_matches_fixture(dev):
    import torch
    import binius_ntt_amd as B
    a, b = M.mul_inputs()
    ta = torch.from_numpy(a.reshape(-1).view(np.int32)).to(dev)
    tb = torch.from_numpy(b.reshape(-1).view(np.int32)).to(dev)
    to = torch.empty_like(ta)
    B.gf128_mul(ta, tb, to)
    torch.cuda.synchronize()
    p = to.cpu().numpy().view(np.uint32).reshape(-1, 4)
    assert O.md5(p) == FX["mul128"]["md5"] and M.words(p[:16]) == FX["mul128"]["head"]
