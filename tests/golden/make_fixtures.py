#!/usr/bin/env python3
"""Generate tests/golden/oracle_fixtures.json: the SURVEY.md §8(c) "fixtures to commit" for the
paths the reference holds no vectors for, produced by the CPU oracle (oracle/*.c, itself pinned to
the reference's MD5 tables and field KATs by tests/test_oracle.py). Committed so that the GPU tests
and later rounds check against stored data, not only against a live oracle run.

Inputs are regenerated from seeds with the oracle's mt19937 / mt19937_64 fills:
limb 0 of element i = std::mt19937(seed0) stream, limbs 1-3 = low 32 bits of
std::mt19937_64(seed64 + j). Nothing of the inputs is stored but the seeds.

  ntt128    GF(2^128) additive NTT, independent limbs: log_h 10 (r 0 and 2), 20, 24 (r 0): MD5 of
            the whole output (u32 LE words), MD5 per limb plane, first and last 16 elements
  sumcheck  transcripts (every round's sum and points 0..d, and the final claim) for
            N in {10, 12}, d in {2, 3, 4}, DATA_IS_TRANSPOSED in {false, true}; columns =
            fill128(0x5C00 + d, 0x5EED0000 + 16 d, d 2^N) column-major compact (bitsliced by
            the oracle for T = true), challenges = fill128(0xC4A1, 0x5EEDC4A1, N)
  mul128    1024 compact GF(2^128) products a_i * b_i, a = fill128(0xA128, 0x5EEDA000, 1024),
            b = fill128(0xB128, 0x5EEDB000, 1024): MD5 of the products and the first 16

  python tests/golden/make_fixtures.py        (about 10 s; the 2^24 transform dominates)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _oracle as O  # noqa: E402

OUT = os.path.join(HERE, "oracle_fixtures.json")
NTT_CASES = [(10, 0), (10, 2), (20, 0), (24, 0)]
SC_CASES = [(n, d, t) for n in (10, 12) for d in (2, 3, 4) for t in (0, 1)]


def words(a):
    return [int(v) for v in np.asarray(a, np.uint32).reshape(-1)]


def ntt_seeds(log_h, r):
    return 0xDEADBEEF + log_h + r, 0x5EED0000


def sc_inputs(n, d):
    cols = O.fill128(0x5C00 + d, 0x5EED0000 + 16 * d, d << n)
    ch = O.fill128(0xC4A1, 0x5EEDC4A1, n)
    return cols, ch


def mul_inputs():
    return O.fill128(0xA128, 0x5EEDA000, 1024), O.fill128(0xB128, 0x5EEDB000, 1024)


def mul_rows(a, b):
    """Row-wise compact GF(2^128) products through the oracle's scalar multiply."""
    to_int = lambda w: sum(int(w[i]) << (32 * i) for i in range(4))  # noqa: E731
    out = np.zeros_like(a)
    for i in range(a.shape[0]):
        v = O.mul128(to_int(a[i]), to_int(b[i]))
        out[i] = [(v >> (32 * k)) & 0xFFFFFFFF for k in range(4)]
    return out


def ntt_entry(log_h, r, out):
    s0, s64 = ntt_seeds(log_h, r)
    return {"log_h": log_h, "log_rate": r, "seed0": s0, "seed64": s64, "md5": O.md5(out),
            "md5_limbs": [O.md5_limb(out, j) for j in range(4)],
            "head": words(out[:16]), "tail": words(out[-16:])}


def main():
    fx = {"generator": "tests/golden/make_fixtures.py (CPU oracle)", "ntt128": [], "sumcheck": [], "mul128": None}
    for log_h, r in NTT_CASES:
        s0, s64 = ntt_seeds(log_h, r)
        x = O.fill128(s0, s64, 1 << log_h)
        fx["ntt128"].append(ntt_entry(log_h, r, O.antt128(x, log_h, r)))
        print("ntt128 log_h %d r %d done" % (log_h, r), flush=True)
    for n, d, t in SC_CASES:
        cols, ch = sc_inputs(n, d)
        inp = O.bitslice128(cols) if t else cols
        sums, pts = O.sumcheck_run(inp, n, d, t, ch)
        fx["sumcheck"].append({"n": n, "d": d, "transposed": t, "sums": words(sums), "points": words(pts),
                               "final_claim": words(O.multilinear_composition(cols, n, d, ch))})
    a, b = mul_inputs()
    p = mul_rows(a, b)
    fx["mul128"] = {"n": 1024, "md5": O.md5(p), "head": words(p[:16])}
    with open(OUT, "w") as f:
        json.dump(fx, f, separators=(",", ":"))
        f.write("\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
