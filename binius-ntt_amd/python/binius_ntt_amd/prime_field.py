"""Prime-field sibling of the sumcheck: QM31 values and the QM31 Sumcheck prover over the C-ABI.

Mirrors src/ulvt/prime_field_sumcheck (sumcheck.cuh:8-96, utils/interpolate.hpp:3-8) and the
field classes src/ulvt/finite_fields/{m31,cm31,qm31}.cuh: CM31 = M31[i]/(i^2 + 1),
QM31 = CM31[u]/(u^2 - (2 + i)). A QM31 is held as 4 canonical M31 ints (lo.a, lo.b, hi.a, hi.b).
"""
import ctypes

import numpy as np

from . import _check, lib

P = (1 << 31) - 1


class QM31:
    """qm31.cuh:8-82. QM31(v) for an int v < p is (v, 0, 0, 0); QM31([a, b, c, d]) takes 4
    components (uint64 sums are reduced, as QM31(uint64_t[4]))."""

    def __init__(self, v=0):
        if isinstance(v, (list, tuple, np.ndarray)):
            self.c = [int(x) % P for x in v]
        else:
            self.c = [int(v) % P, 0, 0, 0]

    @staticmethod
    def _cm(a, b):
        return a[0] * b[0] - a[1] * b[1], a[0] * b[1] + a[1] * b[0]

    def __add__(self, o):
        return QM31([x + y for x, y in zip(self.c, QM31._q(o).c)])

    def __sub__(self, o):
        return QM31([x - y for x, y in zip(self.c, QM31._q(o).c)])

    def __mul__(self, o):
        o = QM31._q(o)
        lo, hi, lo2, hi2 = self.c[:2], self.c[2:], o.c[:2], o.c[2:]
        ll = self._cm(lo, lo2)
        hh = self._cm(hi, hi2)
        rhh = self._cm((2, 1), hh)
        a = self._cm(lo, hi2)
        b = self._cm(hi, lo2)
        return QM31([ll[0] + rhh[0], ll[1] + rhh[1], a[0] + b[0], a[1] + b[1]])

    @staticmethod
    def _q(o):
        return o if isinstance(o, QM31) else QM31(o)

    def __eq__(self, o):
        return isinstance(o, QM31) and self.c == o.c

    def words(self):
        return np.array(self.c, dtype=np.uint32)

    def __repr__(self):
        return "QM31(%s)" % self.c


ONE_HALF = QM31(0x40000000)


def interpolate_at(challenge, evals):
    """utils/interpolate.hpp:3-8: the degree-2 polynomial through (0, e0), (1, e1), (2, e2) at x."""
    c = QM31._q(challenge)
    return (c * (c - 1) * evals[2] * ONE_HALF) - (c * (c - 2) * evals[1]) + ((c - 1) * (c - 2) * evals[0] * ONE_HALF)


class Sumcheck:
    """Sumcheck<NUM_VARS> over QM31 (two columns, product composition)."""

    def __init__(self, num_vars, evals, device=0):
        """evals: column 0 then column 1, 2^num_vars QM31 each, as an (2 * 2^num_vars, 4) or
        flat uint32 array, or a list of QM31 / ints (sumcheck.cuh:24-44)."""
        if isinstance(evals, list):
            evals = np.stack([QM31._q(e).words() for e in evals])
        e = np.ascontiguousarray(evals, dtype=np.uint32).reshape(-1)
        if e.size != 8 << num_vars:
            raise ValueError("expected 2 * 2^%d QM31 values" % num_vars)
        p = ctypes.c_void_p()
        _check(lib().bn_qm31_sumcheck_create(device, num_vars, e.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                             ctypes.byref(p)))
        self._sc = p
        self.num_vars = num_vars

    def close(self):
        if getattr(self, "_sc", None) is not None and self._sc.value:
            lib().bn_qm31_sumcheck_destroy(self._sc)
            self._sc = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def this_round_messages(self):
        out = np.zeros(12, np.uint32)
        _check(lib().bn_qm31_sumcheck_round_messages(self._sc, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
        return [QM31(out[4 * k:4 * k + 4]) for k in range(3)]

    def fold(self, challenge):
        w = QM31._q(challenge).words()
        _check(lib().bn_qm31_sumcheck_fold(self._sc, w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))

    def final_values(self):
        out = np.zeros(8, np.uint32)
        _check(lib().bn_qm31_sumcheck_final_values(self._sc, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
        return QM31(out[:4]), QM31(out[4:])
