"""ctypes bindings to the CPU oracle (oracle/liboracle.so) — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None

_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(path)
        L.orc_init.restype = None
        L.orc_mul.restype = ctypes.c_uint64
        L.orc_mul.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]
        L.orc_square.restype = ctypes.c_uint64
        L.orc_square.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.orc_inv.restype = ctypes.c_uint64
        L.orc_inv.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.orc_mul_alpha.restype = ctypes.c_uint64
        L.orc_mul_alpha.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.orc_mul32.restype = ctypes.c_uint32
        L.orc_mul32.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        for fn in ("orc_mul128",):
            getattr(L, fn).restype = None
            getattr(L, fn).argtypes = [_u32p, _u32p, _u32p]
        L.orc_inv128.restype = None
        L.orc_inv128.argtypes = [_u32p, _u32p]
        L.orc_subspace_evals32.argtypes = [ctypes.c_int, ctypes.c_int, _u32p]
        L.orc_subspace_evals128.argtypes = [ctypes.c_int, ctypes.c_int, _u32p]
        for fn in ("orc_antt32", "orc_antt128", "orc_antt128_limbwise"):
            getattr(L, fn).restype = None
            getattr(L, fn).argtypes = [_u32p, _u32p, ctypes.c_int, ctypes.c_int]
        L.orc_antt128_limbwise_mt.restype = None
        L.orc_antt128_limbwise_mt.argtypes = [_u32p, _u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_antt_mt_threads.restype = ctypes.c_int
        L.orc_antt_mt_threads.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_antt128_limbwise_batch.argtypes = [_u32p, _u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        for fn in ("orc_bitslice_transpose128", "orc_bitslice_untranspose128",
                   "orc_bitslice_transpose32", "orc_bitslice_untranspose32"):
            getattr(L, fn).restype = None
            getattr(L, fn).argtypes = [_u32p]
        L.orc_sumcheck_run.argtypes = [_u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u32p, _u32p, _u32p]
        L.orc_sumcheck_interpolate.argtypes = [_u32p, ctypes.c_int, _u32p, _u32p]
        L.orc_multilinear_composition.argtypes = [_u32p, ctypes.c_int, ctypes.c_int, _u32p, _u32p]
        L.orc_multilinear_composition_fold_mt.restype = None
        L.orc_multilinear_composition_fold_mt.argtypes = [_u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u32p, _u32p,
                                                          ctypes.c_int]
        L.orc_bitslice_many128.restype = None
        L.orc_bitslice_many128.argtypes = [_u32p, ctypes.c_size_t, ctypes.c_int]
        L.orc_mt_fill.argtypes = [ctypes.c_uint32, _u32p, ctypes.c_size_t]
        L.orc_fill128.argtypes = [ctypes.c_uint32, ctypes.c_uint64, _u32p, ctypes.c_size_t]
        L.orc_md5.argtypes = [ctypes.c_void_p, ctypes.c_size_t, _u8p]
        L.orc_md5_limb.argtypes = [_u32p, ctypes.c_size_t, ctypes.c_int, _u8p]
        L.orc_bb31_mul.restype = ctypes.c_uint32
        L.orc_bb31_mul.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.orc_bb31_pow.restype = ctypes.c_uint32
        L.orc_bb31_pow.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
        L.orc_bb31_inv.restype = ctypes.c_uint32
        L.orc_bb31_inv.argtypes = [ctypes.c_uint32]
        L.orc_bb31_ntt.restype = None
        L.orc_bb31_ntt.argtypes = [_u32p, _u32p, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
        L.orc_qm31_mul.restype = None
        L.orc_qm31_mul.argtypes = [_u32p, _u32p, _u32p]
        L.orc_qm31_interpolate.restype = None
        L.orc_qm31_interpolate.argtypes = [_u32p, _u32p, _u32p]
        L.orc_qm31_sumcheck_run.restype = None
        L.orc_qm31_sumcheck_run.argtypes = [_u32p, ctypes.c_int, _u32p, _u32p]
        L.orc_init()
        _LIB = L
    return _LIB


# ---------------- field ----------------
def mul(a, b, h):
    return lib().orc_mul(a, b, h)


def square(a, h):
    return lib().orc_square(a, h)


def inv(a, h):
    return lib().orc_inv(a, h)


def _to_words(x):
    return np.array([(x >> (32 * i)) & 0xFFFFFFFF for i in range(4)], dtype=np.uint32)


def _from_words(w):
    return sum(int(w[i]) << (32 * i) for i in range(4))


def mul128(a, b):
    out = np.zeros(4, np.uint32)
    lib().orc_mul128(_to_words(a), _to_words(b), out)
    return _from_words(out)


def inv128(a):
    out = np.zeros(4, np.uint32)
    lib().orc_inv128(_to_words(a), out)
    return _from_words(out)


# ---------------- NTT ----------------
def subspace_evals(log_h, log_rate, field_bits=32):
    width = log_h + log_rate - 1
    if field_bits == 32:
        s = np.zeros(max(1, log_h * width), np.uint32)
        lib().orc_subspace_evals32(log_h, log_rate, s)
        return s[: log_h * width].reshape(log_h, width)
    s = np.zeros(max(4, 4 * log_h * width), np.uint32)
    lib().orc_subspace_evals128(log_h, log_rate, s)
    return s[: 4 * log_h * width].reshape(log_h, width, 4)


def antt32(x, log_h, log_rate):
    x = np.ascontiguousarray(x, dtype=np.uint32)
    assert x.size == 1 << log_h
    out = np.zeros(1 << (log_h + log_rate), np.uint32)
    lib().orc_antt32(x, out, log_h, log_rate)
    return out


def antt128(x, log_h, log_rate, limbwise=True):
    """x: (2^log_h, 4) uint32 little-endian limbs -> (2^(log_h+log_rate), 4)."""
    x = np.ascontiguousarray(x, dtype=np.uint32)
    assert x.shape == (1 << log_h, 4)
    out = np.zeros((1 << (log_h + log_rate), 4), np.uint32)
    fn = lib().orc_antt128_limbwise if limbwise else lib().orc_antt128
    fn(x.reshape(-1), out.reshape(-1), log_h, log_rate)
    return out


def antt128_batch(x, log_h, log_rate):
    x = np.ascontiguousarray(x, dtype=np.uint32)
    batch = x.shape[0]
    out = np.zeros((batch, 1 << (log_h + log_rate), 4), np.uint32)
    lib().orc_antt128_limbwise_batch(x.reshape(-1), out.reshape(-1), log_h, log_rate, batch)
    return out


# ---------------- inputs / hashing ----------------
def mt_fill(seed, n):
    out = np.zeros(n, np.uint32)
    lib().orc_mt_fill(seed & 0xFFFFFFFF, out, n)
    return out


def fill128(seed0, seed64_base, n):
    out = np.zeros((n, 4), np.uint32)
    lib().orc_fill128(seed0 & 0xFFFFFFFF, seed64_base, out.reshape(-1), n)
    return out


def md5(arr):
    arr = np.ascontiguousarray(arr)
    d = np.zeros(16, np.uint8)
    lib().orc_md5(arr.ctypes.data, arr.nbytes, d)
    return d.tobytes().hex()


def md5_limb(v, limb):
    v = np.ascontiguousarray(v, dtype=np.uint32)
    d = np.zeros(16, np.uint8)
    lib().orc_md5_limb(v.reshape(-1), v.shape[0], limb, d)
    return d.tobytes().hex()


# ---------------- bitslicing ----------------
def bitslice128(blocks):
    b = np.array(blocks, dtype=np.uint32).reshape(-1).copy()
    lib().orc_bitslice_many128(b, b.size // 128, 0)
    return b


def unbitslice128(blocks):
    b = np.array(blocks, dtype=np.uint32).reshape(-1).copy()
    lib().orc_bitslice_many128(b, b.size // 128, 1)
    return b


# ---------------- sumcheck ----------------
def sumcheck_run(evals, n, d, bitsliced, challenges):
    evals = np.ascontiguousarray(evals, dtype=np.uint32).reshape(-1)
    ch = np.ascontiguousarray(challenges, dtype=np.uint32).reshape(-1)
    sums = np.zeros(4 * (n + 1), np.uint32)
    pts = np.zeros(4 * (d + 1) * (n + 1), np.uint32)
    lib().orc_sumcheck_run(evals, n, d, 1 if bitsliced else 0, ch, sums, pts)
    return sums.reshape(n + 1, 4), pts.reshape(n + 1, d + 1, 4)


def interpolate(points, challenge):
    p = np.ascontiguousarray(points, dtype=np.uint32).reshape(-1)
    out = np.zeros(4, np.uint32)
    lib().orc_sumcheck_interpolate(p, p.size // 4, np.ascontiguousarray(challenge, dtype=np.uint32), out)
    return out


def threads():
    """Host threads for the large-size checkers (the GPU box's CPU share is 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(cap) if cap.isdigit() and int(cap) > 0 else 16))


def multilinear_composition_fold(evals, n, d, bitsliced, challenges):
    """prod_j f_j(r) by folding (O(d 2^n) products, multithreaded); evals compact or bitsliced."""
    out = np.zeros(4, np.uint32)
    lib().orc_multilinear_composition_fold_mt(np.ascontiguousarray(evals, dtype=np.uint32).reshape(-1), n, d,
                                              1 if bitsliced else 0,
                                              np.ascontiguousarray(challenges, dtype=np.uint32).reshape(-1), out,
                                              threads())
    return out


def multilinear_composition(evals_compact, n, d, challenges):
    out = np.zeros(4, np.uint32)
    lib().orc_multilinear_composition(np.ascontiguousarray(evals_compact, dtype=np.uint32).reshape(-1), n, d,
                                      np.ascontiguousarray(challenges, dtype=np.uint32).reshape(-1), out)
    return out


BB31_P = 2013265921


def bb31_ntt(x, log_n, gen=137, log_group=27, bit_reversed=False):
    """BabyBear radix-2 NTT (reference NTT<BB31>::apply semantics, gpuntt.cuh:150-183)."""
    x = np.ascontiguousarray(x, dtype=np.uint32)
    out = np.empty(1 << log_n, dtype=np.uint32)
    lib().orc_bb31_ntt(x, out, log_n, gen, log_group, 1 if bit_reversed else 0)
    return out


M31_P = (1 << 31) - 1


def qm31(x):
    """QM31 value as 4 canonical words (lo.a, lo.b, hi.a, hi.b)."""
    return np.array([v % M31_P for v in x], dtype=np.uint32)


def qm31_mul(a, b):
    out = np.zeros(4, np.uint32)
    lib().orc_qm31_mul(qm31(a), qm31(b), out)
    return out


def qm31_interpolate(points, r):
    out = np.zeros(4, np.uint32)
    lib().orc_qm31_interpolate(np.ascontiguousarray(points, dtype=np.uint32).reshape(-1), qm31(r), out)
    return out


def qm31_sumcheck_run(evals, n, challenges):
    """evals: (2, 2^n, 4) uint32 (copied); challenges: (n, 4). Returns points (n, 3, 4)."""
    e = np.ascontiguousarray(evals, dtype=np.uint32).reshape(-1).copy()
    ch = np.ascontiguousarray(challenges, dtype=np.uint32).reshape(-1)
    pts = np.zeros(12 * n, np.uint32)
    lib().orc_qm31_sumcheck_run(e, n, ch, pts)
    return pts.reshape(n, 3, 4)
