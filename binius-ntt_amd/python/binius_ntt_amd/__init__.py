"""Python mirror of the reference's ulvt_gpu / sumcheck library surface over the C-ABI.

The product is the C-ABI shared library (binius-ntt_amd/lib/libbinius_ntt_amd.so, declared in
include/binius_ntt_amd.h); this module binds it with ctypes and mirrors the reference's C++
classes so parity tests read like the reference's own:

  NTTData, DataOrder                  src/ulvt/ntt/nttconf.cuh:9-21
  AdditiveNTTConf(log_h, log_rate)    src/ulvt/ntt/nttconf.cuh:49-60
  AdditiveNTT(conf).apply(in, out)    src/ulvt/ntt/additive_ntt.cuh:175-265
  Sumcheck(num_vars, d, transposed)   src/ulvt/sumcheck/sumcheck.cuh:10-301
  check_gpu_capabilities()            src/ulvt/utils/common.cu:6-43

Device buffers are torch tensors (PyTorch-ROCm is only plumbing here: memory, streams,
torch.distributed). There is no CPU fallback: if the library is missing every call raises.
"""
import ctypes
import enum
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(os.path.dirname(_HERE))  # binius-ntt_amd/
LIB_PATH = os.environ.get("BINIUS_NTT_AMD_LIB") or os.path.join(PKG_ROOT, "lib", "libbinius_ntt_amd.so")  # env: A/B experiments
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "binius_ntt_amd.h")

BN_OK, BN_ERR_INVALID, BN_ERR_HIP, BN_ERR_UNSUPPORTED, BN_ERR_ALLOC = 0, 1, 2, 3, 4
_ERRNAMES = {1: "BN_ERR_INVALID", 2: "BN_ERR_HIP", 3: "BN_ERR_UNSUPPORTED", 4: "BN_ERR_ALLOC"}

_lib = None


class BnError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (_ERRNAMES.get(code, code), msg))
        self.code = code


def lib():
    """Load the HIP engine. Raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libbinius_ntt_amd.so not built (run `make -C binius-ntt_amd` or __graft_entry__.build())")
    # One HIP runtime per process: torch bundles its own libamdhip64 with the same SONAME as
    # ROCm's. If this library were loaded first it would pull in ROCm's copy and torch (which
    # this package uses for device buffers and streams) would then find no GPU. Import torch
    # first so that its runtime is the one both share.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i32, u32p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)
    sig = {
        "bn_last_error": (ctypes.c_char_p, []),
        "bn_version": (ctypes.c_char_p, []),
        "bn_check_gpu_capabilities": (i32, []),
        "bn_antt_plan_create": (i32, [i32, i32, i32, i32, ctypes.POINTER(vp)]),
        "bn_antt_plan_destroy": (i32, [vp]),
        "bn_antt_forward_host": (i32, [vp, vp, sz, vp]),
        "bn_antt_forward_device": (i32, [vp, vp, vp, sz, vp]),
        "bn_antt_get_subspace_evals": (i32, [vp, u32p, sz]),
        "bn_antt_plan_query": (i32, [vp, i32, ctypes.POINTER(ctypes.c_int64)]),
        "bn_antt_plan_set_variant": (i32, [vp, i32]),
        "bn_antt_set_event_timing": (i32, [vp, i32]),
        "bn_antt_get_event_timing": (i32, [vp, ctypes.POINTER(ctypes.c_float), i32, ctypes.POINTER(i32)]),
        "bn_antt_time_passes": (i32, [vp, vp, vp, sz, i32, vp, ctypes.POINTER(ctypes.c_float), i32, ctypes.POINTER(i32)]),
        "bn_antt_pass_kernel_name": (i32, [vp, i32, ctypes.c_char_p, sz]),
        "bn_gf128_mul_device": (i32, [vp, vp, vp, sz, vp]),
        "bn_gf128_mul_bitsliced_device": (i32, [vp, vp, vp, sz, vp]),
        "bn_gf32_mul_device": (i32, [vp, vp, vp, sz, vp]),
        "bn_gf128_mul_repeat_device": (i32, [i32, vp, vp, sz, i32, vp]),
        "bn_bitslice_device": (i32, [vp, sz, i32, vp]),
        "bn_multiply_unrolled": (i32, [i32, u32p, u32p, u32p]),
        "bn_multiply_unrolled_device": (i32, [i32, vp, vp, vp, sz, vp]),
        "bn_mul_binary_tower_32b_simd": (i32, [i32, ctypes.c_uint32, ctypes.c_uint32, u32p]),
        "bn_interleave_32b": (i32, [i32, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p]),
        "bn_xor_adjacent_32b": (i32, [i32, ctypes.c_uint32, u32p]),
        "bn_packed32_device": (i32, [i32, i32, vp, vp, vp, vp, sz, vp]),
        "bn_sumcheck_create": (i32, [i32, i32, i32, i32, u32p, ctypes.POINTER(vp)]),
        "bn_sumcheck_create_device": (i32, [i32, i32, i32, i32, vp, i32, ctypes.POINTER(vp)]),
        "bn_sumcheck_create_staged": (i32, [i32, i32, i32, i32, u32p, ctypes.POINTER(vp)]),
        "bn_sumcheck_prepare": (i32, [vp]),
        "bn_sumcheck_round_messages": (i32, [vp, u32p, u32p]),
        "bn_sumcheck_move_to_next_round": (i32, [vp, u32p]),
        "bn_sumcheck_round": (i32, [vp, ctypes.POINTER(i32)]),
        "bn_sumcheck_set_shard": (i32, [vp, i32, i32]),
        "bn_sumcheck_create_shard_device": (i32, [i32, i32, i32, i32, i32, vp, vp, ctypes.POINTER(vp)]),
        "bn_sumcheck_needs_gather": (i32, [vp, ctypes.POINTER(i32)]),
        "bn_sumcheck_set_message_sink": (i32, [vp, vp]),
        "bn_sumcheck_round_messages_sink": (i32, [vp]),
        "bn_sumcheck_stream": (i32, [vp, ctypes.POINTER(vp)]),
        "bn_sumcheck_export_shard": (i32, [vp, u32p, sz]),
        "bn_sumcheck_import_gathered": (i32, [vp, u32p, sz, i32]),
        "bn_sumcheck_destroy": (i32, [vp]),
        "bn_multilinear_composition_eval": (i32, [i32, i32, i32, i32, u32p, u32p, u32p]),
        "bn_multilinear_composition_eval_device": (i32, [i32, i32, i32, i32, vp, u32p, u32p]),
        "bn_sumcheck_interpolate": (i32, [u32p, i32, u32p, u32p]),
        "bn_bb31_ntt_plan_create": (i32, [i32, ctypes.c_uint32, i32, i32, ctypes.POINTER(vp)]),
        "bn_bb31_ntt_plan_destroy": (i32, [vp]),
        "bn_bb31_ntt_forward_host": (i32, [vp, vp, sz, vp, i32]),
        "bn_bb31_ntt_forward_device": (i32, [vp, vp, vp, sz, i32, vp]),
        "bn_qm31_sumcheck_create": (i32, [i32, i32, u32p, ctypes.POINTER(vp)]),
        "bn_qm31_sumcheck_round_messages": (i32, [vp, u32p]),
        "bn_qm31_sumcheck_fold": (i32, [vp, u32p]),
        "bn_qm31_sumcheck_final_values": (i32, [vp, u32p]),
        "bn_qm31_sumcheck_destroy": (i32, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc):
    if rc != BN_OK:
        raise BnError(rc, lib().bn_last_error().decode())


def exported_symbols():
    """Names declared in include/binius_ntt_amd.h (used by the ABI test)."""
    import re
    with open(HEADER_PATH) as f:
        src = f.read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(bn_\w+)\s*\(", src, re.M)))


def check_gpu_capabilities():
    return bool(lib().bn_check_gpu_capabilities())


def _check_device_tensor(t, words, what):
    """Shape/device/contiguity check before handing a raw pointer to the C-ABI: a short or
    strided tensor would otherwise mean out-of-bounds device accesses."""
    if isinstance(t, int):
        return
    if not t.is_cuda:
        raise ValueError("%s must be a device tensor" % what)
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % what)
    if t.element_size() * t.numel() < 4 * words:
        raise ValueError("%s holds %d bytes, need %d" % (what, t.element_size() * t.numel(), 4 * words))


def _ptr(t):
    """Device pointer of a torch tensor (or an int address)."""
    if isinstance(t, int):
        return ctypes.c_void_p(t)
    return ctypes.c_void_p(t.data_ptr())


def _stream(stream, device=None):
    """hipStream_t for a launch: `stream` (torch stream or raw handle) or, when None, torch's
    current stream of `device` (the plan's device, not whichever device is current)."""
    if stream is None:
        import torch
        dev = torch.device("cuda", device) if device is not None else None
        return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


# ------------------------------------------------------------------ NTT data / config
class DataOrder(enum.IntEnum):
    """nttconf.cuh:9"""
    INVALID = -1
    IN_ORDER = 0
    BIT_REVERSED = 1


class NTTData:
    """Host-owned buffer (nttconf.cuh:11-21). `data` is a numpy array of `size` elements:
    uint32 for GF(2^32), shape (size, 4) uint32 limbs for GF(2^128)."""

    def __init__(self, size, order=DataOrder.INVALID, field_bits=32, data=None):
        self.order = DataOrder(order)
        self.size = int(size)
        self.field_bits = field_bits
        if data is not None:
            self.data = np.ascontiguousarray(data, dtype=np.uint32)
        elif field_bits == 32:
            self.data = np.zeros(self.size, np.uint32)
        else:
            self.data = np.zeros((self.size, field_bits // 32), np.uint32)

    def byte_len(self):
        return self.data.nbytes


class FanPaarTowerField:
    """Field policy tag (binary_tower.cuh:111-128): height 5 = GF(2^32), height 7 = GF(2^128)."""

    def __init__(self, height):
        assert height in (5, 7), "the NTT is built for GF(2^32) and GF(2^128)"
        self.height = height

    def N_BITS(self):
        return 1 << self.height


class AdditiveNTTConf:
    """nttconf.cuh:49-60; the reference ASSERTs (aborts) on bad parameters, this raises."""

    def __init__(self, log_h, log_rate, field=FanPaarTowerField(5), device=0):
        if not log_h >= 1:
            raise ValueError("log_h must be >= 1")
        if not (0 <= log_rate <= 4):
            raise ValueError("log_rate must be in [0, 4]")
        if not log_h + log_rate <= field.N_BITS():
            raise ValueError("log_h + log_rate must be <= N_BITS")
        self.log_h, self.log_rate, self.field, self.device = log_h, log_rate, field, device


class AdditiveNTT:
    """additive_ntt.cuh:175-319 over the C-ABI plan."""

    def __init__(self, conf):
        self.conf = conf
        self.field_bits = conf.field.N_BITS()
        p = ctypes.c_void_p()
        _check(lib().bn_antt_plan_create(conf.device, self.field_bits, conf.log_h, conf.log_rate, ctypes.byref(p)))
        self._plan = p

    def close(self):
        if getattr(self, "_plan", None) is not None and self._plan.value:
            lib().bn_antt_plan_destroy(self._plan)
            self._plan = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def limbs(self):
        return self.field_bits // 32

    def apply(self, inp, out):
        """Reference semantics (additive_ntt.cuh:201-265): False (no other effect) unless
        inp.size == 2^log_h and inp.order == IN_ORDER; fills out (coset-major) synchronously."""
        n = 1 << self.conf.log_h
        if inp.size != n or inp.order != DataOrder.IN_ORDER:
            return False
        src = np.ascontiguousarray(inp.data, dtype=np.uint32)
        assert src.size == n * self.limbs
        n_out = n << self.conf.log_rate
        if out.data.size != n_out * self.limbs:
            out.data = np.zeros((n_out,) if self.limbs == 1 else (n_out, self.limbs), np.uint32)
            out.size = n_out
        dst = out.data
        _check(lib().bn_antt_forward_host(self._plan, src.ctypes.data, n, dst.ctypes.data))
        out.order = DataOrder.IN_ORDER
        return True

    def forward_device(self, d_in, d_out, batch=1, stream=None):
        """Device-resident transform(s) on torch tensors (or raw addresses); async on `stream`
        (default: torch's current stream of the plan's device)."""
        n = (1 << self.conf.log_h) * self.limbs * batch
        _check_device_tensor(d_in, n, "d_in")
        _check_device_tensor(d_out, n << self.conf.log_rate, "d_out")
        _check(lib().bn_antt_forward_device(self._plan, _ptr(d_in), _ptr(d_out), batch,
                                            _stream(stream, self.conf.device)))

    def subspace_evals(self):
        lh, w = self.conf.log_h, self.conf.log_h + self.conf.log_rate - 1
        out = np.zeros(max(1, lh * w), np.uint32)
        _check(lib().bn_antt_get_subspace_evals(self._plan, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), out.size))
        return out[: lh * w].reshape(lh, w)

    def variant(self):
        v = ctypes.c_int64()
        _check(lib().bn_antt_plan_query(self._plan, 4, ctypes.byref(v)))
        return v.value

    def set_variant(self, variant):
        """0: compact tiles, per-butterfly twiddles (default for log_h < 12); 1: bitsliced LDS tiles;
        4: bitsliced register tiles (three to four waves per SIMD) on every pass; 5: register tiles
        for the GF(2^8)-twiddle passes, LDS tiles for the others (default for log_h >= 12).
        Variants 1, 4 and 5 need log_h >= 12; results are identical."""
        _check(lib().bn_antt_plan_set_variant(self._plan, variant))

    def set_event_timing(self, enable):
        _check(lib().bn_antt_set_event_timing(self._plan, 1 if enable else 0))

    def pass_kernel_name(self, i):
        """Demangled name of the kernel pass i launches (bn_antt_pass_kernel_name)."""
        buf = ctypes.create_string_buffer(512)
        _check(lib().bn_antt_pass_kernel_name(self._plan, i, buf, 512))
        return buf.value.decode()

    def time_passes(self, d_in, d_out, reps=10, batch=1, stream=None):
        """Steady-state ms per launch of each pass (bn_antt_time_passes); d_out is scratch."""
        n = (1 << self.conf.log_h) * self.limbs * batch
        _check_device_tensor(d_in, n, "d_in")
        _check_device_tensor(d_out, n << self.conf.log_rate, "d_out")
        arr = (ctypes.c_float * 16)()
        k = ctypes.c_int()
        _check(lib().bn_antt_time_passes(self._plan, _ptr(d_in), _ptr(d_out), batch, reps,
                                         _stream(stream, self.conf.device), arr, 16, ctypes.byref(k)))
        return [arr[i] for i in range(min(k.value, 16))]

    def event_timing(self):
        arr = (ctypes.c_float * 16)()
        n = ctypes.c_int()
        _check(lib().bn_antt_get_event_timing(self._plan, arr, 16, ctypes.byref(n)))
        return [arr[i] for i in range(min(n.value, 16))]


# ------------------------------------------------------------------ BabyBear NTT (prime-field sibling)
class BB31:
    """risc0::Fp value (src/ulvt/finite_fields/risc0_baby_bear.h:40-190), canonical int view:
    BB31(r) == r mod p, asUInt32() returns the canonical value."""
    P = 15 * (1 << 27) + 1

    def __init__(self, v=0):
        self.v = int(v) % self.P

    def asUInt32(self):
        return self.v

    def __mul__(self, o):
        return BB31(self.v * o.v)

    def __add__(self, o):
        return BB31(self.v + o.v)

    def __sub__(self, o):
        return BB31(self.v - o.v)

    def __eq__(self, o):
        return isinstance(o, BB31) and self.v == o.v

    @staticmethod
    def pow(x, n):
        return BB31(pow(x.v, int(n), BB31.P))

    @staticmethod
    def inv(x):
        return BB31(pow(x.v, BB31.P - 2, BB31.P))

    @staticmethod
    def one():
        return BB31(1)


class NTTConfRad2:
    """nttconf.cuh:25-47; the reference ASSERTs on bad parameters, this raises."""

    def __init__(self, generator, log_group_order, log_inp_size, device=0):
        if not 1 <= log_inp_size <= 27:
            raise ValueError("log_inp_size must be in [1, 27]")
        if not log_group_order >= log_inp_size:
            raise ValueError("log_group_order must be >= log_inp_size")
        self.generator = generator if isinstance(generator, BB31) else BB31(generator)
        self.log_group_order, self.log_inp_size, self.device = log_group_order, log_inp_size, device


class NTT:
    """NTT<BB31> (gpuntt.cuh:126-209) over the C-ABI plan: natural-order DFT with
    w = generator^(2^(log_group_order - log_inp_size))."""

    def __init__(self, conf):
        self.conf = conf
        p = ctypes.c_void_p()
        _check(lib().bn_bb31_ntt_plan_create(conf.device, conf.generator.v, conf.log_group_order,
                                             conf.log_inp_size, ctypes.byref(p)))
        self._plan = p

    def close(self):
        if getattr(self, "_plan", None) is not None and self._plan.value:
            lib().bn_bb31_ntt_plan_destroy(self._plan)
            self._plan = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def apply(self, inp, out):
        """Reference semantics: input of 2^log_inp_size canonical words, IN_ORDER or
        BIT_REVERSED; output in order (raises where the reference ASSERTs)."""
        n = 1 << self.conf.log_inp_size
        if inp.size != n:
            raise ValueError("input has %d elements, plan expects %d" % (inp.size, n))
        src = np.ascontiguousarray(inp.data, dtype=np.uint32)
        if out.data.size != n:
            out.data = np.zeros(n, np.uint32)
            out.size = n
        br = 1 if inp.order == DataOrder.BIT_REVERSED else 0
        _check(lib().bn_bb31_ntt_forward_host(self._plan, src.ctypes.data, n, out.data.ctypes.data, br))
        out.order = DataOrder.IN_ORDER

    def forward_device(self, d_in, d_out, batch=1, bit_reversed=False, stream=None):
        _check(lib().bn_bb31_ntt_forward_device(self._plan, _ptr(d_in), _ptr(d_out), batch,
                                                1 if bit_reversed else 0, _stream(stream, self.conf.device)))


# ------------------------------------------------------------------ field / bitslicing
def _dev_index(t):
    return None if isinstance(t, int) else t.device.index


def _same_size(what, *ts):
    sizes = {t.numel() * t.element_size() for t in ts if not isinstance(t, int)}
    if len(sizes) > 1:
        raise ValueError("%s operands differ in size: %s" % (what, sorted(sizes)))


def gf128_mul(a, b, out, stream=None):
    _same_size("gf128_mul", a, b, out)
    for t, w in ((a, "a"), (b, "b"), (out, "out")):
        _check_device_tensor(t, a.numel(), w)
    _check(lib().bn_gf128_mul_device(_ptr(a), _ptr(b), _ptr(out), a.numel() // 4, _stream(stream, _dev_index(a))))


def gf32_mul(a, b, out, stream=None):
    _same_size("gf32_mul", a, b, out)
    for t, w in ((a, "a"), (b, "b"), (out, "out")):
        _check_device_tensor(t, a.numel(), w)
    _check(lib().bn_gf32_mul_device(_ptr(a), _ptr(b), _ptr(out), a.numel(), _stream(stream, _dev_index(a))))


def gf128_mul_bitsliced(a, b, out, stream=None):
    _same_size("gf128_mul_bitsliced", a, b, out)
    for t, w in ((a, "a"), (b, "b"), (out, "out")):
        _check_device_tensor(t, a.numel(), w)
    _check(lib().bn_gf128_mul_bitsliced_device(_ptr(a), _ptr(b), _ptr(out), a.numel() // 128,
                                               _stream(stream, _dev_index(a))))


def gf128_mul_repeat(kind, state, operand, threads, iters, stream=None):
    _check(lib().bn_gf128_mul_repeat_device(kind, _ptr(state), _ptr(operand), threads, iters,
                                            _stream(stream, _dev_index(state))))


def bitslice(buf, untranspose=False, stream=None):
    _check_device_tensor(buf, buf.numel(), "buf")
    _check(lib().bn_bitslice_device(_ptr(buf), buf.numel() // 128, 1 if untranspose else 0,
                                    _stream(stream, _dev_index(buf))))


def multiply_unrolled(height, a, b, dst=None):
    """multiply_unrolled<HEIGHT> (binary_tower_unrolled.cuh:4-5) on host arrays of 2^height
    words (32 bitsliced products); dst may be a (alias-safe). Returns dst."""
    w = 1 << height
    a = np.ascontiguousarray(a, dtype=np.uint32)
    b = np.ascontiguousarray(b, dtype=np.uint32)
    if a.size != w or b.size != w:
        raise ValueError("operands must hold 2^height = %d words" % w)
    if dst is None:
        dst = np.zeros(w, np.uint32)
    _check(lib().bn_multiply_unrolled(height, _u32p(a), _u32p(b), _u32p(dst)))
    return dst


def multiply_unrolled_device(height, a, b, out, stream=None):
    """Device batch of multiply_unrolled<height> over consecutive 2^height-word blocks."""
    _same_size("multiply_unrolled_device", a, b, out)
    w = 1 << height
    for t, nm in ((a, "a"), (b, "b"), (out, "out")):
        _check_device_tensor(t, a.numel(), nm)
    _check(lib().bn_multiply_unrolled_device(height, _ptr(a), _ptr(b), _ptr(out), a.numel() // w,
                                             _stream(stream, _dev_index(a))))


def mul_binary_tower_32b_simd(height, a, b):
    """mul_binary_tower_32b_simd<HEIGHT>(a, b) (binary_tower_simd.cuh:77-127)."""
    out = ctypes.c_uint32()
    _check(lib().bn_mul_binary_tower_32b_simd(height, a, b, ctypes.byref(out)))
    return out.value


def interleave_32b(height, a, b):
    """interleave_32b<HEIGHT>(a, b) -> (c, d) (binary_tower_simd.cuh:129-139)."""
    c, d = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib().bn_interleave_32b(height, a, b, ctypes.byref(c), ctypes.byref(d)))
    return c.value, d.value


def xor_adjacent_32b(height, a):
    """xor_adjacent_32b<HEIGHT>(a) (binary_tower_simd.cuh:141-150)."""
    out = ctypes.c_uint32()
    _check(lib().bn_xor_adjacent_32b(height, a, ctypes.byref(out)))
    return out.value


def packed32_device(op, height, a, b=None, c=None, d=None, stream=None):
    """Device batch of the packed-word primitives: op 0 multiply, 1 interleave, 2 xor_adjacent."""
    n = a.numel()
    for t, nm in ((a, "a"), (b, "b"), (c, "c"), (d, "d")):
        if t is not None:
            _check_device_tensor(t, n, nm)
    _check(lib().bn_packed32_device(op, height, _ptr(a), _ptr(b) if b is not None else None,
                                    _ptr(c), _ptr(d) if d is not None else None, n, _stream(stream, _dev_index(a))))


# ------------------------------------------------------------------ sumcheck
class Sumcheck:
    """Sumcheck<NUM_VARS, COMPOSITION_SIZE, DATA_IS_TRANSPOSED> (sumcheck.cuh:10-301)."""

    def __init__(self, num_vars, composition_size, data_is_transposed, evals, device=0, shard=None, staged=False):
        """staged=True (host evals only): copy the columns but leave compact input untransposed until
        prepare() (or the first round) — the reference constructor's separate Memcpy and Transpose
        phases (sumcheck.cuh:88-124)."""
        self.num_vars, self.d, self.device = num_vars, composition_size, device
        p = ctypes.c_void_p()
        if isinstance(evals, np.ndarray):
            ev = np.ascontiguousarray(evals, dtype=np.uint32).reshape(-1)
            create = lib().bn_sumcheck_create_staged if staged else lib().bn_sumcheck_create
            _check(create(device, num_vars, composition_size, 1 if data_is_transposed else 0,
                          ev.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(p)))
        else:
            _check_device_tensor(evals, composition_size * 4 << num_vars, "evals")
            # the library copies on its own stream: the producer (an NTT, a torch kernel) must be done.
            # A raw device address (int) carries no stream: the caller must have synchronised it.
            if not isinstance(evals, int):
                import torch
                torch.cuda.current_stream(evals.device).synchronize()
            _check(lib().bn_sumcheck_create_device(device, num_vars, composition_size,
                                                   1 if data_is_transposed else 0, _ptr(evals), 0, ctypes.byref(p)))
        self._sc = p
        self._bind()
        if shard is not None:
            _check(lib().bn_sumcheck_set_shard(self._sc, shard[0], shard[1]))

    def prepare(self):
        """The device bit-transpose of a staged prover's compact columns (synchronous; no-op otherwise)."""
        _check(lib().bn_sumcheck_prepare(self._sc))

    def _bind(self):
        # per-round calls are on the protocol's critical path (the GPU waits for the host's
        # challenge): resolve the entry points and the output buffers' pointers once
        L, u32p = lib(), ctypes.POINTER(ctypes.c_uint32)
        self._f_msgs, self._f_next = L.bn_sumcheck_round_messages, L.bn_sumcheck_move_to_next_round
        self._sum_buf = np.zeros(4, np.uint32)
        self._pts_buf = np.zeros(4 * (self.d + 1), np.uint32)
        self._ch_buf = np.zeros(4, np.uint32)
        self._sum_p, self._pts_p, self._ch_p = (b.ctypes.data_as(u32p) for b in (self._sum_buf, self._pts_buf, self._ch_buf))

    @classmethod
    def from_shard(cls, num_vars, composition_size, local_evals, rank, world, device=None, stream=None):
        """Shard prover from this rank's share only (bn_sumcheck_create_shard_device): local_evals
        is a device tensor of composition_size * 4 * 2^num_vars / world words (bitsliced batches
        b with b mod world == rank, in order); the copy is ordered after `stream`. The prover runs
        on local_evals' device (`device`, if given, must name the same one)."""
        _check_device_tensor(local_evals, composition_size * (4 << num_vars) // world, "local_evals")
        if not isinstance(local_evals, int):
            if device is None:
                device = local_evals.device.index
            elif device != local_evals.device.index:
                raise ValueError("device %d does not hold local_evals (cuda:%d)" % (device, local_evals.device.index))
        elif device is None:
            device = 0
        self = cls.__new__(cls)
        self.num_vars, self.d, self.device = num_vars, composition_size, device
        p = ctypes.c_void_p()
        _check(lib().bn_sumcheck_create_shard_device(device, num_vars, composition_size, rank, world,
                                                     _ptr(local_evals), _stream(stream, local_evals.device.index),
                                                     ctypes.byref(p)))
        self._sc = p
        self._bind()
        return self

    def this_round_messages(self):
        rc = self._f_msgs(self._sc, self._sum_p, self._pts_p)
        if rc != BN_OK:
            _check(rc)
        return self._sum_buf.copy(), self._pts_buf.reshape(self.d + 1, 4).copy()

    def move_to_next_round(self, challenge):
        self._ch_buf[:] = np.asarray(challenge, dtype=np.uint32).reshape(4)
        rc = self._f_next(self._sc, self._ch_p)
        if rc != BN_OK:
            _check(rc)

    def round(self):
        r = ctypes.c_int()
        _check(lib().bn_sumcheck_round(self._sc, ctypes.byref(r)))
        return r.value

    # sharded endgame (see bn_sumcheck_needs_gather); driven by binius_ntt_amd.distributed
    def set_message_sink(self, words):
        """bn_sumcheck_set_message_sink: later messages kernels also write the raw point words (and
        the p(1)-skipped flag at word 36) into `words`, a device tensor of >= 37 int32 (None: stop)."""
        if words is None:
            _check(lib().bn_sumcheck_set_message_sink(self._sc, None))
            self._sink = None
            return
        _check_device_tensor(words, 4 * (8 + 1) + 1, "message sink")
        self._sink = words  # keep the buffer alive while the prover writes it
        _check(lib().bn_sumcheck_set_message_sink(self._sc, _ptr(words)))

    def round_messages_sink(self):
        """bn_sumcheck_round_messages_sink: the round's messages kernel is queued (no wait); its raw
        points land in the sink on stream_handle()'s stream."""
        _check(lib().bn_sumcheck_round_messages_sink(self._sc))

    def stream_handle(self):
        """The prover's hipStream_t (as an int), for torch.cuda.ExternalStream."""
        s = ctypes.c_void_p()
        _check(lib().bn_sumcheck_stream(self._sc, ctypes.byref(s)))
        return s.value or 0

    def needs_gather(self):
        f = ctypes.c_int()
        _check(lib().bn_sumcheck_needs_gather(self._sc, ctypes.byref(f)))
        return bool(f.value)

    def export_shard(self):
        out = np.zeros(128 * self.d, np.uint32)
        _check(lib().bn_sumcheck_export_shard(self._sc, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), out.size))
        return out

    def import_gathered(self, words, world):
        w = np.ascontiguousarray(words, dtype=np.uint32).reshape(-1)
        _check(lib().bn_sumcheck_import_gathered(self._sc, w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), w.size,
                                                 world))

    def close(self):
        if getattr(self, "_sc", None) is not None and self._sc.value:
            lib().bn_sumcheck_destroy(self._sc)
            self._sc = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _u32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def evaluate_multilinear_composition(evals, num_vars, composition_size, data_is_transposed, challenges, device=0):
    """evaluate_multilinear_composition (src/ulvt/sumcheck/test/verifier.cu:88-107) on the GPU:
    prod_j f_j(r) for the columns in `evals` (numpy host array or torch device tensor)."""
    ch = np.ascontiguousarray(challenges, dtype=np.uint32).reshape(-1)
    out = np.zeros(4, np.uint32)
    if isinstance(evals, np.ndarray):
        ev = np.ascontiguousarray(evals, dtype=np.uint32).reshape(-1)
        _check(lib().bn_multilinear_composition_eval(device, num_vars, composition_size, 1 if data_is_transposed else 0,
                                                     _u32p(ev), _u32p(ch), _u32p(out)))
    else:
        _check(lib().bn_multilinear_composition_eval_device(device, num_vars, composition_size,
                                                            1 if data_is_transposed else 0, _ptr(evals), _u32p(ch),
                                                            _u32p(out)))
    return out


def evaluate_univariate_given_points(challenge, points):
    """evaluate_univariate_given_points (verifier.cu:9-31): Lagrange interpolation through
    (k, points[k]) evaluated at `challenge` (4-word GF(2^128) values)."""
    p = np.ascontiguousarray(points, dtype=np.uint32).reshape(-1)
    c = np.ascontiguousarray(challenge, dtype=np.uint32).reshape(4)
    out = np.zeros(4, np.uint32)
    _check(lib().bn_sumcheck_interpolate(_u32p(p), p.size // 4, _u32p(c), _u32p(out)))
    return out
