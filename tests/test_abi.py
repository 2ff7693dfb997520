"""CPU: the C-ABI library loads, exports every symbol include/binius_ntt_amd.h declares, and
validates arguments without touching a GPU (no compute calls here)."""
import ctypes

import pytest

import binius_ntt_amd as B


def test_library_exports_every_declared_symbol():
    L = B.lib()
    names = B.exported_symbols()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n


def test_version_and_error_strings():
    L = B.lib()
    assert b"gfx950" in L.bn_version()
    assert isinstance(L.bn_last_error(), bytes)


@pytest.mark.parametrize("field,log_h,log_rate", [(64, 10, 0), (128, 0, 0), (32, 10, 5), (32, 30, 3)])
def test_plan_create_rejects_bad_parameters(field, log_h, log_rate):
    # AdditiveNTTConf asserts (nttconf.cuh:55-60): log_h >= 1, log_h+log_rate <= N_BITS, 0 <= log_rate <= 4
    p = ctypes.c_void_p()
    rc = B.lib().bn_antt_plan_create(0, field, log_h, log_rate, ctypes.byref(p))
    assert rc == B.BN_ERR_INVALID
    assert not p.value
    assert B.lib().bn_last_error()


def test_plan_create_unsupported_sizes():
    # GF(2^128) with log_h + log_rate > 32 is valid for the reference surface but not built here
    p = ctypes.c_void_p()
    assert B.lib().bn_antt_plan_create(0, 128, 31, 2, ctypes.byref(p)) == B.BN_ERR_UNSUPPORTED


def test_conf_mirror_raises_like_reference_asserts():
    with pytest.raises(ValueError):
        B.AdditiveNTTConf(0, 0)
    with pytest.raises(ValueError):
        B.AdditiveNTTConf(10, 5)
    with pytest.raises(ValueError):
        B.AdditiveNTTConf(30, 3, B.FanPaarTowerField(5))


def test_null_arguments_rejected():
    L = B.lib()
    assert L.bn_antt_forward_device(None, None, None, 1, None) == B.BN_ERR_INVALID
    assert L.bn_antt_plan_destroy(None) == B.BN_OK
    assert L.bn_sumcheck_destroy(None) == B.BN_OK
    assert L.bn_gf128_mul_device(None, None, None, 4, None) == B.BN_ERR_INVALID


def test_product_library_has_no_experiment_kernels():
    """Experiments measured and not kept live only in the development / experiment builds (BN_DEV,
    -DBN_SC_FUSED): the product library the driver loads carries none of their kernels."""
    with open(B.LIB_PATH, "rb") as f:
        blob = f.read()
    for name in (b"antt_bs_persist3", b"antt_rr_mid_pf", b"antt_rr_pass_persist", b"sc_fold_msgs"):
        assert name not in blob, name
