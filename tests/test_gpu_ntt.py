"""GPU parity for the additive NTT: HIP path (through the C-ABI) vs the oracle and the
reference's own golden MD5 table (src/ulvt/ntt/tests/test_ntt.cu:52-124, 191-234)."""
import numpy as np
import pytest

import _oracle as O
import binius_ntt_amd as B

pytestmark = pytest.mark.gpu


def _run_device(ntt, x_np, dev, batch=1):
    import torch
    x = torch.from_numpy(x_np.astype(np.uint32).view(np.int32)).to(dev)
    n_out = x_np.size << ntt.conf.log_rate
    y = torch.empty(n_out, dtype=torch.int32, device=dev)
    ntt.forward_device(x, y, batch=batch)
    torch.cuda.synchronize()
    return y.cpu().numpy().view(np.uint32)


def test_capabilities():
    assert B.check_gpu_capabilities(), B.lib().bn_last_error()


@pytest.mark.parametrize("log_h", list(range(1, 25)) + [pytest.param(h, marks=pytest.mark.slow) for h in range(25, 31)])
def test_gf32_r0_reference_md5(ntt_md5, log_h, dev):
    # exactly the reference's run_and_check_additive_ntt(log_h, 0) (test_ntt.cu:191-217): the
    # default range 1-28 and its [slow] cases 29 and 30 (test_ntt.cu:231-234)
    x = O.mt_fill(0xDEADBEEF + log_h, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(5)))
    inp = B.NTTData(1 << log_h, B.DataOrder.IN_ORDER, 32, x)
    out = B.NTTData(1 << log_h, field_bits=32)
    assert ntt.apply(inp, out)
    assert out.order == B.DataOrder.IN_ORDER
    assert O.md5(out.data) == ntt_md5["0"][log_h]


@pytest.mark.parametrize("log_h", list(range(1, 23)) + [pytest.param(h, marks=pytest.mark.slow) for h in range(23, 28)])
def test_gf32_r2_reference_md5(ntt_md5, log_h, dev):
    x = O.mt_fill(0xDEADBEEF + log_h + 2, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 2, B.FanPaarTowerField(5)))
    y = _run_device(ntt, x, dev)
    assert O.md5(y) == ntt_md5["2"][log_h]


@pytest.mark.parametrize("log_h,r", [(1, 0), (2, 1), (3, 0), (5, 2), (8, 0), (10, 0), (10, 2), (11, 1),
                                     (12, 3), (13, 0), (14, 4), (16, 0), (17, 2), (20, 0)])
def test_gf128_matches_oracle(log_h, r, dev):
    # independent random limbs (equal limbs would hide limb-swap bugs)
    x = O.fill128(0xDEADBEEF + log_h + r, 0x5EED0000, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, r, B.FanPaarTowerField(7)))
    y = _run_device(ntt, x.reshape(-1), dev).reshape(-1, 4)
    assert np.array_equal(y, O.antt128(x, log_h, r))


def test_gf128_apply_host_semantics(dev):
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(10, 1, B.FanPaarTowerField(7)))
    x = O.fill128(1, 2, 1 << 10)
    bad = B.NTTData(1 << 9, B.DataOrder.IN_ORDER, 128)
    out = B.NTTData(1 << 11, field_bits=128)
    assert not ntt.apply(bad, out)  # wrong size -> False, no other effect
    wrong_order = B.NTTData(1 << 10, B.DataOrder.BIT_REVERSED, 128, x)
    assert not ntt.apply(wrong_order, out)
    good = B.NTTData(1 << 10, B.DataOrder.IN_ORDER, 128, x)
    assert ntt.apply(good, out)
    assert np.array_equal(out.data, O.antt128(x, 10, 1))


def test_gf128_batched(dev):
    log_h, batch = 12, 5
    xs = np.stack([O.fill128(100 + b, 200 + b, 1 << log_h) for b in range(batch)])
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(7)))
    y = _run_device(ntt, xs.reshape(-1), dev, batch=batch).reshape(batch, -1, 4)
    assert np.array_equal(y, O.antt128_batch(xs, log_h, 0))


@pytest.mark.parametrize("log_h,r,batch", [(20, 2, 2), (21, 1, 1), (19, 3, 3)])
def test_gf128_cosets_at_full_launches(log_h, r, batch, dev):
    # coset bits on launches of many tiles per CU (the LDS-tile passes with their coset twiddle
    # tables, L = 4 limbs); the smaller (log_h, r) cases above run the small-launch kernels
    xs = np.stack([O.fill128(300 + 7 * b + r, 400 + b, 1 << log_h) for b in range(batch)])
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, r, B.FanPaarTowerField(7)))
    y = _run_device(ntt, xs.reshape(-1), dev, batch=batch).reshape(batch, -1, 4)
    assert np.array_equal(y, O.antt128_batch(xs, log_h, r))


@pytest.mark.slow
def test_gf128_north_star_size_limb_md5_and_oracle(ntt_md5, dev):
    # 2^24: limb 0 = the reference's mt19937 stream (MD5-pinned by the reference table),
    # limbs 1..3 = independent mt19937_64 streams (checked against the oracle).
    log_h = 24
    x = O.fill128(0xDEADBEEF + log_h, 0x5EED0000, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(7)))
    y = _run_device(ntt, x.reshape(-1), dev).reshape(-1, 4)
    assert O.md5_limb(y, 0) == ntt_md5["0"][log_h]
    assert np.array_equal(y, O.antt128(x, log_h, 0))


@pytest.mark.slow
def test_c5_batched_256x2p20_at_size(ntt_md5, dev):
    # BASELINE.json configs[4], one GPU's whole batch in ONE forward_device call: 256 x 2^20
    # GF(2^128) transforms (4 GiB in, 4 GiB out). Limb 0 of every transform is the reference's
    # mt19937(0xdeadbeef + 20) stream, so every output limb-0 plane must hash to
    # additive_ntt_hashes[0][20] (test_ntt.cu:52-124, 191-217); limbs 1..3 are independent random
    # words per transform, and transforms 0, 127 and 255 are checked in full against the oracle.
    import hashlib
    import torch
    log_h, batch = 20, 256
    n = 1 << log_h
    limb0 = torch.from_numpy(O.mt_fill(0xDEADBEEF + log_h, n).view(np.int32)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0xC5)
    x = torch.randint(-2**31, 2**31 - 1, (batch, n, 4), dtype=torch.int32, device=dev, generator=g)
    x[:, :, 0] = limb0
    y = torch.empty_like(x)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(7)))
    ntt.forward_device(x.view(-1), y.view(-1), batch=batch)
    torch.cuda.synchronize()
    want_md5 = ntt_md5["0"][log_h]
    planes = y[:, :, 0].contiguous().cpu().numpy().view(np.uint32)
    bad = [b for b in range(batch) if hashlib.md5(planes[b].tobytes()).hexdigest() != want_md5]
    assert not bad, "limb-0 MD5 differs from the reference table for transforms %s" % bad[:16]
    del planes
    for b in (0, 127, 255):
        xb = x[b].cpu().numpy().view(np.uint32)
        want = np.zeros_like(xb)
        O.lib().orc_antt128_limbwise_mt(xb.reshape(-1), want.reshape(-1), log_h, 0, O.threads())
        assert np.array_equal(y[b].cpu().numpy().view(np.uint32), want), "transform %d differs from the oracle" % b


def test_gf128_linearity_at_2_20(dev):
    # size-independent property: NTT(a ^ b) == NTT(a) ^ NTT(b)
    log_h = 20
    a = O.fill128(5, 6, 1 << log_h)
    b = O.fill128(7, 8, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(7)))
    ya = _run_device(ntt, a.reshape(-1), dev)
    yb = _run_device(ntt, b.reshape(-1), dev)
    yab = _run_device(ntt, (a ^ b).reshape(-1), dev)
    assert np.array_equal(ya ^ yb, yab)


@pytest.mark.slow
def test_gf128_2p26_limb_md5_and_oracle(ntt_md5, dev):
    # above the north-star size: limb 0 MD5-pinned by the reference table, all limbs vs the
    # (multithreaded) oracle
    log_h = 26
    x = O.fill128(0xDEADBEEF + log_h, 0x5EED0000, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(7)))
    y = _run_device(ntt, x.reshape(-1), dev).reshape(-1, 4)
    assert O.md5_limb(y, 0) == ntt_md5["0"][log_h]
    want = np.zeros_like(x)
    O.lib().orc_antt128_limbwise_mt(x.reshape(-1), want.reshape(-1), log_h, 0, O.threads())
    assert np.array_equal(y, want)


# Kernel variants: 1 LDS tiles, 4 register tiles on every pass, 5 (the
# default for log_h >= 12) register tiles for the GF(2^8)-only passes and LDS tiles for the others.
# Same passes and layouts; every one parity-green so the A/B numbers stay reproducible.
VARIANTS = [1, 4, 5]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("log_h", [12, 13, 17, 19, 22, 24])
def test_register_tile_variants_gf32_r0_reference_md5(ntt_md5, log_h, variant, dev):
    x = O.mt_fill(0xDEADBEEF + log_h, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(5)))
    ntt.set_variant(variant)
    assert ntt.variant() == variant
    assert O.md5(_run_device(ntt, x, dev)) == ntt_md5["0"][log_h]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("log_h,r", [(12, 3), (13, 0), (14, 4), (17, 2), (20, 0)])
def test_register_tile_variants_gf128_matches_oracle(log_h, r, variant, dev):
    x = O.fill128(0xDEADBEEF + log_h + r, 0x5EED0000, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, r, B.FanPaarTowerField(7)))
    ntt.set_variant(variant)
    y = _run_device(ntt, x.reshape(-1), dev).reshape(-1, 4)
    assert np.array_equal(y, O.antt128(x, log_h, r))


@pytest.mark.parametrize("variant", VARIANTS)
def test_register_tile_variants_gf128_batched(variant, dev):
    log_h, batch = 14, 3
    x = O.fill128(0xB00, 0xC0FFEE, batch << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 1, B.FanPaarTowerField(7)))
    ntt.set_variant(variant)
    y = _run_device(ntt, x.reshape(-1), dev, batch=batch).reshape(batch, -1, 4)
    for b in range(batch):
        assert np.array_equal(y[b], O.antt128(x[b << log_h:(b + 1) << log_h], log_h, 1))


@pytest.mark.parametrize("variant", [1, 4])
def test_variant_gf128_2p24_limb_md5_and_oracle(ntt_md5, variant, dev):
    # the north-star size on the non-default kernels (the default is checked by the fixture test
    # and test_gf128_north_star_size_limb_md5_and_oracle): limb 0 MD5-pinned, all limbs vs the oracle
    log_h = 24
    x = O.fill128(0xDEADBEEF + log_h, 0x5EED0000, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(7)))
    ntt.set_variant(variant)
    y = _run_device(ntt, x.reshape(-1), dev).reshape(-1, 4)
    assert O.md5_limb(y, 0) == ntt_md5["0"][log_h]
    want = np.zeros_like(x)
    O.lib().orc_antt128_limbwise_mt(x.reshape(-1), want.reshape(-1), log_h, 0, O.threads())
    assert np.array_equal(y, want)


@pytest.mark.parametrize("log_h,r", [(20, 0), (19, 1), (18, 2), (16, 2), (12, 0), (14, 4)])
def test_lane_split_passes_gf128(ntt_md5, log_h, r, dev):
    # launches of fewer than two tiles per CU (one 2^20 transform: 256 tiles) run their upper
    # GF(2^16/32) passes lane-split (antt_bs3_pass: each product over two waves, DESIGN.md section
    # 5.1; at 2^17..2^20 there is always such a pass); every size matches the oracle, and limb 0 of
    # an r = 0 transform the reference MD5 table
    x = O.fill128(0xDEADBEEF + log_h + r, 0x5EED0000, 1 << log_h)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, r, B.FanPaarTowerField(7)))
    names = []
    for i in range(4):
        try:
            names.append(ntt.pass_kernel_name(i))
        except B.BnError:
            break
    if log_h >= 17:
        assert any("antt_bs3_pass" in n for n in names), names
        assert "antt_bs3_pass" not in names[-1], names  # the bottom pass keeps one wave per limb
    if len(names) > 1 and (1 << (log_h + r - 12)) < 2 * 256:
        # ... and, fewer than two tiles per CU, runs on register tiles compiled for one wave per SIMD
        # (round 5: no spills)
        import re
        assert re.search(r"antt_rr_pass<4, 2, \d+, 1>", names[-1]), names
    y = _run_device(ntt, x.reshape(-1), dev).reshape(-1, 4)
    assert np.array_equal(y, O.antt128(x, log_h, r))
    if r == 0:
        assert O.md5_limb(y, 0) == ntt_md5["0"][log_h]
