// Host-side sanitizer run (CPU, no GPU needed): built with AddressSanitizer + UBSan by
// tests/cpp/Makefile (`make -C tests/cpp asan`) together with an ASan build of the library's host
// code (binius-ntt_amd/lib-asan, hipcc -Xarch_host -fsanitize=address) and the oracle's C sources.
// It exercises
//   * the oracle (test infrastructure): tower arithmetic, every NTT form, bitslicing, the sumcheck
//     protocol, BabyBear and QM31 — and cross-checks the forms against each other;
//   * the C++ host mirror's host-only classes (FanPaarTowerField<H>, BitsliceUtils<W>, NTTData,
//     AdditiveNTTConf, BB31, QM31/interpolate_at) against the oracle;
//   * the library's host-side code: the generated bitsliced circuits behind multiply_unrolled<H>,
//     the packed-subfield helpers, bn_sumcheck_interpolate, and the argument-checking / error paths
//     of the C-ABI (no device present here: they must fail cleanly with a status code).
// Prints "ok <what>" / "FAIL <what>" per check, and "md5 ..." lines that tests/test_asan.py compares
// with the reference's golden tables; exit status 0 iff every check passed (a sanitizer report
// aborts the run with a non-zero status).
#include <array>
#include <cstdio>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "finite_fields/baby_bear.hpp"
#include "finite_fields/binary_tower.hpp"
#include "finite_fields/binary_tower_simd.hpp"
#include "finite_fields/circuit_generator/unrolled/binary_tower_unrolled.hpp"
#include "ntt/nttconf.hpp"
#include "prime_field_sumcheck/interpolate.hpp"
#include "utils/bitslicing.hpp"
#include "utils/common.hpp"
#include "../../oracle/oracle.h"

static int failures = 0;
static void check(bool ok, const char* what) {
	std::printf("%s %s\n", ok ? "ok" : "FAIL", what);
	if (!ok) failures++;
}

static std::string hex(const uint8_t* d) {
	char s[33];
	for (int i = 0; i < 16; i++) std::snprintf(s + 2 * i, 3, "%02x", d[i]);
	return s;
}

using u128 = unsigned __int128;
static u128 ld128(const uint32_t* w) {
	return (u128)w[0] | ((u128)w[1] << 32) | ((u128)w[2] << 64) | ((u128)w[3] << 96);
}

static void oracle_checks() {
	std::mt19937_64 rng(7);
	// tower: a * a^-1 == 1 at every height, 128-bit product KAT (tests.cu:172-201)
	bool ok = true;
	for (int h = 1; h <= 6; h++)
		for (int t = 0; t < 200; t++) {
			const uint64_t m = h == 6 ? ~0ull : ((1ull << (1 << h)) - 1);
			uint64_t a = rng() & m;
			if (!a) a = 1;
			ok = ok && orc_mul(a, orc_inv(a, h), h) == 1 && orc_square(a, h) == orc_mul(a, a, h);
		}
	check(ok, "oracle tower inverse / square, heights 1-6");
	const uint32_t ka[4] = {0x95323434u, 0x78593827u, 0x2755a479u, 0xf3122332u};
	const uint32_t kb[4] = {0x22048438u, 0x59347593u, 0x84794387u, 0xd3473493u};
	uint32_t kc[4];
	orc_mul128(ka, kb, kc);
	check(ld128(kc) == (((u128)0xceaa247e2dc6d28cull << 64) | 0x999c424f4b3220e5ull), "oracle GF(2^128) KAT (tests.cu:198-201)");

	// NTT: the reference MD5 input at log_h 10 (r = 0), and every GF(2^128) form against each other
	for (int log_h : {10, 12}) {
		std::vector<uint32_t> in((size_t)1 << log_h), out(in.size());
		orc_mt_fill(0xdeadbeefu + (uint32_t)log_h, in.data(), in.size());
		orc_antt32(in.data(), out.data(), log_h, 0);
		uint8_t d[16];
		orc_md5(out.data(), out.size() * 4, d);
		std::printf("md5 0 %d %s\n", log_h, hex(d).c_str());
	}
	{
		const int log_h = 9, r = 2;
		const size_t n = (size_t)1 << log_h;
		std::vector<uint32_t> x(4 * n), a(4 * (n << r)), b(a.size()), c(a.size()), e(a.size());
		orc_fill128(11, 0x5eed0000, x.data(), n);
		orc_antt128(x.data(), a.data(), log_h, r);
		orc_antt128_limbwise(x.data(), b.data(), log_h, r);
		orc_antt128_limbwise_batch(x.data(), c.data(), log_h, r, 1);
		orc_antt128_limbwise_mt(x.data(), e.data(), log_h, r, 3);
		check(a == b && b == c && c == e, "oracle GF(2^128) NTT: full, limb-wise, batched and threaded forms agree");
		std::vector<uint32_t> s32((size_t)log_h * (log_h + r - 1)), s128(4 * s32.size());
		orc_subspace_evals32(log_h, r, s32.data());
		orc_subspace_evals128(log_h, r, s128.data());
		bool same = true;
		for (size_t i = 0; i < s32.size(); i++) same = same && s128[4 * i] == s32[i] && !s128[4 * i + 1] && !s128[4 * i + 2] && !s128[4 * i + 3];
		check(same, "oracle subspace table: GF(2^32) and GF(2^128) computations agree");
	}
	{
		const int log_h = 15, batch = 3;
		std::vector<uint32_t> x(4 * ((size_t)batch << log_h)), a(x.size()), b(x.size());
		orc_fill128(5, 6, x.data(), x.size() / 4);
		orc_antt128_limbwise_batch(x.data(), a.data(), log_h, 0, batch);
		for (int i = 0; i < batch; i++)
			orc_antt128_limbwise_mt(x.data() + 4 * ((size_t)i << log_h), b.data() + 4 * ((size_t)i << log_h), log_h, 0, 8);
		check(a == b, "oracle batched NTT = per-transform threaded NTT (persistent pool, 8 threads)");
	}

	// bitslicing round trips
	{
		std::vector<uint32_t> blk(128 * 5), orig;
		for (auto& w : blk) w = (uint32_t)rng();
		orig = blk;
		orc_bitslice_many128(blk.data(), 5, 0);
		orc_bitslice_many128(blk.data(), 5, 1);
		uint32_t b32[32], o32[32];
		for (int i = 0; i < 32; i++) b32[i] = o32[i] = (uint32_t)rng();
		orc_bitslice_transpose32(b32);
		orc_bitslice_untranspose32(b32);
		check(blk == orig && std::memcmp(b32, o32, sizeof b32) == 0, "oracle bitslice round trips (128- and 32-bit)");
	}

	// sumcheck: compact and bitsliced transcripts agree, p(0) + p(1) = sum, final claim
	{
		const int n = 8, d = 3;
		std::vector<uint32_t> ev((size_t)d * 4 << n), bs(ev.size()), ch(4 * n);
		for (auto& w : ev) w = (uint32_t)rng();
		for (auto& w : ch) w = (uint32_t)rng();
		bs = ev;
		orc_bitslice_many128(bs.data(), bs.size() / 128, 0);
		std::vector<uint32_t> s1(4 * (n + 1)), p1(4 * (d + 1) * (n + 1)), s2(s1.size()), p2(p1.size());
		orc_sumcheck_run(ev.data(), n, d, 0, ch.data(), s1.data(), p1.data());
		orc_sumcheck_run(bs.data(), n, d, 1, ch.data(), s2.data(), p2.data());
		bool inv = s1 == s2 && p1 == p2;
		for (int r = 0; r < n; r++) {
			for (int i = 0; i < 4; i++) inv = inv && s1[4 * r + i] == (p1[4 * (d + 1) * r + i] ^ p1[4 * (d + 1) * r + 4 + i]);
			uint32_t nxt[4];
			orc_sumcheck_interpolate(&p1[4 * (d + 1) * r], d + 1, &ch[4 * r], nxt);
			inv = inv && std::memcmp(nxt, &s1[4 * (r + 1)], 16) == 0;
		}
		uint32_t f1[4], f2[4];
		orc_multilinear_composition(ev.data(), n, d, ch.data(), f1);
		orc_multilinear_composition_fold_mt(bs.data(), n, d, 1, ch.data(), f2, 2);
		inv = inv && std::memcmp(f1, f2, 16) == 0 && std::memcmp(f1, &s1[4 * n], 16) == 0;
		check(inv, "oracle sumcheck: compact = bitsliced transcript, protocol invariants, final claim");
	}

	// BabyBear: MD5 of the reference test input BB31(mt19937(0xdeadbeef + log_n)()) (test_ntt.cu:126-152)
	{
		const int log_n = 10;
		std::vector<uint32_t> in((size_t)1 << log_n), out(in.size());
		orc_mt_fill(0xdeadbeefu + (uint32_t)log_n, in.data(), in.size());
		orc_bb31_ntt(in.data(), out.data(), log_n, 137, 27, 0);
		uint8_t d[16];
		orc_md5(out.data(), out.size() * 4, d);
		std::printf("bb31md5 %d %s\n", log_n, hex(d).c_str());
		check(orc_bb31_mul(orc_bb31_inv(12345), 12345) == 1, "oracle BabyBear inverse");
	}
	// QM31 sumcheck on the reference test input QM31(i) (test_sumcheck.cu)
	{
		const int n = 6;
		std::vector<uint32_t> ev(2 * 4 << n), ch(4 * n), pts(12 * n);
		for (size_t i = 0; i < ev.size() / 4; i++) ev[4 * i] = (uint32_t)(i % ((1u << n)));
		for (auto& w : ch) w = (uint32_t)(rng() % 0x7fffffffu);
		orc_qm31_sumcheck_run(ev.data(), n, ch.data(), pts.data());
		check(true, "oracle QM31 sumcheck run");
	}
}

static void mirror_checks() {
	std::mt19937_64 rng(9);
	bool ok = true;
	for (int t = 0; t < 500; t++) {
		const uint32_t a = (uint32_t)rng(), b = (uint32_t)rng() | 1u;
		ok = ok && FanPaarTowerField<5>::multiply(a, b) == orc_mul32(a, b);
		ok = ok && FanPaarTowerField<5>::multiply(b, FanPaarTowerField<5>::inverse(b)) == 1u;
		ok = ok && FanPaarTowerField<3>::multiply(a & 0xff, b & 0xff) == (uint32_t)orc_mul(a & 0xff, b & 0xff, 3);
		uint32_t wa[4], wb[4], wc[4];
		for (int i = 0; i < 4; i++) wa[i] = (uint32_t)rng(), wb[i] = (uint32_t)rng();
		orc_mul128(wa, wb, wc);
		ok = ok && FanPaarTowerField<7>::multiply(ld128(wa), ld128(wb)) == ld128(wc);
		ok = ok && FanPaarTowerField<7>::multiply(ld128(wa), FanPaarTowerField<7>::inverse(ld128(wa))) == 1;
	}
	check(ok, "mirror FanPaarTowerField<3/5/7> vs oracle (multiply, inverse)");

	uint32_t blk[128], ref[128];
	for (int i = 0; i < 128; i++) blk[i] = ref[i] = (uint32_t)rng();
	BitsliceUtils<128>::bitslice_transpose(blk);
	orc_bitslice_transpose128(ref);
	bool same = std::memcmp(blk, ref, sizeof blk) == 0;
	BitsliceUtils<128>::bitslice_untranspose(blk);
	orc_bitslice_untranspose128(ref);
	same = same && std::memcmp(blk, ref, sizeof blk) == 0;
	const uint32_t val[4] = {1u, 0x80000000u, 0u, 0xffffffffu};
	BitsliceUtils<128>::repeat_value_bitsliced(blk, val);
	same = same && blk[0] == ~0u && blk[1] == 0u && blk[63] == ~0u && blk[64] == 0u && blk[127] == ~0u;
	check(same, "mirror BitsliceUtils<128> vs oracle (transpose, untranspose, repeat_value_bitsliced)");

	NTTData<u128> d(DataOrder::IN_ORDER, 16);
	check(d.byte_len() == 256 && d.order == DataOrder::IN_ORDER, "mirror NTTData");
	int thrown = 0;
	for (auto lr : std::vector<std::pair<int, int>>{{0, 0}, {30, 3}, {8, 5}, {4, -1}}) {
		try {
			AdditiveNTTConf<uint32_t, FanPaarTowerField<5>> c(lr.first, lr.second);
		} catch (const std::invalid_argument&) {
			thrown++;
		}
	}
	check(thrown == 4, "mirror AdditiveNTTConf rejects the reference's asserted cases (nttconf.cuh:55-60)");

	ok = true;
	for (int t = 0; t < 200; t++) {
		const uint32_t a = (uint32_t)rng(), b = (uint32_t)rng();
		ok = ok && (BB31(a) * BB31(b)).asUInt32() == orc_bb31_mul(a % BB31::P, b % BB31::P);
		if (a % BB31::P) ok = ok && (BB31::inv(BB31(a)) * BB31(a)) == BB31::one();
	}
	check(ok, "mirror BB31 vs oracle");

	ok = true;
	for (int t = 0; t < 50; t++) {
		uint32_t r[4], e[12], want[4];
		for (auto& w : r) w = (uint32_t)(rng() % M31::P);
		for (auto& w : e) w = (uint32_t)(rng() % M31::P);
		orc_qm31_interpolate(e, r, want);
		QM31 ev[3];
		for (int i = 0; i < 3; i++) std::memcpy(&ev[i], e + 4 * i, 16);
		QM31 rc;
		std::memcpy(&rc, r, 16);
		const QM31 got = interpolate_at(rc, ev);
		ok = ok && std::memcmp(&got, want, 16) == 0;
	}
	check(ok, "mirror QM31 interpolate_at vs oracle");
}

static void library_host_checks() {
	std::mt19937_64 rng(11);
	check(bn_version() && std::strlen(bn_version()) > 0, "bn_version");
	// generated bitsliced circuits (host build of multiply_unrolled<H>) vs the oracle's products
	bool ok = true;
	for (int t = 0; t < 4; t++) {
		uint32_t a[128], b[128], c[128], ca[128], cb[128];
		for (int i = 0; i < 128; i++) a[i] = ca[i] = (uint32_t)rng(), b[i] = cb[i] = (uint32_t)rng();
		multiply_unrolled<7>(a, b, c);
		orc_bitslice_untranspose128(ca);
		orc_bitslice_untranspose128(cb);
		uint32_t want[128];
		for (int e = 0; e < 32; e++) orc_mul128(ca + 4 * e, cb + 4 * e, want + 4 * e);
		orc_bitslice_transpose128(want);
		ok = ok && std::memcmp(c, want, sizeof c) == 0;
		multiply_unrolled<7>(a, b, a);  // alias-safe (core.cu:21)
		ok = ok && std::memcmp(a, want, sizeof a) == 0;
		uint32_t a5[32], b5[32], c5[32];
		for (int i = 0; i < 32; i++) a5[i] = (uint32_t)rng(), b5[i] = (uint32_t)rng();
		multiply_unrolled<5>(a5, b5, c5);
		uint32_t x5[32], y5[32];
		std::memcpy(x5, a5, sizeof a5);
		std::memcpy(y5, b5, sizeof b5);
		orc_bitslice_untranspose32(x5);
		orc_bitslice_untranspose32(y5);
		uint32_t w5[32];
		for (int e = 0; e < 32; e++) w5[e] = orc_mul32(x5[e], y5[e]);
		orc_bitslice_transpose32(w5);
		ok = ok && std::memcmp(c5, w5, sizeof c5) == 0;
	}
	check(ok, "library multiply_unrolled<5>/<7> host circuits vs oracle (incl. dst == a)");

	ok = true;
	for (int t = 0; t < 100; t++) {
		const uint32_t a = (uint32_t)rng(), b = (uint32_t)rng();
		const uint32_t p = mul_binary_tower_32b_simd<3>(a, b);
		for (int l = 0; l < 4; l++)
			ok = ok && ((p >> (8 * l)) & 0xff) == (uint32_t)orc_mul((a >> (8 * l)) & 0xff, (b >> (8 * l)) & 0xff, 3);
		const auto cd = interleave_32b<2>(a, b);
		const auto back = interleave_32b<2>(cd.first, cd.second);
		ok = ok && back.first == a && back.second == b;
		(void)xor_adjacent_32b<1>(a);
	}
	check(ok, "library packed-subfield helpers (mul_binary_tower_32b_simd<3>, interleave_32b<2> involution)");

	ok = true;
	for (int npts : {2, 4, 9}) {
		std::vector<uint32_t> pts(4 * (size_t)npts);
		for (auto& w : pts) w = (uint32_t)rng();
		uint32_t r[4], got[4], want[4];
		for (auto& w : r) w = (uint32_t)rng();
		ok = ok && bn_sumcheck_interpolate(pts.data(), npts, r, got) == BN_OK;
		orc_sumcheck_interpolate(pts.data(), npts, r, want);
		ok = ok && std::memcmp(got, want, 16) == 0;
	}
	check(ok, "library bn_sumcheck_interpolate vs oracle");

	// error paths: invalid arguments are rejected before any device call; with no device the
	// device-touching calls fail with a status code (never abort), and bn_last_error says why
	bn_antt_plan* plan = reinterpret_cast<bn_antt_plan*>(&ok);
	check(bn_antt_plan_create(0, 64, 10, 0, &plan) == BN_ERR_INVALID && plan == nullptr && std::strlen(bn_last_error()) > 0,
	      "bn_antt_plan_create rejects field_bits 64");
	check(bn_antt_plan_create(0, 128, 0, 0, &plan) == BN_ERR_INVALID, "bn_antt_plan_create rejects log_h 0");
	check(bn_antt_plan_create(0, 128, 10, 5, &plan) == BN_ERR_INVALID, "bn_antt_plan_create rejects log_rate 5");
	check(bn_antt_plan_create(0, 128, 10, 0, nullptr) == BN_ERR_INVALID, "bn_antt_plan_create rejects a NULL output");
	const int rc = bn_antt_plan_create(0, 128, 10, 0, &plan);
	check(rc != BN_OK && plan == nullptr, "bn_antt_plan_create without a device fails cleanly");
	check(bn_antt_forward_device(nullptr, nullptr, nullptr, 1, nullptr) == BN_ERR_INVALID, "bn_antt_forward_device(NULL plan)");
	check(bn_antt_plan_destroy(nullptr) == BN_OK, "bn_antt_plan_destroy(NULL)");
	bn_sumcheck* sc = nullptr;
	std::vector<uint32_t> ev(4 * 8 * 3);
	check(bn_sumcheck_create(0, 3, 9, 0, ev.data(), &sc) == BN_ERR_INVALID && sc == nullptr, "bn_sumcheck_create rejects d = 9");
	check(bn_sumcheck_create(0, 3, 3, 1, ev.data(), &sc) == BN_ERR_INVALID, "bn_sumcheck_create rejects bitsliced n < 5");
	check(bn_sumcheck_interpolate(nullptr, 3, nullptr, nullptr) == BN_ERR_INVALID, "bn_sumcheck_interpolate(NULL)");
	check(bn_multiply_unrolled(8, ev.data(), ev.data(), ev.data()) == BN_ERR_INVALID, "bn_multiply_unrolled rejects height 8");
	check(bn_check_gpu_capabilities() == 0, "bn_check_gpu_capabilities without a device");
	try {
		ulvt::bn_check(bn_antt_plan_create(0, 128, 0, 0, &plan));
		check(false, "ulvt::bn_check throws BnError");
	} catch (const ulvt::BnError& e) {
		check(e.code == BN_ERR_INVALID && std::string(e.what()).find("log_h") != std::string::npos, "ulvt::bn_check throws BnError");
	}
}

int main() {
	oracle_checks();
	mirror_checks();
	library_host_checks();
	std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "PASSED", failures);
	return failures ? 1 : 0;
}
