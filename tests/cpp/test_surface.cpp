// C++ drop-in check: the reference's own test flows (src/ulvt/ntt/tests/test_ntt.cu:189-229,
// src/ulvt/sumcheck/test/test.cu:13-101) written against the host mirror headers
// (binius-ntt_amd/host/ulvt), i.e. against the C-ABI library only. The oracle (test
// infrastructure) is linked as the checker. Prints one line per check; exit status 0 iff all
// pass. The MD5 lines ("md5 <r> <log_h> <hex>") are compared with the reference's tables by
// tests/test_cpp_surface.py.
#include <array>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>  // the sharded test's device message sinks (host API only)

#include "finite_fields/binary_tower.hpp"
#include "finite_fields/binary_tower_simd.hpp"
#include "finite_fields/circuit_generator/unrolled/binary_tower_unrolled.hpp"
#include "ntt/additive_ntt.hpp"
#include "sumcheck/sumcheck.hpp"
#include "sumcheck/verifier.hpp"
#include "utils/bitslicing.hpp"
#include "../../oracle/oracle.h"

static int failures = 0;
static void check(bool ok, const char* what) {
	std::printf("%s %s\n", ok ? "ok" : "FAIL", what);
	if (!ok) failures++;
}

static std::string md5hex(const void* p, size_t n) {
	uint8_t d[16];
	orc_md5(p, n, d);
	char s[33];
	for (int i = 0; i < 16; i++) std::snprintf(s + 2 * i, 3, "%02x", d[i]);
	return s;
}

// test_ntt.cu:191-216: mt19937(0xdeadbeef + log_h + log_rate) input, MD5 of the output words
static void ntt32_md5(int log_h, int log_rate) {
	std::mt19937 gen(0xdeadbeef + log_h + log_rate);
	NTTData<uint32_t> in(DataOrder::IN_ORDER, (size_t)1 << log_h), out((size_t)1 << (log_h + log_rate));
	for (size_t i = 0; i < in.size; i++) in.data[i] = gen();
	AdditiveNTTConf<uint32_t, FanPaarTowerField<5>> conf(log_h, log_rate);
	AdditiveNTT<uint32_t, FanPaarTowerField<5>> ntt(conf);
	const bool ok = ntt.apply(in, out);
	std::printf("md5 %d %d %s\n", log_rate, log_h, ok ? md5hex(out.data.get(), out.byte_len()).c_str() : "apply-failed");
}

static void ntt128_vs_oracle(int log_h, int log_rate) {
	using T = unsigned __int128;
	const size_t n = (size_t)1 << log_h;
	std::vector<uint32_t> words(4 * n);
	orc_fill128(0xdeadbeef + log_h + log_rate, 0x5eed0000, words.data(), n);
	NTTData<T> in(DataOrder::IN_ORDER, n), out(n << log_rate);
	std::memcpy(in.data.get(), words.data(), in.byte_len());
	AdditiveNTT<T, FanPaarTowerField<7>> ntt(AdditiveNTTConf<T, FanPaarTowerField<7>>(log_h, log_rate));
	bool ok = ntt.apply(in, out) && out.order == DataOrder::IN_ORDER;
	std::vector<uint32_t> want(4 * (n << log_rate));
	orc_antt128(words.data(), want.data(), log_h, log_rate);
	ok = ok && std::memcmp(out.data.get(), want.data(), out.byte_len()) == 0;
	char what[96];
	std::snprintf(what, sizeof(what), "AdditiveNTT<u128, FanPaarTowerField<7>> log_h=%d r=%d vs oracle", log_h, log_rate);
	check(ok, what);
}

static void apply_rejects() {
	AdditiveNTT<uint32_t, FanPaarTowerField<5>> ntt(AdditiveNTTConf<uint32_t, FanPaarTowerField<5>>(4, 1));
	NTTData<uint32_t> wrong_size(DataOrder::IN_ORDER, 8), bitrev(DataOrder::BIT_REVERSED, 16), out(32);
	out.data[0] = 0x1234;
	check(!ntt.apply(wrong_size, out) && !ntt.apply(bitrev, out) && out.data[0] == 0x1234 && out.order == DataOrder::INVALID,
		  "apply returns false with no effect on bad size / order (additive_ntt.cuh:206-208)");
	bool threw = false;
	try {
		AdditiveNTTConf<uint32_t, FanPaarTowerField<5>> bad(30, 4);
	} catch (const std::invalid_argument&) {
		threw = true;
	}
	check(threw, "AdditiveNTTConf rejects log_h + log_rate > N_BITS");
}

static void field_policies() {
	std::mt19937_64 g(7);
	bool ok = true;
	for (int i = 0; i < 1000; i++) {
		const uint32_t a = (uint32_t)g(), b = (uint32_t)g();
		ok = ok && FanPaarTowerField<5>::multiply(a, b) == orc_mul32(a, b);
		if (a) ok = ok && FanPaarTowerField<5>::multiply(a, FanPaarTowerField<5>::inverse(a)) == 1;
		uint32_t A[4], B[4], C[4];
		for (int k = 0; k < 4; k++) A[k] = (uint32_t)g(), B[k] = (uint32_t)g();
		orc_mul128(A, B, C);
		unsigned __int128 x = 0, y = 0, z = 0;
		std::memcpy(&x, A, 16), std::memcpy(&y, B, 16), std::memcpy(&z, C, 16);
		ok = ok && FanPaarTowerField<7>::multiply(x, y) == z;
		ok = ok && FanPaarTowerField<7>::multiply(x, FanPaarTowerField<7>::inverse(x)) == 1;
	}
	check(ok, "FanPaarTowerField<5>/<7> multiply/inverse vs oracle");
}

static void bitslicing() {
	std::mt19937 g(3);
	uint32_t blk[128], ref[128];
	for (auto& w : blk) w = g();
	std::memcpy(ref, blk, sizeof(blk));
	BitsliceUtils<128>::bitslice_transpose(blk);
	orc_bitslice_transpose128(ref);
	bool ok = std::memcmp(blk, ref, sizeof(blk)) == 0;
	BitsliceUtils<128>::bitslice_untranspose(blk);
	orc_bitslice_untranspose128(ref);
	ok = ok && std::memcmp(blk, ref, sizeof(blk)) == 0;
	check(ok, "BitsliceUtils<128> transpose / untranspose vs oracle");
}

// multiply_unrolled<H> (binary_tower_unrolled.cuh:4-5, in place as core.cu:21 calls it) and the
// packed-subfield operations (binary_tower_simd.cuh:77-150, KATs of tests.cu:17-95) vs the oracle
template <int H>
static bool unrolled_vs_oracle(std::mt19937& g) {
	constexpr int W = 1 << H;
	uint32_t a[W], b[W];
	for (auto& w : a) w = g();
	for (auto& w : b) w = g();
	uint32_t dst[W];
	std::memcpy(dst, a, sizeof(a));
	multiply_unrolled<H>(dst, b, dst);
	bool ok = true;
	for (int e = 0; e < 32; e++) {
		uint64_t x = 0, y = 0, z = 0;
		for (int i = 0; i < W && i < 64; i++) {
			x |= (uint64_t)((a[i] >> e) & 1) << i;
			y |= (uint64_t)((b[i] >> e) & 1) << i;
			z |= (uint64_t)((dst[i] >> e) & 1) << i;
		}
		if (H <= 6) ok = ok && orc_mul(x, y, H) == z;
	}
	return ok;
}

static void field_simd() {
	std::mt19937 g(77);
	bool ok = unrolled_vs_oracle<2>(g) && unrolled_vs_oracle<5>(g) && unrolled_vs_oracle<6>(g);
	// H = 7: 32 GF(2^128) products through BitsliceUtils<128> vs orc_mul128
	uint32_t a[128], b[128], c[128];
	for (auto& w : a) w = g();
	for (auto& w : b) w = g();
	uint32_t as[128], bs[128];
	std::memcpy(as, a, sizeof(a));
	std::memcpy(bs, b, sizeof(b));
	BitsliceUtils<128>::bitslice_transpose(as);
	BitsliceUtils<128>::bitslice_transpose(bs);
	multiply_unrolled<7>(as, bs, c);
	BitsliceUtils<128>::bitslice_untranspose(c);
	for (int e = 0; e < 32; e++) {
		uint32_t r[4];
		orc_mul128(a + 4 * e, b + 4 * e, r);
		ok = ok && std::memcmp(r, c + 4 * e, 16) == 0;
	}
	check(ok, "multiply_unrolled<2,5,6,7> (in place) vs oracle");
	ok = mul_binary_tower_32b_simd<5>(0xd82c07cdu, 0xd82c07cdu) == 0xafab1b8fu &&
	     mul_binary_tower_32b_simd<3>(0xe0u, 0x76u) == 0x96u && mul_binary_tower_32b_simd<4>(0x4f4bu, 0x4386u) == 0x7202u;
	for (int i = 0; i < 64; i++) {
		const uint32_t x = g(), y = g();
		ok = ok && mul_binary_tower_32b_simd<5>(x, y) == orc_mul32(x, y);
	}
	const auto cd = interleave_32b<0>(0x0000ffffu, 0xffff0000u);
	ok = ok && cd.first == 0xaaaa5555u && cd.second == 0xaaaa5555u;
	const auto ab = interleave_32b<4>(0x11100100u, 0x13120302u);
	ok = ok && ab.first == 0x03020100u && ab.second == 0x13121110u;
	ok = ok && xor_adjacent_32b<3>(0x0000ff0fu) == 0x0000f0f0u;
	check(ok, "mul_binary_tower_32b_simd / interleave_32b / xor_adjacent_32b");
}

// test.cu:13-101 with fixed seeds: per-round verifier checks and the final brute-force claim
template <uint32_t N, uint32_t D, bool T>
static void sumcheck_protocol() {
	using F = FanPaarTowerField<7>;
	using u128 = unsigned __int128;
	const size_t words = 4 * ((size_t)1 << N) * D;
	std::vector<uint32_t> evals(words);
	std::mt19937_64 g(0x5c00 + D);
	for (auto& w : evals) w = (uint32_t)g();
	std::vector<uint32_t> compact = evals;
	if (T)
		for (size_t b = 0; b < words / 128; b++) orc_bitslice_untranspose128(compact.data() + 128 * b);
	Sumcheck<N, D, T> s(evals, false);
	std::vector<uint32_t> challenges(4 * N);
	auto big = [](const uint32_t* w) {
		u128 x = 0;
		std::memcpy(&x, w, 16);
		return x;
	};
	bool ok = true;
	u128 claim = 0;
	for (uint32_t round = 0; round < N; round++) {
		std::array<uint32_t, 4> sum;
		std::array<uint32_t, 4 * (D + 1)> points;
		s.this_round_messages(sum, points);
		if (round > 0) ok = ok && big(sum.data()) == claim;
		ok = ok && big(sum.data()) == (big(points.data()) ^ big(points.data() + 4));
		std::array<uint32_t, 4> ch;
		for (auto& w : ch) w = (uint32_t)g();
		std::memcpy(&challenges[4 * round], ch.data(), 16);
		// evaluate_univariate_given_points: Lagrange through (k, points[k]), k = 0..D, once with the
		// host field policy and once through the library
		const u128 r = big(ch.data());
		u128 acc = 0;
		for (uint32_t i = 0; i <= D; i++) {
			u128 t = big(points.data() + 4 * i);
			for (uint32_t j = 0; j <= D; j++) {
				if (j == i) continue;
				t = F::multiply(t, r ^ (u128)j);
				t = F::multiply(t, F::inverse((u128)(i ^ j)));
			}
			acc ^= t;
		}
		ok = ok && acc == evaluate_univariate_given_points(r, (const u128*)points.data(), D + 1);
		claim = acc;
		s.move_to_next_round(ch);
	}
	std::array<uint32_t, 4> sum;
	std::array<uint32_t, 4 * (D + 1)> points;
	s.this_round_messages(sum, points);
	ok = ok && big(sum.data()) == claim;
	uint32_t brute[4];
	orc_multilinear_composition(compact.data(), N, D, challenges.data(), brute);
	ok = ok && big(brute) == claim;
	// the library's own verifier helpers (verifier.cu:9-31, 88-107)
	const __uint128_t gpu_claim = evaluate_multilinear_composition((const __uint128_t*)compact.data(),
																   (const __uint128_t*)challenges.data(), N, D);
	ok = ok && gpu_claim == claim;
	char what[96];
	std::snprintf(what, sizeof(what), "Sumcheck<%u, %u, %s> protocol checks + final claim", N, D, T ? "true" : "false");
	check(ok, what);
}

// Two shard provers of world 2 in one process, exchanging through their device message sinks (the
// C++ form of ShardedSumcheck's device path): per round the sinks are
// copied back on each prover's stream and XOR-ed, p(1) is completed from the global claim when the
// flag word says it was skipped, and at the endgame the exported batches are gathered. Every round
// must equal the unsharded prover's.
template <uint32_t N, uint32_t D>
static void sharded_sink_protocol() {
	using u128 = unsigned __int128;
	const size_t words = 4 * ((size_t)1 << N) * D;
	std::vector<uint32_t> evals(words);
	std::mt19937_64 g(0x5d00 + D);
	for (auto& w : evals) w = (uint32_t)g();
	Sumcheck<N, D, true> ref(evals, false), s0(evals, false), s1(evals, false);
	s0.set_shard(0, 2);
	s1.set_shard(1, 2);
	constexpr size_t kSink = 40;
	uint32_t* d_sink[2] = {nullptr, nullptr};
	bool ok = hipMalloc((void**)&d_sink[0], kSink * 4) == hipSuccess && hipMalloc((void**)&d_sink[1], kSink * 4) == hipSuccess;
	if (ok) {
		s0.set_message_sink(d_sink[0]);
		s1.set_message_sink(d_sink[1]);
	}
	auto big = [](const uint32_t* w) {
		u128 x = 0;
		std::memcpy(&x, w, 16);
		return x;
	};
	u128 claim = 0;
	bool gathered = false;
	for (uint32_t round = 0; ok && round <= N; round++) {
		std::array<uint32_t, 4> sum{}, rs{};
		std::array<uint32_t, 4 * (D + 1)> points{}, rp{};
		if (!gathered && s0.needs_gather()) {
			std::vector<uint32_t> all = s0.export_shard(), e1 = s1.export_shard();
			all.insert(all.end(), e1.begin(), e1.end());
			s0.import_gathered(all, 2);
			s1.import_gathered(all, 2);
			gathered = true;
		}
		if (gathered) {
			s0.this_round_messages(sum, points);
		} else {
			s0.round_messages_sink();
			s1.round_messages_sink();
			uint32_t h[2][kSink];
			Sumcheck<N, D, true>* sp[2] = {&s0, &s1};
			for (int k = 0; k < 2; k++)
				ok = ok && hipMemcpyAsync(h[k], d_sink[k], sizeof h[k], hipMemcpyDeviceToHost, (hipStream_t)sp[k]->stream()) == hipSuccess &&
				     hipStreamSynchronize((hipStream_t)sp[k]->stream()) == hipSuccess;
			ok = ok && h[0][36] == h[1][36];
			for (size_t i = 0; i < 4 * (D + 1); i++) points[i] = h[0][i] ^ h[1][i];
			if (h[0][36] & 2u) {  // the last call: prod_j f_j(r)
				std::memcpy(sum.data(), points.data(), 16);
				points.fill(0);
			} else if (h[0][36] & 1u) {  // p(1) left out: the global claim completes it
				const u128 p1 = claim ^ big(points.data());
				std::memcpy(points.data() + 4, &p1, 16);
				std::memcpy(sum.data(), &claim, 16);
			} else {
				const u128 sm = big(points.data()) ^ big(points.data() + 4);
				std::memcpy(sum.data(), &sm, 16);
			}
		}
		ref.this_round_messages(rs, rp);
		ok = ok && rs == sum && (round == N || rp == points);
		if (round < N) {
			std::array<uint32_t, 4> ch;
			for (auto& w : ch) w = (uint32_t)g();
			claim = evaluate_univariate_given_points(big(ch.data()), (const u128*)points.data(), D + 1);
			ref.move_to_next_round(ch);
			s0.move_to_next_round(ch);
			if (!gathered) s1.move_to_next_round(ch);
		}
	}
	for (uint32_t* p : d_sink)
		if (p) (void)hipFree(p);
	char what[96];
	std::snprintf(what, sizeof(what), "Sumcheck<%u, %u, true> world-2 shards through device message sinks", N, D);
	check(ok && gathered, what);
}

int main() {
	check(check_gpu_capabilities(), "check_gpu_capabilities");
	for (int log_h = 1; log_h <= 20; log_h++) ntt32_md5(log_h, 0);
	for (int log_h = 1; log_h <= 16; log_h++) ntt32_md5(log_h, 2);
	ntt128_vs_oracle(10, 0);
	ntt128_vs_oracle(10, 2);
	ntt128_vs_oracle(13, 1);
	apply_rejects();
	field_policies();
	bitslicing();
	field_simd();
	sumcheck_protocol<12, 3, true>();
	sumcheck_protocol<11, 2, false>();
	sumcheck_protocol<10, 4, true>();
	sharded_sink_protocol<12, 3>();
	sharded_sink_protocol<11, 2>();
	std::printf("%d failure(s)\n", failures);
	return failures ? 1 : 0;
}
