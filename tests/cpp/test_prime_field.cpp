// C++ drop-in check for the prime-field siblings: the reference's own test flows
// (src/ulvt/ntt/tests/test_ntt.cu:126-187 "NTTBB31 all input lengths" / "NTTBB31 round trip";
// src/ulvt/prime_field_sumcheck/test_sumcheck.cu:9-99 "Prime Field Sumcheck Test") written
// against the host mirror headers (binius-ntt_amd/host/ulvt), i.e. against the C-ABI library
// only. The oracle (test infrastructure) is linked as the checker for the host field classes.
// Prints "bbmd5 <log_n> <hex>" lines (compared with the reference's table by
// tests/test_cpp_surface.py) and ok/FAIL lines; exit status 0 iff every check passes.
#include <array>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "finite_fields/baby_bear.hpp"
#include "ntt/gpuntt.hpp"
#include "prime_field_sumcheck/interpolate.hpp"
#include "prime_field_sumcheck/sumcheck.hpp"
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

// test_ntt.cu:126-152
static void bb31_md5(int log_len) {
	std::mt19937 gen(0xdeadbeef + log_len);
	const size_t inp_size = (size_t)1 << log_len;
	NTTData<BB31> ntt_inp(DataOrder::IN_ORDER, inp_size);
	for (size_t i = 0; i < inp_size; i++) ntt_inp.data[i] = BB31((uint32_t)gen());
	NTTConfRad2<BB31> nttconf(BB31(137), 27, log_len);
	NTT<BB31> ntt(nttconf);
	NTTData<BB31> ntt_out(inp_size);
	ntt.apply(ntt_inp, ntt_out);
	std::vector<uint32_t> words(inp_size);
	for (size_t i = 0; i < inp_size; i++) words[i] = ntt_out.data[i].asUInt32();
	std::printf("bbmd5 %d %s\n", log_len, md5hex(words.data(), 4 * inp_size).c_str());
}

// test_ntt.cu:154-187
static void bb31_round_trip() {
	constexpr int log_inp_len = 24;
	constexpr size_t inp_size = (size_t)1 << log_inp_len;
	NTTData<BB31> ntt_inp(DataOrder::IN_ORDER, inp_size);
	std::mt19937 gen(0xAABBCCDD);
	for (size_t i = 0; i < inp_size; i++) ntt_inp.data[i] = BB31((uint32_t)gen());
	BB31 mul_gen(137);
	NTTConfRad2<BB31> fwdnttconf(mul_gen, 27, log_inp_len);
	NTTConfRad2<BB31> invnttconf(BB31::inv(mul_gen), 27, log_inp_len);
	NTT<BB31> fwdntt(fwdnttconf);
	NTT<BB31> invntt(invnttconf);
	NTTData<BB31> ntt_out(inp_size);
	fwdntt.apply(ntt_inp, ntt_out);
	NTTData<BB31> final_out(inp_size);
	invntt.apply(ntt_out, final_out);
	BB31 inv_log_len = BB31::inv(BB31((uint32_t)inp_size));
	bool ok = std::memcmp(ntt_inp.data.get(), ntt_out.data.get(), ntt_out.byte_len()) != 0;
	for (size_t i = 0; i < inp_size; i++) final_out.data[i] = inv_log_len * final_out.data[i];
	ok = ok && std::memcmp(final_out.data.get(), ntt_inp.data.get(), final_out.byte_len()) == 0;
	check(ok, "NTT<BB31> round trip 2^24 (test_ntt.cu:154-187)");
}

static void apply_rejects() {
	bool threw = false;
	try {
		NTTConfRad2<BB31> bad(BB31(137), 27, 28);
	} catch (const std::invalid_argument&) {
		threw = true;
	}
	NTT<BB31> ntt(NTTConfRad2<BB31>(BB31(137), 27, 10));
	NTTData<BB31> small(DataOrder::IN_ORDER, 512), out(1024);
	bool threw2 = false;
	try {
		ntt.apply(small, out);
	} catch (const std::invalid_argument&) {
		threw2 = true;
	}
	check(threw && threw2, "NTTConfRad2 / NTT::apply reject what the reference ASSERTs");
}

static void fields_vs_oracle() {
	std::mt19937 g(11);
	bool ok = true;
	for (int i = 0; i < 2000; i++) {
		const uint32_t a = g(), b = g();
		const BB31 x(a), y(b);
		ok = ok && (x * y).asUInt32() == orc_bb31_mul(a % BB31::P, b % BB31::P);
		ok = ok && (x.asUInt32() == 0 || x * BB31::inv(x) == BB31::one());
		uint32_t A[4], B[4], C[4], D[4];
		for (int k = 0; k < 4; k++) A[k] = g() % M31::P, B[k] = g() % M31::P;
		orc_qm31_mul(A, B, C);
		(QM31::from_words(A) * QM31::from_words(B)).to_words(D);
		ok = ok && std::memcmp(C, D, 16) == 0;
	}
	check(ok, "BB31 / QM31 host arithmetic vs oracle");
}

// test_sumcheck.cu:9-99, plus the final check f0(r) f1(r) == last claim
template <uint32_t NUM_VARS>
static void prime_sumcheck_flow() {
	QM31 points[3] = {(uint32_t)4, (uint32_t)4, (uint32_t)4};
	bool ok = interpolate_at((uint32_t)7, points) == QM31((uint32_t)4);
	QM31 expected_claim = (uint32_t)0;
	std::vector<QM31> evals;
	for (std::size_t i = 0; i < (1u << NUM_VARS); ++i) evals.push_back(QM31((uint32_t)i));
	for (std::size_t i = 0; i < (1u << NUM_VARS); ++i) evals.push_back(QM31((uint32_t)i));
	for (std::size_t i = 0; i < (1u << NUM_VARS); ++i) expected_claim += evals[i] * evals[i + (1 << NUM_VARS)];
	Sumcheck<NUM_VARS> sumcheck(evals, false);
	for (std::size_t i = 0; i < NUM_VARS; ++i) {
		std::array<QM31, 3> this_round_points;
		sumcheck.template this_round_messages<2048, 32>(this_round_points);
		QM31 this_round_claim = this_round_points[0] + this_round_points[1];
		ok = ok && this_round_claim == expected_claim;
		uint64_t a[4] = {32482843, 85864538, 8348234, 9544334};
		QM31 challenge = QM31(a);
		expected_claim = interpolate_at(challenge, this_round_points.data());
		sumcheck.template fold<2048, 32>(challenge);
	}
	const auto f = sumcheck.final_values();
	ok = ok && f[0] * f[1] == expected_claim;
	char what[96];
	std::snprintf(what, sizeof(what), "Prime Field Sumcheck Test, NUM_VARS=%u (test_sumcheck.cu:9-99) + final claim", NUM_VARS);
	check(ok, what);
}

int main() {
	check(check_gpu_capabilities(), "check_gpu_capabilities");
	for (int log_len = 1; log_len <= 22; log_len++) bb31_md5(log_len);
	bb31_round_trip();
	apply_rejects();
	fields_vs_oracle();
	prime_sumcheck_flow<1>();
	prime_sumcheck_flow<20>();
	prime_sumcheck_flow<24>();
	std::printf("%d failure(s)\n", failures);
	return failures ? 1 : 0;
}
