// The reference's sumcheck benchmark driver (src/ulvt/sumcheck/bench/benchmark.cu:12-85) on this
// build's C++ mirror (binius-ntt_amd/host/ulvt/sumcheck/sumcheck.hpp, the C-ABI underneath):
// the same configurations (NUM_VARS 20/24/28 x COMPOSITION_SIZE 2/3/4), run counts (10/5/2 after
// one warm-up sample), compact input from a host std::vector (DATA_IS_TRANSPOSED = false) and the
// same three phases per sample:
//   Memcpy    = constructor, bn_sumcheck_create_staged: host -> HBM copy (pageable std::vector)
//   Transpose = constructor, bn_sumcheck_prepare: the device compact -> bitsliced transpose
//   Raw       = every round's this_round_messages + move_to_next_round, then the last messages
// Output: the reference's text lines per configuration, then one JSON line with every result.
// Build + run: tools/run_benchmark_sumcheck.sh
#include <array>
#include <chrono>
#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

#include "sumcheck/sumcheck.hpp"

struct Benchmarks {
	double memcpy, transpose, raw;
};

static std::string g_json;

template <uint32_t NUM_VARS, uint32_t COMPOSITION_SIZE>
Benchmarks benchmark_one_sample() {
	constexpr uint32_t INTS = 4;
	constexpr uint32_t POINTS = COMPOSITION_SIZE + 1;
	const size_t total_ints = (size_t)INTS * ((size_t)1 << NUM_VARS) * COMPOSITION_SIZE;
	std::vector<uint32_t> evals(total_ints);
	// a fixed, non-zero input (the reference leaves the vector value-initialised)
	uint32_t x = 0x9E3779B9u;
	for (size_t i = 0; i < total_ints; i++) {
		x ^= x << 13, x ^= x >> 17, x ^= x << 5;
		evals[i] = x;
	}
	Sumcheck<NUM_VARS, COMPOSITION_SIZE, false> s(evals, true);
	std::array<uint32_t, INTS> sum{}, challenge{};
	std::array<uint32_t, POINTS * INTS> points{};
	for (uint32_t round = 0; round < NUM_VARS; ++round) {
		s.this_round_messages(sum, points);
		challenge = {round * 0x01000193u + 1u, 0x85EBCA6Bu ^ round, 0xC2B2AE35u, round};
		s.move_to_next_round(challenge);
	}
	s.this_round_messages(sum, points);
	const auto end = std::chrono::high_resolution_clock::now();
	const std::chrono::duration<double, std::milli> memcpy = s.start_before_transpose - s.start_before_memcpy;
	const std::chrono::duration<double, std::milli> transpose = s.start_raw - s.start_before_transpose;
	const std::chrono::duration<double, std::milli> raw = end - s.start_raw;
	return Benchmarks{memcpy.count(), transpose.count(), raw.count()};
}

template <uint32_t NUM_VARS, uint32_t COMPOSITION_SIZE>
void benchmark(int num_runs) {
	std::cout << "NUM_VARS: " << NUM_VARS << " COMPOSITION_SIZE: " << COMPOSITION_SIZE << std::endl;
	benchmark_one_sample<NUM_VARS, COMPOSITION_SIZE>();
	double m = 0, t = 0, r = 0;
	for (int i = 0; i < num_runs; ++i) {
		const Benchmarks b = benchmark_one_sample<NUM_VARS, COMPOSITION_SIZE>();
		m += b.memcpy, t += b.transpose, r += b.raw;
	}
	m /= num_runs, t /= num_runs, r /= num_runs;
	std::cout << "Memcpy: " << m << std::endl;
	std::cout << "Transpose: " << t << std::endl;
	std::cout << "Raw: " << r << std::endl;
	std::cout << "Total: " << (m + t + r) << std::endl;
	char buf[256];
	snprintf(buf, sizeof buf, "%s{\"num_vars\": %u, \"d\": %u, \"runs\": %d, \"memcpy_ms\": %.4f, \"transpose_ms\": %.4f, \"raw_ms\": %.4f}",
	         g_json.empty() ? "" : ", ", NUM_VARS, COMPOSITION_SIZE, num_runs, m, t, r);
	g_json += buf;
}

int main() {
	benchmark<20, 2>(10);
	benchmark<20, 3>(10);
	benchmark<20, 4>(10);
	benchmark<24, 2>(5);
	benchmark<24, 3>(5);
	benchmark<24, 4>(5);
	benchmark<28, 2>(2);
	benchmark<28, 3>(2);
	benchmark<28, 4>(2);
	std::cout << "{\"harness\": \"tools/cpp/benchmark_sumcheck.cpp (benchmark.cu:12-85 on the C++ mirror)\", \"results\": ["
	          << g_json << "]}" << std::endl;
	return 0;
}
