// Sumcheck<NUM_VARS> over QM31 (src/ulvt/prime_field_sumcheck/sumcheck.cuh:8-96) over the C-ABI
// (bn_qm31_sumcheck_*). Same constructor and protocol methods; the BLOCKS / THREADS_PER_BLOCK
// template arguments of this_round_messages / fold are accepted and ignored (the engine picks its
// own launch geometry). The reference restricts NUM_VARS to {1, 20, 24, 28}; any 1..28 is built.
// Like the reference's, this header defines a class named Sumcheck and is not meant to share a
// translation unit with the GF(2^128) sumcheck/sumcheck.hpp.
#pragma once

#include <array>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "../utils/common.hpp"
#include "qm31.hpp"

template <uint32_t NUM_VARS>
class Sumcheck {
	static_assert(NUM_VARS >= 1 && NUM_VARS <= 28, "NUM_VARS must be in [1, 28]");
	static constexpr uint32_t EVALS_PER_MULTILINEAR = 1u << NUM_VARS;

public:
	std::chrono::time_point<std::chrono::high_resolution_clock> start_before_memcpy;
	std::chrono::time_point<std::chrono::high_resolution_clock> start_raw;

	// evals: column 0 then column 1, 2^NUM_VARS values each (sumcheck.cuh:26-43)
	Sumcheck(const std::vector<QM31>& evals, const bool benchmarking, int device = 0) {
		if (evals.size() != 2 * (size_t)EVALS_PER_MULTILINEAR)
			throw std::invalid_argument("Sumcheck: evals must hold 2 * 2^NUM_VARS values");
		if (benchmarking) start_before_memcpy = std::chrono::high_resolution_clock::now();
		ulvt::bn_check(bn_qm31_sumcheck_create(device, NUM_VARS, reinterpret_cast<const uint32_t*>(evals.data()), &sc));
		if (benchmarking) start_raw = std::chrono::high_resolution_clock::now();
	}
	Sumcheck(const Sumcheck&) = delete;
	Sumcheck& operator=(const Sumcheck&) = delete;
	~Sumcheck() { bn_qm31_sumcheck_destroy(sc); }

	template <uint32_t BLOCKS = 0, uint32_t THREADS_PER_BLOCK = 0>
	void this_round_messages(std::array<QM31, 3>& points_span) {
		uint32_t w[12];
		ulvt::bn_check(bn_qm31_sumcheck_round_messages(sc, w));
		for (int k = 0; k < 3; k++) points_span[k] = QM31::from_words(w + 4 * k);
	}

	template <uint32_t BLOCKS = 0, uint32_t THREADS_PER_BLOCK = 0>
	void fold(QM31 challenge) {
		uint32_t w[4];
		challenge.to_words(w);
		ulvt::bn_check(bn_qm31_sumcheck_fold(sc, w));
	}

	// after NUM_VARS folds: f0(r), f1(r) (no reference counterpart; the verifier's final check)
	std::array<QM31, 2> final_values() {
		uint32_t w[8];
		ulvt::bn_check(bn_qm31_sumcheck_final_values(sc, w));
		return {QM31::from_words(w), QM31::from_words(w + 4)};
	}

private:
	bn_qm31_sumcheck* sc = nullptr;
};
