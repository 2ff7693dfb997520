// Sumcheck<NUM_VARS, COMPOSITION_SIZE, DATA_IS_TRANSPOSED> (src/ulvt/sumcheck/sumcheck.cuh:10-301)
// over the C-ABI. Same constructor and the same two protocol methods; the evaluations are
// COMPOSITION_SIZE columns of 4 * 2^NUM_VARS words, compact (little-endian limbs) or bitsliced
// 128-word batches when DATA_IS_TRANSPOSED (README.md:38-45 of the reference).
#pragma once

#include <array>
#include <chrono>
#include <cstdint>
#include <string>
#include <vector>

#include "../utils/common.hpp"

template <uint32_t NUM_VARS, uint32_t COMPOSITION_SIZE, bool DATA_IS_TRANSPOSED>
class Sumcheck {
	static constexpr uint32_t INTS_PER_VALUE = 4;
	static constexpr uint32_t INTERPOLATION_POINTS = COMPOSITION_SIZE + 1;

public:
	// the reference constructor's phase timestamps (sumcheck.cuh:76-80, 88, 94, 124), read by its
	// benchmark driver (bench/benchmark.cu:39-43): Memcpy = before_transpose - before_memcpy,
	// Transpose = raw - before_transpose
	std::chrono::time_point<std::chrono::high_resolution_clock> start_before_memcpy;
	std::chrono::time_point<std::chrono::high_resolution_clock> start_before_transpose;
	std::chrono::time_point<std::chrono::high_resolution_clock> start_raw;

	Sumcheck(const std::vector<uint32_t>& evals, bool benchmarking, int device = 0) {
		if (evals.size() < (size_t)INTS_PER_VALUE * ((size_t)1 << NUM_VARS) * COMPOSITION_SIZE)
			throw ulvt::BnError(BN_ERR_INVALID, "Sumcheck: evals shorter than COMPOSITION_SIZE * 4 * 2^NUM_VARS words");
		if (benchmarking) start_before_memcpy = std::chrono::high_resolution_clock::now();
		// host -> HBM copy (synchronous), then the device bit-transpose of compact input
		ulvt::bn_check(bn_sumcheck_create_staged(device, NUM_VARS, COMPOSITION_SIZE, DATA_IS_TRANSPOSED ? 1 : 0, evals.data(), &sc));
		if (benchmarking) start_before_transpose = std::chrono::high_resolution_clock::now();
		const int rc = bn_sumcheck_prepare(sc);
		if (rc != BN_OK) {
			const ulvt::BnError err(rc, std::string("binius-ntt-amd: ") + bn_last_error());
			bn_sumcheck_destroy(sc);
			throw err;
		}
		if (benchmarking) start_raw = std::chrono::high_resolution_clock::now();
	}
	Sumcheck(const Sumcheck&) = delete;
	Sumcheck& operator=(const Sumcheck&) = delete;
	~Sumcheck() { bn_sumcheck_destroy(sc); }

	void this_round_messages(std::array<uint32_t, INTS_PER_VALUE>& sum,
							 std::array<uint32_t, INTERPOLATION_POINTS * INTS_PER_VALUE>& points) {
		ulvt::bn_check(bn_sumcheck_round_messages(sc, sum.data(), points.data()));
	}

	void move_to_next_round(const std::array<uint32_t, INTS_PER_VALUE>& challenge) {
		ulvt::bn_check(bn_sumcheck_move_to_next_round(sc, challenge.data()));
	}

	// Multi-GPU sharding and the device-resident round exchange (this build's extensions; see
	// binius_ntt_amd.h and INTEGRATION.md section 4). A shard prover's round messages are partial:
	// the caller XORs them over the ranks; once needs_gather(), the ranks' exported batches are
	// concatenated rank-major and imported by every rank, which then continues unsharded
	// (the reference's hand-over at 32 evaluations, sumcheck.cuh:283-297).
	void set_shard(int rank, int world) { ulvt::bn_check(bn_sumcheck_set_shard(sc, rank, world)); }
	bool needs_gather() const {
		int flag = 0;
		ulvt::bn_check(bn_sumcheck_needs_gather(sc, &flag));
		return flag != 0;
	}
	std::vector<uint32_t> export_shard() const {
		std::vector<uint32_t> out((size_t)COMPOSITION_SIZE * 128);
		ulvt::bn_check(bn_sumcheck_export_shard(sc, out.data(), out.size()));
		return out;
	}
	void import_gathered(const std::vector<uint32_t>& words, int world) {
		ulvt::bn_check(bn_sumcheck_import_gathered(sc, words.data(), words.size(), world));
	}
	// device sink (>= 37 words of device memory): the raw points and the flag word of every later
	// round; round_messages_sink() queues the round on stream() without waiting for it
	void set_message_sink(void* d_words) { ulvt::bn_check(bn_sumcheck_set_message_sink(sc, d_words)); }
	void round_messages_sink() { ulvt::bn_check(bn_sumcheck_round_messages_sink(sc)); }
	void* stream() const {
		void* st = nullptr;
		ulvt::bn_check(bn_sumcheck_stream(sc, &st));
		return st;
	}

private:
	bn_sumcheck* sc = nullptr;
};
