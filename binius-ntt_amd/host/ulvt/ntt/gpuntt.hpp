// NTTConfRad2<E> (src/ulvt/ntt/nttconf.cuh:25-47) and NTT<E> (src/ulvt/ntt/gpuntt.cuh:126-209)
// over the C-ABI (bn_bb31_ntt_*): the BabyBear radix-2 NTT, the prime-field sibling of
// AdditiveNTT. apply() keeps the reference's host semantics: the input may be IN_ORDER (or
// INVALID, which the reference also bit-reverses) or BIT_REVERSED, the output is the
// natural-order DFT X[k] = sum_j x[j] w^(jk), w = generator^(2^(log_group_order - log_inp_size)),
// and output.order becomes IN_ORDER. The reference's ASSERTs become std::invalid_argument.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <type_traits>

#include "../finite_fields/baby_bear.hpp"
#include "../utils/common.hpp"
#include "nttconf.hpp"

template <typename E>
class NTTConfRad2 {
public:
	E generator;
	uint32_t log_group_order;
	int log_inp_size;

	NTTConfRad2(E gen, uint32_t log_grp_order, int inp_log_size)
		: generator(gen), log_group_order(log_grp_order), log_inp_size(inp_log_size) {
		if (!(inp_log_size >= 1)) throw std::invalid_argument("NTTConfRad2: inp_log_size >= 1");
		if (!(inp_log_size <= 27)) throw std::invalid_argument("NTTConfRad2: inp_log_size <= 27");
		if (!(log_grp_order >= (uint32_t)inp_log_size)) throw std::invalid_argument("NTTConfRad2: log_grp_order >= inp_log_size");
	}
};

template <typename E>
class NTT {
	static_assert(std::is_same<E, BB31>::value, "NTT<E>: the engine implements E = BB31 (as the reference's tests)");

public:
	explicit NTT(const NTTConfRad2<E>& nttconf, int device = 0) : ntt_conf(nttconf) {
		ulvt::bn_check(bn_bb31_ntt_plan_create(device, nttconf.generator.asUInt32(), (int)nttconf.log_group_order,
											   nttconf.log_inp_size, &plan));
	}
	NTT(const NTT&) = delete;
	NTT& operator=(const NTT&) = delete;
	~NTT() { bn_bb31_ntt_plan_destroy(plan); }

	void apply(const NTTData<E>& input, NTTData<E>& output) {
		const size_t n = (size_t)1 << ntt_conf.log_inp_size;
		if (input.size != n) throw std::invalid_argument("NTT::apply: input.size must be 2^log_inp_size (gpuntt.cuh:159)");
		if (output.size != n) throw std::invalid_argument("NTT::apply: output.size must be 2^log_inp_size (gpuntt.cuh:181)");
		ulvt::bn_check(bn_bb31_ntt_forward_host(plan, reinterpret_cast<const uint32_t*>(input.data.get()), n,
												reinterpret_cast<uint32_t*>(output.data.get()),
												input.order == DataOrder::BIT_REVERSED ? 1 : 0));
		output.order = DataOrder::IN_ORDER;
	}

	// Device-resident transforms (no reference counterpart): `batch` transforms of 2^log_inp_size
	// canonical u32 words, asynchronous on `stream` (a hipStream_t).
	void forward_device(const uint32_t* d_in, uint32_t* d_out, size_t batch = 1, bool bit_reversed = false,
						void* stream = nullptr) {
		ulvt::bn_check(bn_bb31_ntt_forward_device(plan, d_in, d_out, batch, bit_reversed ? 1 : 0, stream));
	}

	const NTTConfRad2<E>& conf() const { return ntt_conf; }

private:
	NTTConfRad2<E> ntt_conf;
	bn_bb31_ntt_plan* plan = nullptr;
};
