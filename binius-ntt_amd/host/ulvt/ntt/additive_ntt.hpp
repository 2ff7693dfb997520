// AdditiveNTT<T, P> (src/ulvt/ntt/additive_ntt.cuh:175-319) over the C-ABI.
//
//   AdditiveNTT<uint32_t, FanPaarTowerField<5>>            GF(2^32), as the reference
//   AdditiveNTT<unsigned __int128, FanPaarTowerField<7>>   GF(2^128) (4 little-endian u32 limbs)
//
// Construction builds the plan (subspace table precompute + device staging, the reference ctor
// 178-199); apply() has the reference's host semantics (201-265): returns false, with no other
// effect, unless in.size == 2^log_h and in.order == IN_ORDER; otherwise writes 2^(log_h+log_rate)
// elements coset-major into out, sets out.order = IN_ORDER and returns after a full sync.
#pragma once

#include <cstdint>
#include <utility>

#include "../finite_fields/binary_tower.hpp"
#include "../utils/common.hpp"
#include "nttconf.hpp"

template <typename T, typename P>
class AdditiveNTT {
	static_assert(sizeof(T) * 8 == P::N_BITS(), "element type must match the field policy");

public:
	explicit AdditiveNTT(const AdditiveNTTConf<T, P>& conf, int device = 0) : ntt_conf(conf) {
		ulvt::bn_check(bn_antt_plan_create(device, (int)P::N_BITS(), conf.log_h, conf.log_rate, &plan));
	}
	AdditiveNTT(const AdditiveNTT&) = delete;
	AdditiveNTT& operator=(const AdditiveNTT&) = delete;
	~AdditiveNTT() { bn_antt_plan_destroy(plan); }

	bool apply(const NTTData<T>& input, NTTData<T>& output) {
		if (input.size != ((size_t)1 << ntt_conf.log_h) || input.order != DataOrder::IN_ORDER) return false;
		if (output.size < ((size_t)1 << (ntt_conf.log_h + ntt_conf.log_rate))) return false;
		ulvt::bn_check(bn_antt_forward_host(plan, input.data.get(), input.size, output.data.get()));
		output.order = DataOrder::IN_ORDER;
		return true;
	}

	// Device-resident transforms (no reference counterpart): `batch` transforms, asynchronous
	// on `stream` (a hipStream_t).
	void forward_device(const void* d_in, void* d_out, size_t batch = 1, void* stream = nullptr) {
		ulvt::bn_check(bn_antt_forward_device(plan, d_in, d_out, batch, stream));
	}

	// 0: compact tiles, per-butterfly twiddles (default for log_h < 12); 1: bitsliced LDS tiles;
	// 4: bitsliced register tiles; 5: 4 for the GF(2^8)-twiddle passes, 1 for the others (default
	// for log_h >= 12)
	void set_variant(int variant) { ulvt::bn_check(bn_antt_plan_set_variant(plan, variant)); }

	const AdditiveNTTConf<T, P>& conf() const { return ntt_conf; }

private:
	AdditiveNTTConf<T, P> ntt_conf;
	bn_antt_plan* plan = nullptr;
};
