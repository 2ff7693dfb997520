// Packed-subfield operations of the reference (src/ulvt/finite_fields/binary_tower_simd.cuh:77-150)
// for host code: a 32-bit word read as 32 / 2^HEIGHT packed GF(2^(2^HEIGHT)) elements.
//   mul_binary_tower_32b_simd<HEIGHT>(a, b)  lane-wise products (bn_mul_binary_tower_32b_simd)
//   interleave_32b<HEIGHT>(a, b) -> (c, d)   2^HEIGHT-bit block interleave (bn_interleave_32b)
//   xor_adjacent_32b<HEIGHT>(a)              adjacent-block sums (bn_xor_adjacent_32b)
// Device batches of all three: bn_packed32_device.
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>

#include "../utils/common.hpp"

template <size_t HEIGHT>
inline uint32_t mul_binary_tower_32b_simd(uint32_t a, uint32_t b) {
	static_assert(HEIGHT <= 5, "packed subfields of a 32-bit word: HEIGHT <= 5");
	uint32_t out = 0;
	ulvt::bn_check(bn_mul_binary_tower_32b_simd((int)HEIGHT, a, b, &out));
	return out;
}

template <size_t HEIGHT>
inline std::pair<uint32_t, uint32_t> interleave_32b(uint32_t a, uint32_t b) {
	static_assert(HEIGHT < 5, "interleave_32b requires tower height < 5");
	uint32_t c = 0, d = 0;
	ulvt::bn_check(bn_interleave_32b((int)HEIGHT, a, b, &c, &d));
	return {c, d};
}

template <size_t HEIGHT>
inline uint32_t xor_adjacent_32b(uint32_t a) {
	static_assert(HEIGHT < 5, "xor_adjacent_32b requires tower height < 5");
	uint32_t out = 0;
	ulvt::bn_check(bn_xor_adjacent_32b((int)HEIGHT, a, &out));
	return out;
}
