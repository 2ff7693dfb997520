// multiply_unrolled<HEIGHT> of the reference
// (src/ulvt/finite_fields/circuit_generator/unrolled/binary_tower_unrolled.cuh:4-5) for host code:
// 32 bitsliced GF(2^(2^HEIGHT)) products, 2^HEIGHT words per operand (word i = bit i of the 32
// elements, element e in bit e), alias-safe (destination may be an operand, core.cu:21).
// Computed by libbinius_ntt_amd.so's generated circuits (bn_multiply_unrolled); device batches
// go through bn_multiply_unrolled_device.
#pragma once

#include <cstdint>

#include "../../../utils/common.hpp"

template <int HEIGHT>
inline void multiply_unrolled(const uint32_t* field_element_a, const uint32_t* field_element_b, uint32_t* destination) {
	static_assert(HEIGHT >= 2 && HEIGHT <= 7, "multiply_unrolled is built for tower heights 2..7");
	ulvt::bn_check(bn_multiply_unrolled(HEIGHT, field_element_a, field_element_b, destination));
}
