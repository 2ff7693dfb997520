// BitsliceUtils<W> static helpers (src/ulvt/utils/bitslicing.cuh:8-75), host mirror.
// A batch holds 32 elements of W bits: compact = element e at words [e*W/32, (e+1)*W/32)
// (little-endian limbs); bitsliced = word i holds bit i of every element, element e in bit e.
// The device transposes are bn_bitslice_device.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>

template <size_t W>
class BitsliceUtils {
	static_assert(W % 32 == 0 && W >= 32, "W must be a multiple of 32");
	static constexpr size_t LIMBS = W / 32;

public:
	static void bitslice_transpose(uint32_t batch[W]) {
		uint32_t out[W] = {};
		for (size_t e = 0; e < 32; e++)
			for (size_t i = 0; i < W; i++) out[i] |= ((batch[e * LIMBS + i / 32] >> (i % 32)) & 1u) << e;
		std::memcpy(batch, out, sizeof(out));
	}

	static void bitslice_untranspose(uint32_t batch[W]) {
		uint32_t out[W] = {};
		for (size_t i = 0; i < W; i++)
			for (size_t e = 0; e < 32; e++) out[e * LIMBS + i / 32] |= ((batch[i] >> e) & 1u) << (i % 32);
		std::memcpy(batch, out, sizeof(out));
	}

	// every element of the batch = value (bitsliced: word i is all-ones iff bit i of value is set)
	static void repeat_value_bitsliced(uint32_t batch[W], const uint32_t value[LIMBS]) {
		for (size_t i = 0; i < W; i++) batch[i] = 0u - ((value[i / 32] >> (i % 32)) & 1u);
	}
};
