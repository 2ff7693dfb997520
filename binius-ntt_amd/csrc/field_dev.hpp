// Device-side compact tower arithmetic with compile-time heights (fully unrolled).
// Same field as tower.hpp (src/ulvt/finite_fields/binary_tower.cuh:35-105).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bn {

template <int H>
__device__ __forceinline__ uint32_t dmul_alpha(uint32_t a) {
	if constexpr (H == 0) {
		return a & 1u;
	} else {
		constexpr int half = 1 << (H - 1);
		constexpr uint32_t m = (half >= 32) ? 0xffffffffu : ((1u << half) - 1u);
		const uint32_t a0 = a & m, a1 = (a >> half) & m;
		return a1 | ((a0 ^ dmul_alpha<H - 1>(a1)) << half);
	}
}

// Karatsuba down to GF(2^4), GF(16) products by a 4x4 schoolbook-with-reduction network.
template <int H>
__device__ __forceinline__ uint32_t dmul(uint32_t a, uint32_t b) {
	if constexpr (H == 0) {
		return a & b & 1u;
	} else if constexpr (H == 1) {
		// GF(4): (a0 + a1 X)(b0 + b1 X), X^2 = X + 1
		const uint32_t a0 = a & 1, a1 = (a >> 1) & 1, b0 = b & 1, b1 = (b >> 1) & 1;
		const uint32_t z0 = a0 & b0, z2 = a1 & b1, z1 = ((a0 ^ a1) & (b0 ^ b1)) ^ z0 ^ z2;
		return (z0 ^ z2) | ((z1 ^ z2) << 1);
	} else {
		constexpr int half = 1 << (H - 1);
		constexpr uint32_t m = (1u << half) - 1u;
		const uint32_t a0 = a & m, a1 = (a >> half) & m, b0 = b & m, b1 = (b >> half) & m;
		const uint32_t z0 = dmul<H - 1>(a0, b0);
		const uint32_t z2 = dmul<H - 1>(a1, b1);
		const uint32_t z1 = dmul<H - 1>(a0 ^ a1, b0 ^ b1) ^ z0 ^ z2;
		return (z0 ^ z2) | ((z1 ^ dmul_alpha<H - 1>(z2)) << half);
	}
}

// GF(2^64) on u64 and GF(2^128) on 4 x u32 (tower_height_7_mul semantics).
__device__ __forceinline__ uint64_t dmul64_alpha(uint64_t a) {
	const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
	return (uint64_t)a1 | ((uint64_t)(a0 ^ dmul_alpha<5>(a1)) << 32);
}
__device__ __forceinline__ uint64_t dmul64(uint64_t a, uint64_t b) {
	const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
	const uint32_t z0 = dmul<5>(a0, b0), z2 = dmul<5>(a1, b1);
	const uint32_t z1 = dmul<5>(a0 ^ a1, b0 ^ b1) ^ z0 ^ z2;
	return (uint64_t)(z0 ^ z2) | ((uint64_t)(z1 ^ dmul_alpha<5>(z2)) << 32);
}
__device__ __forceinline__ uint4 dmul128(uint4 a, uint4 b) {
	const uint64_t a0 = (uint64_t)a.x | ((uint64_t)a.y << 32), a1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
	const uint64_t b0 = (uint64_t)b.x | ((uint64_t)b.y << 32), b1 = (uint64_t)b.z | ((uint64_t)b.w << 32);
	const uint64_t z0 = dmul64(a0, b0), z2 = dmul64(a1, b1);
	const uint64_t z1 = dmul64(a0 ^ a1, b0 ^ b1) ^ z0 ^ z2;
	const uint64_t lo = z0 ^ z2, hi = z1 ^ dmul64_alpha(z2);
	return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

}  // namespace bn
