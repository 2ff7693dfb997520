// Device-side compact tower arithmetic with compile-time heights (fully unrolled).
// Same field as tower.hpp (src/ulvt/finite_fields/binary_tower.cuh:35-105).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tower.hpp"

namespace bn {

// ---- GF(2^8) of the tower by log/exp tables (compact arithmetic leaves) ----
// lg[0] = 512 (logs of nonzero bytes are 0..254): a product with a zero factor indexes ex at 512 or
// above, where ex is 0, so a leaf is two log reads, an add and one exp read, with no zero test
// (the test cost two 64-bit compares, a select and SGPR mask spills per leaf).
struct Gf8Tables {
	uint16_t lg[256];
	uint8_t ex[1040];  // ex[i] = g^i for i < 510 (no modular reduction for lg[a] + lg[b]), 0 from 510 on
};
constexpr int kGf8ExOffset = 512;  // byte offset of ex in the tables
constexpr Gf8Tables make_gf8_tables() {
	Gf8Tables t{};
	uint64_t g = 2;
	for (;; g++) {  // smallest generator of the tower GF(2^8)^*
		uint64_t x = g;
		int order = 1;
		while (x != 1) {
			x = tw_mul(x, g, 3);
			order++;
		}
		if (order == 255) break;
	}
	uint64_t x = 1;
	for (int i = 0; i < 510; i++) {
		t.ex[i] = (uint8_t)x;
		if (i < 255) t.lg[x] = (uint16_t)i;
		x = tw_mul(x, g, 3);
	}
	t.lg[0] = 512;
	return t;
}
__constant__ constexpr Gf8Tables kGf8 = make_gf8_tables();
constexpr int kGf8LdsBytes = (int)sizeof(Gf8Tables);
static_assert(kGf8LdsBytes % 4 == 0 && kGf8LdsBytes == kGf8ExOffset + 1040, "GF(2^8) table layout");

// Copy the tables into (at least kGf8LdsBytes bytes of 4-byte aligned) LDS; the caller synchronises.
__device__ __forceinline__ void gf8_tables_to_lds(uint8_t* lds_tab) {
	const uint32_t* src = (const uint32_t*)&kGf8;
	for (int i = threadIdx.x; i < kGf8LdsBytes / 4; i += blockDim.x) ((uint32_t*)lds_tab)[i] = src[i];
}

__device__ __forceinline__ uint32_t gf8_mul(uint32_t a, uint32_t b, const uint8_t* tab) {
	const uint16_t* lg = (const uint16_t*)tab;
	return tab[kGf8ExOffset + lg[a] + lg[b]];
}

// multiply_alpha on the low 2^H bits of a u64 (compile-time height, no recursion at run time)
template <int H>
__device__ __forceinline__ uint64_t dmul_alpha_u64(uint64_t a) {
	if constexpr (H == 0) {
		return a & 1u;
	} else {
		constexpr int half = 1 << (H - 1);
		constexpr uint64_t m = (half >= 64) ? ~0ull : ((1ull << half) - 1ull);
		const uint64_t a0 = a & m, a1 = (a >> half) & m;
		return a1 | ((a0 ^ dmul_alpha_u64<H - 1>(a1)) << half);
	}
}

template <int H>
__device__ __forceinline__ uint32_t dmul_alpha(uint32_t a);

// Compact Karatsuba with GF(2^8) table leaves (3 <= H <= 5), values in the low 2^H bits of a u32.
template <int H>
__device__ __forceinline__ uint32_t dmul_t32(uint32_t a, uint32_t b, const uint8_t* tab) {
	if constexpr (H == 3) {
		return gf8_mul(a, b, tab);
	} else {
		constexpr int half = 1 << (H - 1);
		constexpr uint32_t m = (1u << half) - 1u;
		const uint32_t a0 = a & m, a1 = (a >> half) & m, b0 = b & m, b1 = (b >> half) & m;
		const uint32_t z0 = dmul_t32<H - 1>(a0, b0, tab);
		const uint32_t z2 = dmul_t32<H - 1>(a1, b1, tab);
		const uint32_t z1 = dmul_t32<H - 1>(a0 ^ a1, b0 ^ b1, tab) ^ z0 ^ z2;
		return (z0 ^ z2) | ((z1 ^ dmul_alpha<H - 1>(z2)) << half);
	}
}

// The same on a u64 (H <= 6): GF(2^64) splits into u32 halves, so no 64-bit shifts or masks below it.
template <int H>
__device__ __forceinline__ uint64_t dmul_t(uint64_t a, uint64_t b, const uint8_t* tab) {
	if constexpr (H <= 5) {
		return dmul_t32<H>((uint32_t)a, (uint32_t)b, tab);
	} else {
		static_assert(H == 6, "dmul_t: H <= 6 (GF(2^128): dmul128_t)");
		const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
		const uint32_t z0 = dmul_t32<5>(a0, b0, tab);
		const uint32_t z2 = dmul_t32<5>(a1, b1, tab);
		const uint32_t z1 = dmul_t32<5>(a0 ^ a1, b0 ^ b1, tab) ^ z0 ^ z2;
		return (uint64_t)(z0 ^ z2) | ((uint64_t)(z1 ^ dmul_alpha<5>(z2)) << 32);
	}
}
__device__ __forceinline__ uint4 dmul128_t(uint4 a, uint4 b, const uint8_t* tab) {
	const uint64_t a0 = (uint64_t)a.x | ((uint64_t)a.y << 32), a1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
	const uint64_t b0 = (uint64_t)b.x | ((uint64_t)b.y << 32), b1 = (uint64_t)b.z | ((uint64_t)b.w << 32);
	const uint64_t z0 = dmul_t<6>(a0, b0, tab), z2 = dmul_t<6>(a1, b1, tab);
	const uint64_t z1 = dmul_t<6>(a0 ^ a1, b0 ^ b1, tab) ^ z0 ^ z2;
	const uint64_t lo = z0 ^ z2, hi = z1 ^ dmul_alpha_u64<6>(z2);
	return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

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
