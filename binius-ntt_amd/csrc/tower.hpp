// Binary tower field GF(2^(2^h)) in compact form, host + device.
//
// Tower (Fan-Paar / Wiedemann, as src/ulvt/finite_fields/binary_tower.cuh:19-128):
//   level 0 = GF(2); level h = level(h-1)[X_{h-1}] / (X^2 + alpha_{h-1} X + 1),
//   alpha_0 = 1, alpha_h = X_{h-1}. An element of level h is 2^h bits: low half = the
//   level-(h-1) coefficient of 1, high half = the coefficient of X_{h-1}.
// Used on the host for twiddle precomputation and on the device by the v0 kernels,
// the compact GF(2^128) multiply and the sumcheck verifier helpers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bn {

// multiply by alpha of level h (i.e. by X_{h-1}); (a0 + a1 X)X = a1 + (a0 + a1 alpha_{h-1}) X
__host__ __device__ constexpr uint64_t tw_mul_alpha(uint64_t a, int h) {
	if (h == 0) return a & 1;
	const int half = 1 << (h - 1);
	const uint64_t m = half >= 64 ? ~0ull : ((1ull << half) - 1);
	const uint64_t a0 = a & m, a1 = (a >> half) & m;
	return a1 | ((a0 ^ tw_mul_alpha(a1, h - 1)) << half);
}

// Karatsuba recursion to GF(2).
__host__ __device__ constexpr uint64_t tw_mul(uint64_t a, uint64_t b, int h) {
	if (h == 0) return a & b & 1;
	const int half = 1 << (h - 1);
	const uint64_t m = half >= 64 ? ~0ull : ((1ull << half) - 1);
	const uint64_t a0 = a & m, a1 = (a >> half) & m, b0 = b & m, b1 = (b >> half) & m;
	const uint64_t z0 = tw_mul(a0, b0, h - 1);
	const uint64_t z2 = tw_mul(a1, b1, h - 1);
	const uint64_t z1 = tw_mul(a0 ^ a1, b0 ^ b1, h - 1) ^ z0 ^ z2;
	return (z0 ^ z2) | ((z1 ^ tw_mul_alpha(z2, h - 1)) << half);
}

__host__ __device__ constexpr uint64_t tw_square(uint64_t a, int h) { return tw_mul(a, a, h); }

__host__ __device__ constexpr uint64_t tw_inv(uint64_t a, int h) {
	if (h == 0) return a & 1;
	const int half = 1 << (h - 1);
	const uint64_t m = half >= 64 ? ~0ull : ((1ull << half) - 1);
	if ((a >> half) == 0) return tw_inv(a, h - 1);
	const uint64_t a0 = a & m, a1 = (a >> half) & m;
	const uint64_t inter = a0 ^ tw_mul_alpha(a1, h - 1);
	const uint64_t delta = tw_mul(a0, inter, h - 1) ^ tw_square(a1, h - 1);
	const uint64_t dinv = tw_inv(delta, h - 1);
	return tw_mul(dinv, inter, h - 1) | (tw_mul(dinv, a1, h - 1) << half);
}

// GF(2^128) as (lo, hi) u64 pair; schoolbook top level like tower_height_7_mul
// (src/ulvt/sumcheck/test/utils/tower_7_mul.cu:4-20), Karatsuba below.
struct u128p {
	uint64_t lo, hi;
};
__host__ __device__ inline u128p tw_mul128(u128p a, u128p b) {
	const uint64_t z0 = tw_mul(a.lo, b.lo, 6);
	const uint64_t z2 = tw_mul(a.hi, b.hi, 6);
	const uint64_t z1 = tw_mul(a.lo ^ a.hi, b.lo ^ b.hi, 6) ^ z0 ^ z2;
	return u128p{z0 ^ z2, z1 ^ tw_mul_alpha(z2, 6)};
}

// Host-only fast path (round claims, interpolation): the Karatsuba recursion stops at GF(2^8),
// whose products come from a 64 KiB table (built on first use), so a GF(2^128) product is 27
// lookups per GF(2^64) sub-product instead of 729 GF(2) leaves.
__host__ inline const uint8_t* tw_mul8_table() {
	static uint8_t* t = [] {
		static uint8_t tab[256 * 256];
		for (int a = 0; a < 256; a++)
			for (int b = 0; b < 256; b++) tab[a * 256 + b] = (uint8_t)tw_mul((uint64_t)a, (uint64_t)b, 3);
		return tab;
	}();
	return t;
}
// The recursion unrolled at compile time (a runtime-h recursion cost ~1.6 us per GF(2^128)
// product: 26 us per 4-point interpolation, on the critical path of every sumcheck round)
template <int H>
__host__ inline uint64_t tw_alpha_h(uint64_t a) {
	if constexpr (H == 0) {
		return a & 1;
	} else {
		constexpr int half = 1 << (H - 1);
		constexpr uint64_t m = half >= 64 ? ~0ull : ((1ull << half) - 1);
		const uint64_t a0 = a & m, a1 = (a >> half) & m;
		return a1 | ((a0 ^ tw_alpha_h<H - 1>(a1)) << half);
	}
}
template <int H>
__host__ inline uint64_t tw_mul_h(const uint8_t* tab, uint64_t a, uint64_t b) {
	if constexpr (H <= 3) {
		return tab[(a & 0xff) * 256 + (b & 0xff)];
	} else {
		constexpr int half = 1 << (H - 1);
		constexpr uint64_t m = half >= 64 ? ~0ull : ((1ull << half) - 1);
		const uint64_t a0 = a & m, a1 = (a >> half) & m, b0 = b & m, b1 = (b >> half) & m;
		const uint64_t z0 = tw_mul_h<H - 1>(tab, a0, b0);
		const uint64_t z2 = tw_mul_h<H - 1>(tab, a1, b1);
		const uint64_t z1 = tw_mul_h<H - 1>(tab, a0 ^ a1, b0 ^ b1) ^ z0 ^ z2;
		return (z0 ^ z2) | ((z1 ^ tw_alpha_h<H - 1>(z2)) << half);
	}
}
__host__ inline uint64_t tw_mul_host(uint64_t a, uint64_t b, int h) {
	const uint8_t* tab = tw_mul8_table();
	switch (h) {
		case 4: return tw_mul_h<4>(tab, a, b);
		case 5: return tw_mul_h<5>(tab, a, b);
		case 6: return tw_mul_h<6>(tab, a, b);
		default: return h <= 3 ? tw_mul_h<3>(tab, a, b) : tw_mul(a, b, h);
	}
}
__host__ inline u128p tw_mul128_host(u128p a, u128p b) {
	const uint8_t* tab = tw_mul8_table();
	const uint64_t z0 = tw_mul_h<6>(tab, a.lo, b.lo);
	const uint64_t z2 = tw_mul_h<6>(tab, a.hi, b.hi);
	const uint64_t z1 = tw_mul_h<6>(tab, a.lo ^ a.hi, b.lo ^ b.hi) ^ z0 ^ z2;
	return u128p{z0 ^ z2, z1 ^ tw_alpha_h<6>(z2)};
}

}  // namespace bn
