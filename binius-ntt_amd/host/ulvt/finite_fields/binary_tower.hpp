// Field policies of the reference (src/ulvt/finite_fields/binary_tower.cuh:19-262) for host code:
// FanPaarTowerField<H> on uint32_t (H <= 5), plus FanPaarTowerField<7> on unsigned __int128 —
// GF(2^128), the field of this build's NTT and sumcheck (the reference's only 128-bit multiply is
// tower_height_7_mul, src/ulvt/sumcheck/test/utils/tower_7_mul.cu:4-20).
//
// Static API as the reference: ZERO() ONE() N_BITS() add multiply square inverse. Host
// arithmetic only (used for twiddle-style host precomputation and verifier-side checks); the
// device kernels live behind the C-ABI.
#pragma once

#include <cstddef>
#include <cstdint>

namespace ulvt_tower {

// level h = level(h-1)[X] / (X^2 + alpha X + 1), alpha_0 = 1, alpha_h = X_{h-1}
constexpr uint64_t mul_alpha(uint64_t a, int h) {
	if (h == 0) return a & 1;
	const int half = 1 << (h - 1);
	const uint64_t m = half >= 64 ? ~0ull : ((1ull << half) - 1);
	const uint64_t a0 = a & m, a1 = (a >> half) & m;
	return a1 | ((a0 ^ mul_alpha(a1, h - 1)) << half);
}

constexpr uint64_t mul(uint64_t a, uint64_t b, int h) {
	if (h == 0) return a & b & 1;
	const int half = 1 << (h - 1);
	const uint64_t m = half >= 64 ? ~0ull : ((1ull << half) - 1);
	const uint64_t a0 = a & m, a1 = (a >> half) & m, b0 = b & m, b1 = (b >> half) & m;
	const uint64_t z0 = mul(a0, b0, h - 1), z2 = mul(a1, b1, h - 1);
	const uint64_t z1 = mul(a0 ^ a1, b0 ^ b1, h - 1) ^ z0 ^ z2;
	return (z0 ^ z2) | ((z1 ^ mul_alpha(z2, h - 1)) << half);
}

constexpr uint64_t inv(uint64_t a, int h) {
	if (h == 0) return a & 1;
	const int half = 1 << (h - 1);
	const uint64_t m = half >= 64 ? ~0ull : ((1ull << half) - 1);
	if ((a >> half) == 0) return inv(a, h - 1);
	const uint64_t a0 = a & m, a1 = (a >> half) & m;
	const uint64_t inter = a0 ^ mul_alpha(a1, h - 1);
	const uint64_t delta = mul(a0, inter, h - 1) ^ mul(a1, a1, h - 1);
	const uint64_t dinv = inv(delta, h - 1);
	return mul(dinv, inter, h - 1) | (mul(dinv, a1, h - 1) << half);
}

using u128 = unsigned __int128;

inline u128 mul128(u128 a, u128 b) {
	const uint64_t al = (uint64_t)a, ah = (uint64_t)(a >> 64), bl = (uint64_t)b, bh = (uint64_t)(b >> 64);
	const uint64_t z0 = mul(al, bl, 6), z2 = mul(ah, bh, 6);
	const uint64_t z1 = mul(al ^ ah, bl ^ bh, 6) ^ z0 ^ z2;
	return (u128)(z0 ^ z2) | ((u128)(z1 ^ mul_alpha(z2, 6)) << 64);
}

inline u128 inv128(u128 a) {
	const uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64);
	if (a1 == 0) return inv(a0, 6);
	const uint64_t inter = a0 ^ mul_alpha(a1, 6);
	const uint64_t delta = mul(a0, inter, 6) ^ mul(a1, a1, 6);
	const uint64_t dinv = inv(delta, 6);
	return (u128)mul(dinv, inter, 6) | ((u128)mul(dinv, a1, 6) << 64);
}

}  // namespace ulvt_tower

template <size_t HEIGHT>
class FanPaarTowerField {
	static_assert(HEIGHT <= 5, "uint32_t policy: height <= 5 (use FanPaarTowerField<7> for GF(2^128))");

public:
	using T = uint32_t;
	static constexpr uint32_t ONE() { return 1; }
	static constexpr uint32_t ZERO() { return 0; }
	static constexpr uint32_t N_BITS() { return 1u << HEIGHT; }
	static constexpr bool is_valid(uint32_t a) { return HEIGHT == 5 || (a >> N_BITS()) == 0; }
	static constexpr uint32_t add(uint32_t a, uint32_t b) { return a ^ b; }
	static constexpr uint32_t multiply(uint32_t a, uint32_t b) { return (uint32_t)ulvt_tower::mul(a, b, HEIGHT); }
	static constexpr uint32_t square(uint32_t a) { return multiply(a, a); }
	static constexpr uint32_t inverse(uint32_t a) { return (uint32_t)ulvt_tower::inv(a, HEIGHT); }
	static constexpr uint32_t multiply_alpha(uint32_t a) { return (uint32_t)ulvt_tower::mul_alpha(a, HEIGHT); }
};

template <>
class FanPaarTowerField<7> {
public:
	using T = unsigned __int128;
	static constexpr T ONE() { return 1; }
	static constexpr T ZERO() { return 0; }
	static constexpr uint32_t N_BITS() { return 128; }
	static constexpr bool is_valid(T) { return true; }
	static constexpr T add(T a, T b) { return a ^ b; }
	static T multiply(T a, T b) { return ulvt_tower::mul128(a, b); }
	static T square(T a) { return multiply(a, a); }
	static T inverse(T a) { return ulvt_tower::inv128(a); }
};
