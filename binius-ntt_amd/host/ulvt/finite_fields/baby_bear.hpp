// BB31, the BabyBear prime field p = 15 * 2^27 + 1 (src/ulvt/finite_fields/baby_bear.cuh, which
// aliases RISC Zero's Fp, risc0_baby_bear.h:40-192), host mirror. The reference stores values
// Montgomery-encoded; the mirror stores them canonical, so the 4-byte element *is* asUInt32() and
// arrays of BB31 go to the C-ABI (bn_bb31_ntt_*) as plain u32 words. BB31(x) reduces x mod p, as
// the reference's encode does for any u32.
#pragma once

#include <cstddef>
#include <cstdint>

class BB31 {
public:
	static constexpr uint32_t P = 15u * (1u << 27) + 1u;

	constexpr BB31() : val(0) {}
	constexpr BB31(uint32_t v) : val(v % P) {}

	static constexpr BB31 one() { return BB31(1u); }
	static constexpr BB31 zero() { return BB31(0u); }
	constexpr uint32_t asUInt32() const { return val; }

	constexpr BB31 operator+(BB31 r) const { return raw(val + r.val >= P ? val + r.val - P : val + r.val); }
	constexpr BB31 operator-(BB31 r) const { return raw(val >= r.val ? val - r.val : val + P - r.val); }
	constexpr BB31 operator-() const { return raw(val ? P - val : 0u); }
	constexpr BB31 operator*(BB31 r) const { return raw((uint32_t)((uint64_t)val * r.val % P)); }
	BB31& operator+=(BB31 r) { return *this = *this + r; }
	BB31& operator-=(BB31 r) { return *this = *this - r; }
	BB31& operator*=(BB31 r) { return *this = *this * r; }
	constexpr bool operator==(BB31 r) const { return val == r.val; }
	constexpr bool operator!=(BB31 r) const { return val != r.val; }

	// Fp::pow / Fp::inv (risc0_baby_bear.h:133-149); inv(0) == 0 as there
	static constexpr BB31 pow(BB31 x, size_t n) {
		BB31 r = one();
		while (n) {
			if (n & 1) r = r * x;
			x = x * x;
			n >>= 1;
		}
		return r;
	}
	static constexpr BB31 inv(BB31 x) { return pow(x, P - 2); }

private:
	static constexpr BB31 raw(uint32_t v) {
		BB31 b;
		b.val = v;
		return b;
	}
	uint32_t val;
};

static_assert(sizeof(BB31) == 4, "BB31 is one u32 word");
