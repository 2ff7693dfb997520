// Bitsliced layout helpers (device): 32x32 bit transposes in registers and the
// BitsliceUtils<128> block mapping of the reference (src/ulvt/utils/bitslicing.cuh:32-64):
// compact element e, limb l (word 4e+l of a 128-word block) <-> word 32l+i, bit e.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bitsliced_gen.hpp"

namespace bn {

// A uniform value (a constant, a loop-uniform mask or shift count) as a VGPR operand. On gfx950 a
// VALU instruction that reads an SGPR issues at ~0.21 wave-instructions per SIMD-cycle against
// ~0.35 for VGPR / inline-constant operands (tools/microbench5.hip), and the compiler puts every
// non-inline constant and uniform value of these loops into an SGPR: the empty asm ties the value
// to a VGPR the compiler cannot see through, so it stays there (and is hoisted out of the loops).
__device__ __forceinline__ uint32_t vgpr(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
	asm("" : "=v"(x) : "0"(x));
#endif
	return x;
}

// In-place 32x32 bit transpose (recursive block swap): afterwards bit j of word i is bit i of
// word j of the input. Fully unrolled: all indices are compile-time constants. The 16- and 8-bit
// levels are byte permutes (one v_perm_b32 per word), the others two selects (v_bitop3) and two
// shifts per word pair: 256 instructions instead of 400 for the XOR-swap form.
__device__ __forceinline__ void transpose32(uint32_t* a) {
	// masks and byte selectors as VGPR operands (see vgpr())
	const uint32_t m2 = vgpr(0x0F0F0F0Fu), m1 = vgpr(0x33333333u), m0 = vgpr(0x55555555u);
	const uint32_t p4a = vgpr(0x05040100u), p4b = vgpr(0x07060302u), p3a = vgpr(0x06020400u), p3b = vgpr(0x07030501u);
#pragma unroll
	for (int lj = 4; lj >= 0; lj--) {
		const int j = 1 << lj;
		const uint32_t m = lj == 2 ? m2 : lj == 1 ? m1 : m0;
#pragma unroll
		for (int kk = 0; kk < 16; kk++) {
			const int k = ((kk & ~(j - 1)) << 1) | (kk & (j - 1));  // the 16 words with bit lj clear
			const uint32_t x = a[k], y = a[k + j];
			if (lj >= 3) {
				// v_perm_b32(S0 = y, S1 = x, sel): selector bytes 0-3 pick x's bytes, 4-7 y's
				a[k] = __builtin_amdgcn_perm(y, x, lj == 4 ? p4a : p3a);
				a[k + j] = __builtin_amdgcn_perm(y, x, lj == 4 ? p4b : p3b);
			} else {
				a[k] = __builtin_amdgcn_bitop3_b32(m, x, y << j, 0xCA);      // m ? x : y << j
				a[k + j] = __builtin_amdgcn_bitop3_b32(m, x >> j, y, 0xCA);  // m ? x >> j : y
			}
		}
	}
}

__device__ __forceinline__ void bs_transpose128(uint32_t* r) {
	uint32_t t[128];
#pragma unroll
	for (int i = 0; i < 128; i++) t[32 * (i & 3) + (i >> 2)] = r[i];
#pragma unroll
	for (int c = 0; c < 4; c++) transpose32(t + 32 * c);
#pragma unroll
	for (int i = 0; i < 128; i++) r[i] = t[i];
}

__device__ __forceinline__ void bs_untranspose128(uint32_t* r) {
	uint32_t t[128];
#pragma unroll
	for (int i = 0; i < 128; i++) t[i] = r[i];
#pragma unroll
	for (int c = 0; c < 4; c++) transpose32(t + 32 * c);
#pragma unroll
	for (int i = 0; i < 128; i++) r[4 * (i & 31) + (i >> 5)] = t[i];
}

// 32 GF(2^128) products on bitsliced blocks (multiply_unrolled<7> semantics), alias-safe.
__device__ __forceinline__ void bs_mul128(const uint32_t* a, const uint32_t* b, uint32_t* out) { bsm7_mul(a, b, out); }

}  // namespace bn
