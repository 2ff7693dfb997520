/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * BabyBear (p = 15 * 2^27 + 1) radix-2 NTT, restating the reference's prime-field sibling
 * path: the field ops of risc0::Fp (src/ulvt/finite_fields/risc0_baby_bear.h:40-190, values
 * kept canonical here instead of Montgomery-encoded; BB31(r) == r mod p), the twiddle
 * precomputation NTT::pre_compute (src/ulvt/ntt/gpuntt.cuh:186-205: w = g^(2^(log_group - log_n)),
 * tw[i] = w^i, i < n/2, then bit-reversed over log_n - 1 bits, gpuntt.cuh:135-139), the input
 * bit reversal of NTT::apply (gpuntt.cuh:157-163) and the stage loop of ntt_kernel
 * (gpuntt.cuh:65-124, dif_butterfly 36-44): stage s pairs (i, i + 2^s), i with bit s clear,
 * U = u + v, V = (u - v) * tw_br[i >> (s + 1)], stages 0 .. log_n - 1; output in order.
 * Pinned by the reference's MD5 table bb31_ntt_hashes (src/ulvt/ntt/tests/test_ntt.cu:21-50).
 */
#include <stdlib.h>

#include "oracle.h"

#define BB_P 2013265921u

uint32_t orc_bb31_mul(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) % BB_P); }

uint32_t orc_bb31_pow(uint32_t x, uint64_t n) {
	uint32_t r = 1;
	x %= BB_P;
	while (n) {
		if (n & 1) r = orc_bb31_mul(r, x);
		x = orc_bb31_mul(x, x);
		n >>= 1;
	}
	return r;
}

uint32_t orc_bb31_inv(uint32_t x) { return orc_bb31_pow(x, BB_P - 2); }

static uint32_t rev_bits(uint32_t v, int bits) {
	uint32_t r = 0;
	for (int i = 0; i < bits; i++) r |= ((v >> i) & 1u) << (bits - 1 - i);
	return r;
}

void orc_bb31_ntt(const uint32_t* in, uint32_t* out, int log_n, uint32_t gen, int log_group, int in_bit_reversed) {
	const size_t n = (size_t)1 << log_n;
	for (size_t i = 0; i < n; i++) {
		const size_t src = in_bit_reversed ? i : rev_bits((uint32_t)i, log_n);
		out[i] = in[src] % BB_P;
	}
	const size_t half = n / 2;
	uint32_t* tw = (uint32_t*)malloc(sizeof(uint32_t) * (half ? half : 1));
	const uint32_t w = orc_bb31_pow(gen, (uint64_t)1 << (log_group - log_n));
	uint32_t cur = 1;
	for (size_t i = 0; i < half; i++) {
		tw[rev_bits((uint32_t)i, log_n - 1)] = cur;
		cur = orc_bb31_mul(cur, w);
	}
	for (int s = 0; s < log_n; s++) {
		const size_t d = (size_t)1 << s;
		for (size_t p = 0; p < half; p++) {
			const size_t i = (p & (d - 1)) | ((p >> s) << (s + 1));
			const uint32_t u = out[i], v = out[i + d];
			const uint32_t t = tw[p >> s];
			const uint32_t sum = u + v >= BB_P ? u + v - BB_P : u + v;
			const uint32_t dif = u >= v ? u - v : u + BB_P - v;
			out[i] = sum;
			out[i + d] = orc_bb31_mul(dif, t);
		}
	}
	free(tw);
}
