/*
 * CPU ORACLE (test infrastructure only) — binary tower field arithmetic.
 * Restates src/ulvt/finite_fields/binary_tower.cuh:19-128 (compact Fan-Paar tower,
 * recursive Karatsuba) and src/ulvt/sumcheck/test/utils/unbitsliced_mul.cuh:19-262
 * (the same tower on u64, heights <= 6), plus tower_height_7_mul
 * (src/ulvt/sumcheck/test/utils/tower_7_mul.cu:4-20) for GF(2^128).
 * Leaf products are computed from the recursive definition down to GF(2); a
 * GF(2^8) table built from that definition only speeds the recursion up.
 */
#include "oracle.h"

#include <string.h>

static uint8_t g_mul8[256][256];
static int g_inited = 0;

static uint64_t mask_bits(int bits) { return bits >= 64 ? ~0ull : ((1ull << bits) - 1); }

/* Pure recursion (binary_tower.cuh:35-50, 83-93). */
static uint64_t rec_mul_alpha(uint64_t a, int h);
static uint64_t rec_mul(uint64_t a, uint64_t b, int h) {
	if (h == 0) return a & b & 1;
	int half = 1 << (h - 1);
	uint64_t m = mask_bits(half);
	uint64_t a0 = a & m, a1 = (a >> half) & m, b0 = b & m, b1 = (b >> half) & m;
	uint64_t z0 = rec_mul(a0, b0, h - 1);
	uint64_t z2 = rec_mul(a1, b1, h - 1);
	uint64_t z1 = rec_mul(a0 ^ a1, b0 ^ b1, h - 1) ^ z0 ^ z2;
	uint64_t z2a = rec_mul_alpha(z2, h - 1);
	return (z0 ^ z2) | ((z1 ^ z2a) << half);
}
static uint64_t rec_mul_alpha(uint64_t a, int h) {
	if (h == 0) return a & 1;
	int half = 1 << (h - 1);
	uint64_t m = mask_bits(half);
	uint64_t a0 = a & m, a1 = (a >> half) & m;
	return a1 | ((a0 ^ rec_mul_alpha(a1, h - 1)) << half);
}

void orc_init(void) {
	if (g_inited) return;
	for (int a = 0; a < 256; a++)
		for (int b = 0; b < 256; b++) g_mul8[a][b] = (uint8_t)rec_mul((uint64_t)a, (uint64_t)b, 3);
	g_inited = 1;
}

uint64_t orc_mul_alpha(uint64_t a, int h) { return rec_mul_alpha(a, h); }

uint64_t orc_mul(uint64_t a, uint64_t b, int h) {
	if (h <= 3) {
		if (!g_inited) orc_init();
		uint64_t m = mask_bits(1 << h);
		return g_mul8[a & m][b & m];
	}
	int half = 1 << (h - 1);
	uint64_t m = mask_bits(half);
	uint64_t a0 = a & m, a1 = (a >> half) & m, b0 = b & m, b1 = (b >> half) & m;
	uint64_t z0 = orc_mul(a0, b0, h - 1);
	uint64_t z2 = orc_mul(a1, b1, h - 1);
	uint64_t z1 = orc_mul(a0 ^ a1, b0 ^ b1, h - 1) ^ z0 ^ z2;
	uint64_t z2a = rec_mul_alpha(z2, h - 1);
	return (z0 ^ z2) | ((z1 ^ z2a) << half);
}

/* generic_square (binary_tower.cuh:52-61) */
uint64_t orc_square(uint64_t a, int h) {
	if (h == 0) return a & 1;
	int half = 1 << (h - 1);
	uint64_t m = mask_bits(half);
	uint64_t a0 = a & m, a1 = (a >> half) & m;
	uint64_t z0 = orc_square(a0, h - 1);
	uint64_t z2 = orc_square(a1, h - 1);
	return (z0 ^ z2) | (rec_mul_alpha(z2, h - 1) << half);
}

/* generic_inverse (binary_tower.cuh:63-81) */
uint64_t orc_inv(uint64_t a, int h) {
	if (h == 0) return a & 1;
	int half = 1 << (h - 1);
	uint64_t m = mask_bits(half);
	if ((a >> half) == 0 && h >= 1) {
		/* element of the subfield: its inverse lives in the subfield */
		return orc_inv(a, h - 1);
	}
	uint64_t a0 = a & m, a1 = (a >> half) & m;
	uint64_t inter = a0 ^ rec_mul_alpha(a1, h - 1);
	uint64_t delta = orc_mul(a0, inter, h - 1) ^ orc_square(a1, h - 1);
	uint64_t dinv = orc_inv(delta, h - 1);
	uint64_t inv0 = orc_mul(dinv, inter, h - 1);
	uint64_t inv1 = orc_mul(dinv, a1, h - 1);
	return inv0 | (inv1 << half);
}

/* GF(2^32) with a GF(2^8)-table leaf: Karatsuba over GF(2^16) -> GF(2^8). */
static inline uint32_t mul16(uint32_t a, uint32_t b) {
	uint32_t a0 = a & 0xff, a1 = (a >> 8) & 0xff, b0 = b & 0xff, b1 = (b >> 8) & 0xff;
	uint32_t z0 = g_mul8[a0][b0];
	uint32_t z2 = g_mul8[a1][b1];
	uint32_t z1 = g_mul8[a0 ^ a1][b0 ^ b1] ^ z0 ^ z2;
	/* multiply_alpha at level 3: alpha_3 = X_2 = 0x10 in GF(2^8) */
	uint32_t z2a = g_mul8[z2][0x10];
	return (z0 ^ z2) | ((z1 ^ z2a) << 8);
}
static inline uint32_t mul_alpha16(uint32_t a) { /* multiply by X_3 = 0x100 in GF(2^16) */
	uint32_t a0 = a & 0xff, a1 = (a >> 8) & 0xff;
	return a1 | ((a0 ^ g_mul8[a1][0x10]) << 8);
}
uint32_t orc_mul32(uint32_t a, uint32_t b) {
	if (!g_inited) orc_init();
	uint32_t a0 = a & 0xffff, a1 = a >> 16, b0 = b & 0xffff, b1 = b >> 16;
	uint32_t z0 = mul16(a0, b0);
	uint32_t z2 = mul16(a1, b1);
	uint32_t z1 = mul16(a0 ^ a1, b0 ^ b1) ^ z0 ^ z2;
	return (z0 ^ z2) | ((z1 ^ mul_alpha16(z2)) << 16);
}

/* ---- GF(2^128) ---- */
typedef struct { uint64_t lo, hi; } u128p;
static u128p load128(const uint32_t a[4]) {
	u128p r;
	r.lo = (uint64_t)a[0] | ((uint64_t)a[1] << 32);
	r.hi = (uint64_t)a[2] | ((uint64_t)a[3] << 32);
	return r;
}
static void store128(u128p v, uint32_t out[4]) {
	out[0] = (uint32_t)v.lo;
	out[1] = (uint32_t)(v.lo >> 32);
	out[2] = (uint32_t)v.hi;
	out[3] = (uint32_t)(v.hi >> 32);
}

/* tower_height_7_mul (tower_7_mul.cu:4-20): schoolbook at the top level. */
void orc_mul128(const uint32_t a[4], const uint32_t b[4], uint32_t out[4]) {
	u128p A = load128(a), B = load128(b);
	uint64_t a0b0 = orc_mul(A.lo, B.lo, 6);
	uint64_t a0b1 = orc_mul(A.lo, B.hi, 6);
	uint64_t a1b0 = orc_mul(A.hi, B.lo, 6);
	uint64_t a1b1 = orc_mul(A.hi, B.hi, 6);
	u128p r;
	r.lo = a0b0 ^ a1b1;
	r.hi = a0b1 ^ a1b0 ^ rec_mul_alpha(a1b1, 6);
	store128(r, out);
}

/* generic_inverse one level up (binary_tower.cuh:63-81 pattern at height 7). */
void orc_inv128(const uint32_t a[4], uint32_t out[4]) {
	u128p A = load128(a);
	u128p r;
	if (A.hi == 0) {
		r.lo = orc_inv(A.lo, 6);
		r.hi = 0;
		store128(r, out);
		return;
	}
	uint64_t inter = A.lo ^ rec_mul_alpha(A.hi, 6);
	uint64_t delta = orc_mul(A.lo, inter, 6) ^ orc_square(A.hi, 6);
	uint64_t dinv = orc_inv(delta, 6);
	r.lo = orc_mul(dinv, inter, 6);
	r.hi = orc_mul(dinv, A.hi, 6);
	store128(r, out);
}
