/*
 * CPU ORACLE (test infrastructure only) — GF(2^128) sumcheck prover.
 * Restates the semantics of Sumcheck<NUM_VARS, COMPOSITION_SIZE, DATA_IS_TRANSPOSED>
 * (src/ulvt/sumcheck/sumcheck.cuh:10-301) on compact values:
 *   this_round_messages :130-246  sum = sum_x prod_j f_j(x);
 *                                 points[k] = sum_{x<h} prod_j (f_j(x) + k (f_j(x) + f_j(x+h))), k = 0..d
 *                                 (interpolation point k = tower element with integer value k,
 *                                  sumcheck.cuh:103-115)
 *   move_to_next_round  :248-300  f_j(x) <- f_j(x) + r (f_j(x) + f_j(x+h))  (highest variable first;
 *                                 fold_batch core.cu:25-56, fold_small core.cu:58-82)
 * plus the verifier helpers of src/ulvt/sumcheck/test/verifier.cu.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct { uint32_t w[4]; } f128;

static inline f128 fadd(f128 a, f128 b) {
	f128 r;
	for (int i = 0; i < 4; i++) r.w[i] = a.w[i] ^ b.w[i];
	return r;
}
static inline f128 fmul(f128 a, f128 b) {
	f128 r;
	orc_mul128(a.w, b.w, r.w);
	return r;
}
static inline f128 fconst(uint32_t k) {
	f128 r = {{k, 0, 0, 0}};
	return r;
}

void orc_sumcheck_run(const uint32_t* evals, int n, int d, int bitsliced, const uint32_t* challenges, uint32_t* sums,
					  uint32_t* points) {
	orc_init();
	const size_t N = (size_t)1 << n;
	f128* cols = (f128*)malloc(sizeof(f128) * N * (size_t)d);
	for (int j = 0; j < d; j++) {
		const uint32_t* src = evals + (size_t)j * 4 * N;
		if (!bitsliced) {
			memcpy(cols + (size_t)j * N, src, sizeof(f128) * N);
		} else {
			for (size_t b = 0; b < N / 32; b++) {
				uint32_t blk[128];
				memcpy(blk, src + 128 * b, sizeof(blk));
				orc_bitslice_untranspose128(blk);
				memcpy(cols + (size_t)j * N + 32 * b, blk, sizeof(blk));
			}
		}
	}
	size_t cur = N;
	for (int round = 0; round <= n; round++) {
		const size_t h = cur / 2;
		f128 sum = fconst(0);
		for (size_t x = 0; x < cur; x++) {
			f128 p = cols[x];
			for (int j = 1; j < d; j++) p = fmul(p, cols[(size_t)j * N + x]);
			sum = fadd(sum, p);
		}
		memcpy(sums + 4 * (size_t)round, sum.w, 16);
		for (int k = 0; k <= d; k++) {
			f128 acc = fconst(0);
			f128 kk = fconst((uint32_t)k);
			for (size_t x = 0; x < h; x++) {
				f128 p = fconst(1);
				for (int j = 0; j < d; j++) {
					f128 lo = cols[(size_t)j * N + x], hi = cols[(size_t)j * N + x + h];
					f128 f = fadd(lo, fmul(kk, fadd(lo, hi)));
					p = fmul(p, f);
				}
				acc = fadd(acc, p);
			}
			memcpy(points + 4 * ((size_t)round * (size_t)(d + 1) + (size_t)k), acc.w, 16);
		}
		if (round == n) break;
		f128 r;
		memcpy(r.w, challenges + 4 * (size_t)round, 16);
		for (int j = 0; j < d; j++)
			for (size_t x = 0; x < h; x++) {
				f128 lo = cols[(size_t)j * N + x], hi = cols[(size_t)j * N + x + h];
				cols[(size_t)j * N + x] = fadd(lo, fmul(r, fadd(lo, hi)));
			}
		cur = h;
	}
	free(cols);
}

/* evaluate_univariate_given_points (verifier.cu:9-31): Lagrange interpolation through
 * (k, points[k]) for k = 0..num_points-1, evaluated at the challenge. */
void orc_sumcheck_interpolate(const uint32_t* points, int num_points, const uint32_t challenge[4], uint32_t out[4]) {
	orc_init();
	f128 r, acc = fconst(0);
	memcpy(r.w, challenge, 16);
	for (int i = 0; i < num_points; i++) {
		f128 t;
		memcpy(t.w, points + 4 * i, 16);
		for (int j = 0; j < num_points; j++) {
			if (j == i) continue;
			t = fmul(t, fadd(r, fconst((uint32_t)j)));
			t = fmul(t, fconst((uint32_t)orc_inv((uint64_t)(i ^ j), 2)));
		}
		acc = fadd(acc, t);
	}
	memcpy(out, acc.w, 16);
}

/* evaluate_multilinear_composition (verifier.cu:33-107) with lagrange_basis_eval
 * (kernel/verifier_kernel.cu:4-37): bit v of x pairs with challenge r[n-1-v]. */
void orc_multilinear_composition(const uint32_t* evals_compact, int n, int d, const uint32_t* challenges, uint32_t out[4]) {
	orc_init();
	const size_t N = (size_t)1 << n;
	f128 prod = fconst(1);
	for (int j = 0; j < d; j++) {
		f128 acc = fconst(0);
		for (size_t x = 0; x < N; x++) {
			f128 p;
			memcpy(p.w, evals_compact + 4 * ((size_t)j * N + x), 16);
			for (int v = 0; v < n; v++) {
				f128 r;
				memcpy(r.w, challenges + 4 * (size_t)(n - 1 - v), 16);
				if (!((x >> v) & 1)) r.w[0] ^= 1;
				p = fmul(p, r);
			}
			acc = fadd(acc, p);
		}
		prod = fmul(prod, acc);
	}
	memcpy(out, prod.w, 16);
}
