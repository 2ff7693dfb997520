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
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
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

/*
 * Large-size checker for the final claim (evaluate_multilinear_composition, verifier.cu:88-107):
 * prod_j f_j(r) with f_j(r) computed by folding the column with r[0], r[1], ..., r[n-1]
 * (highest variable first: f(x) <- f(x) + r (f(x) + f(x + h)), which is the Lagrange-basis sum
 * sum_x f(x) prod_v (bit v of x ? r[n-1-v] : 1 + r[n-1-v]) evaluated one variable at a time).
 * Columns are compact, or bitsliced 128-word batches when `bitsliced`; the folds are split over
 * `nthreads` pthreads. O(d 2^n) products instead of orc_multilinear_composition's O(d n 2^n).
 */
typedef struct {
	f128* col;
	const uint32_t* src;
	int bitsliced;
	size_t lo, hi, h;
	const f128* tab; /* x -> r x as 16 byte tables: tab[256 k + b] = r (b << 8k) (linearity) */
	int phase;       /* 0: load (untranspose), 1: fold */
} ml_arg;

static void mul_tables(f128 r, f128* tab) {
	for (int k = 0; k < 16; k++) {
		f128 basis[8];
		for (int i = 0; i < 8; i++) {
			f128 e = fconst(0);
			e.w[(8 * k + i) / 32] = 1u << ((8 * k + i) % 32);
			basis[i] = fmul(r, e);
		}
		tab[256 * k] = fconst(0);
		for (int b = 1; b < 256; b++) {
			const int low = __builtin_ctz((unsigned)b);
			tab[256 * k + b] = fadd(tab[256 * k + (b & (b - 1))], basis[low]);
		}
	}
}

static inline f128 tab_mul(const f128* tab, f128 x) {
	f128 acc = fconst(0);
	for (int k = 0; k < 16; k++) acc = fadd(acc, tab[256 * k + ((x.w[k / 4] >> (8 * (k % 4))) & 0xFF)]);
	return acc;
}

static void* ml_worker(void* p) {
	ml_arg* a = (ml_arg*)p;
	if (a->phase == 0) {
		for (size_t b = a->lo; b < a->hi; b++) {
			uint32_t blk[128];
			memcpy(blk, a->src + 128 * b, sizeof(blk));
			if (a->bitsliced) orc_bitslice_untranspose128(blk);
			memcpy(a->col + 32 * b, blk, sizeof(blk));
		}
	} else {
		for (size_t x = a->lo; x < a->hi; x++) a->col[x] = fadd(a->col[x], tab_mul(a->tab, fadd(a->col[x], a->col[x + a->h])));
	}
	return NULL;
}

static void ml_parallel(ml_arg* proto, size_t total, int nthreads) {
	pthread_t th[256];
	ml_arg args[256];
	if (nthreads > 256) nthreads = 256;
	if ((size_t)nthreads > total) nthreads = total ? (int)total : 1;
	for (int i = 0; i < nthreads; i++) {
		args[i] = *proto;
		args[i].lo = total * (size_t)i / (size_t)nthreads;
		args[i].hi = total * (size_t)(i + 1) / (size_t)nthreads;
		pthread_create(&th[i], NULL, ml_worker, &args[i]);
	}
	for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
}

void orc_multilinear_composition_fold_mt(const uint32_t* evals, int n, int d, int bitsliced, const uint32_t* challenges,
                                         uint32_t out[4], int nthreads) {
	orc_init();
	const size_t N = (size_t)1 << n;
	f128* col = (f128*)malloc(sizeof(f128) * (N < 32 ? 32 : N));
	f128* tab = (f128*)malloc(sizeof(f128) * 16 * 256);
	f128 prod = fconst(1);
	for (int j = 0; j < d; j++) {
		const uint32_t* src = evals + (size_t)j * 4 * N;
		if (N < 32 || !bitsliced) {
			memcpy(col, src, sizeof(f128) * N);
		} else {
			ml_arg a = {col, src, bitsliced, 0, 0, 0, NULL, 0};
			ml_parallel(&a, N / 32, nthreads);
		}
		size_t cur = N;
		for (int v = 0; v < n; v++) {
			f128 r;
			memcpy(r.w, challenges + 4 * (size_t)v, 16);
			mul_tables(r, tab);
			ml_arg a = {col, NULL, 0, 0, 0, cur / 2, tab, 1};
			ml_parallel(&a, cur / 2, cur >= (1u << 16) ? nthreads : 1);
			cur /= 2;
		}
		prod = fmul(prod, col[0]);
	}
	free(tab);
	free(col);
	memcpy(out, prod.w, 16);
}
