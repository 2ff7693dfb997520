/*
 * CPU ORACLE (test infrastructure only) — additive NTT.
 * Restates src/ulvt/ntt/additive_ntt.cuh:
 *   subspace_map            :16-19   x^2 + c*x
 *   calculate_twiddle       :59-77   XOR of s[stage][k] over set bits of (coset<<(log_h-1-stage))|blk
 *   antt_butterfly          :10-14   u += w*v ; v += u
 *   additive_ntt_kernel     :91-160  stages end-1 .. start on a 2^stage butterfly block
 *   AdditiveNTT::apply      :201-265 2^log_rate coset copies, kernels in reverse order,
 *                                    coset-major output
 *   precompute_subspace_evals :273-309
 * The multi-launch / shared-memory tiling of the reference only changes the order in which
 * independent butterflies run; the serial loop below computes the same values (pinned by
 * the reference's MD5 table, test_ntt.cu:52-124).
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define SIDX(i, j, width) ((size_t)(i) * (size_t)(width) + (size_t)(j))

void orc_subspace_evals32(int log_h, int log_rate, uint32_t* s) {
	orc_init();
	const int width = log_h + log_rate - 1;
	uint32_t* norm = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(log_h > 0 ? log_h : 1));
	memset(s, 0, sizeof(uint32_t) * (size_t)log_h * (size_t)(width > 0 ? width : 1));
	for (int i = 1; i < log_h + log_rate; i++) s[SIDX(0, i - 1, width)] = 1u << i;
	norm[0] = 1;
	for (int i = 1; i < log_h; i++) {
		uint32_t np = norm[i - 1];
		uint32_t p0 = s[SIDX(i - 1, 0, width)];
		norm[i] = (uint32_t)(orc_square(p0, 5) ^ orc_mul32(np, p0));
		for (int j = 1; j < log_h + log_rate - i; j++) {
			uint32_t sp = s[SIDX(i - 1, j, width)];
			s[SIDX(i, j - 1, width)] = (uint32_t)(orc_square(sp, 5) ^ orc_mul32(np, sp));
		}
	}
	for (int i = 0; i < log_h; i++) {
		uint32_t inv = (uint32_t)orc_inv(norm[i], 5);
		for (int j = 0; j < log_h + log_rate - i - 1; j++) s[SIDX(i, j, width)] = orc_mul32(inv, s[SIDX(i, j, width)]);
	}
	free(norm);
}

/* Same table computed with GF(2^128) arithmetic (the field policy P = GF(2^128)). */
void orc_subspace_evals128(int log_h, int log_rate, uint32_t* s) {
	orc_init();
	const int width = log_h + log_rate - 1;
	uint32_t(*norm)[4] = (uint32_t(*)[4])calloc((size_t)(log_h > 0 ? log_h : 1), sizeof(uint32_t[4]));
	memset(s, 0, sizeof(uint32_t) * 4 * (size_t)log_h * (size_t)(width > 0 ? width : 1));
	for (int i = 1; i < log_h + log_rate; i++) {
		uint32_t* e = s + 4 * SIDX(0, i - 1, width);
		e[i / 32] = 1u << (i % 32);   /* T(1 << i) as a 128-bit integer */
	}
	norm[0][0] = 1;
	for (int i = 1; i < log_h; i++) {
		uint32_t* np = norm[i - 1];
		for (int j = 0; j < log_h + log_rate - i; j++) {
			const uint32_t* sp = s + 4 * SIDX(i - 1, j, width);
			uint32_t sq[4], t[4], r[4];
			orc_mul128(sp, sp, sq);
			orc_mul128(np, sp, t);
			for (int k = 0; k < 4; k++) r[k] = sq[k] ^ t[k];
			if (j == 0)
				memcpy(norm[i], r, sizeof(r));
			else
				memcpy(s + 4 * SIDX(i, j - 1, width), r, sizeof(r));
		}
	}
	for (int i = 0; i < log_h; i++) {
		uint32_t inv[4];
		orc_inv128(norm[i], inv);
		for (int j = 0; j < log_h + log_rate - i - 1; j++) {
			uint32_t* e = s + 4 * SIDX(i, j, width);
			uint32_t r[4];
			orc_mul128(inv, e, r);
			memcpy(e, r, sizeof(r));
		}
	}
	free(norm);
}

static inline uint32_t twiddle32(const uint32_t* s, int width, int log_h, int log_rate, int coset, int stage, size_t blk) {
	uint64_t indicator = ((uint64_t)coset << (log_h - 1 - stage)) | (uint64_t)blk;
	uint32_t sum = 0;
	for (int k = 0; k < log_h + log_rate - 1 - stage; k++)
		if ((indicator >> k) & 1) sum ^= s[SIDX(stage, k, width)];
	return sum;
}

void orc_antt32(const uint32_t* in, uint32_t* out, int log_h, int log_rate) {
	orc_init();
	const int width = log_h + log_rate - 1;
	uint32_t* s = (uint32_t*)calloc((size_t)log_h * (size_t)(width > 0 ? width : 1), sizeof(uint32_t));
	orc_subspace_evals32(log_h, log_rate, s);
	const size_t n = (size_t)1 << log_h;
	for (int c = 0; c < (1 << log_rate); c++) {
		uint32_t* d = out + (size_t)c * n;
		memcpy(d, in, n * sizeof(uint32_t));
		for (int stage = log_h - 1; stage >= 0; stage--) {
			const size_t half = (size_t)1 << stage;
			const size_t nblk = n >> (stage + 1);
			for (size_t blk = 0; blk < nblk; blk++) {
				uint32_t w = twiddle32(s, width, log_h, log_rate, c, stage, blk);
				uint32_t* u = d + (blk << (stage + 1));
				uint32_t* v = u + half;
				for (size_t k = 0; k < half; k++) {
					u[k] ^= orc_mul32(w, v[k]);
					v[k] ^= u[k];
				}
			}
		}
	}
	free(s);
}

void orc_antt128(const uint32_t* in, uint32_t* out, int log_h, int log_rate) {
	orc_init();
	const int width = log_h + log_rate - 1;
	uint32_t* s = (uint32_t*)calloc(4 * (size_t)log_h * (size_t)(width > 0 ? width : 1), sizeof(uint32_t));
	orc_subspace_evals128(log_h, log_rate, s);
	const size_t n = (size_t)1 << log_h;
	for (int c = 0; c < (1 << log_rate); c++) {
		uint32_t* d = out + 4 * (size_t)c * n;
		memcpy(d, in, 4 * n * sizeof(uint32_t));
		for (int stage = log_h - 1; stage >= 0; stage--) {
			const size_t half = (size_t)1 << stage;
			const size_t nblk = n >> (stage + 1);
			for (size_t blk = 0; blk < nblk; blk++) {
				uint64_t indicator = ((uint64_t)c << (log_h - 1 - stage)) | (uint64_t)blk;
				uint32_t w[4] = {0, 0, 0, 0};
				for (int k = 0; k < log_h + log_rate - 1 - stage; k++)
					if ((indicator >> k) & 1)
						for (int q = 0; q < 4; q++) w[q] ^= s[4 * SIDX(stage, k, width) + q];
				for (size_t k = 0; k < half; k++) {
					uint32_t* u = d + 4 * ((blk << (stage + 1)) + k);
					uint32_t* v = u + 4 * half;
					uint32_t t[4];
					orc_mul128(w, v, t);
					for (int q = 0; q < 4; q++) {
						u[q] ^= t[q];
						v[q] ^= u[q];
					}
				}
			}
		}
	}
	free(s);
}

void orc_antt128_limbwise_batch(const uint32_t* in, uint32_t* out, int log_h, int log_rate, int batch) {
	orc_init();
	const int width = log_h + log_rate - 1;
	uint32_t* s = (uint32_t*)calloc((size_t)log_h * (size_t)(width > 0 ? width : 1), sizeof(uint32_t));
	orc_subspace_evals32(log_h, log_rate, s);
	const size_t n = (size_t)1 << log_h;
	for (int b = 0; b < batch; b++) {
		const uint32_t* src = in + (size_t)b * 4 * n;
		uint32_t* dstb = out + (size_t)b * 4 * n * ((size_t)1 << log_rate);
		for (int c = 0; c < (1 << log_rate); c++) {
			uint32_t* d = dstb + 4 * (size_t)c * n;
			memcpy(d, src, 4 * n * sizeof(uint32_t));
			for (int stage = log_h - 1; stage >= 0; stage--) {
				const size_t half = (size_t)1 << stage;
				const size_t nblk = n >> (stage + 1);
				for (size_t blk = 0; blk < nblk; blk++) {
					uint32_t w = twiddle32(s, width, log_h, log_rate, c, stage, blk);
					uint32_t* u = d + 4 * (blk << (stage + 1));
					uint32_t* v = u + 4 * half;
					for (size_t k = 0; k < 4 * half; k++) {
						u[k] ^= orc_mul32(w, v[k]);
						v[k] ^= u[k];
					}
				}
			}
		}
	}
	free(s);
}

void orc_antt128_limbwise(const uint32_t* in, uint32_t* out, int log_h, int log_rate) {
	orc_antt128_limbwise_batch(in, out, log_h, log_rate, 1);
}

/*
 * All-cores CPU baseline (bench.py cpu_baseline): the same serial algorithm as
 * orc_antt128_limbwise, with the butterflies of each stage split into contiguous ranges over
 * worker threads (a barrier between stages, as the reference's kernel launches are). The workers
 * are a persistent pool, created on first use and reused by every later call and stage, and a
 * call uses at most one thread per kMinBfPerThread butterflies of a stage (orc_antt_mt_threads),
 * so a small transform is not timed as thread start-up and barrier traffic.
 * Flattened butterfly t of a stage: blk = t >> stage, k = t & (2^stage - 1).
 */
enum { kMinBfPerThread = 1 << 12, kPoolMax = 256 };

typedef struct {
	const uint32_t* s;
	uint32_t* d;
	int width, log_h, log_rate, coset, nthreads;
} mt_job;

static struct {
	pthread_mutex_t mu;
	pthread_cond_t start, done;
	pthread_t th[kPoolMax];
	int size;            /* threads in the pool, the caller included */
	unsigned long gen;   /* job generation */
	int pending;         /* workers of the current job still running */
	const mt_job* job;   /* valid until pending reaches 0 */
	int job_n;           /* its thread count (read under the lock: late non-participants never touch job) */
	pthread_barrier_t bar;
	int bar_n;           /* participants the stage barrier is set up for (0: none) */
} pool = {.mu = PTHREAD_MUTEX_INITIALIZER, .start = PTHREAD_COND_INITIALIZER, .done = PTHREAD_COND_INITIALIZER};
/* held for a whole orc_antt128_limbwise_mt call: concurrent callers (ctypes releases the GIL) take
 * turns instead of overwriting each other's job */
static pthread_mutex_t pool_call = PTHREAD_MUTEX_INITIALIZER;

static void mt_run(const mt_job* a, int id) {
	const size_t n = (size_t)1 << a->log_h;
	const size_t nbf = n / 2;
	const size_t lo = nbf * (size_t)id / (size_t)a->nthreads, hi = nbf * (size_t)(id + 1) / (size_t)a->nthreads;
	for (int stage = a->log_h - 1; stage >= 0; stage--) {
		const size_t half = (size_t)1 << stage;
		size_t cur_blk = (size_t)-1;
		uint32_t w = 0;
		for (size_t t = lo; t < hi; t++) {
			const size_t blk = t >> stage, k = t & (half - 1);
			if (blk != cur_blk) {
				cur_blk = blk;
				w = twiddle32(a->s, a->width, a->log_h, a->log_rate, a->coset, stage, blk);
			}
			uint32_t* u = a->d + 4 * ((blk << (stage + 1)) + k);
			uint32_t* v = u + 4 * half;
			for (int q = 0; q < 4; q++) {
				u[q] ^= orc_mul32(w, v[q]);
				v[q] ^= u[q];
			}
		}
		if (a->nthreads > 1) pthread_barrier_wait(&pool.bar);
	}
}

static void* pool_worker(void* p) {
	const int id = (int)(intptr_t)p;
	unsigned long seen = 0;
	for (;;) {
		pthread_mutex_lock(&pool.mu);
		while (pool.gen == seen) pthread_cond_wait(&pool.start, &pool.mu);
		seen = pool.gen;
		const mt_job* job = pool.job;
		const int n = pool.job_n;
		pthread_mutex_unlock(&pool.mu);
		if (id < n) {
			mt_run(job, id);
			pthread_mutex_lock(&pool.mu);
			if (--pool.pending == 0) pthread_cond_signal(&pool.done);
			pthread_mutex_unlock(&pool.mu);
		}
	}
	return NULL;
}

int orc_antt_mt_threads(int log_h, int nthreads) {
	const size_t nbf = ((size_t)1 << log_h) / 2;
	size_t cap = nbf / kMinBfPerThread;
	if (cap < 1) cap = 1;
	if (nthreads < 1) nthreads = 1;
	if (nthreads > kPoolMax) nthreads = kPoolMax;
	return (size_t)nthreads > cap ? (int)cap : nthreads;
}

void orc_antt128_limbwise_mt(const uint32_t* in, uint32_t* out, int log_h, int log_rate, int nthreads) {
	orc_init();
	nthreads = orc_antt_mt_threads(log_h, nthreads);
	const int width = log_h + log_rate - 1;
	uint32_t* s = (uint32_t*)calloc((size_t)log_h * (size_t)(width > 0 ? width : 1), sizeof(uint32_t));
	orc_subspace_evals32(log_h, log_rate, s);
	const size_t n = (size_t)1 << log_h;
	pthread_mutex_lock(&pool_call);
	pthread_mutex_lock(&pool.mu);
	if (pool.size == 0) pool.size = 1;  /* the caller is thread 0 */
	while (pool.size < nthreads) {
		/* a thread that cannot be created caps this call's participants (no stage barrier ever
		 * waits for a worker that does not exist) */
		if (pthread_create(&pool.th[pool.size], NULL, pool_worker, (void*)(intptr_t)pool.size) != 0) break;
		pool.size++;
	}
	if (nthreads > pool.size) nthreads = pool.size;
	if (nthreads > 1 && pool.bar_n != nthreads) {
		/* no job is running (pool_call serialises the calls), so the barrier is idle */
		if (pool.bar_n) pthread_barrier_destroy(&pool.bar);
		pthread_barrier_init(&pool.bar, NULL, (unsigned)nthreads);
		pool.bar_n = nthreads;
	}
	pthread_mutex_unlock(&pool.mu);
	for (int c = 0; c < (1 << log_rate); c++) {
		uint32_t* d = out + 4 * (size_t)c * n;
		memcpy(d, in, 4 * n * sizeof(uint32_t));
		const mt_job job = {s, d, width, log_h, log_rate, c, nthreads};
		if (nthreads > 1) {
			pthread_mutex_lock(&pool.mu);
			pool.job = &job;
			pool.job_n = nthreads;
			pool.pending = nthreads - 1;
			pool.gen++;
			pthread_cond_broadcast(&pool.start);
			pthread_mutex_unlock(&pool.mu);
		}
		mt_run(&job, 0);
		if (nthreads > 1) {
			pthread_mutex_lock(&pool.mu);
			while (pool.pending > 0) pthread_cond_wait(&pool.done, &pool.mu);
			pthread_mutex_unlock(&pool.mu);
		}
	}
	pthread_mutex_unlock(&pool_call);
	free(s);
}
