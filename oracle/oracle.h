/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference (shourovrm/binius-NTT) algorithms on the
 * GF(2^128) additive-NTT hot path. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker /
 * reported CPU baseline. The product (binius-ntt_amd/) never links or calls it.
 *
 * Parity pinning: the NTT restatement is checked against the reference's own
 * golden MD5 tables (src/ulvt/ntt/tests/test_ntt.cu:52-124) and the field code
 * against the reference's known-answer tests (src/ulvt/finite_fields/tests/
 * test_fanpaartower.cu:9-273, tests.cu:172-201). The reference itself is not
 * buildable here (its headers need <cuda/std/utility> and nvcc), so there is no
 * oracle/_ref build; see DESIGN.md "Oracle".
 */
#ifndef BINIUS_NTT_ORACLE_H
#define BINIUS_NTT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- binary tower field (Fan-Paar / Wiedemann) ----------------
 * Level 0 = GF(2); level h = level(h-1)[X_{h-1}] / (X^2 + alpha_{h-1} X + 1),
 * alpha_0 = 1, alpha_h = X_{h-1} (the top generator of level h).
 * Follows src/ulvt/finite_fields/binary_tower.cuh:35-105 (generic_multiply,
 * generic_square, generic_inverse, generic_multiply_alpha).                    */
void     orc_init(void);
uint64_t orc_mul(uint64_t a, uint64_t b, int h);   /* h <= 6 */
uint64_t orc_mul_alpha(uint64_t a, int h);          /* h <= 6 */
uint64_t orc_square(uint64_t a, int h);             /* h <= 6 */
uint64_t orc_inv(uint64_t a, int h);                /* h <= 6, a != 0 */
uint32_t orc_mul32(uint32_t a, uint32_t b);         /* GF(2^32) fast path */

/* GF(2^128): 4 x u32 little-endian limbs (word 0 = bits 0..31), exactly the
 * layout of src/ulvt/sumcheck/test/utils/bigints.cu:6-13.
 * orc_mul128 follows tower_height_7_mul (src/ulvt/sumcheck/test/utils/tower_7_mul.cu:4-20). */
void orc_mul128(const uint32_t a[4], const uint32_t b[4], uint32_t out[4]);
void orc_inv128(const uint32_t a[4], uint32_t out[4]);

/* ---------------- additive NTT ----------------
 * precompute_subspace_evals (src/ulvt/ntt/additive_ntt.cuh:273-309):
 * s is a log_h x (log_h+log_rate-1) row-major table. field_bits is 32 or 128
 * (the table is identical; the 128-bit variant computes it in GF(2^128)).     */
void orc_subspace_evals32(int log_h, int log_rate, uint32_t* s);
void orc_subspace_evals128(int log_h, int log_rate, uint32_t* s /* 4 words per entry */);

/* Serial restatement of additive_ntt_kernel (additive_ntt.cuh:91-160) run over
 * every launch of AdditiveNTT::apply (additive_ntt.cuh:201-265): every coset c
 * gets a copy of the input, stages log_h-1 .. 0, butterfly u += w v; v += u
 * (antt_butterfly, :10-14), twiddle per calculate_twiddle (:59-77). The output
 * is coset-major, 2^(log_h+log_rate) elements.                                  */
void orc_antt32(const uint32_t* in, uint32_t* out, int log_h, int log_rate);
/* GF(2^128) field policy: full 128-bit multiplies of the (embedded) twiddle. */
void orc_antt128(const uint32_t* in, uint32_t* out, int log_h, int log_rate);
/* Same transform computed limb-plane by limb-plane with GF(2^32) arithmetic
 * (valid because every twiddle lies in GF(2^32) when log_h+log_rate <= 32).    */
void orc_antt128_limbwise(const uint32_t* in, uint32_t* out, int log_h, int log_rate);

/* Batched variant used by the CPU baseline: `batch` independent transforms,
 * element stride 4 words, transform stride 4 << log_h words.                  */
void orc_antt128_limbwise_batch(const uint32_t* in, uint32_t* out, int log_h, int log_rate, int batch);
void orc_antt128_limbwise_mt(const uint32_t* in, uint32_t* out, int log_h, int log_rate, int nthreads);
/* Threads orc_antt128_limbwise_mt actually uses for a 2^log_h transform when asked for nthreads
 * (at most one per 4096 butterflies of a stage; persistent pool, at most 256). */
int orc_antt_mt_threads(int log_h, int nthreads);

/* ---------------- bitslicing (src/ulvt/utils/bitslicing.cuh:32-74) ---------------- */
void orc_bitslice_transpose128(uint32_t blk[128]);
void orc_bitslice_untranspose128(uint32_t blk[128]);
void orc_bitslice_transpose32(uint32_t blk[32]);   /* BitsliceUtils<32> */
void orc_bitslice_untranspose32(uint32_t blk[32]);

/* ---------------- sumcheck (src/ulvt/sumcheck/sumcheck.cuh:10-301) ----------------
 * evals: d columns, each 4*2^n words, column-major; compact (bitsliced==0) or
 * bitsliced 128-word batches (bitsliced==1). Runs the whole protocol with the
 * given challenges (n x 4 words) and writes, per round r = 0..n:
 *   sums[4*r..]            = this round's sum
 *   points[4*(d+1)*r ..]   = round polynomial at 0..d
 * (round n is the final call with one evaluation left; its points are zero).   */
void orc_sumcheck_run(const uint32_t* evals, int n, int d, int bitsliced,
                      const uint32_t* challenges, uint32_t* sums, uint32_t* points);
/* evaluate_univariate_given_points (src/ulvt/sumcheck/test/verifier.cu:9-31)   */
void orc_sumcheck_interpolate(const uint32_t* points, int num_points, const uint32_t challenge[4], uint32_t out[4]);
/* evaluate_multilinear_composition (verifier.cu:88-107) on compact columns.     */
void orc_multilinear_composition_fold_mt(const uint32_t* evals, int n, int d, int bitsliced, const uint32_t* challenges,
                                         uint32_t out[4], int nthreads);
void orc_bitslice_many128(uint32_t* blocks, size_t n_blocks, int untranspose);
void orc_multilinear_composition(const uint32_t* evals_compact, int n, int d, const uint32_t* challenges, uint32_t out[4]);

/* ---------------- test helpers ---------------- */
typedef struct { uint32_t mt[624]; int idx; } orc_mt19937;
void     orc_mt_seed(orc_mt19937* g, uint32_t seed);
uint32_t orc_mt_next(orc_mt19937* g);
typedef struct { uint64_t mt[312]; int idx; } orc_mt19937_64;
void     orc_mt64_seed(orc_mt19937_64* g, uint64_t seed);
uint64_t orc_mt64_next(orc_mt19937_64* g);
/* fills n words from std::mt19937(seed) (one gen() per word) */
void orc_mt_fill(uint32_t seed, uint32_t* out, size_t n);
/* fills n elements of a 4-limb GF(2^128) vector: limb 0 from mt19937(seed0),
 * limb j (j=1..3) from the low 32 bits of mt19937_64(seed64_base + j)           */
void orc_fill128(uint32_t seed0, uint64_t seed64_base, uint32_t* out, size_t n);
/* RFC 1321 MD5 over len bytes */
void orc_md5(const void* data, size_t len, uint8_t digest[16]);
/* MD5 of one limb plane (limb in 0..3) of a 4-word-per-element vector */
void orc_md5_limb(const uint32_t* v, size_t n_elems, int limb, uint8_t digest[16]);


/* ---------------- BabyBear radix-2 NTT (prime-field sibling path, bb31.c) ----------------
 * Canonical u32 values (< 2013265921); inputs are reduced mod p as BB31(r) does.            */
uint32_t orc_bb31_mul(uint32_t a, uint32_t b);
uint32_t orc_bb31_pow(uint32_t x, uint64_t n);
uint32_t orc_bb31_inv(uint32_t x);
void     orc_bb31_ntt(const uint32_t* in, uint32_t* out, int log_n, uint32_t gen, int log_group, int in_bit_reversed);


/* ---------------- QM31 sumcheck (prime-field sibling path, qm31.c) ----------------
 * QM31 element = 4 canonical M31 words (lo.a, lo.b, hi.a, hi.b) as qm31.cuh's member order.  */
void orc_qm31_mul(const uint32_t* a, const uint32_t* b, uint32_t* out);
void orc_qm31_interpolate(const uint32_t* points, const uint32_t* r, uint32_t* out);
void orc_qm31_sumcheck_run(uint32_t* evals, int n, const uint32_t* challenges, uint32_t* points);

#ifdef __cplusplus
}
#endif
#endif
