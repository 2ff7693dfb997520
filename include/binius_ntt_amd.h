/*
 * binius_ntt_amd.h — the C-ABI drop-in boundary of the MI355X (gfx950) binary-tower /
 * additive-NTT engine. Plain pointers and sizes only; every entry point returns an int
 * status (0 = BN_OK) and never aborts; bn_last_error() describes the last failure on the
 * calling thread.
 *
 * Each entry point names the reference interface it replaces (shourovrm/binius-NTT,
 * paths relative to its repository root). The C++ mirror of the reference surface
 * (AdditiveNTT<T,P>, NTTData, Sumcheck<N,d,T>, ...) lives in binius-ntt_amd/host/ulvt and
 * calls only these functions.
 *
 * Element layouts (bit-exact with the reference):
 *   GF(2^32) element  : one uint32_t.
 *   GF(2^128) element : four uint32_t limbs, little-endian (limb 0 = bits 0..31),
 *                       as src/ulvt/sumcheck/test/utils/bigints.cu:6-13.
 *   bitsliced block   : 128 uint32_t words; word i holds bit i of 32 consecutive GF(2^128)
 *                       elements, element e in bit e (src/ulvt/utils/bitslicing.cuh:32-47).
 */
#ifndef BINIUS_NTT_AMD_H
#define BINIUS_NTT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
	BN_OK = 0,
	BN_ERR_INVALID = 1,     /* bad argument (reference: ASSERT / apply() returning false) */
	BN_ERR_HIP = 2,         /* HIP runtime failure (reference: CUDA_CHECK, common.cuh:18-29) */
	BN_ERR_UNSUPPORTED = 3, /* valid in the reference surface but not built here */
	BN_ERR_ALLOC = 4        /* device or host allocation failure */
};

/* Description of the last error on this thread ("" if none). */
const char* bn_last_error(void);
/* Library version string. */
const char* bn_version(void);

/* Replaces bool check_gpu_capabilities() (src/ulvt/utils/common.cu:6-43): returns 1 if a
 * gfx950 device with enough LDS for the kernels is visible, else 0. */
int bn_check_gpu_capabilities(void);

/* ------------------------------------------------------------------------------------
 * Additive NTT (src/ulvt/ntt/additive_ntt.cuh, src/ulvt/ntt/nttconf.cuh)
 * ------------------------------------------------------------------------------------ */
typedef struct bn_antt_plan bn_antt_plan;

/* Replaces AdditiveNTTConf<T,P>(log_h, log_rate) (nttconf.cuh:55-60) + the AdditiveNTT
 * constructor (additive_ntt.cuh:178-199): validates 1 <= log_h, 0 <= log_rate <= 4,
 * log_h + log_rate <= field_bits (and <= 32: every twiddle must lie in GF(2^32)),
 * precomputes the normalised subspace evaluations on the host and stages them on
 * `device`. field_bits is 32 (T=uint32_t, P=FanPaarTowerField<5>) or 128 (GF(2^128)). */
int bn_antt_plan_create(int device, int field_bits, int log_h, int log_rate, bn_antt_plan** plan);
/* Replaces ~AdditiveNTT (additive_ntt.cuh:267-270). NULL is accepted. */
int bn_antt_plan_destroy(bn_antt_plan* plan);

/* Replaces bool AdditiveNTT::apply(const NTTData<T>& in, NTTData<T>& out)
 * (additive_ntt.cuh:201-265): host buffers, synchronous. in_elems must equal 2^log_h
 * (the reference returns false otherwise: here BN_ERR_INVALID with no other effect);
 * `out` receives 2^(log_h+log_rate) elements, coset-major. */
int bn_antt_forward_host(bn_antt_plan* plan, const void* in, size_t in_elems, void* out);

/* Device-resident entry (no reference counterpart; used by benchmarks, batched and
 * multi-GPU callers): `batch` independent transforms, transform b reads
 * d_in + b*2^log_h elements and writes d_out + b*2^(log_h+log_rate) elements.
 * d_in and d_out must not overlap. Asynchronous on `stream` (a hipStream_t, may be 0). */
int bn_antt_forward_device(bn_antt_plan* plan, const void* d_in, void* d_out, size_t batch, void* stream);

/* Copies the plan's normalised subspace-evaluation table s[i][j] (GF(2^32) values,
 * log_h rows x (log_h+log_rate-1) columns, row-major) to host memory. */
int bn_antt_get_subspace_evals(const bn_antt_plan* plan, uint32_t* out, size_t out_words);

/* Plan introspection: 0 log_h, 1 log_rate, 2 field_bits, 3 device, 4 kernel variant. */
int bn_antt_plan_query(const bn_antt_plan* plan, int what, int64_t* value);
/* Kernel selection, the analogue of choosing AdditiveNTT vs ModifiedAdditiveNTT
 * (src/ulvt/ntt/modified_antt.cuh:223-427, benchmark_antt.cu): 0 = compact tiles with the twiddle
 * recomputed per butterfly from the subspace table (the reference kernel's scheme), 1 = bitsliced
 * LDS tiles with host-tabulated twiddle contributions, 4 = bitsliced register tiles (three to four
 * waves per SIMD) on every pass, 5 = variant 4 for the passes whose twiddles all lie in GF(2^8)
 * and variant 1 for the others (default when log_h >= 12). Other values
 * return BN_ERR_INVALID. Variants 1, 4 and 5 need log_h >= 12; results are identical. */
int bn_antt_plan_set_variant(bn_antt_plan* plan, int variant);

/* Profiling hook for bench.py: records hipEvents around every kernel launch of the next
 * bn_antt_forward_device call on its stream and returns per-launch-kind mean durations. */
int bn_antt_set_event_timing(bn_antt_plan* plan, int enable);
int bn_antt_get_event_timing(bn_antt_plan* plan, float* ms_per_kind, int max_kinds, int* n_kinds);
/* Profiling (no reference counterpart; bench.py's roofline): every pass of the transform is
 * launched `reps` times back to back on `stream` between two hipEvents, giving its steady-state
 * duration per launch in ms_per_pass[pass]. d_out's contents are meaningless afterwards (passes
 * are re-applied to their own output; their cost does not depend on the values). Variants
 * 1, 4 and 5. Synchronous. */
int bn_antt_time_passes(bn_antt_plan* plan, const void* d_in, void* d_out, size_t batch, int reps,
                        void* stream, float* ms_per_pass, int max_passes, int* n_passes);
/* Profiling (no reference counterpart): the demangled name of the kernel that pass `pass` of the
 * plan's current variant launches, as rocprofv3 reports it (e.g. "void bn::antt_bs_pass<4, 2, 32,
 * false>(bn::BsParams)"), so committed counter summaries can be matched to the launches exactly.
 * BN_ERR_UNSUPPORTED for variant 0. */
int bn_antt_pass_kernel_name(bn_antt_plan* plan, int pass, char* buf, size_t cap);

/* ------------------------------------------------------------------------------------
 * Binary tower field arithmetic (src/ulvt/finite_fields/)
 * ------------------------------------------------------------------------------------ */
/* Elementwise GF(2^128) product of compact vectors, n elements, device pointers.
 * Semantics of tower_height_7_mul (src/ulvt/sumcheck/test/utils/tower_7_mul.cu:4-20). Any n;
 * alias-safe (d_out == d_a or d_out == d_b). Runs on the bitsliced quad-lane product behind
 * in-LDS bit transposes (78 KB of dynamic LDS per work-group). */
int bn_gf128_mul_device(const void* d_a, const void* d_b, void* d_out, size_t n, void* stream);
/* Same on bitsliced 128-word blocks: multiply_unrolled<7> (circuit_generator/unrolled/
 * binary_tower_unrolled7.cu), n_blocks blocks of 32 products each. Alias-safe (d_out == d_a). */
int bn_gf128_mul_bitsliced_device(const void* d_a, const void* d_b, void* d_out, size_t n_blocks, void* stream);
/* Elementwise GF(2^32) product (FanPaarTowerField<5>::multiply, binary_tower.cuh:113-115). */
int bn_gf32_mul_device(const void* d_a, const void* d_b, void* d_out, size_t n, void* stream);
/* Register-resident repeat-loop microbenchmarks in the style of bitsliced_repeat
 * (src/ulvt/finite_fields/tests/profiling/kernels/bitsliced_repeat.cu:5-32):
 * kind 0 = compact GF(2^128), kind 1 = bitsliced GF(2^128) (32 products per lane-block,
 * multiply_unrolled<7> per lane), kind 2 = bitsliced GF(2^128) on the quad-lane product of the
 * sumcheck (one 32-product block per quad of lanes).
 * Each of `threads` lanes (kinds 0, 1) or blocks (kind 2) performs `iters` dependent products;
 * d_state holds threads*4 (kind 0) or threads*128 (kinds 1, 2) words, updated in place, and
 * d_operand holds the multipliers in the same shape. */
int bn_gf128_mul_repeat_device(int kind, void* d_state, const void* d_operand, size_t threads, int iters, void* stream);

/* ------------------------------------------------------------------------------------
 * Bitslicing (src/ulvt/utils/bitslicing.cuh:89-105)
 * ------------------------------------------------------------------------------------ */
/* In-place compact -> bitsliced (untranspose == 0) or bitsliced -> compact (untranspose != 0)
 * over n_blocks 128-word blocks. Replaces transpose_kernel / untranspose_kernel. */
int bn_bitslice_device(void* d_buf, size_t n_blocks, int untranspose, void* stream);

/* ------------------------------------------------------------------------------------
 * Field primitives beside the hot path (src/ulvt/finite_fields)
 * ------------------------------------------------------------------------------------ */
/* Replaces multiply_unrolled<HEIGHT>(a, b, dst) (circuit_generator/unrolled/
 * binary_tower_unrolled.cuh:4-5): 32 bitsliced GF(2^(2^height)) products, 2^height words per
 * operand (word i = bit i of the 32 elements). Host computation; alias-safe (dst may be a or b,
 * as core.cu:21 uses it). 2 <= height <= 7. */
int bn_multiply_unrolled(int height, const uint32_t* a, const uint32_t* b, uint32_t* dst);
/* Device batch of the same: nblocks blocks of 2^height words per operand. Async on `stream`. */
int bn_multiply_unrolled_device(int height, const void* a, const void* b, void* dst, size_t nblocks, void* stream);
/* Replaces mul_binary_tower_32b_simd<HEIGHT>(a, b) (binary_tower_simd.cuh:77-127): the words as
 * 32/2^height packed GF(2^(2^height)) elements, multiplied lane by lane. 0 <= height <= 5. */
int bn_mul_binary_tower_32b_simd(int height, uint32_t a, uint32_t b, uint32_t* out);
/* Replaces interleave_32b<HEIGHT>(a, b) -> (c, d) and xor_adjacent_32b<HEIGHT>(a)
 * (binary_tower_simd.cuh:129-150); 0 <= height <= 4. */
int bn_interleave_32b(int height, uint32_t a, uint32_t b, uint32_t* c, uint32_t* d);
int bn_xor_adjacent_32b(int height, uint32_t a, uint32_t* out);
/* Device batch over n words: op 0 = mul_binary_tower_32b_simd (c = a*b), 1 = interleave_32b
 * ((c, d) from (a, b)), 2 = xor_adjacent_32b (c from a; b, d unused). Async on `stream`. */
int bn_packed32_device(int op, int height, const void* a, const void* b, void* c, void* d, size_t n, void* stream);

/* ------------------------------------------------------------------------------------
 * Sumcheck over GF(2^128) (src/ulvt/sumcheck/sumcheck.cuh:10-301)
 * ------------------------------------------------------------------------------------ */
typedef struct bn_sumcheck bn_sumcheck;

/* Replaces Sumcheck<NUM_VARS, COMPOSITION_SIZE, DATA_IS_TRANSPOSED>(evals, benchmarking)
 * (sumcheck.cuh:82-126). evals: composition_size columns of 4*2^num_vars words each,
 * column-major; compact when data_is_transposed == 0 (converted on the device), bitsliced
 * 128-word blocks otherwise. 1 <= num_vars <= 30 (>= 5 for bitsliced input),
 * 1 <= composition_size <= 8.
 * The host copy is made synchronously. */
int bn_sumcheck_create(int device, int num_vars, int composition_size, int data_is_transposed,
                       const uint32_t* evals, bn_sumcheck** sc);
/* bn_sumcheck_create in the reference constructor's two timed phases (sumcheck.cuh:88-124:
 * start_before_memcpy, start_before_transpose, start_raw): _staged allocates and copies the host
 * columns (synchronous, the "Memcpy" phase) and leaves compact input untransposed;
 * bn_sumcheck_prepare runs the device bit-transpose and synchronises (the "Transpose" phase; a
 * no-op for bitsliced input or a prepared prover). A staged prover used without prepare is
 * prepared by its first round call. */
int bn_sumcheck_create_staged(int device, int num_vars, int composition_size, int data_is_transposed,
                              const uint32_t* evals, bn_sumcheck** sc);
int bn_sumcheck_prepare(bn_sumcheck* sc);
/* As above but from device memory already holding the columns (no host copy). The buffer
 * is copied into the prover's own storage unless take_ownership != 0, in which case the
 * prover folds it in place and frees it with hipFree on destroy (so it must come from
 * hipMalloc). The copy (or first use) runs on the prover's own stream, ordered after the work
 * queued on the legacy default stream; a producer on any other stream must have completed
 * (the Python mirror synchronises the tensor's current stream first). */
int bn_sumcheck_create_device(int device, int num_vars, int composition_size, int data_is_transposed,
                              void* d_evals, int take_ownership, bn_sumcheck** sc);
/* Replaces Sumcheck::this_round_messages(sum, points) (sumcheck.cuh:130-246):
 * sum[4], points[4*(composition_size+1)] (round polynomial at 0..d). Blocks until the round's
 * points are posted (the calling thread polls host memory). */
int bn_sumcheck_round_messages(bn_sumcheck* sc, uint32_t* sum, uint32_t* points);
/* Replaces Sumcheck::move_to_next_round(challenge) (sumcheck.cuh:248-300). Asynchronous: queues
 * the fold and the next round's messages kernel on the prover's stream and returns. */
int bn_sumcheck_move_to_next_round(bn_sumcheck* sc, const uint32_t* challenge);
/* Current round (0 .. num_vars). */
int bn_sumcheck_round(const bn_sumcheck* sc, int* round);
/* Multi-GPU sharding: this prover holds shard `rank` of `world` (interleaved by 32-element
 * batch index); round messages are then partial and must be XOR-combined across ranks by
 * the caller (the Python/RCCL layer does allgather + XOR). world must be a power of two
 * with 32*world <= 2^num_vars. Must be called before the first round. */
int bn_sumcheck_set_shard(bn_sumcheck* sc, int rank, int world);
/* A shard prover built directly from this rank's share (no reference counterpart): d_local
 * holds the bitsliced batches b with b mod world == rank, in order (4*2^num_vars/world words per
 * column, columns back to back). The copy is ordered after the work queued on `stream` (a
 * hipStream_t; NULL = default stream). Equivalent to bn_sumcheck_create_device on the whole
 * input followed by bn_sumcheck_set_shard(rank, world), without any rank holding the whole. */
int bn_sumcheck_create_shard_device(int device, int num_vars, int composition_size, int rank, int world,
                                    const void* d_local, void* stream, bn_sumcheck** sc);
/* Sharded endgame (no reference counterpart; the reference's analogue is the hand-over to the
 * CPU at 32 evaluations, sumcheck.cuh:283-297): once every shard is down to one 32-element
 * batch (*flag = 1), folds pair elements of different ranks. Each rank exports its batch
 * (composition_size * 128 words), the caller all-gathers them rank-major and every rank
 * imports the concatenation; the prover then continues unsharded. */
int bn_sumcheck_needs_gather(const bn_sumcheck* sc, int* flag);
/* Device-resident round exchange (no reference counterpart): every later round-messages kernel also
 * writes the round's raw point words into d_words (device memory, >= 4*(8+1)+1 words, or NULL to
 * stop): words 0 .. 4*(composition_size+1)-1 = the kernel's points 0..d (p(1) zero when it was not
 * computed), word 36 = flags: bit 0 set if p(1) was left out (the caller then has p(1) = claim + p(0)
 * and sum = claim with the round's claim, which for XOR-combined shards is the global one; clear:
 * sum = p(0) + p(1)); bit 1 set for the last call (one evaluation left: words 0-3 are the sum,
 * prod_j f_j(r), and there are no points). The words are written before the posted sequence number, so they are complete
 * once bn_sumcheck_round_messages has returned; consumers on other streams order themselves after
 * the prover's stream (bn_sumcheck_stream) to read them. A prover with a sink never starts the
 * resident round server; while a server started earlier runs (an unsharded prover's last rounds),
 * setting a sink returns BN_ERR_INVALID. */
int bn_sumcheck_set_message_sink(bn_sumcheck* sc, void* d_words);
/* Sharded drivers with a message sink: replaces bn_sumcheck_round_messages without waiting for the
 * round. Makes sure the round's messages kernel is queued on the prover's stream and returns; the
 * raw points and flags reach the sink in stream order, so a consumer orders itself after
 * bn_sumcheck_stream (e.g. enqueues its collective there) and never polls the host. The caller
 * then holds the round's global points: the next round skips p(1) when the prover derives it
 * (sink word 36 bit 0) and the caller completes it from the global claim. Once used, the rounds
 * up to the endgame gather must all be read this way. BN_ERR_INVALID while a round server runs. */
int bn_sumcheck_round_messages_sink(bn_sumcheck* sc);
int bn_sumcheck_stream(const bn_sumcheck* sc, void** stream);
int bn_sumcheck_export_shard(const bn_sumcheck* sc, uint32_t* out, size_t out_words);
int bn_sumcheck_import_gathered(bn_sumcheck* sc, const uint32_t* words, size_t n_words, int world);
int bn_sumcheck_destroy(bn_sumcheck* sc);

/* ------------------------------------------------------------------------------------
 * Verifier side of the sumcheck (src/ulvt/sumcheck/test/verifier.cu)
 * ------------------------------------------------------------------------------------ */
/* Replaces evaluate_multilinear_composition(evals, challenges, num_vars, composition_size)
 * (verifier.cu:88-107, with evaluate_multilinear_given_point :33-86 and lagrange_basis_eval,
 * kernel/verifier_kernel.cu:4-37): out = prod_j sum_x f_j(x) prod_v (x_v ? r[n-1-v] : 1 + r[n-1-v]),
 * i.e. every column folded at the challenges (highest variable first), multiplied together.
 * Computed on `device` by the sumcheck fold kernels. evals as bn_sumcheck_create (host memory,
 * compact or bitsliced); challenges: num_vars x 4 words. Synchronous. */
int bn_multilinear_composition_eval(int device, int num_vars, int composition_size, int data_is_transposed,
                                    const uint32_t* evals, const uint32_t* challenges, uint32_t* out);
/* Same with the columns already in device memory (left untouched). */
int bn_multilinear_composition_eval_device(int device, int num_vars, int composition_size, int data_is_transposed,
                                           const void* d_evals, const uint32_t* challenges, uint32_t* out);
/* Replaces evaluate_univariate_given_points(challenge, points, num_points) (verifier.cu:9-31):
 * Lagrange interpolation through (k, points[k]), k = 0..num_points-1 (tower elements), evaluated
 * at `challenge`. Host arithmetic; 1 <= num_points <= 16. */
int bn_sumcheck_interpolate(const uint32_t* points, int num_points, const uint32_t* challenge, uint32_t* out);


/* ------------------------------------------------------------------------------------
 * BabyBear radix-2 NTT, the prime-field sibling path (src/ulvt/ntt/gpuntt.cuh,
 * NTTConfRad2 in src/ulvt/ntt/nttconf.cuh:25-47, BB31 = risc0::Fp,
 * src/ulvt/finite_fields/risc0_baby_bear.h:40-190). Elements are uint32_t holding the
 * canonical value (BB31::asUInt32(); inputs are reduced mod p = 15*2^27+1 as BB31(r) does).
 * The transform is the natural-order DFT X[k] = sum_j x[j] w^(jk), w = g^(2^(log_group-log_n)).
 * Raw risc0 Fp words (Montgomery form, val = x * 2^32 mod p, the bytes of NTTData<BB31> in the
 * reference) are accepted as well: the transform is linear and multiplies data only by
 * Montgomery-encoded twiddles, so Montgomery words (< p) in give the reference's Montgomery
 * words out (tests/test_bb31.py::test_gpu_montgomery_words_in_montgomery_words_out).
 * ------------------------------------------------------------------------------------ */
typedef struct bn_bb31_ntt_plan bn_bb31_ntt_plan;

/* Replaces NTTConfRad2<BB31>(generator, log_group_order, log_inp_size) (nttconf.cuh:31-38:
 * 1 <= log_n <= 27, log_group_order >= log_n) + the NTT<BB31> constructor (gpuntt.cuh:128-146,
 * twiddle precomputation). generator is a canonical value (BB31(137) -> 137). */
int bn_bb31_ntt_plan_create(int device, uint32_t generator, int log_group_order, int log_n, bn_bb31_ntt_plan** plan);
int bn_bb31_ntt_plan_destroy(bn_bb31_ntt_plan* plan);

/* Replaces NTT<BB31>::apply(input, output) (gpuntt.cuh:150-183): host in -> host out,
 * synchronous, output in order. in_bit_reversed = 1 for NTTData::order == BIT_REVERSED (the
 * input is used as stored), 0 for IN_ORDER. BN_ERR_INVALID if in_elems != 2^log_n (the
 * reference ASSERTs). */
int bn_bb31_ntt_forward_host(bn_bb31_ntt_plan* plan, const uint32_t* in, size_t in_elems, uint32_t* out,
                             int in_bit_reversed);

/* Device-resident, asynchronous on `stream` (hipStream_t, NULL = default): batch transforms of
 * 2^log_n words each, contiguous; d_in and d_out must not overlap. Multi-pass sizes
 * (log_n >= 14) stage their data in the plan's scratch buffer, so a plan is used by one stream
 * at a time (and not concurrently with forward_host); use one plan per stream. */
int bn_bb31_ntt_forward_device(bn_bb31_ntt_plan* plan, const uint32_t* d_in, uint32_t* d_out, size_t batch,
                               int in_bit_reversed, void* stream);


/* ------------------------------------------------------------------------------------
 * QM31 sumcheck, the prime-field sibling of the GF(2^128) sumcheck
 * (src/ulvt/prime_field_sumcheck/sumcheck.cuh:8-96, core/kernels.cu:5-77). A QM31 element
 * is 4 uint32_t M31 words (lo.a, lo.b, hi.a, hi.b), canonical (< 2^31 - 1) on output.
 * ------------------------------------------------------------------------------------ */
typedef struct bn_qm31_sumcheck bn_qm31_sumcheck;

/* Replaces Sumcheck<NUM_VARS>(evals, benchmarking) (sumcheck.cuh:24-44): evals = column 0 then
 * column 1, 2^num_vars QM31 each (8 * 2^num_vars words); 1 <= num_vars <= 28 (the reference
 * instantiates 1, 20, 24, 28). */
int bn_qm31_sumcheck_create(int device, int num_vars, const uint32_t* evals, bn_qm31_sumcheck** sc);
/* Replaces this_round_messages<BLOCKS, THREADS>(points) (sumcheck.cuh:46-86): points 0, 1, 2
 * (12 words). */
int bn_qm31_sumcheck_round_messages(bn_qm31_sumcheck* sc, uint32_t* points);
/* Replaces fold<BLOCKS, THREADS>(challenge) (sumcheck.cuh:88-96). */
int bn_qm31_sumcheck_fold(bn_qm31_sumcheck* sc, const uint32_t* challenge);
/* After the last fold: the two remaining values f0(r), f1(r) (8 words). */
int bn_qm31_sumcheck_final_values(bn_qm31_sumcheck* sc, uint32_t* out);
int bn_qm31_sumcheck_destroy(bn_qm31_sumcheck* sc);

#ifdef __cplusplus
}
#endif
#endif
