// GF(2^128) sumcheck prover on bitsliced columns (Sumcheck<N, d, T>, src/ulvt/sumcheck/sumcheck.cuh).
//
// Semantics (sumcheck.cuh:130-300, fold_batch / compute_sum in core/core.cu): with columns
// f_0..f_{d-1} of cur evaluations and h = cur / 2,
//   points[k] = sum_{x<h} prod_j (f_j(x) + k (f_j(x) + f_j(x+h))),  k = 0..d (tower element k)
//   sum       = points[0] + points[1]   (= sum_{x<cur} prod_j f_j(x); for cur == 1: prod_j f_j(0))
//   fold(r)   : f_j(x) <- f_j(x) + r (f_j(x) + f_j(x+h))   (highest variable first)
//
// Layout: each column is a run of bitsliced 128-word batches (32 elements; word i = bit i of
// the 32 elements, element e in bit e), columns back to back. While cur >= 64 a butterfly pairs
// whole batches x and x + cur/64; below that the single remaining batch pairs bit-lanes.
//
// Arithmetic: one GF(2^128) bitsliced product is spread over a quad of lanes (lane l holds limb
// l = words 32l..32l+31 of each operand and of the result). With A = A_hi X + A_lo the tower's
// top level is done schoolbook (as tower_height_7_mul, tower_7_mul.cu:4-20): lane q computes one
// GF(2^64) product P_q = A_i B_j, (i,j) = (0,0), (1,1), (0,1), (1,0), by Karatsuba over three
// generated GF(2^32) circuits (bsm5_mul); then
//   c_lo = P00 + P11,  c_hi = P01 + P10 + alpha(P11)
// and the quad trades halves through LDS. Operands and partial products travel through a
// 1 KiB LDS slot per quad, so a lane never holds more than ~4 x 32 words of field data.
// The big folds, whose second operand is the wave-uniform challenge, run on lane pairs with
// constant-operand circuits instead (sc_fold_pair).
//
// Round messages are reduced without ever forming 128-word sums: after each product a lane
// folds its 32 result words into one word of parities (bit i = XOR over the elements of bit i),
// which is exactly the limb of the element-sum that the reference's compute_sum produces.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "bitsliced.hpp"
#include "common.hpp"
#include "quad_mul.hpp"
#include "tower.hpp"

int bitslice_launch(const void* src, void* dst, size_t nblk, int untranspose, hipStream_t st);  // field.hip

namespace bn {
namespace {

#ifndef BN_SC_THREADS
#define BN_SC_THREADS 256
#endif
constexpr int kScThreads = BN_SC_THREADS;  // (512-thread workgroups, one per CU: 6 % slower on c4)
constexpr int kScMinWG = 512 / kScThreads;  // 2 waves per SIMD (256 VGPRs)
constexpr int kQuadsPerWG = kScThreads / 4;
// Round messages are XOR-accumulated into kAccCopies copies of the (kMaxD + 1) x 4-word point
// set, workgroup b into copy b % kAccCopies, each copy on its own 256-B lines: device-scope
// atomics on one line serialise across the whole grid (about 0.4 ms per c4 run with a single
// copy), spread over 64 lines they overlap. The host XORs the copies.
constexpr int kAccCopies = 64;
constexpr int kAccStride = 64;  // words per copy (>= 4 * (kMaxD + 1))
constexpr int kAccSet = kAccCopies * kAccStride;
// Word kAccStride - 1 of copy 0 counts the finished workgroups; the last one XORs the copies and
// posts the points straight to host-mapped memory, then the round's sequence number in word
// kResSeq (so the host polls one word instead of queueing a copy and synchronising the stream).
constexpr int kAccCount = kAccStride - 1;
constexpr size_t kPostInKernelMaxWG = 64;  // grids up to this post in-kernel (else sc_post)
static_assert(kPostInKernelMaxWG <= (size_t)kAccCopies, "an in-kernel posting grid stores one copy per workgroup");
constexpr size_t kHexMaxItems = 8192;      // launches up to this many items use 16-lane products
constexpr size_t kWideMaxItems = 1024;     // ... and up to this many the 64-lane product
using namespace quad;
static_assert(kAccStride > 4 * (kMaxD + 1), "accumulator copy too small");
constexpr int kResSeq = 4 * (kMaxD + 1);

// out = k * x for a tower constant k < 16 acting on the 8 GF(2^4) coordinates of a limb; c[a]
// is the GF(2^4) product k * 2^a (host-computed, ScArgs::kcol). Alias-safe.
__device__ __forceinline__ void mul_small(const uint32_t* c, const uint32_t* x, uint32_t* out) {
#pragma unroll
	for (int g = 0; g < 8; g++) {
		uint32_t r[4];
#pragma unroll
		for (int b = 0; b < 4; b++) {
			r[b] = 0;
#pragma unroll
			for (int a = 0; a < 4; a++) r[b] ^= x[4 * g + a] & (0u - ((c[a] >> b) & 1u));
		}
#pragma unroll
		for (int b = 0; b < 4; b++) out[4 * g + b] = r[b];
	}
}

// x <- k x for k = 2 or 3 (m = 0 or ~0: k = 2 + (m & 1)), the same map as mul_small with 8 XORs
// per 4-word group instead of 16 AND-XORs: with X0^2 = X0 + 1, X0 (a0 + a1 X0) = a1 + (a0 + a1) X0 on
// both GF(2^2) halves of each GF(2^4) coordinate, plus m & x
__device__ __forceinline__ void mul_23(uint32_t m, uint32_t* x) {
#pragma unroll
	for (int g = 0; g < 8; g++) {
		const uint32_t b0 = x[4 * g], b1 = x[4 * g + 1], b2 = x[4 * g + 2], b3 = x[4 * g + 3];
		x[4 * g] = b1 ^ (b0 & m);
		x[4 * g + 1] = b0 ^ (b1 & ~m);
		x[4 * g + 2] = b3 ^ (b2 & m);
		x[4 * g + 3] = b2 ^ (b3 & ~m);
	}
}

// bit i = parity of (w[i] & mask): the limb of the sum over the batch's (masked) elements
__device__ __forceinline__ uint32_t parity_word(const uint32_t* w, uint32_t mask) {
	uint32_t r = 0;
#pragma unroll
	for (int i = 0; i < 32; i++) r |= (uint32_t)(__popc(w[i] & mask) & 1) << i;
	return r;
}

struct ScArgs {
	uint32_t* cols;
	size_t col_stride;  // words between columns
	int d;
	size_t n_pairs;     // batch pairs (big mode) or 1 (small modes)
	size_t hb;          // batch distance of a pair (big mode)
	int h;              // element distance of a pair inside the batch (small modes)
	int mode;           // 0 big, 1 in-batch pairs, 2 single element (cur == 1)
	int kmax;           // points 0..kmax
	int skip1;          // point 1 is not computed (the host derives it from the round claim)
	uint32_t r[4];      // fold challenge
	uint32_t* acc;      // kAccCopies x (kmax + 1) x 4 words, XOR-accumulated (this round's set)
	uint32_t* clr;      // the other accumulator set: cleared here for the next round
	uint32_t* res;      // host-mapped: 4 (kMaxD + 1) point words, then the sequence word
	uint32_t* sink;     // optional device copy of the raw point words + flags (bn_sumcheck_set_message_sink)
	uint32_t seq;       // this launch's sequence number
	int post;           // 1: the last workgroup posts the points (small grids), 0: sc_post does
	uint32_t kcol[kMaxD + 1][4];  // GF(2^4) products k * 2^a (interpolation point k)
#ifdef BN_SC_FUSED
	int fm_p;                     // sc_fold_msgs: pairs per work-group P
	uint32_t fm_magic;            // ... ceil(2^32 / (2 P)): item / (2 P) = umulhi(item, fm_magic) for items < 2^16
#endif
	int dbg;  // development build (BN_DEV) only: BN_SC_DBG bit 0 = synthetic operands instead of
	          // column loads, bit 1 = no products, bit 2 = no k-multiples, bit 3 = no parity
	          // reduction (wrong results; for timing experiments)
};

// lo/hi limbs of column j for pair p (this lane's limb l)
template <int MODE>
__device__ __forceinline__ void load_pair(const ScArgs& A, int j, size_t p, int l, uint32_t* lo, uint32_t* hi, uint32_t& emask) {
	const uint32_t* c = A.cols + (size_t)j * A.col_stride;
#ifdef BN_DEV
	if (A.dbg & 1) {
#pragma unroll
		for (int i = 0; i < 32; i++) {
			lo[i] = (uint32_t)p * 0x9E3779B9u + (uint32_t)(i * 7 + l + j);
			hi[i] = lo[i] * 0x85EBCA6Bu;
		}
		emask = ~0u;
		return;
	}
#endif
	if constexpr (MODE == 0) {
		ld32(lo, c + 128 * p + 32 * l);
		ld32(hi, c + 128 * (p + A.hb) + 32 * l);
		emask = ~0u;
	} else if constexpr (MODE == 1) {
		const uint32_t m = (1u << A.h) - 1u;
		uint32_t w[32];
		ld32(w, c + 32 * l);
#pragma unroll
		for (int i = 0; i < 32; i++) {
			lo[i] = w[i] & m;
			hi[i] = (w[i] >> A.h) & m;
		}
		emask = m;
	} else {
		ld32(lo, c + 32 * l);
#pragma unroll
		for (int i = 0; i < 32; i++) {
			lo[i] &= 1u;
			hi[i] = lo[i];  // k = 0 only: f = lo
		}
		emask = 1u;
	}
}

// Reduce the accumulator copies and post the points + sequence word to host-mapped memory.
__device__ __forceinline__ void post_points(const ScArgs& A, int t) {
	if (t < 4 * (A.kmax + 1)) {
		uint32_t v = 0;
		for (int c = 0; c < kAccCopies; c++)
			v ^= __hip_atomic_load(A.acc + c * kAccStride + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		A.res[t] = v;
		if (A.sink) A.sink[t] = v;
	}
	if (A.sink && t == 0) A.sink[kResSeq] = (uint32_t)A.skip1 | (A.mode == 2 ? 2u : 0u);
	__threadfence_system();
	__syncthreads();
	if (t == 0) __hip_atomic_store(A.res + kResSeq, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Timing-experiment builds only (make BUILD=build-x LIBDIR=lib-x EXTRA=-DBN_SC_SKIP_MID): the
// big rounds' quad products run 8 of their 12 GF(2^32) circuits (wrong results), the upper bound
// on what a 9-circuit Karatsuba top level could save (EXPERIMENTS.md section 5.3, round 5).
#ifdef BN_SC_SKIP_MID
constexpr bool kSkipMid = true;
#else
constexpr bool kSkipMid = false;
#endif

// Products run on a group of G lanes: G = 4 (quad_mul, throughput) for launches that fill the
// GPU, G = 16 (hex_mul, about a third of the latency) for the last rounds' small launches, G = 64
// (wide_mul, GF(2^16) circuits on 36 lanes) for the smallest. Lanes l < 4 of a group hold the
// limbs of the operands and results.
template <int G>
struct Grp {
	static constexpr int kGroups = kScThreads / G;
	static constexpr int kSlotWords = G == 4 ? kQuadWords : G == 16 ? kHexWords : kWideWords;
	static constexpr int kSlotsWords = kGroups * kSlotWords;
};
template <int G, bool B_SHARED>
__device__ __forceinline__ void grp_mul(const Slot& S, const uint32_t* B, int l, bool skip_mid = false) {
	if constexpr (G == 4)
		quad_mul<B_SHARED>(S, B, l, skip_mid);
	else if constexpr (G == 16)
		hex_mul<B_SHARED>(S, B, l);
	else
		wide_mul<B_SHARED>(S, B, l);
}

// One (pair, point k) per group, k fastest: the kmax+1 groups of a pair run side by side, so the
// pair's columns are read from HBM once and hit in cache for the other points.
template <int MODE, int G>
__global__ __launch_bounds__(kScThreads, kScMinWG) void sc_messages(ScArgs A) {
	extern __shared__ uint32_t lds[];
	const int l = threadIdx.x % G, qw = threadIdx.x / G;
	const Slot S{lds + qw * Grp<G>::kSlotWords};
	uint32_t* accL = lds + Grp<G>::kSlotsWords + 128;  // (kMaxD + 1) x 4 words
	if (threadIdx.x < 4 * (kMaxD + 1)) accL[threadIdx.x] = 0;
	// rounds alternate between two accumulator sets; the other set was last read back by the
	// previous round's copy (ordered before this launch), so no memset is queued per round
	if (blockIdx.x == 0)
		for (int i = threadIdx.x; i < kAccSet; i += kScThreads) A.clr[i] = 0;
	__syncthreads();
	const int npts = A.kmax + 1 - A.skip1;
	const size_t item = (size_t)blockIdx.x * Grp<G>::kGroups + qw;
	const size_t p = item / npts;
	const int ki = (int)(item % npts);
	const int k = (A.skip1 && ki >= 1) ? ki + 1 : ki;
	if (p < A.n_pairs) {
		uint32_t emask = 0;
		for (int j = 0; j < A.d; j++) {
			// f_j at point k: lo + k (lo + hi), written into the A (j == 0) or B operand
			if (l < 4) {
			uint32_t lo[32], hi[32];
			load_pair<MODE>(A, j, p, l, lo, hi, emask);
			if (k == 0) {
			} else if (k == 1) {
#pragma unroll
				for (int i = 0; i < 32; i++) lo[i] = hi[i];
			} else {
#pragma unroll
				for (int i = 0; i < 32; i++) hi[i] ^= lo[i];
#ifdef BN_DEV
				if (!(A.dbg & 4))
#endif
				{
					if (A.kmax <= 3)  // d <= 3: every k here is 2 or 3 (launch-uniform branch)
						mul_23(0u - (uint32_t)(k & 1), hi);
					else
						mul_small(A.kcol[k], hi, hi);
				}
#pragma unroll
				for (int i = 0; i < 32; i++) lo[i] ^= hi[i];
			}
			sst(S, (j == 0 ? 0 : 4) + l, lo);
			}
#ifdef BN_DEV
			if (A.dbg & 2) continue;
#endif
			if (j > 0) grp_mul<G, false>(S, nullptr, l, kSkipMid);
		}
		wsync();
		if (l < 4) {
		uint32_t t[32];
		sld(t, S, l);
#ifdef BN_DEV
		const uint32_t acc = (A.dbg & 8) ? t[0] ^ t[31] : parity_word(t, emask);
#else
		const uint32_t acc = parity_word(t, emask);
#endif
		if (acc) atomicXor(accL + 4 * k + l, acc);  // LDS atomic
		}
	}
	__syncthreads();
	if (!A.post) {
		if (threadIdx.x < 4 * (A.kmax + 1) && accL[threadIdx.x])
			atomicXor(A.acc + (blockIdx.x % kAccCopies) * kAccStride + threadIdx.x, accL[threadIdx.x]);
		return;  // sc_post follows
	}
	if (gridDim.x == 1) {  // a single workgroup posts its own sums
		if (threadIdx.x < 4 * (A.kmax + 1)) {
			A.res[threadIdx.x] = accL[threadIdx.x];
			if (A.sink) A.sink[threadIdx.x] = accL[threadIdx.x];
		}
		if (A.sink && threadIdx.x == 0) A.sink[kResSeq] = (uint32_t)A.skip1 | (A.mode == 2 ? 2u : 0u);
		__threadfence_system();
		__syncthreads();
		if (threadIdx.x == 0) __hip_atomic_store(A.res + kResSeq, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
		return;
	}
	// small grids (<= kAccCopies workgroups): workgroup b stores its sums into copy b with plain
	// stores, the last one to finish XORs the gridDim.x copies and posts the points itself
	const int nw = 4 * (A.kmax + 1);
	if (threadIdx.x < nw) A.acc[blockIdx.x * kAccStride + threadIdx.x] = accL[threadIdx.x];
	uint32_t* last = accL + 4 * (kMaxD + 1);  // (a static __shared__ word cost a workgroup per CU)
	__syncthreads();
	if (threadIdx.x == 0)
		// acq_rel: release orders this workgroup's stores before its count, acquire makes every other
		// workgroup's stores visible to the last one
		*last = __hip_atomic_fetch_add(A.acc + kAccCount, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
	__syncthreads();
	if (!*last) return;
	__threadfence();
	uint32_t* red = last + 1;  // 4 (kMaxD + 1) words
	if (threadIdx.x < nw) red[threadIdx.x] = 0;
	__syncthreads();
	// every (copy, word) by one thread, XOR-reduced in LDS
	for (int i = threadIdx.x; i < (int)gridDim.x * nw; i += kScThreads) {
		const int b = i / nw, w = i - b * nw;
		const uint32_t v = __hip_atomic_load(A.acc + b * kAccStride + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (v) atomicXor(red + w, v);
	}
	__syncthreads();
	if (threadIdx.x < nw) {
		A.res[threadIdx.x] = red[threadIdx.x];
		if (A.sink) A.sink[threadIdx.x] = red[threadIdx.x];
	}
	if (A.sink && threadIdx.x == 0) A.sink[kResSeq] = (uint32_t)A.skip1 | (A.mode == 2 ? 2u : 0u);
	__threadfence_system();
	__syncthreads();
	if (threadIdx.x == 0) __hip_atomic_store(A.res + kResSeq, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#ifdef BN_SC_FUSED
// sc_messages's body as device functions for the fused experiment kernel (sc_fold_msgs). The
// product kernel above keeps its own copy: the product build is round 5's code.
// the work-group's point sums in LDS (after the product slots); the accumulator set of the next
// round is cleared by workgroup 0 (rounds alternate between two sets; the other set was last read
// back by the previous round's post, ordered before this launch, so no memset is queued per round)
template <int G>
__device__ __forceinline__ uint32_t* messages_init(const ScArgs& A, uint32_t* lds) {
	uint32_t* accL = lds + Grp<G>::kSlotsWords + 128;  // (kMaxD + 1) x 4 words
	if (threadIdx.x < 4 * (kMaxD + 1)) accL[threadIdx.x] = 0;
	if (blockIdx.x == 0)
		for (int i = threadIdx.x; i < kAccSet; i += kScThreads) A.clr[i] = 0;
	return accL;
}

// point k of pair p on this group (when `valid`), then the work-group's reduction and posting
template <int MODE, int G>
__device__ __forceinline__ void messages_run(const ScArgs& A, uint32_t* lds, uint32_t* accL, size_t p, int k, bool valid) {
	const int l = threadIdx.x % G, qw = threadIdx.x / G;
	const Slot S{lds + qw * Grp<G>::kSlotWords};
	if (valid) {
		uint32_t emask = 0;
		for (int j = 0; j < A.d; j++) {
			// f_j at point k: lo + k (lo + hi), written into the A (j == 0) or B operand
			if (l < 4) {
			uint32_t lo[32], hi[32];
			load_pair<MODE>(A, j, p, l, lo, hi, emask);
			if (k == 0) {
			} else if (k == 1) {
#pragma unroll
				for (int i = 0; i < 32; i++) lo[i] = hi[i];
			} else {
#pragma unroll
				for (int i = 0; i < 32; i++) hi[i] ^= lo[i];
#ifdef BN_DEV
				if (!(A.dbg & 4))
#endif
				{
					if (A.kmax <= 3)  // d <= 3: every k here is 2 or 3 (launch-uniform branch)
						mul_23(0u - (uint32_t)(k & 1), hi);
					else
						mul_small(A.kcol[k], hi, hi);
				}
#pragma unroll
				for (int i = 0; i < 32; i++) lo[i] ^= hi[i];
			}
			sst(S, (j == 0 ? 0 : 4) + l, lo);
			}
#ifdef BN_DEV
			if (A.dbg & 2) continue;
#endif
			if (j > 0) grp_mul<G, false>(S, nullptr, l, kSkipMid);
		}
		wsync();
		if (l < 4) {
		uint32_t t[32];
		sld(t, S, l);
#ifdef BN_DEV
		const uint32_t acc = (A.dbg & 8) ? t[0] ^ t[31] : parity_word(t, emask);
#else
		const uint32_t acc = parity_word(t, emask);
#endif
		if (acc) atomicXor(accL + 4 * k + l, acc);  // LDS atomic
		}
	}
	__syncthreads();
	if (!A.post) {
		if (threadIdx.x < 4 * (A.kmax + 1) && accL[threadIdx.x])
			atomicXor(A.acc + (blockIdx.x % kAccCopies) * kAccStride + threadIdx.x, accL[threadIdx.x]);
		return;  // sc_post follows
	}
	if (gridDim.x == 1) {  // a single workgroup posts its own sums
		if (threadIdx.x < 4 * (A.kmax + 1)) {
			A.res[threadIdx.x] = accL[threadIdx.x];
			if (A.sink) A.sink[threadIdx.x] = accL[threadIdx.x];
		}
		if (A.sink && threadIdx.x == 0) A.sink[kResSeq] = (uint32_t)A.skip1 | (A.mode == 2 ? 2u : 0u);
		__threadfence_system();
		__syncthreads();
		if (threadIdx.x == 0) __hip_atomic_store(A.res + kResSeq, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
		return;
	}
	// small grids (<= kAccCopies workgroups): workgroup b stores its sums into copy b with plain
	// stores, the last one to finish XORs the gridDim.x copies and posts the points itself
	const int nw = 4 * (A.kmax + 1);
	if (threadIdx.x < nw) A.acc[blockIdx.x * kAccStride + threadIdx.x] = accL[threadIdx.x];
	uint32_t* last = accL + 4 * (kMaxD + 1);  // (a static __shared__ word cost a workgroup per CU)
	__syncthreads();
	if (threadIdx.x == 0)
		// acq_rel: release orders this workgroup's stores before its count, acquire makes every other
		// workgroup's stores visible to the last one
		*last = __hip_atomic_fetch_add(A.acc + kAccCount, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
	__syncthreads();
	if (!*last) return;
	__threadfence();
	uint32_t* red = last + 1;  // 4 (kMaxD + 1) words
	if (threadIdx.x < nw) red[threadIdx.x] = 0;
	__syncthreads();
	// every (copy, word) by one thread, XOR-reduced in LDS
	for (int i = threadIdx.x; i < (int)gridDim.x * nw; i += kScThreads) {
		const int b = i / nw, w = i - b * nw;
		const uint32_t v = __hip_atomic_load(A.acc + b * kAccStride + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (v) atomicXor(red + w, v);
	}
	__syncthreads();
	if (threadIdx.x < nw) {
		A.res[threadIdx.x] = red[threadIdx.x];
		if (A.sink) A.sink[threadIdx.x] = red[threadIdx.x];
	}
	if (A.sink && threadIdx.x == 0) A.sink[kResSeq] = (uint32_t)A.skip1 | (A.mode == 2 ? 2u : 0u);
	__threadfence_system();
	__syncthreads();
	if (threadIdx.x == 0) __hip_atomic_store(A.res + kResSeq, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#endif  // BN_SC_FUSED

// Big grids: a one-wave kernel after sc_messages reduces the copies and posts the points (one
// counter shared by thousands of workgroups serialised them: 2x the kernel time).
__global__ __launch_bounds__(64) void sc_post(ScArgs A) { post_points(A, threadIdx.x); }

template <int MODE, int G>
__global__ __launch_bounds__(kScThreads, kScMinWG) void sc_fold(ScArgs A) {
	extern __shared__ uint32_t lds[];
	const int l = threadIdx.x % G, qw = threadIdx.x / G;
	const Slot S{lds + qw * Grp<G>::kSlotWords};
	uint32_t* R = lds + Grp<G>::kSlotsWords;  // the challenge, broadcast-bitsliced, shared
	if (threadIdx.x < 128) R[threadIdx.x] = 0u - ((A.r[threadIdx.x / 32] >> (threadIdx.x % 32)) & 1u);
	__syncthreads();
	const size_t items = (size_t)A.d * A.n_pairs;
	const size_t it = (size_t)blockIdx.x * Grp<G>::kGroups + qw;
	if (it < items) {  // one item per group (no grid-stride loop: it costs registers)
		const int j = (int)(it / A.n_pairs);
		const size_t p = it % A.n_pairs;
		uint32_t lo[32], hi[32], emask;
		if (l < 4) {
			load_pair<MODE>(A, j, p, l, lo, hi, emask);
#pragma unroll
			for (int i = 0; i < 32; i++) hi[i] ^= lo[i];
			sst(S, l, hi);
		}
#ifdef BN_DEV
		if (!(A.dbg & 2))
#endif
		grp_mul<G, true>(S, R, l, kSkipMid);
		if (l >= 4) return;
		// lo is re-read (cache-resident) rather than kept live across the quad product; the hex
		// product leaves the registers for it
		if constexpr (G == 4) load_pair<MODE>(A, j, p, l, lo, hi, emask);
		sld(hi, S, l);
#pragma unroll
		for (int i = 0; i < 32; i++) lo[i] = (lo[i] ^ hi[i]) & emask;
		wsync();
		st32(A.cols + (size_t)j * A.col_stride + 128 * p + 32 * l, lo);
	}
}

// Big-mode fold with wave-coalesced global traffic (n_pairs % 16 == 0): a wave's 16 quads take
// 16 consecutive pairs of one column, so its lo and hi batches are two contiguous 8 KiB runs.
// Lane t moves 16 B at byte 16 t + 1 KiB i (i < 8) and the LDS slots do the transposition to
// the quads' limb rows (sc_fold<0>, one 128-B line per lane per instruction, took 13% longer:
// c4 d=3 round 0, 434 -> 384 us).
__device__ __forceinline__ uint32_t* coal_addr(uint32_t* wslots, int lane, int i) {
	const int w = 4 * lane + 256 * i;  // word offset in the wave's 16-batch run
	return wslots + (w >> 7) * kQuadWords + kRowWords * ((w >> 5) & 3) + (w & 31);
}

__global__ __launch_bounds__(kScThreads, kScMinWG) void sc_fold_coal(ScArgs A) {
	extern __shared__ uint32_t lds[];
	const int l = threadIdx.x & 3, qw = threadIdx.x >> 2, lane = threadIdx.x & 63;
	const Slot S{lds + qw * kQuadWords};
	uint32_t* wslots = lds + (qw & ~15) * kQuadWords;
	uint32_t* R = lds + kQuadsPerWG * kQuadWords;
	if (threadIdx.x < 128) R[threadIdx.x] = 0u - ((A.r[threadIdx.x / 32] >> (threadIdx.x % 32)) & 1u);
	__syncthreads();
	const size_t it0 = (size_t)blockIdx.x * kQuadsPerWG + (qw & ~15);  // the wave's first item
	if (it0 >= (size_t)A.d * A.n_pairs) return;
	const int j = (int)(it0 / A.n_pairs);
	const size_t p0 = it0 % A.n_pairs;
	uint32_t* lo = A.cols + (size_t)j * A.col_stride + 128 * p0;
	const uint32_t* hi = lo + 128 * A.hb;
#pragma unroll
	for (int i = 0; i < 8; i++) {
		const uint4 a = *(const uint4*)(lo + 4 * lane + 256 * i), b = *(const uint4*)(hi + 4 * lane + 256 * i);
		*(uint4*)coal_addr(wslots, lane, i) = make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
	}
#ifdef BN_DEV
	if (!(A.dbg & 2))
#endif
	quad_mul<true>(S, R, l, kSkipMid);
	wsync();
#pragma unroll
	for (int i = 0; i < 8; i++) {
		const uint4 a = *(const uint4*)(lo + 4 * lane + 256 * i), q = *(const uint4*)coal_addr(wslots, lane, i);
		*(uint4*)(lo + 4 * lane + 256 * i) = make_uint4(a.x ^ q.x, a.y ^ q.y, a.z ^ q.z, a.w ^ q.w);
	}
}

// Big-mode fold on lane PAIRS (n_pairs % 32 == 0): the product r (lo + hi) has a constant operand,
// the same challenge r for every lane, so its Karatsuba leaves and sums are scalar work. Lane u of
// a pair holds the GF(2^64) half a_u (words 64u..64u+63) of s = lo + hi and forms, with r = r0 +
// r1 X (compact words A.r[0..3]),
//   T = a_u r1            (bsm6_fma_w2: three GF(2^32) circuits whose twiddle side is SGPR bits)
//   the pair swaps T (DPP): lane 0 gets a_1 r1, lane 1 gets a_0 r1
//   lane 0: a_0 r0 + a_1 r1                 = c_lo
//   lane 1: a_1 r0 + a_0 r1 + alpha64(a_1 r1) = c_hi
// (the schoolbook top level of quad_mul with P_ij = a_i r_j). Per product: 6 constant-operand
// GF(2^32) circuits on 2 lanes instead of 12 general ones on 4, and no operand rows in LDS.
// A wave takes 32 consecutive pairs of one column: coalesced 16-B loads as sc_fold_coal, staged
// in LDS rows of 64 words padded to 68 (16 lanes of a ds_read_b128 then hit distinct banks). The
// rows hold s until every lane has read its row, then lo (kept in registers from the loads), so
// the result lo + r s needs no second read of lo from HBM (that re-read was a third of the
// kernel's HBM reads); x stays in registers through both products, opaque to the compiler so the
// two products do not share (and keep live) their data-side sums.
constexpr int kPairRowWords = 68;
constexpr int kPairWaveWords = 64 * kPairRowWords;  // 64 lane rows per wave
constexpr int kPairItemsPerWG = kScThreads / 2;
constexpr size_t kPairMinItems = 384 * (size_t)kPairItemsPerWG;
__device__ __forceinline__ uint32_t* pair_addr(uint32_t* slot, int w) { return slot + (w >> 6) * kPairRowWords + (w & 63); }

#ifdef BN_SC_FUSED
// One wave's 32 lane-pair folds. Item q < 32 of the wave folds batch lo_of(q) (nullptr: no item)
// with the batch 2 A.n_pairs further on, in place. Lane t of the wave moves 16 B of item (t >> 5) + 2 i at
// word (4 t) & 127 for i < 16: coalesced 512-B pieces.
// (sc_fold_pair keeps its own copy of this body with one base pointer per wave: a per-item pointer
// here made the product kernel 35 % slower, round 6)
template <bool MAYBE_NULL, class LoOf>
__device__ __forceinline__ void fold_pair_wave(const ScArgs& A, uint32_t* slot, int lane, LoOf lo_of) {
	const int u = lane & 1;
	uint4 la[16];
#pragma unroll
	for (int i = 0; i < 16; i++) {
		const int w = 4 * lane + 256 * i;
		const uint32_t* lo = lo_of(w >> 7);
		uint4 b = make_uint4(0, 0, 0, 0);
		la[i] = b;
		if (!MAYBE_NULL || lo) {
			b = *(const uint4*)(lo + 256 * A.n_pairs + (w & 127));  // old pair distance 2 hb'

			la[i] = *(const uint4*)(lo + (w & 127));
		}
		*(uint4*)pair_addr(slot, w) = make_uint4(la[i].x ^ b.x, la[i].y ^ b.y, la[i].z ^ b.z, la[i].w ^ b.w);
	}
	wsync();
	uint32_t* row = slot + lane * kPairRowWords;
	uint32_t x[64], t[64];
#pragma unroll
	for (int i = 0; i < 64; i += 4) {
		const uint4 v = *(const uint4*)(row + i);
		x[i] = v.x, x[i + 1] = v.y, x[i + 2] = v.z, x[i + 3] = v.w;
	}
	wsync();  // every row read: the rows take lo
#pragma unroll
	for (int i = 0; i < 16; i++) *(uint4*)pair_addr(slot, 4 * lane + 256 * i) = la[i];
#pragma unroll
	for (int i = 0; i < 64; i++) t[i] = 0;
#ifdef BN_DEV
	if (!(A.dbg & 2))
#endif
	bsm6_fma_w2(x, A.r[2], A.r[3], t);  // a_u r1
	const uint32_t m = 0u - (uint32_t)u;
	uint32_t o[64];
	{
		uint32_t ah[32];
		bs_alpha<5>(t + 32, ah);
#pragma unroll
		for (int i = 0; i < 32; i++) {
			o[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)t[i], 0xB1, 0xF, 0xF, false) ^ (t[32 + i] & m);
			o[32 + i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)t[32 + i], 0xB1, 0xF, 0xF, false) ^ ((t[i] ^ ah[i]) & m);
		}
	}
	// (x opaque: the compiler would otherwise share the two products' data-side sums)
#pragma unroll
	for (int i = 0; i < 64; i++) asm volatile("" : "+v"(x[i]));
#ifdef BN_DEV
	if (!(A.dbg & 2))
#endif
	bsm6_fma_w2(x, A.r[0], A.r[1], o);  // + a_u r0
	wsync();
#pragma unroll
	for (int i = 0; i < 64; i += 4) {
		const uint4 v = *(const uint4*)(row + i);
		*(uint4*)(row + i) = make_uint4(o[i] ^ v.x, o[i + 1] ^ v.y, o[i + 2] ^ v.z, o[i + 3] ^ v.w);
	}
	wsync();
#pragma unroll
	for (int i = 0; i < 16; i++) {
		const int w = 4 * lane + 256 * i;
		uint32_t* lo = lo_of(w >> 7);
		if (!MAYBE_NULL || lo) *(uint4*)(lo + (w & 127)) = *(const uint4*)pair_addr(slot, w);
	}
}

#endif  // BN_SC_FUSED

__global__ __launch_bounds__(kScThreads, kScMinWG) void sc_fold_pair(ScArgs A) {
	extern __shared__ uint32_t lds[];
	const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, u = lane & 1;
	uint32_t* slot = lds + wave * kPairWaveWords;
	const size_t it0 = (size_t)blockIdx.x * kPairItemsPerWG + 32 * wave;  // the wave's first item
	if (it0 >= (size_t)A.d * A.n_pairs) return;
	const int j = (int)(it0 / A.n_pairs);
	const size_t p0 = it0 % A.n_pairs;
	uint32_t* lo = A.cols + (size_t)j * A.col_stride + 128 * p0;
	const uint32_t* hi = lo + 128 * A.hb;
	uint4 la[16];
#pragma unroll
	for (int i = 0; i < 16; i++) {
		const int w = 4 * lane + 256 * i;
		const uint4 b = *(const uint4*)(hi + w);
		la[i] = *(const uint4*)(lo + w);
		*(uint4*)pair_addr(slot, w) = make_uint4(la[i].x ^ b.x, la[i].y ^ b.y, la[i].z ^ b.z, la[i].w ^ b.w);
	}
	wsync();
	uint32_t* row = slot + lane * kPairRowWords;
	uint32_t x[64], t[64];
#pragma unroll
	for (int i = 0; i < 64; i += 4) {
		const uint4 v = *(const uint4*)(row + i);
		x[i] = v.x, x[i + 1] = v.y, x[i + 2] = v.z, x[i + 3] = v.w;
	}
	wsync();  // every row read: the rows take lo
#pragma unroll
	for (int i = 0; i < 16; i++) *(uint4*)pair_addr(slot, 4 * lane + 256 * i) = la[i];
#pragma unroll
	for (int i = 0; i < 64; i++) t[i] = 0;
#ifdef BN_DEV
	if (!(A.dbg & 2))
#endif
	bsm6_fma_w2(x, A.r[2], A.r[3], t);  // a_u r1
	const uint32_t m = 0u - (uint32_t)u;
	uint32_t o[64];
	{
		uint32_t ah[32];
		bs_alpha<5>(t + 32, ah);
#pragma unroll
		for (int i = 0; i < 32; i++) {
			o[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)t[i], 0xB1, 0xF, 0xF, false) ^ (t[32 + i] & m);
			o[32 + i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)t[32 + i], 0xB1, 0xF, 0xF, false) ^ ((t[i] ^ ah[i]) & m);
		}
	}
	// (x opaque: the compiler would otherwise share the two products' data-side sums)
#pragma unroll
	for (int i = 0; i < 64; i++) asm volatile("" : "+v"(x[i]));
#ifdef BN_DEV
	if (!(A.dbg & 2))
#endif
	bsm6_fma_w2(x, A.r[0], A.r[1], o);  // + a_u r0
	wsync();
#pragma unroll
	for (int i = 0; i < 64; i += 4) {
		const uint4 v = *(const uint4*)(row + i);
		*(uint4*)(row + i) = make_uint4(o[i] ^ v.x, o[i + 1] ^ v.y, o[i + 2] ^ v.z, o[i + 3] ^ v.w);
	}
	wsync();
#pragma unroll
	for (int i = 0; i < 16; i++) {
		const int w = 4 * lane + 256 * i;
		*(uint4*)(lo + w) = *(const uint4*)pair_addr(slot, w);
	}
}

#ifdef BN_SC_FUSED
// Round i's fold fused with round i + 1's messages (the QM31 sibling's
// qm_fold_messages in GF(2^128) form). A work-group owns P = kGroups / npts consecutive pairs
// p0 .. p0 + P - 1 of the folded columns (pair distance hb' = A.n_pairs). Phase 1 folds the 2 P d
// batches they consist of, p' and p' + hb' of every column (old pairs (b, b + 2 hb')), on lane
// pairs as sc_fold_pair, and writes them in place. Phase 2 runs the
// messages of those P pairs on the quads as sc_messages, reading the batches the work-group has
// just written (L2) instead of a second kernel reading them back from HBM; one launch per round
// instead of two. No other work-group reads what this one writes: pair p' reads old batches p',
// p' + hb', p' + 2 hb', p' + 3 hb' and writes p', p' + hb' only.
__global__ __launch_bounds__(kScThreads, kScMinWG) void sc_fold_msgs(ScArgs A) {
	extern __shared__ uint32_t lds[];
	const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	const int npts = A.kmax + 1 - A.skip1;
	const int P = A.fm_p;
	const size_t p0 = (size_t)blockIdx.x * P;
	const size_t hbn = A.n_pairs;
	uint32_t* accL = messages_init<4>(A, lds);
	// phase 1: item v of column j (v < 2 P) folds batch p0 + v (v < P) or hb' + p0 + v - P
	const int items = 2 * P * A.d;
	if (32 * wave < items) {
		fold_pair_wave<true>(A, lds + wave * kPairWaveWords, lane, [&](int q) -> uint32_t* {
			const int it = 32 * wave + q;
			if (it >= items) return nullptr;
			const int j = (int)__umulhi((uint32_t)it, A.fm_magic), v = it - j * 2 * P;
			const size_t pp = p0 + (size_t)(v < P ? v : v - P);
			if (pp >= hbn) return nullptr;
			return A.cols + (size_t)j * A.col_stride + 128 * (v < P ? pp : pp + hbn);
		});
	}
	// every fold of the work-group is in memory (L2) and the fold's LDS rows are free
	__syncthreads();
	const int qw = threadIdx.x / 4;
	const int lp = qw / npts, ki = qw - lp * npts;
	const int k = (A.skip1 && ki >= 1) ? ki + 1 : ki;
	messages_run<0, 4>(A, lds, accL, p0 + (size_t)lp, k, lp < P && p0 + (size_t)lp < hbn);
}
#endif  // BN_SC_FUSED
// ---------------------------------------------------------------------------------------
// Round server for the last rounds (at most kServerMaxCur evaluations per column left): ONE
// resident 768-thread workgroup runs every remaining round by itself. It waits for the host's
// challenge in host-mapped control words, folds, computes the next round's messages on 64-lane
// products (wide_mul) and posts them exactly as sc_messages does (points, then the sequence word). A small
// round then costs no kernel launch, no dispatch ramp and no cross-workgroup reduction: with one
// fold and one messages launch per round the last rounds of c4 took ~10 us (fold) + ~18 us
// (messages) of kernel time plus ~12 us of host launches each (round-4 trace).
// A waiting server holds its hardware queue, and work that other streams of the process queue
// behind it on the same queue (HIP maps streams onto a few queues) waits too. So the wait is short
// (kSrvTimeoutTicks of s_memrealtime): a server that gets no challenge in time records the last
// ticket it served (kCtlExit) and ends, and the host relaunches one when it next needs it
// (bn_sumcheck_round_messages). bn_sumcheck_destroy posts kSrvStop.
// ---------------------------------------------------------------------------------------
constexpr int kSrvThreads = 768;  // 12 waves: three per SIMD (the wide product fits 168 VGPRs)
constexpr int kSrvG = 64;  // wide_mul: latency is all that counts here (a few items per round)
constexpr int kSrvGroups = kSrvThreads / kSrvG;
#ifndef BN_SC_SERVER_MAX
#define BN_SC_SERVER_MAX 512
#endif
constexpr size_t kServerMaxCur = BN_SC_SERVER_MAX;  // (-DBN_SC_SERVER_MAX=0: no server, A/B builds)
constexpr uint32_t kSrvStop = 0xFFFFFFFFu;
constexpr int kCtlR = 0, kCtlSkip = 4, kCtlTicket = 5, kCtlExit = 6, kCtlWords = 8;  // host-mapped control words
constexpr uint32_t kSrvRunning = 0xFFFFFFFEu;                   // kCtlExit while a server may be alive
constexpr unsigned long long kSrvTimeoutTicks = 20000ull;        // 200 us at 100 MHz

struct SrvArgs {
	uint32_t* cols;
	size_t col_stride;
	int d;
	size_t cur;           // evaluations per column before the first fold
	uint32_t* res;        // host-mapped points + sequence word (as ScArgs::res)
	const uint32_t* ctl;  // host-mapped control words: challenge, skip-p(1) flag, ticket
	uint32_t* ctl_exit;   // ... kCtlExit: the last ticket served by a server that timed out
	uint32_t seq;         // sequence number of the first posted round
	uint32_t ticket;      // ticket of the first challenge
	uint32_t kcol[kMaxD + 1][4];
	unsigned long long* trace;  // development build: per round, s_memrealtime at wake, fold, messages, post
};

template <int MODE>
__device__ __forceinline__ void srv_fold(const ScArgs& a, const Slot& S, const uint32_t* R, int qw, int l) {
	const size_t items = (size_t)a.d * a.n_pairs;
	for (size_t it = qw; it < items; it += kSrvGroups) {
		const int j = (int)(it / a.n_pairs);
		const size_t p = it % a.n_pairs;
		uint32_t lo[32], hi[32], emask = 0;
		if (l < 4) {
			load_pair<MODE>(a, j, p, l, lo, hi, emask);
#pragma unroll
			for (int i = 0; i < 32; i++) hi[i] ^= lo[i];
			sst(S, l, hi);
		}
		grp_mul<kSrvG, true>(S, R, l);
		if (l < 4) {
			sld(hi, S, l);
			uint32_t* o = a.cols + (size_t)j * a.col_stride + (MODE == 0 ? 128 * p : 0) + 32 * l;
			if (MODE == 0) {
#pragma unroll
				for (int i = 0; i < 32; i++) lo[i] ^= hi[i];
			} else {
				// in-batch pairs: the folded values replace the low half's bit-lanes
#pragma unroll
				for (int i = 0; i < 32; i++) lo[i] = (lo[i] ^ hi[i]) & emask;
			}
			st32(o, lo);
		}
		wsync();
	}
}

template <int MODE>
__device__ __forceinline__ void srv_messages(const ScArgs& a, const uint32_t (*kcol)[4], const Slot& S, uint32_t* accL, int qw,
                                             int l) {
	const int npts = a.kmax + 1 - a.skip1;
	const size_t items = a.n_pairs * (size_t)npts;
	for (size_t item = qw; item < items; item += kSrvGroups) {
		const size_t p = item / npts;
		const int ki = (int)(item % npts);
		const int k = (a.skip1 && ki >= 1) ? ki + 1 : ki;
		uint32_t emask = 0;
		for (int j = 0; j < a.d; j++) {
			if (l < 4) {
				uint32_t lo[32], hi[32];
				load_pair<MODE>(a, j, p, l, lo, hi, emask);
				if (k == 1) {
#pragma unroll
					for (int i = 0; i < 32; i++) lo[i] = hi[i];
				} else if (k > 1) {
#pragma unroll
					for (int i = 0; i < 32; i++) hi[i] ^= lo[i];
					if (a.kmax <= 3)
						mul_23(0u - (uint32_t)(k & 1), hi);
					else
						mul_small(kcol[k], hi, hi);
#pragma unroll
					for (int i = 0; i < 32; i++) lo[i] ^= hi[i];
				}
				sst(S, (j == 0 ? 0 : 4) + l, lo);
			}
			if (j > 0) grp_mul<kSrvG, false>(S, nullptr, l);
		}
		wsync();
		if (l < 4) {
			uint32_t t[32];
			sld(t, S, l);
			const uint32_t acc = parity_word(t, emask);
			if (acc) atomicXor(accL + 4 * k + l, acc);
		}
		wsync();
	}
}

__global__ __launch_bounds__(kSrvThreads, 1) void sc_server(SrvArgs P) {
	extern __shared__ uint32_t lds[];
	const int l = threadIdx.x % kSrvG, qw = threadIdx.x / kSrvG;
	const Slot S{lds + qw * Grp<kSrvG>::kSlotWords};
	uint32_t* R = lds + kSrvGroups * Grp<kSrvG>::kSlotWords;  // the challenge, broadcast-bitsliced
	uint32_t* accL = R + 128;                    // (kMaxD + 1) x 4 point words
	uint32_t* ctlL = accL + 4 * (kMaxD + 1);     // [0] wake-up reason, [1] skip-p(1) flag, [2..5] challenge
	ScArgs a{};
	a.cols = P.cols;
	a.col_stride = P.col_stride;
	a.d = P.d;
	size_t cur = P.cur;
	uint32_t seq = P.seq, ticket = P.ticket;
	for (;;) {
		// ---- the host's challenge for the fold of this round
		if (threadIdx.x == 0) {
			const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
			uint32_t why = 2;  // timed out
			for (;;) {
				const uint32_t t = __hip_atomic_load(P.ctl + kCtlTicket, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
				if (t == ticket) { why = 0; break; }
				if (t == kSrvStop) { why = 1; break; }
				if (__builtin_amdgcn_s_memrealtime() - t0 > kSrvTimeoutTicks) break;
				__builtin_amdgcn_s_sleep(2);
			}
			ctlL[0] = why;
			// the words the ticket publishes, read by the thread whose acquire saw it
			ctlL[1] = __hip_atomic_load(P.ctl + kCtlSkip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			for (int i = 0; i < 4; i++)
				ctlL[2 + i] = __hip_atomic_load(P.ctl + kCtlR + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		}
		__syncthreads();
#ifdef BN_DEV
		unsigned long long* trw = P.trace ? P.trace + 4 * (size_t)(ticket % 64) : nullptr;
		if (trw && threadIdx.x == 0) trw[0] = __builtin_amdgcn_s_memrealtime();
#endif
		if (ctlL[0] != 0) {
			// timed out: tell the host which ticket was served last (it relaunches for the next)
			if (ctlL[0] == 2 && threadIdx.x == 0)
				__hip_atomic_store(P.ctl_exit, ticket - 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
			return;
		}
		if (threadIdx.x < 128) R[threadIdx.x] = 0u - ((ctlL[2 + threadIdx.x / 32] >> (threadIdx.x % 32)) & 1u);
		if (threadIdx.x < 4 * (kMaxD + 1)) accL[threadIdx.x] = 0;
		__syncthreads();
		// ---- fold: cur -> cur / 2
		a.n_pairs = cur >= 64 ? cur / 64 : 1;
		a.hb = cur / 64;
		a.h = (int)(cur / 2);
		if (cur >= 64)
			srv_fold<0>(a, S, R, qw, l);
		else
			srv_fold<1>(a, S, R, qw, l);
		cur /= 2;
		__syncthreads();  // every folded column word is written (one CU: the workgroup's fence suffices)
#ifdef BN_DEV
		if (trw && threadIdx.x == 0) trw[1] = __builtin_amdgcn_s_memrealtime();
#endif
		// ---- the next round's messages
		const int mode = cur >= 64 ? 0 : cur >= 2 ? 1 : 2;
		a.mode = mode;
		a.n_pairs = cur >= 64 ? cur / 64 : 1;
		a.hb = cur / 64;
		a.h = (int)(cur / 2);
		a.kmax = mode == 2 ? 0 : a.d;
		a.skip1 = mode == 2 ? 0 : (int)(ctlL[1] & 1u);
		if (mode == 0)
			srv_messages<0>(a, P.kcol, S, accL, qw, l);
		else if (mode == 1)
			srv_messages<1>(a, P.kcol, S, accL, qw, l);
		else
			srv_messages<2>(a, P.kcol, S, accL, qw, l);
		__syncthreads();
#ifdef BN_DEV
		if (trw && threadIdx.x == 0) trw[2] = __builtin_amdgcn_s_memrealtime();
#endif
		if (threadIdx.x < 4 * (a.kmax + 1)) P.res[threadIdx.x] = accL[threadIdx.x];
		__threadfence_system();
		__syncthreads();
#ifdef BN_DEV
		if (trw && threadIdx.x == 0) trw[3] = __builtin_amdgcn_s_memrealtime();
#endif
		if (threadIdx.x == 0) __hip_atomic_store(P.res + kResSeq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
		if (cur == 1) return;  // the final evaluation is posted: no fold left
		seq++;
		ticket++;
	}
}

size_t srv_lds_bytes() { return ((size_t)kSrvGroups * Grp<kSrvG>::kSlotWords + 128 + 4 * (kMaxD + 1) + 6) * sizeof(uint32_t); }

// quad slots + the fold's broadcast challenge (128 words) + the messages' accumulators, flag and
// last-workgroup reduction
template <int G>
size_t lds_bytes() { return ((size_t)Grp<G>::kSlotsWords + 128 + 8 * (kMaxD + 1) + 1) * sizeof(uint32_t); }

struct DeviceScope {
	int prev = -1;
	bool ok = true;
	explicit DeviceScope(int dev) {
		if (hipGetDevice(&prev) != hipSuccess) prev = -1;
		if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
	}
	~DeviceScope() {
		int cur = -1;
		if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
	}
};

}  // namespace
}  // namespace bn

struct bn_sumcheck {
	int device = 0;
	int num_vars = 0, d = 0;
	int rank = 0, world = 1;
	int round = 0;
	size_t cur = 0;         // evaluations per column held by this prover
	size_t col_words = 0;   // words between columns (allocation)
	uint32_t* cols = nullptr;
	uint32_t* acc = nullptr;    // 2 sets of kAccSet words (see kAccCopies), alternating rounds
	int par = 0;                // set used by the next round_messages
	uint32_t* h_res = nullptr;  // host-mapped, GPU-coherent: the round's points + sequence word
	uint32_t* sink = nullptr;   // caller's device buffer for the raw point words (sharded exchange)
	uint32_t* d_res = nullptr;  // its device address
	uint32_t seq = 0;
	hipStream_t stream = nullptr;
	bool sharded_used = false;
	// bn_sumcheck_create_staged leaves compact input untransposed until bn_sumcheck_prepare (the
	// reference constructor's separate Memcpy and Transpose phases, sumcheck.cuh:88-124)
	bool prepared = true;
	int compact_input = 0;
	// Round claim: once round i's points are known, move_to_next_round(r) interpolates them at r,
	// which is this prover's sum for round i + 1 (p_i(r) = sum_x prod_j f_j'(x), per shard too).
	// Round i + 1 then skips point 1 (p(1) = claim + p(0)): (d - 1) fewer products per pair.
	// The interpolation itself runs in the next round_messages, while its kernel is in flight.
	bool have_pts = false, have_claim = false, claim_pending = false;
	// bn_sumcheck_round_messages_sink: the round's points went to the sink unread by the prover; the
	// caller (the sharded driver) holds the GLOBAL points and completes a skipped p(1) itself
	bool pts_external = false;
	uint32_t last_pts[4 * (bn::quad::kMaxD + 1)];
	uint32_t claim[4], pending_r[4];
	// move_to_next_round queues the next round's messages kernel right behind the fold, so the
	// GPU never waits for the host's next call (composition_eval, which only folds, does not)
	bool msgs_queued = false, eager = true;
	// BN_SUMCHECK_FULL_POINTS=1 (read when the prover is created): every round computes p(1) and
	// the sum from the data instead of deriving them from the claim, so the verifier's
	// p(0) + p(1) == previous p(r) check also tests the folds (tests/test_gpu_sumcheck.py)
	bool derive_p1 = !(getenv("BN_SUMCHECK_FULL_POINTS") && atoi(getenv("BN_SUMCHECK_FULL_POINTS")) != 0);
	// round server (sc_server) for the last rounds: running once launched until cur == 1
	uint32_t* h_ctl = nullptr;  // host-mapped control words (challenge, skip flag, ticket)
	bool server = false;
	uint32_t ticket = 0;
	size_t server_max_cur = bn::kServerMaxCur;  // BN_SC_SERVER_MAX_CUR (development build) overrides
	uint32_t last_sum[4] = {0, 0, 0, 0}, last_points[4 * (bn::quad::kMaxD + 1)];  // the round read last
	unsigned long long* h_trace = nullptr;  // development build (BN_SC_TIMING): the server's phase stamps
	double t_post = 0;                      // ... and the host's time of the last challenge post
	bool read_this_round = false;
	bool gathered = false;  // built by bn_sumcheck_import_gathered (no round server: server_eligible)
};

namespace {

using namespace bn;
using namespace bn::quad;

int sc_launch(bn_sumcheck* sc, bool fold, const uint32_t* r) {
	ScArgs A{};
	A.cols = sc->cols;
	A.col_stride = sc->col_words;
	A.d = sc->d;
	if (sc->cur >= 64) {
		A.mode = 0;
		A.n_pairs = sc->cur / 64;
		A.hb = sc->cur / 64;
		A.kmax = sc->d;
	} else if (sc->cur >= 2) {
		A.mode = 1;
		A.n_pairs = 1;
		A.h = (int)(sc->cur / 2);
		A.kmax = sc->d;
	} else {
		A.mode = 2;
		A.n_pairs = 1;
		A.kmax = 0;
	}
	A.skip1 = (!fold && (sc->have_claim || sc->claim_pending) && A.mode != 2) ? 1 : 0;
	A.res = sc->d_res;
	A.sink = fold ? nullptr : sc->sink;
	if (!fold) A.seq = ++sc->seq;
	A.acc = sc->acc + kAccSet * sc->par;
	A.clr = sc->acc + kAccSet * (1 - sc->par);
	if (fold) memcpy(A.r, r, 16);
#ifdef BN_DEV
	{
		static const int dbg = getenv("BN_SC_DBG") ? atoi(getenv("BN_SC_DBG")) : 0;
		A.dbg = dbg;
	}
#endif
	// GF(2^4) products k * 2^a, tabulated once (36 recursive tower products per launch were ~1 us of
	// host time on every round's critical path)
	struct KCol {
		uint32_t v[kMaxD + 1][4];
		KCol() {
			for (int k = 0; k <= kMaxD; k++)
				for (int a = 0; a < 4; a++) v[k][a] = (uint32_t)tw_mul((uint64_t)k, 1ull << a, 2);
		}
	};
	static const KCol kc;
	memcpy(A.kcol, kc.v, sizeof A.kcol);
	// one item per lane group: fold (column, pair), messages (pair, point)
	const size_t items = fold ? (size_t)sc->d * A.n_pairs : A.n_pairs * (size_t)(A.kmax + 1 - A.skip1);
	size_t hex_max = kHexMaxItems, wide_max = kWideMaxItems, post_max = kPostInKernelMaxWG;
#ifdef BN_DEV
	{
		static const char *eh = getenv("BN_SC_HEX_MAX"), *ew = getenv("BN_SC_WIDE_MAX"), *ep = getenv("BN_SC_POST_MAX");
		if (eh) hex_max = (size_t)atol(eh);
		if (ew) wide_max = (size_t)atol(ew);
		if (ep) post_max = std::min((size_t)atol(ep), (size_t)kAccCopies);
	}
#endif
	// 64-, 16-, 4-lane products; folds stay on 16 lanes (one product each: the 64-lane product's
	// extra combine phase cost what its shorter circuit saved, c4 trace of round 4)
	const int tier = (!fold && items <= wide_max) ? 2 : items <= hex_max ? 1 : 0;
	const size_t per_wg = tier == 2 ? Grp<64>::kGroups : tier == 1 ? Grp<16>::kGroups : Grp<4>::kGroups;
	size_t grid = (items + per_wg - 1) / per_wg;
	void* args[] = {&A};
	const bool coal = fold && tier == 0 && A.mode == 0 && A.n_pairs % 16 == 0;
	// (lane pairs take 128 items per workgroup, half of sc_fold_coal's grid: below ~1.5 workgroups per
	// CU the quad fold's wider grid wins, c4 rounds 5-6: 28.0 / 24.6 vs 22.6 / 16.3 us)
	bool pair = fold && tier == 0 && A.mode == 0 && A.n_pairs % 32 == 0 && items >= kPairMinItems;
#ifdef BN_DEV
	{
		static const char* ep = getenv("BN_SC_FOLD_PAIR");
		if (ep && atoi(ep) == 0) pair = false;
	}
#endif
	if (pair) {  // lane-pair products with a scalar challenge (sc_fold_pair)
		grid = (items + kPairItemsPerWG - 1) / kPairItemsPerWG;
		BN_HIP(hipLaunchKernel((const void*)sc_fold_pair, dim3((unsigned)grid), dim3(kScThreads), args,
		                       sizeof(uint32_t) * 4 * kPairWaveWords, sc->stream));
		return BN_OK;
	}
	const void* fns[3][2][3] = {
		{{(const void*)sc_messages<0, 4>, (const void*)sc_messages<1, 4>, (const void*)sc_messages<2, 4>},
		 {coal ? (const void*)sc_fold_coal : (const void*)sc_fold<0, 4>, (const void*)sc_fold<1, 4>, (const void*)sc_fold<2, 4>}},
		{{(const void*)sc_messages<0, 16>, (const void*)sc_messages<1, 16>, (const void*)sc_messages<2, 16>},
		 {(const void*)sc_fold<0, 16>, (const void*)sc_fold<1, 16>, (const void*)sc_fold<2, 16>}},
		{{(const void*)sc_messages<0, 64>, (const void*)sc_messages<1, 64>, (const void*)sc_messages<2, 64>},
		 {(const void*)sc_fold<0, 16>, (const void*)sc_fold<1, 16>, (const void*)sc_fold<2, 16>}}};  // (not used)
	A.post = grid <= post_max;
	const size_t lds = tier == 2 ? lds_bytes<64>() : tier == 1 ? lds_bytes<16>() : lds_bytes<4>();
	BN_HIP(hipLaunchKernel(fns[tier][fold ? 1 : 0][A.mode], dim3((unsigned)grid), dim3(kScThreads), args, lds, sc->stream));
	if (!fold && !A.post) BN_HIP(hipLaunchKernel((const void*)sc_post, dim3(1), dim3(64), args, 0, sc->stream));
	return BN_OK;
}

// Round i's fold with r fused into round i + 1's messages (sc_fold_msgs): the big rounds whose
// messages run on quads. Called after move_to_next_round has halved cur and updated the claim state.
// Measured slower than separate fold + messages launches on c4 (d = 3: 3.59-3.67 vs 3.40-3.44 ms,
// DESIGN.md section 10): the batches a work-group folds leave L2 before its messages phase reads
// them, so the product keeps the two launches; -DBN_SC_FUSED builds the fused path (experiments).
#ifdef BN_SC_FUSED
constexpr bool kFusedFold = true;
#else
constexpr bool kFusedFold = false;
#endif
bool fused_eligible(const bn_sumcheck* sc) {
	if (!kFusedFold || !sc->eager || sc->cur < 64 || (sc->world > 1 && sc->cur <= 32)) return false;
	const int npts = sc->d + 1 - ((sc->have_claim || sc->claim_pending) ? 1 : 0);
	return (sc->cur / 64) * (size_t)npts > kHexMaxItems && npts <= Grp<4>::kGroups;
}

int launch_fused(bn_sumcheck* sc, const uint32_t* r) {
#ifndef BN_SC_FUSED
	(void)sc, (void)r;
	BN_FAIL(BN_ERR_UNSUPPORTED, "fused fold + messages: experiment builds only (-DBN_SC_FUSED)");
#else
	ScArgs A{};
	A.cols = sc->cols;
	A.col_stride = sc->col_words;
	A.d = sc->d;
	A.mode = 0;
	A.n_pairs = sc->cur / 64;  // pairs of the folded columns (the fold's pairs are 2 n_pairs apart)
	A.hb = A.n_pairs;
	A.kmax = sc->d;
	A.skip1 = (sc->have_claim || sc->claim_pending) ? 1 : 0;
	A.res = sc->d_res;
	A.sink = sc->sink;
	A.seq = ++sc->seq;
	A.acc = sc->acc + kAccSet * sc->par;
	A.clr = sc->acc + kAccSet * (1 - sc->par);
	memcpy(A.r, r, 16);
#ifdef BN_DEV
	{
		static const int dbg = getenv("BN_SC_DBG") ? atoi(getenv("BN_SC_DBG")) : 0;
		A.dbg = dbg;
	}
#endif
	for (int k = 0; k <= kMaxD; k++)
		for (int a = 0; a < 4; a++) A.kcol[k][a] = (uint32_t)tw_mul((uint64_t)k, 1ull << a, 2);
	const int npts = A.kmax + 1 - A.skip1;
	const size_t P = Grp<4>::kGroups / npts;
	A.fm_p = (int)P;
	A.fm_magic = (uint32_t)(((1ull << 32) + 2 * P - 1) / (2 * P));
	const size_t grid = (A.n_pairs + P - 1) / P;
	A.post = grid <= kPostInKernelMaxWG;
	void* args[] = {&A};
	const size_t lds = std::max(lds_bytes<4>(), sizeof(uint32_t) * 4 * kPairWaveWords);
	BN_HIP(hipLaunchKernel((const void*)sc_fold_msgs, dim3((unsigned)grid), dim3(kScThreads), args, lds, sc->stream));
	if (!A.post) BN_HIP(hipLaunchKernel((const void*)sc_post, dim3(1), dim3(64), args, 0, sc->stream));
	sc->par ^= 1;
	sc->msgs_queued = true;
	return BN_OK;
#endif
}

#ifdef BN_DEV
double host_us() {
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}
#endif

// The round server takes over once at most server_max_cur evaluations per column are left (an
// unsharded, eager prover without a message sink; composition_eval only folds)
// (not for a replica built by import_gathered: the sharded driver runs one per rank in lockstep, and
// several servers waiting in one process would block each other's queues for up to the timeout)
bool server_eligible(const bn_sumcheck* sc) {
	return sc->eager && sc->world == 1 && !sc->sink && !sc->gathered && sc->prepared && sc->cur >= 2 && sc->cur <= sc->server_max_cur;
}

// a server that folds `cur` evaluations per column on `ticket` and posts those messages as `seq`
int server_launch(bn_sumcheck* sc, size_t cur, uint32_t seq, uint32_t ticket) {
	SrvArgs P{};
	P.cols = sc->cols;
	P.col_stride = sc->col_words;
	P.d = sc->d;
	P.cur = cur;
	P.res = sc->d_res;
	uint32_t* d_ctl = nullptr;
	BN_HIP(hipHostGetDevicePointer((void**)&d_ctl, sc->h_ctl, 0));
	P.ctl = d_ctl;
	P.ctl_exit = d_ctl + kCtlExit;
	P.seq = seq;
	P.ticket = ticket;
	P.trace = nullptr;
#ifdef BN_DEV
	if (getenv("BN_SC_TIMING")) {
		if (!sc->h_trace) {
			BN_HIP(hipHostMalloc((void**)&sc->h_trace, 64 * 4 * sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent));
			memset(sc->h_trace, 0, 64 * 4 * sizeof(unsigned long long));
		}
		BN_HIP(hipHostGetDevicePointer((void**)&P.trace, sc->h_trace, 0));
	}
#endif
	((volatile uint32_t*)sc->h_ctl)[kCtlExit] = kSrvRunning;
	for (int k = 0; k <= kMaxD; k++)
		for (int a = 0; a < 4; a++) P.kcol[k][a] = (uint32_t)tw_mul((uint64_t)k, 1ull << a, 2);
	void* args[] = {&P};
	BN_HIP(hipLaunchKernel((const void*)sc_server, dim3(1), dim3(kSrvThreads), args, srv_lds_bytes(), sc->stream));
	sc->server = true;
	return BN_OK;
}

// hand the server its next challenge (the fold of this round, then the next round's messages)
void server_post(bn_sumcheck* sc, const uint32_t* r, bool skip1) {
	volatile uint32_t* c = sc->h_ctl;
	for (int i = 0; i < 4; i++) c[kCtlR + i] = r[i];
	c[kCtlSkip] = skip1 ? 1u : 0u;
	std::atomic_thread_fence(std::memory_order_release);
	c[kCtlTicket] = ++sc->ticket;
	sc->seq++;  // the server posts this round's messages with the next sequence number
#ifdef BN_DEV
	sc->t_post = host_us();
#endif
}

// Wait for the round's posted sequence number (the stream is queried between polls, so a failed
// kernel is reported rather than waited for); relaunches a round server that timed out before
// taking this round's challenge.
int wait_posted(bn_sumcheck* sc) {
	const volatile uint32_t* posted = sc->h_res + kResSeq;
	for (;;) {
		bool seen = false;
		for (int i = 0; i < 4096 && !(seen = *posted == sc->seq); i++) {
		}
		if (seen) {
#ifdef BN_DEV
			if (sc->server && sc->h_trace && sc->ticket > 0) {
				const unsigned long long* t = sc->h_trace + 4 * (size_t)(sc->ticket % 64);
				fprintf(stderr, "server round cur=%zu: post->seen %.1f us | wake->fold %.1f fold->msgs %.1f msgs->post %.1f us\n", sc->cur,
				        host_us() - sc->t_post, (t[1] - t[0]) / 100.0, (t[2] - t[1]) / 100.0, (t[3] - t[2]) / 100.0);
			}
#endif
			return BN_OK;
		}
		if (sc->server && ((volatile uint32_t*)sc->h_ctl)[kCtlExit] == sc->ticket - 1) {
			// the challenge and the ticket are already posted: the new server folds 2 cur down to cur
			std::atomic_thread_fence(std::memory_order_acquire);
			const int lrc = server_launch(sc, sc->cur * 2, sc->seq, sc->ticket);
			if (lrc != BN_OK) return lrc;
			continue;
		}
		const hipError_t e = hipStreamQuery(sc->stream);
		if (e == hipSuccess) {
			if (*posted == sc->seq) return BN_OK;
			// the server may have timed out between the kCtlExit read above and the query (it then
			// records ticket - 1 and ends, so the stream drains without a post): relaunch it
			std::atomic_thread_fence(std::memory_order_acquire);
			if (sc->server && ((volatile uint32_t*)sc->h_ctl)[kCtlExit] == sc->ticket - 1) continue;
			BN_FAIL(BN_ERR_HIP, "round messages were not posted (sequence %u)", sc->seq);
		}
		if (e != hipErrorNotReady) BN_FAIL(BN_ERR_HIP, "round messages kernel: %s", hipGetErrorString(e));
	}
}

int queue_messages(bn_sumcheck* sc) {
	int rc = sc_launch(sc, false, nullptr);
	if (rc != BN_OK) return rc;
	sc->par ^= 1;
	sc->msgs_queued = true;
	return BN_OK;
}

int sc_alloc(bn_sumcheck* sc, size_t col_words) {
	sc->col_words = col_words;
	BN_HIP(hipMalloc(&sc->cols, sizeof(uint32_t) * col_words * (size_t)sc->d));
	return BN_OK;
}

int sc_common_init(bn_sumcheck* sc) {
	BN_HIP(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
	BN_HIP(hipMalloc(&sc->acc, sizeof(uint32_t) * 2 * kAccSet));
	BN_HIP(hipMemsetAsync(sc->acc, 0, sizeof(uint32_t) * 2 * kAccSet, sc->stream));
	BN_HIP(hipHostMalloc((void**)&sc->h_res, sizeof(uint32_t) * (kResSeq + 1), hipHostMallocMapped | hipHostMallocCoherent));
	memset(sc->h_res, 0, sizeof(uint32_t) * (kResSeq + 1));
	BN_HIP(hipHostGetDevicePointer((void**)&sc->d_res, sc->h_res, 0));
	BN_HIP(hipHostMalloc((void**)&sc->h_ctl, sizeof(uint32_t) * kCtlWords, hipHostMallocMapped | hipHostMallocCoherent));
	memset(sc->h_ctl, 0, sizeof(uint32_t) * kCtlWords);
	BN_HIP(hipFuncSetAttribute((const void*)sc_server, hipFuncAttributeMaxDynamicSharedMemorySize, (int)srv_lds_bytes()));
#ifdef BN_DEV
	if (const char* e = getenv("BN_SC_SERVER_MAX_CUR")) sc->server_max_cur = (size_t)atol(e);
#endif
	const void* fns[17] = {(const void*)sc_messages<0, 4>,  (const void*)sc_messages<1, 4>,  (const void*)sc_messages<2, 4>,
						   (const void*)sc_fold<0, 4>,      (const void*)sc_fold<1, 4>,      (const void*)sc_fold<2, 4>,
						   (const void*)sc_messages<0, 16>, (const void*)sc_messages<1, 16>, (const void*)sc_messages<2, 16>,
						   (const void*)sc_fold<0, 16>,     (const void*)sc_fold<1, 16>,     (const void*)sc_fold<2, 16>,
						   (const void*)sc_messages<0, 64>, (const void*)sc_messages<1, 64>, (const void*)sc_messages<2, 64>,
						   (const void*)sc_fold_coal, (const void*)sc_fold_pair};
	const int lds_max = (int)std::max(lds_bytes<4>(), std::max(lds_bytes<16>(), lds_bytes<64>()));
	for (const void* f : fns) BN_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max));
	return BN_OK;
}

void sc_free(bn_sumcheck* sc) {
	if (!sc) return;
	if (sc->server && sc->h_ctl) {  // a server still waiting for a challenge: release it
		std::atomic_thread_fence(std::memory_order_release);
		((volatile uint32_t*)sc->h_ctl)[kCtlTicket] = kSrvStop;
	}
	if (sc->stream) (void)hipStreamSynchronize(sc->stream);
	if (sc->cols) (void)hipFree(sc->cols);
	if (sc->acc) (void)hipFree(sc->acc);
	if (sc->h_res) (void)hipHostFree(sc->h_res);
	if (sc->h_ctl) (void)hipHostFree(sc->h_ctl);
	if (sc->h_trace) (void)hipHostFree(sc->h_trace);
	if (sc->stream) (void)hipStreamDestroy(sc->stream);
	delete sc;
}

int check_shape(int num_vars, int d, int transposed) {
	BN_CHECK_ARG(d >= 1 && d <= kMaxD, "composition_size must be in [1, %d]", kMaxD);
	BN_CHECK_ARG(num_vars >= 1 && num_vars <= 30, "num_vars must be in [1, 30]");
	BN_CHECK_ARG(!transposed || num_vars >= 5, "bitsliced input needs num_vars >= 5 (whole 32-element batches)");
	return BN_OK;
}

// Device bit-transpose of compact input (the reference constructor's transpose_kernel,
// sumcheck.cuh:97-101), then a stream synchronisation: the prover is ready for round 0.
int sc_prepare(bn_sumcheck* sc) {
	if (sc->prepared) return BN_OK;
	if (sc->compact_input) {
		const size_t blocks = sc->col_words / 128 * (size_t)sc->d;
		int rc = bn_bitslice_device(sc->cols, blocks, 0, sc->stream);
		if (rc != BN_OK) return rc;
	}
	BN_HIP(hipStreamSynchronize(sc->stream));
	sc->prepared = true;
	return BN_OK;
}

// Common tail of both constructors: the d columns (4*2^n words each, compact or bitsliced) are in
// the prover's storage; compact ones are converted in place unless `stage_only`.
int sc_finish_create(bn_sumcheck* sc, int transposed, bool stage_only = false) {
	const size_t n = (size_t)1 << sc->num_vars;
	sc->compact_input = !transposed;
	sc->prepared = false;
	sc->cur = n;
	sc->round = 0;
	if (stage_only) {
		BN_HIP(hipStreamSynchronize(sc->stream));
		return BN_OK;
	}
	return sc_prepare(sc);
}

}  // namespace

static int create_from_host(int device, int num_vars, int d, int transposed, const uint32_t* evals, bool stage_only,
                            bn_sumcheck** out) {
	BN_CHECK_ARG(out, "NULL output pointer");
	*out = nullptr;
	BN_CHECK_ARG(evals, "NULL evals");
	int rc = check_shape(num_vars, d, transposed);
	if (rc != BN_OK) return rc;
	DeviceScope ds(device);
	if (!ds.ok) BN_FAIL(BN_ERR_HIP, "hipSetDevice(%d) failed", device);
	bn_sumcheck* sc = new bn_sumcheck;
	sc->device = device;
	sc->num_vars = num_vars;
	sc->d = d;
	const size_t n = (size_t)1 << num_vars;
	const size_t in_words = 4 * n;
	const size_t col_words = in_words < 128 ? 128 : in_words;  // pad to one batch
	if ((rc = sc_common_init(sc)) != BN_OK || (rc = sc_alloc(sc, col_words)) != BN_OK) {
		sc_free(sc);
		return rc;
	}
	hipError_t e = hipSuccess;
	if (col_words != in_words) e = hipMemsetAsync(sc->cols, 0, sizeof(uint32_t) * col_words * (size_t)d, sc->stream);
	for (int j = 0; j < d && e == hipSuccess; j++)
		e = hipMemcpyAsync(sc->cols + (size_t)j * col_words, evals + (size_t)j * in_words, sizeof(uint32_t) * in_words,
						   hipMemcpyHostToDevice, sc->stream);
	if (e != hipSuccess) {
		sc_free(sc);
		BN_FAIL(BN_ERR_HIP, "copying evals to the device: %s", hipGetErrorString(e));
	}
	if ((rc = sc_finish_create(sc, transposed, stage_only)) != BN_OK) {
		sc_free(sc);
		return rc;
	}
	*out = sc;
	return BN_OK;
}

extern "C" int bn_sumcheck_create(int device, int num_vars, int d, int transposed, const uint32_t* evals,
								  bn_sumcheck** out) {
	return create_from_host(device, num_vars, d, transposed, evals, false, out);
}

extern "C" int bn_sumcheck_create_staged(int device, int num_vars, int d, int transposed, const uint32_t* evals,
                                         bn_sumcheck** out) {
	return create_from_host(device, num_vars, d, transposed, evals, true, out);
}

extern "C" int bn_sumcheck_prepare(bn_sumcheck* sc) {
	BN_CHECK_ARG(sc, "NULL prover");
	DeviceScope ds(sc->device);
	return sc_prepare(sc);
}

extern "C" int bn_sumcheck_create_device(int device, int num_vars, int d, int transposed, void* d_evals, int take,
										 bn_sumcheck** out) {
	BN_CHECK_ARG(out, "NULL output pointer");
	*out = nullptr;
	BN_CHECK_ARG(d_evals, "NULL evals");
	int rc = check_shape(num_vars, d, transposed);
	if (rc != BN_OK) return rc;
	DeviceScope ds(device);
	if (!ds.ok) BN_FAIL(BN_ERR_HIP, "hipSetDevice(%d) failed", device);
	bn_sumcheck* sc = new bn_sumcheck;
	sc->device = device;
	sc->num_vars = num_vars;
	sc->d = d;
	const size_t n = (size_t)1 << num_vars;
	const size_t in_words = 4 * n;
	if ((rc = sc_common_init(sc)) != BN_OK) {
		sc_free(sc);
		return rc;
	}
	{
		// order the prover's stream after the work already queued on the legacy default stream
		// (producers on other streams must still complete first: see the header)
		hipEvent_t ready = nullptr;
		hipError_t e = hipEventCreateWithFlags(&ready, hipEventDisableTiming);
		if (e == hipSuccess) e = hipEventRecord(ready, 0);
		if (e == hipSuccess) e = hipStreamWaitEvent(sc->stream, ready, 0);
		if (ready) (void)hipEventDestroy(ready);
		if (e != hipSuccess) {
			sc_free(sc);
			BN_FAIL(BN_ERR_HIP, "ordering after the default stream: %s", hipGetErrorString(e));
		}
	}
	if (take && in_words >= 128) {
		sc->cols = (uint32_t*)d_evals;
		sc->col_words = in_words;
	} else {
		const size_t col_words = in_words < 128 ? 128 : in_words;
		if ((rc = sc_alloc(sc, col_words)) != BN_OK) {
			sc_free(sc);
			return rc;
		}
		hipError_t e = hipSuccess;
		if (!transposed && col_words == in_words) {
			// compact columns of whole blocks: bit-transposed straight from the caller's buffer into the
			// prover's storage (one pass over HBM instead of a copy and an in-place transpose)
			rc = bitslice_launch(d_evals, sc->cols, col_words / 128 * (size_t)d, 0, sc->stream);
			if (rc != BN_OK) {
				sc_free(sc);
				return rc;
			}
			transposed = 1;
		} else {
			if (col_words != in_words) e = hipMemsetAsync(sc->cols, 0, sizeof(uint32_t) * col_words * (size_t)d, sc->stream);
			for (int j = 0; j < d && e == hipSuccess; j++)
				e = hipMemcpyAsync(sc->cols + (size_t)j * col_words, (const uint32_t*)d_evals + (size_t)j * in_words,
								   sizeof(uint32_t) * in_words, hipMemcpyDeviceToDevice, sc->stream);
		}
		if (e == hipSuccess && take) e = hipStreamSynchronize(sc->stream);
		if (e == hipSuccess && take) e = hipFree(d_evals);
		if (e != hipSuccess) {
			sc_free(sc);
			BN_FAIL(BN_ERR_HIP, "copying device evals: %s", hipGetErrorString(e));
		}
	}
	if ((rc = sc_finish_create(sc, transposed)) != BN_OK) {
		sc_free(sc);
		return rc;
	}
	*out = sc;
	return BN_OK;
}

// A shard prover built straight from this rank's share of bitsliced columns (the batches b with
// b mod world == rank, in order: 4 * 2^num_vars / world words per column, columns back to back),
// so no rank ever holds the whole input. The copy is ordered after the work queued on `stream`
// (the caller's producer stream; NULL = the legacy default stream).
extern "C" int bn_sumcheck_create_shard_device(int device, int num_vars, int d, int rank, int world,
                                               const void* d_local, void* stream, bn_sumcheck** out) {
	BN_CHECK_ARG(out, "NULL output pointer");
	*out = nullptr;
	BN_CHECK_ARG(d_local, "NULL evals");
	int rc = check_shape(num_vars, d, 1);
	if (rc != BN_OK) return rc;
	BN_CHECK_ARG(world >= 1 && (world & (world - 1)) == 0, "world must be a power of two");
	BN_CHECK_ARG(rank >= 0 && rank < world, "rank out of range");
	const size_t n = (size_t)1 << num_vars;
	BN_CHECK_ARG(n >= (size_t)32 * world, "need at least one 32-element batch per rank");
	DeviceScope ds(device);
	if (!ds.ok) BN_FAIL(BN_ERR_HIP, "hipSetDevice(%d) failed", device);
	bn_sumcheck* sc = new bn_sumcheck;
	sc->device = device;
	sc->num_vars = num_vars;
	sc->d = d;
	const size_t col_words = 4 * n / (size_t)world;
	if ((rc = sc_common_init(sc)) != BN_OK || (rc = sc_alloc(sc, col_words)) != BN_OK) {
		sc_free(sc);
		return rc;
	}
	hipEvent_t ready = nullptr;
	hipError_t e = hipEventCreateWithFlags(&ready, hipEventDisableTiming);
	if (e == hipSuccess) e = hipEventRecord(ready, (hipStream_t)stream);
	if (e == hipSuccess) e = hipStreamWaitEvent(sc->stream, ready, 0);
	if (e == hipSuccess)
		e = hipMemcpyAsync(sc->cols, d_local, sizeof(uint32_t) * col_words * (size_t)d, hipMemcpyDeviceToDevice, sc->stream);
	if (e == hipSuccess) e = hipStreamSynchronize(sc->stream);
	if (ready) (void)hipEventDestroy(ready);
	if (e != hipSuccess) {
		sc_free(sc);
		BN_FAIL(BN_ERR_HIP, "copying the shard: %s", hipGetErrorString(e));
	}
	sc->cur = n / (size_t)world;
	sc->round = 0;
	sc->rank = rank;
	sc->world = world;
	sc->sharded_used = world > 1;
	*out = sc;
	return BN_OK;
}

extern "C" int bn_sumcheck_set_shard(bn_sumcheck* sc, int rank, int world) {
	BN_CHECK_ARG(sc, "NULL prover");
	BN_CHECK_ARG(sc->round == 0 && !sc->sharded_used, "set_shard must precede the first round");
	BN_CHECK_ARG(world >= 1 && (world & (world - 1)) == 0, "world must be a power of two");
	BN_CHECK_ARG(rank >= 0 && rank < world, "rank out of range");
	const size_t n = (size_t)1 << sc->num_vars;
	BN_CHECK_ARG(n >= (size_t)32 * world, "need at least one 32-element batch per rank");
	if (world == 1) return BN_OK;
	DeviceScope ds(sc->device);
	if (!sc->prepared) {  // a staged prover transposes on first use
		const int prc = sc_prepare(sc);
		if (prc != BN_OK) return prc;
	}
	// keep the batches b with b mod world == rank, in order
	const size_t nb_local = n / 32 / world;
	uint32_t* local = nullptr;
	BN_HIP(hipMalloc(&local, sizeof(uint32_t) * 128 * nb_local * (size_t)sc->d));
	for (int j = 0; j < sc->d; j++)
		BN_HIP(hipMemcpy2DAsync(local + (size_t)j * 128 * nb_local, 128 * sizeof(uint32_t),
								sc->cols + (size_t)j * sc->col_words + 128 * (size_t)rank, 128 * sizeof(uint32_t) * world,
								128 * sizeof(uint32_t), nb_local, hipMemcpyDeviceToDevice, sc->stream));
	BN_HIP(hipStreamSynchronize(sc->stream));
	BN_HIP(hipFree(sc->cols));
	sc->cols = local;
	sc->col_words = 128 * nb_local;
	sc->cur = n / world;
	sc->rank = rank;
	sc->world = world;
	sc->sharded_used = true;
	return BN_OK;
}

extern "C" int bn_sumcheck_needs_gather(const bn_sumcheck* sc, int* flag) {
	BN_CHECK_ARG(sc && flag, "NULL argument");
	*flag = (sc->world > 1 && sc->cur <= 32) ? 1 : 0;
	return BN_OK;
}

extern "C" int bn_sumcheck_export_shard(const bn_sumcheck* sc, uint32_t* out, size_t out_words) {
	BN_CHECK_ARG(sc && out, "NULL argument");
	BN_CHECK_ARG(sc->world > 1 && sc->cur <= 32, "export_shard is only valid once a shard is down to one batch");
	BN_CHECK_ARG(out_words >= (size_t)128 * sc->d, "output needs composition_size * 128 words");
	DeviceScope ds(sc->device);
	for (int j = 0; j < sc->d; j++)
		BN_HIP(hipMemcpyAsync(out + 128 * (size_t)j, sc->cols + (size_t)j * sc->col_words, 128 * sizeof(uint32_t),
							  hipMemcpyDeviceToHost, sc->stream));
	BN_HIP(hipStreamSynchronize(sc->stream));
	return BN_OK;
}

extern "C" int bn_sumcheck_import_gathered(bn_sumcheck* sc, const uint32_t* words, size_t n_words, int world) {
	BN_CHECK_ARG(sc && words, "NULL argument");
	BN_CHECK_ARG(world == sc->world && sc->world > 1 && sc->cur <= 32, "import_gathered needs the exported state of every rank");
	BN_CHECK_ARG(n_words >= (size_t)world * 128 * sc->d, "need world * composition_size * 128 words");
	DeviceScope ds(sc->device);
	// rank r's batch becomes global batch r (r < world, so batch r is owned by rank r)
	const size_t col_words = 128 * (size_t)world;
	std::vector<uint32_t> host((size_t)sc->d * col_words);
	for (int r = 0; r < world; r++)
		for (int j = 0; j < sc->d; j++)
			memcpy(&host[(size_t)j * col_words + 128 * (size_t)r], words + ((size_t)r * sc->d + j) * 128, 128 * sizeof(uint32_t));
	uint32_t* cols = nullptr;
	BN_HIP(hipMalloc(&cols, sizeof(uint32_t) * host.size()));
	hipError_t e = hipMemcpyAsync(cols, host.data(), sizeof(uint32_t) * host.size(), hipMemcpyHostToDevice, sc->stream);
	if (e == hipSuccess) e = hipStreamSynchronize(sc->stream);
	if (e != hipSuccess) {
		(void)hipFree(cols);
		BN_FAIL(BN_ERR_HIP, "uploading gathered state: %s", hipGetErrorString(e));
	}
	BN_HIP(hipFree(sc->cols));
	sc->cols = cols;
	sc->col_words = col_words;
	sc->cur = (size_t)32 * world;
	sc->rank = 0;
	sc->world = 1;
	sc->gathered = true;
	sc->have_pts = sc->have_claim = sc->claim_pending = sc->pts_external = false;  // the shards' claims are partial: recompute point 1
	sc->msgs_queued = false;
	return BN_OK;
}

extern "C" int bn_sumcheck_set_message_sink(bn_sumcheck* sc, void* d_words) {
	BN_CHECK_ARG(sc, "NULL prover");
	// a running round server posts to the host words only: switching the prover to a sink then would
	// hand the caller words no kernel wrote
	BN_CHECK_ARG(!sc->server || d_words == sc->sink, "the round server is running: set the sink before the last rounds");
	sc->sink = (uint32_t*)d_words;
	return BN_OK;
}

extern "C" int bn_sumcheck_stream(const bn_sumcheck* sc, void** stream) {
	BN_CHECK_ARG(sc && stream, "NULL argument");
	*stream = (void*)sc->stream;
	return BN_OK;
}

extern "C" int bn_sumcheck_round_messages(bn_sumcheck* sc, uint32_t* sum, uint32_t* points) {
	BN_CHECK_ARG(sc && sum && points, "NULL argument");
	BN_CHECK_ARG(!(sc->world > 1 && sc->cur <= 32), "shard exhausted: gather (export_shard/import_gathered) first");
	DeviceScope ds(sc->device);
	if (!sc->prepared) {  // a staged prover transposes on first use
		const int prc = sc_prepare(sc);
		if (prc != BN_OK) return prc;
	}
	if (!sc->msgs_queued && sc->server) {
		// this round was read already and the server is waiting for the next challenge (no launch
		// may queue behind it): the same messages again
		if (!sc->read_this_round) BN_FAIL(BN_ERR_INVALID, "round server: no messages for this round");
		memcpy(sum, sc->last_sum, 16);
		memcpy(points, sc->last_points, sizeof(uint32_t) * 4 * (sc->d + 1));
		return BN_OK;
	}
	if (sc->claim_pending && sc->pts_external)  // checked before anything is queued
		BN_FAIL(BN_ERR_INVALID, "the previous round's points went to the message sink: read this round there too");
	if (!sc->msgs_queued) {
		int rc = queue_messages(sc);
		if (rc != BN_OK) return rc;
	}
	sc->msgs_queued = false;
	int rc = BN_OK;
	if (sc->claim_pending) {  // last round's claim, computed while this round's kernel runs
		rc = bn_sumcheck_interpolate(sc->last_pts, sc->d + 1, sc->pending_r, sc->claim);
		if (rc != BN_OK) return rc;
		sc->claim_pending = false;
		sc->have_claim = sc->cur > 1;
	}
	if ((rc = wait_posted(sc)) != BN_OK) return rc;
	std::atomic_thread_fence(std::memory_order_acquire);
	const int npts = sc->d + 1;
	uint32_t acc[4 * (kMaxD + 1)];
	for (int i = 0; i < 4 * npts; i++) acc[i] = ((const volatile uint32_t*)sc->h_res)[i];
	if (sc->cur == 1) {
		memcpy(sum, acc, 16);  // mode 2 computed prod_j f_j(0) as "point 0"
		memset(points, 0, sizeof(uint32_t) * 4 * npts);
		sc->have_pts = false;
	} else {
		memcpy(points, acc, sizeof(uint32_t) * 4 * npts);
		if (sc->have_claim) {
			// point 1 was skipped: p(1) = claim + p(0)
			for (int i = 0; i < 4; i++) points[4 + i] = sc->claim[i] ^ acc[i];
			memcpy(sum, sc->claim, 16);
		} else {
			for (int i = 0; i < 4; i++) sum[i] = acc[i] ^ acc[4 + i];
		}
		memcpy(sc->last_pts, points, sizeof(uint32_t) * 4 * npts);
		sc->have_pts = true;
		sc->pts_external = false;
	}
	sc->have_claim = false;
	sc->sharded_used = true;
	memcpy(sc->last_sum, sum, 16);
	memcpy(sc->last_points, points, sizeof(uint32_t) * 4 * npts);
	sc->read_this_round = true;
	return BN_OK;
}

extern "C" int bn_sumcheck_round_messages_sink(bn_sumcheck* sc) {
	BN_CHECK_ARG(sc, "NULL prover");
	BN_CHECK_ARG(sc->sink, "no message sink set (bn_sumcheck_set_message_sink)");
	BN_CHECK_ARG(!(sc->world > 1 && sc->cur <= 32), "shard exhausted: gather (export_shard/import_gathered) first");
	BN_CHECK_ARG(!sc->server, "the round server is running: read this round with bn_sumcheck_round_messages");
	DeviceScope ds(sc->device);
	if (!sc->prepared) {
		const int prc = sc_prepare(sc);
		if (prc != BN_OK) return prc;
	}
	if (!sc->msgs_queued) {
		const int rc = queue_messages(sc);
		if (rc != BN_OK) return rc;
	}
	// no poll: the words reach the sink on the prover's stream, where the caller orders its reads.
	// The caller holds this round's global points, so the next round may skip p(1) (flag bit 0 of
	// sink word 36 says when it did)
	sc->msgs_queued = false;
	sc->claim_pending = sc->have_claim = false;
	sc->have_pts = sc->cur > 1;
	sc->pts_external = true;
	sc->sharded_used = true;
	return BN_OK;
}

extern "C" int bn_sumcheck_move_to_next_round(bn_sumcheck* sc, const uint32_t* challenge) {
	BN_CHECK_ARG(sc && challenge, "NULL argument");
	BN_CHECK_ARG(sc->cur >= 2, "no variables left to fold");
	BN_CHECK_ARG(!(sc->world > 1 && sc->cur <= 32), "shard exhausted: gather (export_shard/import_gathered) first");
	DeviceScope ds(sc->device);
	if (!sc->prepared) {  // a staged prover transposes on first use
		const int prc = sc_prepare(sc);
		if (prc != BN_OK) return prc;
	}
	const bool to_server = sc->server || server_eligible(sc);
	// no sync: the fold is ordered before the next round's messages on the prover's stream
	sc->have_claim = false;  // a claim not consumed by this round's messages is stale now
	sc->claim_pending = sc->have_pts && sc->derive_p1;
	sc->cur /= 2;
	const bool fused = !to_server && fused_eligible(sc);  // decided on the folded size
	sc->cur *= 2;
	if (!to_server && !fused) {  // (a fold launch does not read the claim state)
		int rc = sc_launch(sc, true, challenge);
		if (rc != BN_OK) return rc;
	}
	if (sc->claim_pending) memcpy(sc->pending_r, challenge, 16);
	sc->have_pts = false;
	sc->read_this_round = false;
	if (fused) {
		sc->cur /= 2;
		sc->round++;
		sc->sharded_used = true;
		sc->msgs_queued = false;  // a queued, unread messages kernel ran before the fold: dropped
		return launch_fused(sc, challenge);
	}
	if (to_server) {
		// the round server folds and computes the next round's messages (p(1) skipped when the
		// claim is derived; never for the final evaluation, which the server decides itself)
		if (sc->server && sc->msgs_queued) {
			// the previous challenge's messages were not read: let them land first (one ticket at a
			// time, so a relaunched server never misses an overwritten challenge)
			const int wrc = wait_posted(sc);
			if (wrc != BN_OK) return wrc;
		}
		if (!sc->server || ((volatile uint32_t*)sc->h_ctl)[kCtlExit] == sc->ticket) {
			const int rc = server_launch(sc, sc->cur, sc->seq + 1, sc->ticket + 1);
			if (rc != BN_OK) return rc;
		}
		server_post(sc, challenge, sc->claim_pending && sc->cur / 2 >= 2);
		sc->cur /= 2;
		sc->round++;
		sc->sharded_used = true;
		sc->msgs_queued = true;
		return BN_OK;
	}
	sc->cur /= 2;
	sc->round++;
	sc->sharded_used = true;
	sc->msgs_queued = false;  // a queued, unread messages kernel ran before the fold: dropped
	if (sc->eager && !(sc->world > 1 && sc->cur <= 32)) return queue_messages(sc);
	return BN_OK;
}

extern "C" int bn_sumcheck_round(const bn_sumcheck* sc, int* round) {
	BN_CHECK_ARG(sc && round, "NULL argument");
	*round = sc->round;
	return BN_OK;
}

extern "C" int bn_sumcheck_destroy(bn_sumcheck* sc) {
	if (!sc) return BN_OK;
	DeviceScope ds(sc->device);
	sc_free(sc);
	return BN_OK;
}

// ---------------------------------------------------------------------------------------
// Verifier side
// ---------------------------------------------------------------------------------------
namespace {

int composition_eval(bn_sumcheck* sc, const uint32_t* challenges, uint32_t* out) {
	// folding every column at r_0, r_1, ... (highest variable first) leaves f_j(r); the last
	// round's "sum" is then prod_j f_j(r)
	sc->eager = false;
	for (int i = 0; i < sc->num_vars; i++) {
		int rc = bn_sumcheck_move_to_next_round(sc, challenges + 4 * (size_t)i);
		if (rc != BN_OK) return rc;
	}
	uint32_t pts[4 * (kMaxD + 1)];
	return bn_sumcheck_round_messages(sc, out, pts);
}

}  // namespace

extern "C" int bn_multilinear_composition_eval(int device, int num_vars, int d, int transposed, const uint32_t* evals,
											   const uint32_t* challenges, uint32_t* out) {
	BN_CHECK_ARG(challenges && out, "NULL argument");
	bn_sumcheck* sc = nullptr;
	int rc = bn_sumcheck_create(device, num_vars, d, transposed, evals, &sc);
	if (rc != BN_OK) return rc;
	rc = composition_eval(sc, challenges, out);
	bn_sumcheck_destroy(sc);
	return rc;
}

extern "C" int bn_multilinear_composition_eval_device(int device, int num_vars, int d, int transposed,
													  const void* d_evals, const uint32_t* challenges, uint32_t* out) {
	BN_CHECK_ARG(challenges && out, "NULL argument");
	bn_sumcheck* sc = nullptr;
	int rc = bn_sumcheck_create_device(device, num_vars, d, transposed, const_cast<void*>(d_evals), 0, &sc);
	if (rc != BN_OK) return rc;
	rc = composition_eval(sc, challenges, out);
	bn_sumcheck_destroy(sc);
	return rc;
}

namespace {

// Interpolation on the nodes 0..n-1 (tower elements of GF(2^4)) by the coefficient form:
// c = V^-1 points with V[i][k] = i^k over GF(2^4), then p(r) = sum_k c_k r^k by Horner. V^-1 has
// GF(2^4) entries, and a GF(2^4) scalar times a GF(2^128) element acts on its 32 GF(2^4) coordinates
// (nibbles) one by one, so this is n^2 table-driven scalar products and n - 1 GF(2^128) products
// instead of the Lagrange form's n^2 GF(2^128) products (5.3 -> ~1 us for n = 4: on the host's
// critical path of every sumcheck round).
struct InterpTables {
	uint8_t vinv[17][16][16];  // [n][k][i]
	uint8_t smul[16][256];     // [c][byte]: the two GF(2^4) coordinates of the byte times c
	InterpTables() {
		for (int c = 0; c < 16; c++)
			for (int x = 0; x < 256; x++)
				smul[c][x] = (uint8_t)(tw_mul((uint64_t)c, (uint64_t)(x & 15), 2) | (tw_mul((uint64_t)c, (uint64_t)(x >> 4), 2) << 4));
		for (int n = 1; n <= 16; n++) {
			// Gauss-Jordan on [V | I] over GF(2^4); V is invertible (distinct nodes)
			uint8_t m[16][32] = {};
			for (int i = 0; i < n; i++) {
				uint64_t p = 1;
				for (int k = 0; k < n; k++) {
					m[i][k] = (uint8_t)p;
					p = tw_mul(p, (uint64_t)i, 2);
				}
				m[i][n + i] = 1;
			}
			for (int col = 0; col < n; col++) {
				int piv = col;
				while (m[piv][col] == 0) piv++;
				for (int k = 0; k < 2 * n; k++) std::swap(m[col][k], m[piv][k]);
				const uint64_t inv = tw_inv(m[col][col], 2);
				for (int k = 0; k < 2 * n; k++) m[col][k] = (uint8_t)tw_mul(m[col][k], inv, 2);
				for (int row = 0; row < n; row++) {
					if (row == col || m[row][col] == 0) continue;
					const uint64_t f = m[row][col];
					for (int k = 0; k < 2 * n; k++) m[row][k] ^= (uint8_t)tw_mul(f, m[col][k], 2);
				}
			}
			// V c = points  =>  c = V^-1 points; vinv[n][k][i] = (V^-1)[k][i]
			for (int k = 0; k < n; k++)
				for (int i = 0; i < n; i++) vinv[n][k][i] = m[k][n + i];
		}
	}
};

const InterpTables& interp_tables() {
	static const InterpTables t;
	return t;
}

}  // namespace

extern "C" int bn_sumcheck_interpolate(const uint32_t* points, int num_points, const uint32_t* challenge, uint32_t* out) {
	BN_CHECK_ARG(points && challenge && out, "NULL argument");
	BN_CHECK_ARG(num_points >= 1 && num_points <= 16, "num_points must be in [1, 16]");
	const InterpTables& T = interp_tables();
	const int n = num_points;
	// coefficients c_k = sum_i vinv[k][i] points_i (byte-wise scalar products)
	uint8_t c[16][16];
	for (int k = 0; k < n; k++) {
		uint8_t acc[16] = {};
		for (int i = 0; i < n; i++) {
			const uint8_t s = T.vinv[n][k][i];
			if (!s) continue;
			const uint8_t* pb = (const uint8_t*)(points + 4 * i);
			const uint8_t* tab = T.smul[s];
			for (int b = 0; b < 16; b++) acc[b] ^= tab[pb[b]];
		}
		memcpy(c[k], acc, 16);
	}
	auto ld = [](const uint8_t* p) {
		uint64_t lo, hi;
		memcpy(&lo, p, 8);
		memcpy(&hi, p + 8, 8);
		return bn::u128p{lo, hi};
	};
	const bn::u128p r{(uint64_t)challenge[0] | ((uint64_t)challenge[1] << 32), (uint64_t)challenge[2] | ((uint64_t)challenge[3] << 32)};
	bn::u128p acc = ld(c[n - 1]);
	for (int k = n - 2; k >= 0; k--) {
		acc = bn::tw_mul128_host(acc, r);
		const bn::u128p ck = ld(c[k]);
		acc.lo ^= ck.lo;
		acc.hi ^= ck.hi;
	}
	out[0] = (uint32_t)acc.lo;
	out[1] = (uint32_t)(acc.lo >> 32);
	out[2] = (uint32_t)acc.hi;
	out[3] = (uint32_t)(acc.hi >> 32);
	return BN_OK;
}
