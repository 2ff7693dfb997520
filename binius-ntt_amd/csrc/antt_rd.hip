// Round-scheduled bitsliced additive NTT for gfx950 (kernel variant 3, the default for log_h >= 12).
//
// What it computes: AdditiveNTT::apply (src/ulvt/ntt/additive_ntt.cuh:201-265), i.e. the butterflies
// u ^= w*v, v ^= u (antt_butterfly, :10-14) for stage = log_h-1 .. 0 with the twiddle of
// calculate_twiddle (:59-77). Every twiddle lies in GF(2^32) (basis 1 << i, :281-283) and multiplies
// each 32-bit limb of a GF(2^128) element on its own, so a GF(2^128) transform is four GF(2^32)
// transforms sharing twiddles; with a GF(2^8) / GF(2^16) twiddle a limb splits further into 4 / 2
// independent sub-field coordinates (bytes / halves of the tower representation).
//
// Layouts
//   * HBM: compact AoS in and out (4 x u32 per element); between passes the output buffer holds
//     bitsliced 32-element blocks in element order: block q = 128 words, limb l at 32 l, word i =
//     bit i of limb l of the 32 elements (BitsliceUtils<128>, src/ulvt/utils/bitslicing.cuh:32-47).
//   * Tile: 128 blocks (2^12 elements) of one pass; tile bit m <-> index bit bb[m], the other index
//     bits are fixed per work-group. LDS holds one 16 KiB plane per limb, unpadded, with 16-byte
//     chunks XOR-swizzled: chunk c of block q sits at byte 256 (q >> 1) + 16 (key(q) ^ c), key a
//     linear 4-bit function of q (kKey*) chosen by search so that every ds_read_b128 / ds_write_b128
//     of every round type, of the tile load / store and of the in-word stages is bank-conflict free
//     (gfx950 b128 lane groups, MI355X_MICROARCH.md section LDS).
//
// Rounds (block stages, index bits >= 5): a round runs K consecutive stages on K tile bits in
// registers, radix 2^K. A lane owns one "slice" of SW = 64 / 2^K words of one limb for the 2^K
// blocks of a group (the other 7 - K tile bits), so every round type holds exactly 64 data VGPRs:
//   K = 3, SW = 8 : all three stages with GF(2^8) twiddles (one byte coordinate per lane)
//   K = 2, SW = 16: GF(2^8)/GF(2^16) twiddles (one half-limb per lane)
//   K = 1, SW = 32: any twiddle (one limb per lane)
// Wave w always owns limb plane w, so rounds never synchronise across waves; LDS traffic per stage
// falls from one read + one write of the plane per stage to one per round. The host (rd_plan) picks
// K greedily from the stages' twiddle fields.
//
// In-word stages (index bits 0..4, bottom pass): lane (x, y) = (block pair, limb): it keeps blocks
// qa, qb = qa + 64 of limb y in registers for all five stages (one packed multiply per stage serves
// both blocks), transposes them back to compact words, and a 4x4 permlane16/32 swap across the limb
// lanes gives each lane whole 16-byte elements, stored straight to HBM. The compact input of the
// first pass takes the same path backwards (16-byte loads, permlane swap, transpose, planes).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "antt_plan.hpp"
#include "bitsliced.hpp"

namespace bn {
namespace rd {

constexpr int kBlkBits = 7;
constexpr int kTileBlocks = 1 << kBlkBits;
constexpr int kPlaneBytes = kTileBlocks * 128;
constexpr int kMinLogH = kBlkBits + 5;
constexpr int kMaxStages = kBlkBits + 5;
constexpr int kMaxOuter = 32 - 5 - kBlkBits;
constexpr int kMaxRateBits = 4;
constexpr int kMaxRounds = kBlkBits;

enum { ROLE_FIRST = 0, ROLE_MID = 1, ROLE_LAST = 2, ROLE_SINGLE = 3 };

// LDS swizzle key: bit b (b < 3) = parity(q & kKey[b]) XORs the chunk index, bit 3 = parity(q & kKey[3])
// picks the half of the 256-byte row shared by blocks q and q ^ 1 (kKey[3] has bit 0, so they differ)
constexpr uint32_t kKey[4] = {0x74, 0x2A, 0x52, 0x2F};
__host__ __device__ constexpr uint32_t par(uint32_t x) { return (uint32_t)__builtin_popcount(x) & 1u; }
__host__ __device__ constexpr uint32_t sw_key(uint32_t q) {
	return par(q & kKey[0]) | (par(q & kKey[1]) << 1) | (par(q & kKey[2]) << 2) | (par(q & kKey[3]) << 3);
}
// byte offset of chunk 0 of block q within a plane; chunk c of q is at blk_byte(q) ^ (16 c). Linear
// over XOR for blocks with disjoint bits, which the rounds use to split lane and register parts.
__host__ __device__ constexpr uint32_t blk_byte(uint32_t q) { return 256u * (q >> 1) | 16u * sw_key(q); }

// Lane -> round task maps (found together with kKey): g-bit b of the group is lane bit kGPos[K][b],
// slice bit b is lane bit kSPos[K][b].
__host__ __device__ constexpr int gpos(int K, int b) {
	return K == 1 ? (b == 0 ? 2 : b == 1 ? 0 : b == 2 ? 3 : b == 3 ? 1 : b == 4 ? 5 : 4)
	     : K == 2 ? (b == 0 ? 2 : b == 1 ? 0 : b == 2 ? 1 : b == 3 ? 5 : 3)
	              : (b == 0 ? 0 : b == 1 ? 5 : b == 2 ? 2 : 3);
}
__host__ __device__ constexpr int spos(int K, int b) { return K == 2 ? 4 : (b == 0 ? 1 : 4); }

struct RdRound {
	int k, j0, fld, pad;
	uint32_t V[6];        // byte-offset contribution of group bit b (its tile bit's blk_byte)
	uint32_t U[8];        // byte-offset contribution of register block r
	uint32_t tau[3][6];   // twiddle contribution of group bit b to stage j0 + i
	uint32_t rho[3][8];   // twiddle contribution of register block r to stage j0 + i
};

// One pass = stages lo .. lo + k - 1 over every tile (device-resident, read with scalar loads).
struct RdPass {
	int lo, k, role, n_outer, n_rounds, pad;
	int bb[kBlkBits];                        // index bit of tile bit m
	int ob[kMaxOuter];                       // fixed (outer) index bits, ascending
	int field[kMaxStages];                   // 8/16/32: sub-field holding every twiddle of stage lo + j
	uint32_t twt[kMaxStages][kBlkBits];      // twiddle contribution of tile bit m
	uint32_t two[kMaxStages][kMaxOuter];     // ... of outer bit m
	uint32_t twc[kMaxStages][kMaxRateBits];  // ... of coset bit c
	uint32_t pat[5][32];                     // in-word stages: bit-lane part of the twiddle words
	RdRound rounds[kMaxRounds];
};

struct RdParams {
	const uint32_t* src;
	uint32_t* dst;
	int log_h, log_rate;
	int outmode;  // EXPERIMENT
	int dbg;      // EXPERIMENT: 1 skip in-word stages, 2 skip rounds, 4 skip K=1 rounds
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_stream(const uint32_t* p) {
	const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
	return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_stream(uint32_t* p, uint4 g) {
	u32x4 v;
	v.x = g.x;
	v.y = g.y;
	v.z = g.z;
	v.w = g.w;
	__builtin_nontemporal_store(v, (u32x4*)p);
}
__device__ __forceinline__ void lds_rd4(const char* lds, uint32_t off, uint32_t* r) {
	const uint4 v = *(const uint4*)(lds + off);
	r[0] = v.x, r[1] = v.y, r[2] = v.z, r[3] = v.w;
}
__device__ __forceinline__ void lds_wr4(char* lds, uint32_t off, const uint32_t* r) {
	*(uint4*)(lds + off) = make_uint4(r[0], r[1], r[2], r[3]);
}
// compiler ordering for a wave's own LDS traffic (the hardware executes it in order)
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

__host__ __device__ constexpr uint32_t lane_mask(int j) {
	return j == 0 ? 0xAAAAAAAAu : j == 1 ? 0xCCCCCCCCu : j == 2 ? 0xF0F0F0F0u : j == 3 ? 0xFF00FF00u : 0xFFFF0000u;
}

// P = t*v on SW-word slices (SW = 8: one byte coordinate, 16: a half, 32: a limb); `field`
// (uniform) is the smallest sub-field holding the twiddle, FMAX the largest of the kernel's pass.
template <int SW, int FMAX>
__device__ __forceinline__ void mul_slice(int field, uint32_t t, const uint32_t* v, uint32_t* P) {  // P may be v
	uint32_t W[32];
#ifdef RD_EXP_K1ONLY
	if (FMAX <= 8) {
#else
	if (SW == 8 || FMAX <= 8 || field <= 8) {
#endif
#pragma unroll
		for (int b = 0; b < 8; b++) W[b] = (uint32_t)__builtin_amdgcn_sbfe(t, b, 1);
#pragma unroll
		for (int g = 0; g < SW / 8; g++) bsm3_mul(v + 8 * g, W, P + 8 * g);
	} else if (SW == 16 || FMAX <= 16
#ifndef RD_EXP_K1ONLY
	           || field <= 16
#endif
	           ) {
#pragma unroll
		for (int b = 0; b < 16; b++) W[b] = (uint32_t)__builtin_amdgcn_sbfe(t, b, 1);
#pragma unroll
		for (int g = 0; g < SW / 16; g++) bsm4_mul(v + 16 * g, W, P + 16 * g);
	} else {
		// operands complete before the circuit: with a load still in flight the scheduler hoists the
		// w-side Karatsuba sums (up to 243 live leaves) to cover its latency, and spills
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int b = 0; b < 32; b++) W[b] = (uint32_t)__builtin_amdgcn_sbfe(t, b, 1);
		bsm5_mul(v, W, P);
		__builtin_amdgcn_sched_barrier(0);
	}
}
template <int SW, int FMAX>
__device__ __forceinline__ void bfly(int field, uint32_t t, uint32_t* u, uint32_t* v) {
	uint32_t P[SW];
	mul_slice<SW, FMAX>(field, t, v, P);
#pragma unroll
	for (int i = 0; i < SW; i++) {
		u[i] ^= P[i];
		v[i] ^= u[i];
	}
}

// One round: K stages (R.j0 + K - 1 down to R.j0) on this wave's plane, radix 2^K in registers.
template <int K, int FMAX>
__device__ __forceinline__ void rd_round(const RdRound& R, char* pl, int lane, uint32_t cuv) {
	constexpr int SW = 64 >> K, NCH = SW / 4, NB = 1 << K, GB = kBlkBits - K;
	uint32_t gm[GB];
	uint32_t A = 0;
#pragma unroll
	for (int b = 0; b < GB; b++) {
		gm[b] = 0u - (uint32_t)((lane >> gpos(K, b)) & 1);
		A ^= R.V[b] & gm[b];
	}
	uint32_t s = 0;
#pragma unroll
	for (int b = 0; b < K - 1; b++) s |= (uint32_t)((lane >> spos(K, b)) & 1) << b;
	A ^= 16u * NCH * s;
	uint32_t X[NB][SW];
	if (K == 1) {
		// one limb per lane, for register pressure at two waves per SIMD: only v and the twiddle are
		// live during the (GF(2^32)) multiply, which overwrites v with w*v; u and the old v are then
		// streamed through the butterfly chunk by chunk from the plane
		uint32_t tg = (uint32_t)__builtin_amdgcn_readlane((int)cuv, R.j0);
#pragma unroll
		for (int b = 0; b < GB; b++) tg ^= R.tau[0][b] & gm[b];
		uint32_t* Pr = X[1];
#pragma unroll
		for (int c = 0; c < NCH; c++) lds_rd4(pl, A ^ (R.U[1] ^ (16u * c)), Pr + 4 * c);
		mul_slice<SW, FMAX>(R.fld, tg, Pr, Pr);
		// all u and old-v reads in flight together (one LDS latency), then the butterfly
		uint32_t Uo[SW], Vo[SW];
#pragma unroll
		for (int c = 0; c < NCH; c++) {
			lds_rd4(pl, A ^ (R.U[0] ^ (16u * c)), Uo + 4 * c);
			lds_rd4(pl, A ^ (R.U[1] ^ (16u * c)), Vo + 4 * c);
		}
#pragma unroll
		for (int i = 0; i < SW; i++) {
			Uo[i] ^= Pr[i];
			Vo[i] ^= Uo[i];
		}
#pragma unroll
		for (int c = 0; c < NCH; c++) {
			lds_wr4(pl, A ^ (R.U[0] ^ (16u * c)), Uo + 4 * c);
			lds_wr4(pl, A ^ (R.U[1] ^ (16u * c)), Vo + 4 * c);
		}
		lds_order();
		return;
	} else {
#pragma unroll
	for (int r = 0; r < NB; r++)
#pragma unroll
		for (int c = 0; c < NCH; c++) lds_rd4(pl, A ^ (R.U[r] ^ (16u * c)), &X[r][4 * c]);
#pragma unroll
	for (int jj = K - 1; jj >= 0; jj--) {
		uint32_t tg = (uint32_t)__builtin_amdgcn_readlane((int)cuv, R.j0 + jj);
#pragma unroll
		for (int b = 0; b < GB; b++) tg ^= R.tau[jj][b] & gm[b];
#pragma unroll
		for (int r = 0; r < NB; r++) {
			if ((r >> jj) & 1) continue;
			// GF(2^16) butterflies one at a time (register pressure); the small GF(2^8) ones interleave
			if (SW == 16) __builtin_amdgcn_sched_barrier(0);
			bfly<SW, FMAX>(R.fld, tg ^ R.rho[jj][r], X[r], X[r | (1 << jj)]);
		}
	}
	}
#pragma unroll
	for (int r = 0; r < NB; r++)
#pragma unroll
		for (int c = 0; c < NCH; c++) lds_wr4(pl, A ^ (R.U[r] ^ (16u * c)), &X[r][4 * c]);
	lds_order();
}

// 4x4 transpose of (limb register j) x (lane bits 4, 5): lane with lane bits (5,4) = y, register j
// <-> lane j, register y. Involution; used both ways for the compact <-> limb-plane I/O.
__device__ __forceinline__ void limb_swap(uint32_t* g) {
	auto a = __builtin_amdgcn_permlane32_swap(g[0], g[2], false, false);
	auto b = __builtin_amdgcn_permlane32_swap(g[1], g[3], false, false);
	auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
	auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
	g[0] = c[0], g[1] = c[1], g[2] = d[0], g[3] = d[1];
}

template <int L, int ROLE, int FMAX>
__global__ __launch_bounds__(64 * L, 2) void antt_rd_pass(RdParams P, const RdPass* __restrict__ tab) {
	extern __shared__ __attribute__((aligned(16))) uint32_t lds_words[];
	char* lds = (char*)lds_words;
	constexpr bool IN_COMPACT = ROLE == ROLE_FIRST || ROLE == ROLE_SINGLE;
	constexpr bool LAST = ROLE == ROLE_LAST || ROLE == ROLE_SINGLE;
	const RdPass& ps = *tab;
	const int tid = threadIdx.x;
	const int w = tid >> 6, lane = tid & 63;
	char* pl = lds + w * kPlaneBytes;  // wave w owns limb plane w in the rounds
	const size_t n = (size_t)1 << P.log_h;

	// tile -> (outer bits, coset, batch)
	const size_t t = blockIdx.x;
	const size_t outer = t & (((size_t)1 << ps.n_outer) - 1);
	const size_t rest = t >> ps.n_outer;
	const int coset = (int)(rest & ((1u << P.log_rate) - 1));
	const size_t batch = rest >> P.log_rate;
	size_t ooff = 0;
	for (int m = 0; m < ps.n_outer; m++) ooff |= ((outer >> m) & 1) << ps.ob[m];
	uint32_t* dst = P.dst + (((batch << P.log_rate) + (size_t)coset) * n) * L;
	const uint32_t* src = IN_COMPACT ? (P.src + batch * n * L) : dst;
	auto tile_off = [&](uint32_t q) -> size_t {  // element offset of block q
		size_t off = 0;
#pragma unroll
		for (int m = 0; m < kBlkBits; m++) off |= (size_t)((q >> m) & 1) << ps.bb[m];
		return off;
	};

	// workgroup-uniform twiddle part (outer and coset bits) of stage j, held by lane j
	uint32_t cuv = 0;
	if (lane < ps.k) {
		for (int m = 0; m < ps.n_outer; m++)
			if ((outer >> m) & 1) cuv ^= ps.two[lane][m];
		for (int b = 0; b < P.log_rate; b++)
			if ((coset >> b) & 1) cuv ^= ps.twc[lane][b];
	}

	// ---- tile in
	if (IN_COMPACT) {
		// blocks of this lane in the compact I/O and in-word phases: qa and qb = qa + 64 of limb y
		const int x = L == 4 ? (lane & 15) : lane;
		const int y = L == 4 ? (lane >> 4) : 0;
		const uint32_t qa = L == 4 ? (uint32_t)(16 * w + x) : (uint32_t)x;
#pragma unroll
		for (int h = 0; h < 2; h++) {
			const uint32_t q = qa + 64u * h;
			const uint32_t* sp = src + (ooff | tile_off(q)) * L;
			uint32_t a[32];
			if (L == 4) {
				// load r: lane (x, k) takes element 4 r + k of block q; the limb swap leaves limb y of
				// elements 4 r .. 4 r + 3 in registers 4 r .. 4 r + 3
				uint4 g[8];
#pragma unroll
				for (int r = 0; r < 8; r++) g[r] = *(const uint4*)(sp + 4 * (4 * r + y));  // 64-byte half lines: plain loads
#pragma unroll
				for (int r = 0; r < 8; r++) {
					uint32_t v[4] = {g[r].x, g[r].y, g[r].z, g[r].w};
					limb_swap(v);
#pragma unroll
					for (int j = 0; j < 4; j++) a[4 * r + j] = v[j];
				}
			} else {
#pragma unroll
				for (int r = 0; r < 8; r++) {
					const uint4 v = ld_stream(sp + 4 * r);
					a[4 * r] = v.x, a[4 * r + 1] = v.y, a[4 * r + 2] = v.z, a[4 * r + 3] = v.w;
				}
			}
			transpose32(a);
			char* yp = lds + y * kPlaneBytes;
			const uint32_t bq = blk_byte(q);
#pragma unroll
			for (int c = 0; c < 8; c++) lds_wr4(yp, bq ^ (16u * c), a + 4 * c);
		}
		__syncthreads();
	} else {
		// bitsliced: limb w of block q is 128 contiguous bytes; wave w loads its own plane
		uint4 g[16];
#pragma unroll
		for (int r = 0; r < 16; r++) {
			const int u = lane + 64 * r;
			const uint32_t q = (uint32_t)(u >> 3), c = (uint32_t)(u & 7);
			g[r] = ld_stream(src + (ooff | tile_off(q)) * L + 32 * w + 4 * c);
		}
#pragma unroll
		for (int r = 0; r < 16; r++) {
			const int u = lane + 64 * r;
			const uint32_t q = (uint32_t)(u >> 3), c = (uint32_t)(u & 7);
			*(uint4*)(pl + (blk_byte(q) ^ (16u * c))) = g[r];
		}
		lds_order();
	}

	// ---- block stages, in rounds (each wave on its own plane)
	for (int i = 0; i < ps.n_rounds; i++) {
		if (P.dbg & 2) break;
		const RdRound& R = ps.rounds[i];
		if ((P.dbg & 4) && R.k == 1) continue;
#ifdef RD_EXP_K1ONLY
		rd_round<1, FMAX>(R, pl, lane, cuv);
#else
		if (R.k == 3)
			rd_round<3, 8>(R, pl, lane, cuv);
		else if (R.k == 2)
			rd_round<2, (FMAX < 16 ? FMAX : 16)>(R, pl, lane, cuv);
		else
			rd_round<1, FMAX>(R, pl, lane, cuv);
#endif
	}

	if (LAST) {
		// ---- stages 4..0 inside the words: lane (x, y) keeps blocks qa, qb of limb y in registers.
		// Per stage both blocks share one multiply: qa's v-lanes move down onto the u positions,
		// qb's stay on the v positions (a pair's twiddle depends only on index bits above s).
		__syncthreads();  // the rounds of every wave have written their planes
		// lane-derived values of this phase are recomputed here from an opaque copy of the lane id,
		// so the compiler cannot keep them live (in VGPRs) across the rounds' circuits
		int tid2;
		asm volatile("v_mov_b32 %0, %1" : "=v"(tid2) : "v"(tid));
		const int x = L == 4 ? (tid2 & 15) : (tid2 & 63);
		const int y = L == 4 ? ((tid2 >> 4) & 3) : 0;
		const uint32_t qa = L == 4 ? (uint32_t)(16 * w + x) : (uint32_t)x;
		const uint32_t qb = qa + 64u;
		const char* yp = lds + y * kPlaneBytes;
		uint32_t A[32], B[32];
		{
			const uint32_t ba = blk_byte(qa), bb = blk_byte(qb);
#pragma unroll
			for (int c = 0; c < 8; c++) {
				lds_rd4(yp, ba ^ (16u * c), A + 4 * c);
				lds_rd4(yp, bb ^ (16u * c), B + 4 * c);
			}
		}
		for (int s = 4; s >= ((P.dbg & 1) ? 5 : 0); s--) {
			const int d = 1 << s;
			const uint32_t um = ~lane_mask(s);  // u-lanes (bit s clear)
			uint32_t cb = (uint32_t)__builtin_amdgcn_readlane((int)cuv, s);  // bottom pass: lo = 0, j = s
#pragma unroll
			for (int m = 0; m < kBlkBits; m++) cb ^= ps.twt[s][m] & (0u - ((qb >> m) & 1u));
			uint32_t W[32], T[32];
#pragma unroll
			for (int i = 0; i < 32; i++) {
				T[i] = __builtin_amdgcn_bitop3_b32(A[i] >> d, B[i], um, 0xe4);  // (A>>d & um) | (B & ~um)
				// twiddle word i: bit-lane pattern (bits s+1..4, qa/qb difference on A's lanes) ^ qb's part
				W[i] = ps.pat[s][i] ^ (uint32_t)__builtin_amdgcn_sbfe(cb, i, 1);
			}
			const int f = ps.field[s];
#ifdef RD_EXP_K1ONLY
			if (FMAX <= 8) {
#else
			if (FMAX <= 8 || f <= 8) {
#endif
#pragma unroll
				for (int g = 0; g < 4; g++) bsm3_mul(T + 8 * g, W, T + 8 * g);
			} else if (FMAX <= 16
#ifndef RD_EXP_K1ONLY
			           || f <= 16
#endif
			           ) {
#pragma unroll
				for (int g = 0; g < 2; g++) bsm4_mul(T + 16 * g, W, T + 16 * g);
			} else {
				__builtin_amdgcn_sched_barrier(0);
				bsm5_mul(T, W, T);
				__builtin_amdgcn_sched_barrier(0);
			}
#pragma unroll
			for (int i = 0; i < 32; i++) {
				// u ^= w*v on the u-lanes, then v ^= u: (x & um) << d == (x << d) & ~um and
				// (x & ~um) >> d == (x >> d) & um for these lane masks
				const uint32_t a = __builtin_amdgcn_bitop3_b32(T[i], um, A[i], 0x6a);       // A ^ (T & um)
				const uint32_t b = __builtin_amdgcn_bitop3_b32(T[i] >> d, um, B[i], 0x6a);  // B ^ ((T >> d) & um)
				A[i] = __builtin_amdgcn_bitop3_b32(a << d, um, a, 0x9a);                    // a ^ ((a << d) & ~um)
				B[i] = __builtin_amdgcn_bitop3_b32(b << d, um, b, 0x9a);
			}
		}
		// ---- back to compact words, then whole elements straight to HBM
		transpose32(A);
		transpose32(B);
		if (P.outmode == 1) {
			// EXPERIMENT: stage through the planes, gather 16-byte elements, coalesced stores
			{
				char* ypw = lds + y * kPlaneBytes;
				const uint32_t ba = blk_byte(qa), bb = blk_byte(qb);
#pragma unroll
				for (int c = 0; c < 8; c++) {
					lds_wr4(ypw, ba ^ (16u * c), A + 4 * c);
					lds_wr4(ypw, bb ^ (16u * c), B + 4 * c);
				}
			}
			__syncthreads();
#pragma unroll 4
			for (int r = 0; r < kTileBlocks * 32 / (64 * L); r++) {
				const int u = tid + 64 * L * r;  // element of the tile
				const uint32_t q = (uint32_t)(u >> 5), e = (uint32_t)(u & 31);
				const uint32_t o = (blk_byte(q) ^ (16u * (e >> 2))) + 4u * (e & 3);
				uint32_t v[4];
#pragma unroll
				for (int l = 0; l < L; l++) v[l] = *(const uint32_t*)(lds + l * kPlaneBytes + o);
				uint32_t* dp = dst + (ooff | tile_off(q)) * L + (size_t)e * L;
				if (L == 4)
					st_stream(dp, make_uint4(v[0], v[1], v[2], v[3]));
				else
					*dp = v[0];
			}
			return;
		}
#pragma unroll
		for (int h = 0; h < 2; h++) {
			const uint32_t* Z = h ? B : A;
			uint32_t* dp = dst + (ooff | tile_off(h ? qb : qa)) * L;
			if (L == 4) {
#pragma unroll
				for (int r = 0; r < 8; r++) {
					uint32_t v[4] = {Z[4 * r], Z[4 * r + 1], Z[4 * r + 2], Z[4 * r + 3]};
					limb_swap(v);  // lane (x, k): limbs 0..3 of element 4 r + k
					// plain (temporal) stores: an instruction writes 64-byte halves of lines, the next
					// one the other halves, which meet in L2
					*(uint4*)(dp + 4 * (4 * r + y)) = make_uint4(v[0], v[1], v[2], v[3]);
				}
			} else {
#pragma unroll
				for (int r = 0; r < 8; r++) st_stream(dp + 4 * r, make_uint4(Z[4 * r], Z[4 * r + 1], Z[4 * r + 2], Z[4 * r + 3]));
			}
		}
	} else {
		// ---- bitsliced tile out: wave w stores its own plane
#pragma unroll
		for (int r = 0; r < 16; r++) {
			const int u = lane + 64 * r;
			const uint32_t q = (uint32_t)(u >> 3), c = (uint32_t)(u & 7);
			const uint4 g = *(const uint4*)(pl + (blk_byte(q) ^ (16u * c)));
			st_stream(dst + (ooff | tile_off(q)) * L + 32 * w + 4 * c, g);
		}
	}
}

// ------------------------------------------------------------------------------------
// host: pass and round planning
// ------------------------------------------------------------------------------------
static std::vector<RdPass> rd_plan(const bn_antt_plan* plan) {
	const int log_h = plan->log_h;
	const int width = plan->width;
	auto S = [&](int s, int kk) -> uint32_t {  // s[s][kk], 0 outside the table
		if (kk < 0 || kk >= width - s) return 0u;
		return plan->s_host[(size_t)s * width + kk];
	};
	std::vector<RdPass> passes;
	auto make = [&](int lo, int k, bool bottom) {
		RdPass p;
		memset(&p, 0, sizeof(p));
		p.lo = lo;
		p.k = k;
		std::vector<int> bits;
		if (bottom) {
			for (int b = 5; b < 5 + kBlkBits; b++) bits.push_back(b);
		} else {
			// the lowest non-word index bits (adjacent blocks in memory), then the stage bits
			for (int b = 5; (int)bits.size() < kBlkBits - k; b++) bits.push_back(b);
			for (int b = lo; b < lo + k; b++) bits.push_back(b);
		}
		for (int m = 0; m < kBlkBits; m++) p.bb[m] = bits[m];
		p.n_outer = 0;
		for (int b = 5; b < log_h; b++)
			if (std::find(bits.begin(), bits.end(), b) == bits.end()) p.ob[p.n_outer++] = b;
		int tile_bit[kMaxStages];  // tile bit of stage lo + j (>= 5), -1 for the in-word stages
		for (int j = 0; j < k; j++) {
			const int s = lo + j;
			// twiddle of a butterfly block = XOR of s[s][kk] over the set bits kk of
			// (coset << (log_h-1-s)) | (index >> (s+1)); index bit b contributes s[s][b-s-1]
			uint32_t acc = 0;
			for (int kk = 0; kk < width - s; kk++) acc |= S(s, kk);
			p.field[j] = acc < 256u ? 8 : acc < 65536u ? 16 : 32;
			tile_bit[j] = -1;
			for (int m = 0; m < kBlkBits; m++) {
				if (p.bb[m] == s) tile_bit[j] = m;
				p.twt[j][m] = S(s, p.bb[m] - s - 1);
			}
			for (int m = 0; m < p.n_outer; m++) p.two[j][m] = S(s, p.ob[m] - s - 1);
			for (int c = 0; c < plan->log_rate; c++) p.twc[j][c] = S(s, log_h - 1 - s + c);
			if (s < 5) {
				// bit-lane e of a word has index bits 0..4 = e: bits s+1..4 contribute per bit-lane
				for (int i = 0; i < 32; i++) {
					uint32_t wv = 0;
					for (int b = s + 1; b < 5; b++)
						if ((S(s, b - s - 1) >> i) & 1) wv ^= lane_mask(b);
					// qa's v-lanes sit on the u positions with twiddle cb ^ twt[s][6] (qa and qb
					// differ in tile bit 6 only): fold that uniform difference in
					if ((p.twt[j][kBlkBits - 1] >> i) & 1) wv ^= ~lane_mask(s);
					p.pat[s][i] = wv;
				}
			}
		}
		// rounds over the block stages, highest first: K = 3 when three consecutive stages have
		// GF(2^8) twiddles, K = 2 for two with GF(2^16) ones, else K = 1
		const int jlo = bottom ? 5 : 0;
		int j = k - 1;
		p.n_rounds = 0;
		while (j >= jlo) {
			auto fits = [&](int kk, int f) {
				if (j - kk + 1 < jlo) return false;
				for (int i = 0; i < kk; i++)
					if (p.field[j - i] > f) return false;
				return true;
			};
			static const int kmax = getenv("BN_RD_KMAX") ? atoi(getenv("BN_RD_KMAX")) : 3;  // EXPERIMENT
			const int K = (kmax >= 3 && fits(3, 8)) ? 3 : (kmax >= 2 && fits(2, 16)) ? 2 : 1;
			RdRound& R = p.rounds[p.n_rounds++];
			R.k = K;
			R.j0 = j - K + 1;
			R.fld = 8;
			int M[3];
			for (int i = 0; i < K; i++) {
				R.fld = std::max(R.fld, p.field[R.j0 + i]);
				M[i] = tile_bit[R.j0 + i];
			}
			std::vector<int> fr;
			for (int m = 0; m < kBlkBits; m++)
				if (std::find(M, M + K, m) == M + K) fr.push_back(m);
			for (int b = 0; b < kBlkBits - K; b++) {
				R.V[b] = blk_byte(1u << fr[b]);
				for (int i = 0; i < K; i++) R.tau[i][b] = p.twt[R.j0 + i][fr[b]];
			}
			for (int r = 0; r < (1 << K); r++) {
				uint32_t rb = 0;
				for (int i = 0; i < K; i++)
					if ((r >> i) & 1) rb |= 1u << M[i];
				R.U[r] = blk_byte(rb);
				for (int i = 0; i < K; i++) {
					uint32_t rho = 0;
					for (int i2 = i + 1; i2 < K; i2++)
						if ((r >> i2) & 1) rho ^= p.twt[R.j0 + i][M[i2]];
					R.rho[i][r] = rho;
				}
			}
			j -= K;
		}
		return p;
	};
	const int rest = log_h - kMinLogH;
	const int n_up = (rest + kBlkBits - 1) / kBlkBits;
	int hi = log_h;
	for (int i = 0; i < n_up; i++) {
		const int remaining_up = n_up - i;
		const int k = (hi - kMinLogH + remaining_up - 1) / remaining_up;
		passes.push_back(make(hi - k, k, false));
		hi -= k;
	}
	passes.push_back(make(0, kMinLogH, true));
	for (size_t i = 0; i < passes.size(); i++) {
		const bool first = i == 0, last = i + 1 == passes.size();
		passes[i].role = first && last ? ROLE_SINGLE : first ? ROLE_FIRST : last ? ROLE_LAST : ROLE_MID;
	}
	return passes;
}

template <int L, int FMAX>
static const void* kernel_for_f(int role) {
	switch (role) {
		case ROLE_FIRST: return (const void*)antt_rd_pass<L, ROLE_FIRST, FMAX>;
		case ROLE_MID: return (const void*)antt_rd_pass<L, ROLE_MID, FMAX>;
		case ROLE_LAST: return (const void*)antt_rd_pass<L, ROLE_LAST, FMAX>;
		default: return (const void*)antt_rd_pass<L, ROLE_SINGLE, FMAX>;
	}
}
static const void* kernel_for(int L, int role, int fmax) {
	if (L == 4) return fmax <= 8 ? kernel_for_f<4, 8>(role) : kernel_for_f<4, 32>(role);
	return fmax <= 8 ? kernel_for_f<1, 8>(role) : kernel_for_f<1, 32>(role);
}
static int pass_fmax(const RdPass& p) {
	int f = 8;
	for (int j = 0; j < p.k; j++) f = std::max(f, p.field[j]);
	return f;
}
static size_t lds_bytes(int L) { return (size_t)L * kPlaneBytes; }

}  // namespace rd

bool rd_supports(const bn_antt_plan* plan) {
	return plan->log_h >= rd::kMinLogH && plan->log_h - 5 - rd::kBlkBits <= rd::kMaxOuter &&
	       plan->log_rate <= rd::kMaxRateBits;
}

int rd_prepare(bn_antt_plan* plan) {
	for (int L : {1, 4})
		for (int role = 0; role < 4; role++)
			for (int f : {8, 32})
				BN_HIP(hipFuncSetAttribute(rd::kernel_for(L, role, f), hipFuncAttributeMaxDynamicSharedMemorySize,
				                           (int)rd::lds_bytes(L)));
	if (plan->rd_tables == nullptr) {
		const auto ps = rd::rd_plan(plan);
		plan->rd_n_passes = (int)ps.size();
		plan->rd_host.resize(ps.size() * sizeof(rd::RdPass));
		memcpy(plan->rd_host.data(), ps.data(), plan->rd_host.size());
		BN_HIP(hipMalloc(&plan->rd_tables, plan->rd_host.size()));
		BN_HIP(hipMemcpy(plan->rd_tables, plan->rd_host.data(), plan->rd_host.size(), hipMemcpyHostToDevice));
	}
	return BN_OK;
}

int bs_launch_pass(bn_antt_plan* plan, int i, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st);

// one launch of pass i
static int rd_launch_one(bn_antt_plan* plan, int i, const uint32_t* d_in, uint32_t* d_out, size_t batch,
                         hipStream_t st) {
	const rd::RdPass& pass = ((const rd::RdPass*)plan->rd_host.data())[i];
	static const int hyb = getenv("BN_RD_HYB") ? atoi(getenv("BN_RD_HYB")) : 1;  // EXPERIMENT
	if (hyb && pass.role == rd::ROLE_LAST) return bs_launch_pass(plan, i, d_in, d_out, batch, st);
	const rd::RdPass* tab = (const rd::RdPass*)plan->rd_tables + i;
	static const int outmode = getenv("BN_RD_OUT") ? atoi(getenv("BN_RD_OUT")) : 0;  // EXPERIMENT
	static const int dbg = getenv("BN_RD_DBG") ? atoi(getenv("BN_RD_DBG")) : 0;  // EXPERIMENT
	rd::RdParams prm{d_in, d_out, plan->log_h, plan->log_rate, outmode, dbg};
	const int L = plan->limbs;
	const size_t ntiles = (batch << plan->log_rate) << pass.n_outer;
	int rc = timing_begin(plan, i, st);
	if (rc != BN_OK) return rc;
	void* args[] = {&prm, &tab};
	BN_HIP(hipLaunchKernel(rd::kernel_for(L, pass.role, rd::pass_fmax(pass)), dim3((unsigned)ntiles), dim3(64 * L),
	                       args, rd::lds_bytes(L), st));
	return timing_end(plan, i, st);
}

int launch_rd(bn_antt_plan* plan, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st) {
	for (int i = 0; i < plan->rd_n_passes; i++) {
		int rc = rd_launch_one(plan, i, d_in, d_out, batch, st);
		if (rc != BN_OK) return rc;
	}
	return BN_OK;
}

// Profiling: each pass launched `reps` times back to back between two hipEvents on `st` (steady-
// state duration per launch). The output buffer holds no meaningful values afterwards; the cost of
// a pass does not depend on the values (bitwise arithmetic, no data-dependent control flow).
int rd_time_passes(bn_antt_plan* plan, const uint32_t* d_in, uint32_t* d_out, size_t batch, int reps, hipStream_t st,
                   float* ms, int max_passes, int* n_out) {
	const int saved = plan->timing;
	plan->timing = 0;
	hipEvent_t e0 = nullptr, e1 = nullptr;
	int rc = BN_OK;
	if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) rc = BN_ERR_HIP;
	for (int i = 0; rc == BN_OK && i < plan->rd_n_passes; i++) {
		rc = rd_launch_one(plan, i, d_in, d_out, batch, st);  // untimed: steady-state input layout
		if (rc == BN_OK && hipEventRecord(e0, st) != hipSuccess) rc = BN_ERR_HIP;
		for (int r = 0; rc == BN_OK && r < reps; r++) rc = rd_launch_one(plan, i, d_in, d_out, batch, st);
		if (rc == BN_OK && hipEventRecord(e1, st) != hipSuccess) rc = BN_ERR_HIP;
		float t = 0.f;
		if (rc == BN_OK && (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&t, e0, e1) != hipSuccess))
			rc = BN_ERR_HIP;
		if (rc == BN_OK && i < max_passes) ms[i] = t / (float)reps;
	}
	if (e0) (void)hipEventDestroy(e0);
	if (e1) (void)hipEventDestroy(e1);
	plan->timing = saved;
	if (rc != BN_OK) BN_FAIL(rc, "timing the passes failed");
	*n_out = plan->rd_n_passes;
	return BN_OK;
}

}  // namespace bn
