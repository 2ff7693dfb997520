// Register-resident bitsliced additive NTT for gfx950 (kernel variant 4).
//
// What it computes: the passes of AdditiveNTT::apply (src/ulvt/ntt/additive_ntt.cuh:201-265), the
// butterflies u ^= w*v, v ^= u (antt_butterfly, :10-14) with the twiddle of calculate_twiddle
// (:59-77), over the same passes, tiles and HBM layouts as variant 1 (antt_bs.hip): a pass owns
// tiles of 128 bitsliced 32-element blocks, the output buffer holds bitsliced blocks between passes.
//
// Why registers: in the LDS-tile kernel every stage reads and writes the tile plane once
// (ds_write_b128 moves ~80 B/clk/CU, half the read rate), waits for LDS twice per stage, and a
// 74 KB tile allows only 2 work-groups (2 waves per SIMD) per CU. Here the tile lives in VGPRs:
//   * wave w owns limb plane w, lane L holds two blocks R0, R1 (64 VGPRs); the 7 tile bits are the
//     register index plus six lane coordinates c0 = L0^L2, c1 = L1^L2, c2..c5 = L2..L5;
//   * before the stage on tile bit m < 6 the register bit is exchanged with coordinate m: one
//     v_permlane32_swap / v_permlane16_swap per word pair for c5 / c4, and DPP reads (row_ror:8,
//     row_half_mirror, quad_perm) plus two selects for c3..c0 (partners L^8, L^7, L^2, L^1);
//   * the product accumulates straight into u (bsmN_mul_acc: u ^= w*v), so no product array;
//   * the in-word stages (bottom pass, index bits 0..4) keep the pair of blocks packed as
//     X = u-values, Y = v-values of both blocks (X ^= w*Y, Y ^= X), repacked between stages.
// LDS only stages the tile's HBM traffic, half a tile at a time (36 KB per work-group): the compact
// (16-byte element) input of the first pass and output of the last pass, and the bitsliced lines of
// the others (coalesced 1 KiB per wave-instruction, re-read lane-private). VGPRs set the occupancy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "antt_bs.hpp"
#include "bitsliced.hpp"

namespace bn {
namespace rr {

// minimum waves per SIMD the compiler must fit (VGPR budget 512 / n): the bottom pass needs 170
// registers unconstrained and fits 168 (three waves) without spills; the upper passes are left
// unconstrained (114-164 registers, three or four waves: forcing three made the scheduler spill)
template <int ROLE>
struct RrOcc {
	static constexpr int value = (ROLE == ROLE_LAST || ROLE == ROLE_SINGLE) ? 3 : 1;
};

struct RrParams {
	const uint32_t* src;
	uint32_t* dst;
	int log_h, log_rate;
	size_t ntiles;  // antt_rr_mid_pf (persistent grid): tiles of the pass
	RtPass p;
#ifdef BN_DEV
	int dbg;  // BN_DEBUG_FLAGS bit 0 = no tile loads, bit 1 = no tile stores (wrong results; timing
	          // experiments on antt_rr_pass)
#endif
};
#ifdef BN_DEV
#define RR_DBG(P) ((P).dbg)
#else
#define RR_DBG(P) 0
#endif

constexpr int kSlot = 36;                 // LDS words per staged block (32 + 4 pad: conflict-free b128 writes)
constexpr int kStagePlane = 64 * kSlot;   // one limb plane of a half tile

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ld4(const uint32_t* p, uint32_t* r) {
	const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
	r[0] = v.x, r[1] = v.y, r[2] = v.z, r[3] = v.w;
}
__device__ __forceinline__ void st4(uint32_t* p, const uint32_t* r) {
	u32x4 v;
	v.x = r[0], v.y = r[1], v.z = r[2], v.w = r[3];
	__builtin_nontemporal_store(v, (u32x4*)p);
}

__host__ __device__ constexpr uint32_t lane_mask(int j) {
	return j == 0 ? 0xAAAAAAAAu : j == 1 ? 0xCCCCCCCCu : j == 2 ? 0xF0F0F0F0u : j == 3 ? 0xFF00FF00u : 0xFFFF0000u;
}
__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t a, uint32_t b) {  // m ? a : b, bitwise
	return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}
__device__ __forceinline__ uint32_t bitmask(int x, int b) { return 0u - (uint32_t)((x >> b) & 1); }

// lane coordinates as a 6-bit number (tile bits of R0 in the initial mapping)
__device__ __forceinline__ int coords(int lane) {
	const int c0 = (lane ^ (lane >> 2)) & 1, c1 = ((lane >> 1) ^ (lane >> 2)) & 1;
	return c0 | (c1 << 1) | (lane & 0x3c);
}

// Exchange of the register bit with lane coordinate k (one code path for every k: a switch over
// per-coordinate DPP / permlane variants makes the register allocator copy R0/R1 at the merge):
// lanes with c_k = 0 keep R0 and take the partner's R0 into R1, lanes with c_k = 1 keep R1 and take
// the partner's R1 into R0. The partner is lane L ^ pi_k (pi = 1, 2, 7, 8, 16, 32), read with
// ds_bpermute (the LDS crossbar, no LDS memory); c_k = parity(L & kappa_k).
__device__ __forceinline__ void xchg(uint32_t* R0, uint32_t* R1, int lane, int k) {
	const int pi = k == 5 ? 32 : k == 4 ? 16 : k == 3 ? 8 : k == 2 ? 7 : k == 1 ? 2 : 1;
	const int kappa = k == 5 ? 32 : k == 4 ? 16 : k == 3 ? 8 : k == 2 ? 4 : k == 1 ? 6 : 5;
	const uint32_t cm = 0u - (uint32_t)(__builtin_popcount(lane & kappa) & 1);
	const int addr = (lane ^ pi) << 2;
#pragma unroll
	for (int i = 0; i < 32; i++) {
		const uint32_t x = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)sel(cm, R0[i], R1[i]));
		R0[i] = sel(cm, x, R0[i]);
		R1[i] = sel(cm, R1[i], x);
	}
}

// u ^= w * v on 32 bitsliced GF(2^32) limbs, w in GF(2^field) given compactly (the same twiddle in
// every bit-lane; field uniform per stage); v, u distinct. A GF(2^8) / GF(2^16) twiddle acts on each
// byte / half of the tower representation on its own.
template <int FMAX>
__device__ __forceinline__ void fma_tw(int field, uint32_t tw, const uint32_t* v, uint32_t* u) {
	if (FMAX <= 8 || field <= 8) {
		bsm3x4_fma_tw(v, tw, u);
	} else if (FMAX <= 16 || field <= 16) {
		bsm4x2_fma_tw(v, tw, u);
	} else {
		bsm5_fma_tw(v, tw, u);
	}
}

template <int L, int ROLE, int FMAX, int OCC = RrOcc<ROLE>::value>
__global__ __launch_bounds__(64 * L, OCC) void antt_rr_pass(RrParams P) {
	extern __shared__ uint32_t lds[];
	constexpr bool IN_COMPACT = ROLE == ROLE_FIRST || ROLE == ROLE_SINGLE;
	constexpr bool LAST = ROLE == ROLE_LAST || ROLE == ROLE_SINGLE;
	constexpr int NT = 64 * L;
	const RtPass& ps = P.p;
	const int tid = threadIdx.x;
	const int w = tid >> 6, lane = tid & 63;
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
	auto tile_off = [&](int q) -> size_t {
		size_t off = 0;
#pragma unroll
		for (int m = 0; m < kBlkBits; m++) off |= (size_t)((q >> m) & 1) << ps.bb[m];
		return off;
	};
	// work-group-uniform twiddle part (outer and coset bits) of stage j, held by lane j
	uint32_t cuv = 0;
	if (lane < ps.k) {
		for (int m = 0; m < ps.n_outer; m++)
			if ((outer >> m) & 1) cuv ^= ps.two[lane][m];
		for (int b = 0; b < P.log_rate; b++)
			if ((coset >> b) & 1) cuv ^= ps.twc[lane][b];
	}
	auto ucu = [&](int j) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)cuv, j); };

	const int G = coords(lane);
	uint32_t R0[32], R1[32];

	// ---- tile in. Initial mapping: register bit <-> tile bit 6, c_k <-> tile bit k, so R_h holds
	// block G + 64 h.
	if (IN_COMPACT && L == 4) {
		// compact 16-byte elements, half a tile (64 blocks) at a time through LDS: coalesced loads,
		// limb l of block slot s at plane l, word s * kSlot + element. Both halves' loads are issued
		// up front (64 VGPRs, below the stages' peak), so the second half's latency hides behind the
		// first half's LDS round trip and transposes.
		uint32_t gv[2][8][4];
#pragma unroll
		for (int h = 0; h < 2; h++)
#pragma unroll
			for (int r = 0; r < 8; r++) {
				const int idx = tid + NT * r, s = idx >> 5, e = idx & 31;
				if (RR_DBG(P) & 1)
					gv[h][r][0] = idx, gv[h][r][1] = s, gv[h][r][2] = e, gv[h][r][3] = tid;
				else
					ld4(src + (ooff | tile_off(s + 64 * h) | (size_t)e) * 4, gv[h][r]);
			}
#pragma unroll
		for (int h = 0; h < 2; h++) {
			if (h) __syncthreads();  // every wave has read the first half
#pragma unroll
			for (int r = 0; r < 8; r++) {
				const int idx = tid + NT * r, s = idx >> 5, e = idx & 31;
#pragma unroll
				for (int l = 0; l < 4; l++) lds[l * kStagePlane + s * kSlot + e] = gv[h][r][l];
			}
			__syncthreads();
			uint32_t* R = h ? R1 : R0;
			const uint32_t* sp = lds + w * kStagePlane + G * kSlot;
#pragma unroll
			for (int c = 0; c < 8; c++) {
				const uint4 v = *(const uint4*)(sp + 4 * c);
				R[4 * c] = v.x, R[4 * c + 1] = v.y, R[4 * c + 2] = v.z, R[4 * c + 3] = v.w;
			}
			transpose32(R);
		}
	} else {
		// bitsliced limb plane w of a block (128 contiguous bytes; or a compact GF(2^32) block), half
		// a tile at a time by LDS-DMA into this wave's LDS region (no VGPRs): instruction r fetches
		// slots 8 r .. 8 r + 7, lane L chunk (L & 7) ^ f(slot) of slot 8 r + L / 8, so every
		// instruction reads eight whole 128-byte lines and its 1 KiB lands lane-linear; the chunk
		// swizzle f(s) = (s >> 1) & 7 makes the lane-private re-reads (lane G: slot G) conflict-free
		char* wr = (char*)(lds + w * kStagePlane);
#pragma unroll
		for (int h = 0; h < 2; h++) {
			if (h) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // half 0 read out before the overwrite
#pragma unroll
			for (int r = 0; r < 8; r++) {
				const int sl = 8 * r + (lane >> 3), c = (lane & 7) ^ ((sl >> 1) & 7);
				if (RR_DBG(P) & 1) continue;
				__builtin_amdgcn_global_load_lds((const void*)(src + (ooff | tile_off(sl + 64 * h)) * L + 32 * w + 4 * c),
				                                 (__attribute__((address_space(3))) void*)(wr + 1024 * r), 16, 0, 0);
			}
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			uint32_t* R = h ? R1 : R0;
#pragma unroll
			for (int c = 0; c < 8; c++) {
				const uint4 v = *(const uint4*)(wr + 128 * G + 16 * (c ^ ((G >> 1) & 7)));
				R[4 * c] = v.x, R[4 * c + 1] = v.y, R[4 * c + 2] = v.z, R[4 * c + 3] = v.w;
			}
		}
		if (IN_COMPACT) {
			transpose32(R0);
			transpose32(R1);
		}
	}

	// ---- block stages on tile bits 6 .. mlow (the bottom pass runs all seven)
	const int mlow = LAST ? 0 : ps.mlow;
#pragma unroll 1
	for (int m = kBlkBits - 1; m >= mlow; m--) {
		if (m < kBlkBits - 1) xchg(R0, R1, lane, m);
		uint32_t tw = ucu(ps.jm[m]);
#pragma unroll
		for (int b = 0; b < 6; b++) tw ^= ps.tau[m][b] & bitmask(lane, b);
		__builtin_amdgcn_sched_barrier(0);
		fma_tw<FMAX>(ps.field_m[m], tw, R1, R0);  // u ^= w * v
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int i = 0; i < 32; i++) R1[i] ^= R0[i];  // v ^= u
	}

	if (LAST) {
		// ---- stages 4..0 inside the words. Mapping now: register bit <-> tile bit 0, c_k <-> tile
		// bit k + 1. The pair (A, B) = (R0, R1) is held packed per stage: X = u-values (A's on the
		// u-lanes, B's moved up onto the v-lanes), Y = v-values (A's moved down, B's in place);
		// one multiply then serves both blocks, with the twiddle words of variant 1's in-word stages.
#pragma unroll 1
		for (int s = 4; s >= 0; s--) {
			// shift count and lane mask as VGPR operands (an SGPR operand halves the issue rate)
			const uint32_t d = vgpr(1u << s);
			const uint32_t um = vgpr(~lane_mask(s));  // u-lanes (bit s clear)
#pragma unroll
			for (int i = 0; i < 32; i++) {
				const uint32_t x = sel(um, R0[i], R1[i] << d);
				const uint32_t y = sel(um, R0[i] >> d, R1[i]);
				R0[i] = x;
				R1[i] = y;
			}
			uint32_t cb = ucu(s - ps.lo) ^ ps.cb_const[s];
#pragma unroll
			for (int b = 0; b < 6; b++) cb ^= ps.tau_iw[s][b] & bitmask(lane, b);
			{
				// one circuit for every in-word stage, the pass's largest field (a sub-field twiddle is a
				// GF(2^32) value with zero upper bits; per-stage field branches here would make the
				// register allocator copy R0/R1 at their merge)
				uint32_t W[32];
				__builtin_amdgcn_sched_barrier(0);
				if (FMAX <= 8) {
#pragma unroll
					for (int i = 0; i < 8; i++) W[i] = ps.pat[s][i] ^ (uint32_t)__builtin_amdgcn_sbfe(cb, i, 1);
					bsm3x4_mul_acc(R1, W, R0);
				} else if (FMAX <= 16) {
#pragma unroll
					for (int i = 0; i < 16; i++) W[i] = ps.pat[s][i] ^ (uint32_t)__builtin_amdgcn_sbfe(cb, i, 1);
					bsm4x2_mul_acc(R1, W, R0);
				} else {
#pragma unroll
					for (int i = 0; i < 32; i++) W[i] = ps.pat[s][i] ^ (uint32_t)__builtin_amdgcn_sbfe(cb, i, 1);
					bsm5_mul_acc(R1, W, R0);
				}
				__builtin_amdgcn_sched_barrier(0);
			}
#pragma unroll
			for (int i = 0; i < 32; i++) {
				const uint32_t x = R0[i], y = R1[i] ^ x;  // v ^= u
				R0[i] = sel(um, x, y << d);                // A: u-lanes from X, v-lanes from Y
				R1[i] = sel(um, x >> d, y);                // B
			}
		}
		transpose32(R0);
		transpose32(R1);
		// lane holds limb w of blocks 2G (R0) and 2G + 1 (R1)
		if (L == 4) {
			// half a tile at a time through LDS: gather whole 16-byte elements, coalesced stores
#pragma unroll
			for (int h = 0; h < 2; h++) {
				if (h) __syncthreads();
				const uint32_t* R = h ? R1 : R0;
				uint32_t* sp = lds + w * kStagePlane + G * kSlot;
#pragma unroll
				for (int c = 0; c < 8; c++) *(uint4*)(sp + 4 * c) = make_uint4(R[4 * c], R[4 * c + 1], R[4 * c + 2], R[4 * c + 3]);
				__syncthreads();
#pragma unroll
				for (int r = 0; r < 8; r++) {
					const int idx = tid + NT * r, s = idx >> 5, e = idx & 31;
					uint32_t v[4];
#pragma unroll
					for (int l = 0; l < 4; l++) v[l] = lds[l * kStagePlane + s * kSlot + e];
					if (!(RR_DBG(P) & 2)) st4(dst + (ooff | tile_off(2 * s + h) | (size_t)e) * 4, v);
				}
			}
		} else {
#pragma unroll
			for (int c = 0; c < 8; c++) {
				st4(dst + (ooff | tile_off(2 * G)) + 4 * c, R0 + 4 * c);
				st4(dst + (ooff | tile_off(2 * G + 1)) + 4 * c, R1 + 4 * c);
			}
		}
	} else {
		// ---- bitsliced out. Final mapping: register bit <-> tile bit mlow, c_k <-> k (k < mlow) or
		// k + 1 (k >= mlow): R_h holds the block with tile bit mlow = h and G in the other bits
		// (through this wave's LDS region: coalesced stores of eight whole lines per instruction)
		const int lowm = (1 << mlow) - 1;
		uint32_t* wp = lds + w * kStagePlane;
#pragma unroll
		for (int h = 0; h < 2; h++) {
			const uint32_t* R = h ? R1 : R0;
#pragma unroll
			for (int c = 0; c < 8; c++) *(uint4*)(wp + G * kSlot + 4 * c) = make_uint4(R[4 * c], R[4 * c + 1], R[4 * c + 2], R[4 * c + 3]);
#pragma unroll
			for (int r = 0; r < 8; r++) {
				const int sl = 8 * r + (lane >> 3), c = lane & 7;
				const int q = ((sl & ~lowm) << 1) | (h << mlow) | (sl & lowm);
				const uint4 v = *(const uint4*)(wp + sl * kSlot + 4 * c);
				const uint32_t o[4] = {v.x, v.y, v.z, v.w};
				if (!(RR_DBG(P) & 2)) st4(dst + (ooff | tile_off(q)) * L + 32 * w + 4 * c, o);
			}
		}
	}
}

// ------------------------------------------------------------------------------------
// Middle passes with the next tile's loads hidden (persistent grid, two work-groups per CU). The
// LDS-tile kernel (antt_bs_pass) has no room to overlap a tile's loads with its stages: the tile
// fills the LDS (74 KB, two per CU) and the circuits the VGPRs, so each tile's loads are exposed
// (the dev build's no-load run of pass 1 at 2^24 is 17 % faster). Here the tile lives in VGPRs (as
// antt_rr_pass) and the LDS holds, per wave,
//   * 16 KB: the NEXT tile's limb plane, requested by LDS-DMA (global_load_lds, no VGPRs) as soon as
//     this tile's plane has been read out of the same region, landing while this tile computes;
//   * 4 KB: output staging, 32 blocks at a time (coalesced 1 KiB stores of whole lines).
// 4 x 20 KB = 80 KB per work-group, two per CU. Same tiles, tables and HBM layout as antt_rr_pass.
// Development build only (BN_MID_PF=1): parity green (GF(2^128) suite + MD5 tables), but pass 1 at
// 2^24 measured 0.224-0.229 ms against 0.189-0.193 ms for antt_bs_pass (three A/B pairs, round 5):
// the register tile's exchanges cost more than the hidden loads give back.
// ------------------------------------------------------------------------------------
#ifdef BN_DEV
__device__ __forceinline__ int opaque_lane() {
	int x = (int)threadIdx.x & 63;
	asm volatile("" : "=v"(x) : "0"(x));
	return x;
}
constexpr int kPreWords = 128 * 32;  // per wave: a whole limb plane, chunk-swizzled (no padding)
constexpr int kOutWords = 32 * 32;   // per wave: 32 blocks of output staging, chunk-swizzled

template <int FMAX>
__global__ __launch_bounds__(256, 2) void antt_rr_mid_pf(RrParams P) {
	extern __shared__ uint32_t lds[];
	constexpr int L = 4;
	const RtPass& ps = P.p;
	const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
	// the lane index is re-read opaquely at every tile: lane-derived addresses hoisted out of the tile
	// loop would stay live through the circuits and spill
	int lane = threadIdx.x & 63;
	const size_t n = (size_t)1 << P.log_h;
	char* pre = (char*)(lds + w * kPreWords);
	uint32_t* ost = lds + L * kPreWords + w * kOutWords;
	auto tile_off = [&](int q) -> size_t {
		size_t off = 0;
#pragma unroll
		for (int m = 0; m < kBlkBits; m++) off |= (size_t)((q >> m) & 1) << ps.bb[m];
		return off;
	};
	struct Geo {
		size_t outer, ooff;
		int coset;
		uint32_t* d;
	};
	auto geo = [&](size_t t) -> Geo {
		Geo g;
		g.outer = t & (((size_t)1 << ps.n_outer) - 1);
		const size_t rest = t >> ps.n_outer;
		g.coset = (int)(rest & ((1u << P.log_rate) - 1));
		const size_t batch = rest >> P.log_rate;
		g.ooff = 0;
		for (int m = 0; m < ps.n_outer; m++) g.ooff |= ((g.outer >> m) & 1) << ps.ob[m];
		g.d = P.dst + (((batch << P.log_rate) + (size_t)g.coset) * n) * L;
		return g;
	};
	// the tile's limb plane w by LDS-DMA into `pre`: instruction 8 h + r fetches slots 8 r .. 8 r + 7 of
	// half h (blocks + 64 h), lane L chunk (L & 7) ^ f(slot) of slot 8 r + L / 8 (antt_rr_pass's layout)
	auto dma = [&](const Geo& g) {
#pragma unroll
		for (int h = 0; h < 2; h++)
#pragma unroll
			for (int r = 0; r < 8; r++) {
				const int sl = 8 * r + (lane >> 3), c = (lane & 7) ^ ((sl >> 1) & 7);
				__builtin_amdgcn_global_load_lds((const void*)(g.d + (g.ooff | tile_off(sl + 64 * h)) * L + 32 * w + 4 * c),
				                                 (__attribute__((address_space(3))) void*)(pre + 8192 * h + 1024 * r), 16, 0, 0);
			}
	};
	size_t tile = blockIdx.x;
	Geo cur = geo(tile);
	dma(cur);
	const int mlow = ps.mlow;
	for (;;) {
		lane = opaque_lane();
		const int G = coords(lane);
		// work-group-uniform twiddle part (outer and coset bits) of stage j, held by lane j
		uint32_t cuv = 0;
		if (lane < ps.k) {
			for (int m = 0; m < ps.n_outer; m++)
				if ((cur.outer >> m) & 1) cuv ^= ps.two[lane][m];
			for (int b = 0; b < P.log_rate; b++)
				if ((cur.coset >> b) & 1) cuv ^= ps.twc[lane][b];
		}
		auto ucu = [&](int j) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)cuv, j); };
		// ---- this tile's plane: its DMA is done once all but the previous tile's 16 stores are
		uint32_t R0[32], R1[32];
#ifdef BN_MID_PF_ASM
		{
			// read in inline asm: the compiler cannot tell this tile's DMA from the previous tile's
			// stores and would wait for both (vmcnt(0)) before an LDS read it can see
			typedef unsigned int v4u __attribute__((ext_vector_type(4)));
			v4u x[16];
			const uint32_t a0 = (uint32_t)(uintptr_t)(pre + 128 * G);
			const uint32_t sw = 16u * (uint32_t)((G >> 1) & 7);
			uint32_t ad[8];
#pragma unroll
			for (int c = 0; c < 8; c++) ad[c] = a0 + ((16u * c) ^ sw);
			asm volatile(
			    "s_waitcnt vmcnt(16)\n"
			    "ds_read_b128 %0, %16\n ds_read_b128 %1, %17\n ds_read_b128 %2, %18\n ds_read_b128 %3, %19\n"
			    "ds_read_b128 %4, %20\n ds_read_b128 %5, %21\n ds_read_b128 %6, %22\n ds_read_b128 %7, %23\n"
			    "ds_read_b128 %8, %16 offset:8192\n ds_read_b128 %9, %17 offset:8192\n ds_read_b128 %10, %18 offset:8192\n"
			    "ds_read_b128 %11, %19 offset:8192\n ds_read_b128 %12, %20 offset:8192\n ds_read_b128 %13, %21 offset:8192\n"
			    "ds_read_b128 %14, %22 offset:8192\n ds_read_b128 %15, %23 offset:8192\n"
			    "s_waitcnt lgkmcnt(0)"
			    : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), "=&v"(x[7]),
			      "=&v"(x[8]), "=&v"(x[9]), "=&v"(x[10]), "=&v"(x[11]), "=&v"(x[12]), "=&v"(x[13]), "=&v"(x[14]), "=&v"(x[15])
			    : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7])
			    : "memory");
#pragma unroll
			for (int c = 0; c < 8; c++) {
				R0[4 * c] = x[c].x, R0[4 * c + 1] = x[c].y, R0[4 * c + 2] = x[c].z, R0[4 * c + 3] = x[c].w;
				R1[4 * c] = x[8 + c].x, R1[4 * c + 1] = x[8 + c].y, R1[4 * c + 2] = x[8 + c].z, R1[4 * c + 3] = x[8 + c].w;
			}
		}
#else
		asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
#pragma unroll
		for (int h = 0; h < 2; h++) {
			uint32_t* R = h ? R1 : R0;
#pragma unroll
			for (int c = 0; c < 8; c++) {
				const uint4 v = *(const uint4*)(pre + 8192 * h + 128 * G + 16 * (c ^ ((G >> 1) & 7)));
				R[4 * c] = v.x, R[4 * c + 1] = v.y, R[4 * c + 2] = v.z, R[4 * c + 3] = v.w;
			}
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read out: the region takes the next tile
#endif
		const size_t next = tile + gridDim.x;
		const bool has_next = next < P.ntiles;
		Geo nxt = cur;
		if (has_next) {
			nxt = geo(next);
			dma(nxt);
		}

		// ---- block stages on tile bits 6 .. mlow (antt_rr_pass)
#pragma unroll 1
		for (int m = kBlkBits - 1; m >= mlow; m--) {
			if (m < kBlkBits - 1) xchg(R0, R1, lane, m);
			uint32_t tw = ucu(ps.jm[m]);
#pragma unroll
			for (int b = 0; b < 6; b++) tw ^= ps.tau[m][b] & bitmask(lane, b);
			__builtin_amdgcn_sched_barrier(0);
			fma_tw<FMAX>(ps.field_m[m], tw, R1, R0);  // u ^= w * v
			__builtin_amdgcn_sched_barrier(0);
#pragma unroll
			for (int i = 0; i < 32; i++) R1[i] ^= R0[i];  // v ^= u
		}

		// ---- bitsliced out, 32 blocks per round through this wave's 4 KB: round (h, hh) stages the
		// blocks of R_h held by lanes 32 hh .. 32 hh + 31 (slot G & 31, chunk-swizzled), then the wave
		// stores them as four 1 KiB runs of whole 128-byte lines (antt_rr_pass's block mapping)
		const int lowm = (1 << mlow) - 1;
#pragma unroll
		for (int h = 0; h < 2; h++) {
			const uint32_t* R = h ? R1 : R0;
#pragma unroll
			for (int hh = 0; hh < 2; hh++) {
				if ((G >> 5) == hh) {
					const int so = G & 31;
#pragma unroll
					for (int c = 0; c < 8; c++)
						*(uint4*)(ost + 32 * so + 4 * (c ^ ((so >> 1) & 7))) = make_uint4(R[4 * c], R[4 * c + 1], R[4 * c + 2], R[4 * c + 3]);
				}
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
				for (int r = 0; r < 4; r++) {
					const int so = 8 * r + (lane >> 3), c = lane & 7;
					const int sl = 32 * hh + so;
					const int q = ((sl & ~lowm) << 1) | (h << mlow) | (sl & lowm);
					const uint4 v = *(const uint4*)(ost + 32 * so + 4 * (c ^ ((so >> 1) & 7)));
					const uint32_t o[4] = {v.x, v.y, v.z, v.w};
					st4(cur.d + (cur.ooff | tile_off(q)) * L + 32 * w + 4 * c, o);
				}
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read out before the next round's writes
			}
		}
		if (!has_next) break;
		tile = next;
		cur = nxt;
	}
}

static size_t mid_pf_lds_bytes() { return (size_t)4 * (kPreWords + kOutWords) * sizeof(uint32_t); }
#endif  // BN_DEV

template <int L, int FMAX>
static const void* kernel_f(int role) {
	switch (role) {
		case ROLE_FIRST: return (const void*)antt_rr_pass<L, ROLE_FIRST, FMAX>;
		case ROLE_MID: return (const void*)antt_rr_pass<L, ROLE_MID, FMAX>;
		case ROLE_LAST: return (const void*)antt_rr_pass<L, ROLE_LAST, FMAX>;
		default: return (const void*)antt_rr_pass<L, ROLE_SINGLE, FMAX>;
	}
}
static const void* kernel_for(int L, int role, int fmax) {
	if (L == 4) return fmax <= 8 ? kernel_f<4, 8>(role) : fmax <= 16 ? kernel_f<4, 16>(role) : kernel_f<4, 32>(role);
	return fmax <= 8 ? kernel_f<1, 8>(role) : fmax <= 16 ? kernel_f<1, 16>(role) : kernel_f<1, 32>(role);
}
// The bottom pass of a launch with fewer tiles than two per CU runs one wave per SIMD whatever its
// register count, so it is compiled without the three-waves bound (no spills)
static bool small_last(int L, int role, size_t ntiles, int num_cus) {
	return L == 4 && role == ROLE_LAST && ntiles < (size_t)2 * (size_t)num_cus;
}
static const void* kernel_small_last(int fmax) {
	return fmax <= 8 ? (const void*)antt_rr_pass<4, ROLE_LAST, 8, 1> : fmax <= 16 ? (const void*)antt_rr_pass<4, ROLE_LAST, 16, 1>
	                                                                              : (const void*)antt_rr_pass<4, ROLE_LAST, 32, 1>;
}
// every role stages through LDS: compact elements (first / last pass) or coalesced bitsliced lines
static size_t lds_bytes(int L, int role) {
	(void)role;
	return (size_t)L * kStagePlane * sizeof(uint32_t);
}

}  // namespace rr

int rr_prepare(bn_antt_plan* plan) {
	(void)plan;
#ifdef BN_DEV
	for (const void* f : {(const void*)rr::antt_rr_mid_pf<16>, (const void*)rr::antt_rr_mid_pf<32>})
		BN_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)rr::mid_pf_lds_bytes()));
#endif
	for (int L : {1, 4})
		for (int role = 0; role < 4; role++)
			for (int f : {8, 16, 32})
				BN_HIP(hipFuncSetAttribute(rr::kernel_for(L, role, f), hipFuncAttributeMaxDynamicSharedMemorySize,
				                           (int)std::max<size_t>(rr::lds_bytes(L, role), 1)));
	for (int f : {8, 16, 32})
		BN_HIP(hipFuncSetAttribute(rr::kernel_small_last(f), hipFuncAttributeMaxDynamicSharedMemorySize,
		                           (int)rr::lds_bytes(4, ROLE_LAST)));
	return BN_OK;
}

const void* rr_pass_kernel(bn_antt_plan* plan, const BsPass& pass) {
	const size_t ntiles = ((size_t)1 << plan->log_rate) << pass.n_outer;  // one transform (see bs_pass_kernel)
	if (rr::small_last(plan->limbs, pass.role, ntiles, plan->num_cus)) return rr::kernel_small_last(pass_fmax(pass));
	return rr::kernel_for(plan->limbs, pass.role, pass_fmax(pass));
}

// pass i of variant 4 (same pass split and tables as variant 1)
int rr_launch_pass(bn_antt_plan* plan, int i, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st) {
	size_t n_passes = 0;
	const BsPass* passes = bs_passes(plan, &n_passes);
	if (i < 0 || (size_t)i >= n_passes) BN_FAIL(BN_ERR_INVALID, "pass %d out of range", i);
	const BsPass& pass = passes[i];
	const bool bottom = pass.role == ROLE_LAST || pass.role == ROLE_SINGLE;
	rr::RrParams prm;
	prm.src = d_in;
	prm.dst = d_out;
	prm.log_h = plan->log_h;
	prm.log_rate = plan->log_rate;
	prm.ntiles = (batch << plan->log_rate) << pass.n_outer;
#ifdef BN_DEV
	prm.dbg = 0;
	if (const char* e = getenv("BN_DEBUG_FLAGS")) prm.dbg = atoi(e) & 3;
#endif
	int rc = make_rt(pass, bottom, &prm.p);
	if (rc != BN_OK) BN_FAIL(rc, "register-tile pass table: stage bits are not the top tile bits");
	const int L = plan->limbs;
	const size_t ntiles = (batch << plan->log_rate) << pass.n_outer;
	rc = timing_begin(plan, i, st);
	if (rc != BN_OK) return rc;
	void* args[] = {&prm};
	const void* k = rr::small_last(L, pass.role, ntiles, plan->num_cus) ? rr::kernel_small_last(pass_fmax(pass))
	                                                                    : rr::kernel_for(L, pass.role, pass_fmax(pass));
	BN_HIP(hipLaunchKernel(k, dim3((unsigned)ntiles), dim3(64 * L), args, rr::lds_bytes(L, pass.role), st));
	return timing_end(plan, i, st);
}

#ifdef BN_DEV
// a middle pass (bitsliced in and out, GF(2^16/32) twiddles) on the prefetching register-tile kernel
int rr_launch_mid_pf(bn_antt_plan* plan, int i, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st) {
	size_t n_passes = 0;
	const BsPass* passes = bs_passes(plan, &n_passes);
	if (i < 0 || (size_t)i >= n_passes) BN_FAIL(BN_ERR_INVALID, "pass %d out of range", i);
	const BsPass& pass = passes[i];
	if (pass.role != ROLE_MID || plan->limbs != 4) BN_FAIL(BN_ERR_UNSUPPORTED, "prefetching kernel: middle passes of GF(2^128) plans only");
	rr::RrParams prm;
	prm.src = d_in;
	prm.dst = d_out;
	prm.log_h = plan->log_h;
	prm.log_rate = plan->log_rate;
	int rc = make_rt(pass, false, &prm.p);
	if (rc != BN_OK) BN_FAIL(rc, "register-tile pass table: stage bits are not the top tile bits");
	const size_t ntiles = (batch << plan->log_rate) << pass.n_outer;
	prm.ntiles = ntiles;
	prm.dbg = 0;  // (development build only: this launcher exists only there)
	const size_t grid = std::min(ntiles, (size_t)2 * (size_t)plan->num_cus);
	rc = timing_begin(plan, i, st);
	if (rc != BN_OK) return rc;
	void* args[] = {&prm};
	const void* k = pass_fmax(pass) <= 16 ? (const void*)rr::antt_rr_mid_pf<16> : (const void*)rr::antt_rr_mid_pf<32>;
	BN_HIP(hipLaunchKernel(k, dim3((unsigned)grid), dim3(256), args, rr::mid_pf_lds_bytes(), st));
	return timing_end(plan, i, st);
}

const void* rr_mid_pf_kernel(const BsPass& pass) {
	return pass_fmax(pass) <= 16 ? (const void*)rr::antt_rr_mid_pf<16> : (const void*)rr::antt_rr_mid_pf<32>;
}

#endif  // BN_DEV

int launch_rr(bn_antt_plan* plan, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st) {
	size_t n_passes = 0;
	bs_passes(plan, &n_passes);
	for (size_t i = 0; i < n_passes; i++) {
		const int rc = rr_launch_pass(plan, (int)i, d_in, d_out, batch, st);
		if (rc != BN_OK) return rc;
	}
	return BN_OK;
}

}  // namespace bn
