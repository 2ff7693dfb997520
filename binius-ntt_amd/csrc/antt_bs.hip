// Bitsliced, LDS-tiled additive NTT for gfx950 (kernel variant 1).
//
// Data layout
//   * A "block" is 32 consecutive elements. In bitsliced form (the same layout as the
//     reference's BitsliceUtils<128>, src/ulvt/utils/bitslicing.cuh:32-47) block word
//     32*l + i holds bit i of limb l of the 32 elements, element e in bit e.
//   * Between passes the transform lives in HBM as bitsliced blocks in element order (our own
//     scratch layout); the first pass reads the caller's compact AoS input and the last pass
//     writes compact AoS output, so exactly two bit-transposes happen per transform.
//   * A workgroup owns a tile of 128 blocks (2^12 elements, 72 KiB of LDS at GF(2^128), two
//     workgroups per CU so one loads/stores while the other computes): index bits 0..4 inside
//     each word plus 7 "block bits" bb[0..6]; the remaining index bits are fixed per workgroup.
//
// Arithmetic
//   Every twiddle lies in GF(2^32) and multiplies each GF(2^32) limb separately, so a
//   GF(2^128) butterfly is four GF(2^32) bitsliced butterflies sharing one twiddle. Products
//   use the generated Karatsuba circuits (bitsliced_gen.hpp, v_bitop3-fused); the host picks,
//   per stage, the smallest sub-field (GF(2^8)/GF(2^16)/GF(2^32)) that holds every twiddle
//   (multiplication by a sub-field scalar acts on each sub-field coordinate independently).
//   Twiddles are linear in the butterfly-block index (calculate_twiddle, additive_ntt.cuh:
//   59-77): the host tabulates, per stage, the contribution of every tile bit, every fixed
//   (workgroup) index bit and every coset bit, so a twiddle is a handful of masked XORs.
//
// Stage schedule: block-bit stages go through LDS (partners change every stage). In the bottom
// pass the 5 stages on index bits 0..4 pair bit-lanes of one word, so each thread keeps its two
// blocks in registers for all of them and transposes them back to compact form in registers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <type_traits>
#include <vector>

#include "antt_bs.hpp"
#include "bitsliced.hpp"
#include "quad_mul.hpp"

namespace bn {

struct BsParams {
	const uint32_t* src;
	uint32_t* dst;
	size_t ntiles;  // tiles of the pass; the (persistent) grid may be smaller
	int log_h, log_rate;
	unsigned long long* trace;  // BN_TRACE=1: per-wave phase timestamps (dev tool)
	int dbg;  // timing experiments only (BN_DEBUG_FLAGS): 1 no loads, 2 no stores, 4 no multiplies,
	          // 8 no stage barriers, 16 no in-word stages, 32 no tile-bit stages,
	          // 64 no lgkmcnt wait between stages
	BsPass p;
};

// timing switches and phase traces exist only in the development build (make BN_DEV=1)
#ifdef BN_DEV
#define BS_DBG(P) ((P).dbg)
#define BS_TRACE(P) ((P).trace != nullptr)
#else
#define BS_DBG(P) 0
#define BS_TRACE(P) false
#endif

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// streaming (non-temporal) 16-byte global accesses: every byte is touched once per pass
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

// bit masks of the bit-lanes p with bit j of p set
__host__ __device__ constexpr uint32_t lane_mask(int j) {
	return j == 0 ? 0xAAAAAAAAu : j == 1 ? 0xCCCCCCCCu : j == 2 ? 0xF0F0F0F0u : j == 3 ? 0xFF00FF00u : 0xFFFF0000u;
}

// out = w*x for 32 bitsliced GF(2^32) limbs (alias-safe: out may be x). W holds bit i of each
// lane's twiddle in word i; `field` (uniform per stage) selects the sub-field circuit, FMAX (the
// largest field of the pass) removes the circuits a pass never uses.
template <int FMAX>
__device__ __forceinline__ void mul_tw(int field, const uint32_t* x, const uint32_t* W, uint32_t* out) {
	if (FMAX <= 8 || field <= 8) {
#pragma unroll
		for (int g = 0; g < 4; g++) bsm3_mul(x + 8 * g, W, out + 8 * g);
	} else if (FMAX <= 16 || field <= 16) {
#pragma unroll
		for (int g = 0; g < 2; g++) bsm4_mul(x + 16 * g, W, out + 16 * g);
	} else {
		bsm5_mul(x, W, out);
	}
}

// LDS image of a tile: one plane per limb, block q of limb l at l*kPlane + q*kLimbStride (stride 36
// words: 16 consecutive blocks of one plane hit 16 distinct 4-bank groups, so a wave's
// ds_read_b128 over consecutive blocks is conflict-free).
constexpr int kPlane = kTileBlocks * kLimbStride;
constexpr int kLoads = kTileBlocks * 8 / 64;  // 16-byte global loads per lane per tile

// Stage-to-stage ordering inside one wave: a wave's LDS operations execute in order, so only the
// compiler must not move accesses across this point (the wait also bounds the LDS queue).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// One pass over every tile. Without PF a workgroup transforms tile blockIdx.x. With PF the grid
// is persistent (workgroup b takes tiles b, b + grid, ...) and the next tile's global loads are
// issued into registers right after the current tile reaches LDS, so they are in flight during
// the stages instead of exposed at the start of the next tile.
template <int L, int ROLE, int FMAX, bool PF>
__device__ __forceinline__ void bs_pass_body(const BsParams& P, size_t tile0) {
	extern __shared__ uint32_t lds[];
	constexpr int NT = 64 * L;
	constexpr bool IN_COMPACT = ROLE == ROLE_FIRST || ROLE == ROLE_SINGLE;
	constexpr bool LAST = ROLE == ROLE_LAST || ROLE == ROLE_SINGLE;  // bottom pass, compact out
	const BsPass& ps = P.p;
	const int tid = threadIdx.x;
	// wave w owns limb w of the tile for every stage: the waves never wait for each other
	// between stages (the four GF(2^32) limb transforms share only their twiddles)
	const int l = tid >> 6, lane = tid & 63;
	uint32_t* plane = lds + l * kPlane;
	uint32_t* cu_w = lds + L * kPlane + l * kMaxStages;  // this wave's copy of the uniform twiddle parts
	const size_t n = (size_t)1 << P.log_h;
	const bool TR = BS_TRACE(P);
	unsigned long long tr[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // load, block, in-word, store, tiles, pre, mul, post
	auto ts = [&]() -> unsigned long long {
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		return __builtin_amdgcn_s_memtime();
	};

	auto tile_off = [&](int q) -> size_t {
		size_t off = 0;
#pragma unroll
		for (int m = 0; m < kBlkBits; m++) off |= (size_t)((q >> m) & 1) << ps.bb[m];
		return off;
	};
	// tile -> (outer bits, coset, batch) -> addresses
	size_t outer, outer_off;
	int coset;
	uint32_t* dst;
	const uint32_t* src;
	auto geo = [&](size_t t, size_t& o, size_t& ooff, int& c, uint32_t*& d, const uint32_t*& s) {
		o = t & (((size_t)1 << ps.n_outer) - 1);
		const size_t rest = t >> ps.n_outer;
		c = (int)(rest & ((1u << P.log_rate) - 1));
		const size_t batch = rest >> P.log_rate;
		ooff = 0;
		for (int m = 0; m < ps.n_outer; m++) ooff |= ((o >> m) & 1) << ps.ob[m];
		d = P.dst + (((batch << P.log_rate) + (size_t)c) * n) * L;
		s = IN_COMPACT ? (P.src + batch * n * L) : d;
	};
	uint4 gbuf[kLoads];
	auto issue = [&](const uint32_t* s, size_t ooff) {
#pragma unroll
		for (int r = 0; r < kLoads; r++) {
			if (IN_COMPACT) {
				// compact elements: 16-byte loads, 8*L lanes per 32-element block
				const int u = tid + r * NT;
				const int q = u / (8 * L), j = u % (8 * L);
				gbuf[r] = (BS_DBG(P) & 1) ? make_uint4(u, j, q, tid) : ld_stream(s + (ooff | tile_off(q)) * L + 4 * j);
			} else {
				// bitsliced: limb l of block q is 128 contiguous bytes, each wave loads its own plane
				const int u = lane + r * 64;
				const int q = u >> 3, j = u & 7;
				gbuf[r] = (BS_DBG(P) & 1) ? make_uint4(u, j, q, tid) : ld_stream(s + (ooff | tile_off(q)) * L + 32 * l + 4 * j);
			}
		}
	};

	auto tile_tw = [&](int j, int q) -> uint32_t {
		uint32_t w = 0;
#pragma unroll
		for (int m = 0; m < kBlkBits; m++) w ^= ps.twt[j][m] & (uint32_t)__builtin_amdgcn_sbfe(q, m, 1);
		return w;
	};

	// ---- tile-bit stages (index bits >= 5), high to low. Lane = block pair of the wave's limb;
	// only V and the twiddle are live during the multiply, U is read afterwards.
	auto block_stage = [&](int j, int pair) {
		unsigned long long t_a = TR ? ts() : 0;
		const int m = ps.stage_m[j];
		const int qu = ((pair >> m) << (m + 1)) | (pair & ((1 << m) - 1));
		const int qv = qu | (1 << m);
		const uint32_t w = cu_w[j] ^ tile_tw(j, qu);
		uint32_t* pu = plane + qu * kLimbStride;
		uint32_t* pv = plane + qv * kLimbStride;
		uint32_t W[32], V[32], Pr[32], U[32];
#pragma unroll
		for (int i = 0; i < 32; i += 4) *(uint4*)(V + i) = *(const uint4*)(pv + i);
		// with the small GF(2^8) circuits there are registers for U: request it before the multiply
		if (FMAX <= 8) {
#pragma unroll
			for (int i = 0; i < 32; i += 4) *(uint4*)(U + i) = *(const uint4*)(pu + i);
		}
		// the stage on the top tile bit: qu's bits 0..5 are the lane's, and when none of them moves
		// the twiddle (twt[j][0..5] = 0: the tile's other bits are lower stages) it is the
		// workgroup-uniform part alone, so the circuit's twiddle side is scalar (bsm5_mul_w)
		bool uni = FMAX == 32 && m == kBlkBits - 1 && ps.field[j] == 32 && !(BS_DBG(P) & 4);
#pragma unroll
		for (int mm = 0; mm < kBlkBits - 1; mm++) uni = uni && ps.twt[j][mm] == 0u;
		if (uni) {
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			__builtin_amdgcn_sched_barrier(0);
			bsm5_mul_w(V, (uint32_t)__builtin_amdgcn_readfirstlane((int)cu_w[j]), Pr);
			__builtin_amdgcn_sched_barrier(0);
		} else {
#pragma unroll
		for (int i = 0; i < 32; i++) W[i] = (uint32_t)__builtin_amdgcn_sbfe(w, i, 1);
		if (TR) {
			const unsigned long long t = ts();
			tr[5] += t - t_a;
			t_a = t;
		}
		if (BS_DBG(P) & 4) {
#pragma unroll
			for (int i = 0; i < 32; i++) Pr[i] = V[i] ^ W[i];
		} else {
			// V complete before the circuit: with its loads in flight the scheduler hoists the w-side
			// Karatsuba sums to cover their latency, and runs out of registers
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			__builtin_amdgcn_sched_barrier(0);
			mul_tw<FMAX>(ps.field[j], V, W, Pr);  // sub-field circuits reuse W: Pr must not alias it
			__builtin_amdgcn_sched_barrier(0);
		}
		}
		if (TR) {
			uint32_t acc = 0;
#pragma unroll
			for (int i = 0; i < 32; i++) acc ^= Pr[i];
			asm volatile("" ::"v"(acc));
			const unsigned long long t = ts();
			tr[6] += t - t_a;
			t_a = t;
		}
#pragma unroll
		for (int i = 0; i < 32; i += 4) {
			uint4 u = FMAX <= 8 ? *(const uint4*)(U + i) : *(const uint4*)(pu + i);
			u.x ^= Pr[i];
			u.y ^= Pr[i + 1];
			u.z ^= Pr[i + 2];
			u.w ^= Pr[i + 3];
			*(uint4*)(pu + i) = u;
			*(uint4*)(pv + i) = make_uint4(V[i] ^ u.x, V[i + 1] ^ u.y, V[i + 2] ^ u.z, V[i + 3] ^ u.w);
		}
		if (TR) tr[7] += ts() - t_a;
	};

	size_t tile = tile0;
	geo(tile, outer, outer_off, coset, dst, src);
	if (PF) issue(src, outer_off);
	for (;;) {
		unsigned long long t0 = TR ? ts() : 0;
		// the previous tile's cross-plane LDS readers (compact store) / writers (compact load)
		// are done before this tile's planes are overwritten
		if (IN_COMPACT || LAST) __syncthreads();
		if (!PF) issue(src, outer_off);

		// workgroup-uniform twiddle part of every stage (outer + coset bits), one lane per stage
		if (lane < ps.k) {
			uint32_t c = 0;
			for (int m = 0; m < ps.n_outer; m++) c ^= ps.two[lane][m] & (0u - (uint32_t)((outer >> m) & 1));
			for (int b = 0; b < P.log_rate; b++) c ^= ps.twc[lane][b] & (0u - (uint32_t)((coset >> b) & 1));
			cu_w[lane] = c;
		}

		// ---- tile into LDS
#pragma unroll
		for (int r = 0; r < kLoads; r++) {
			const uint4 g = gbuf[r];
			if (IN_COMPACT) {
				// split by limb into the planes
				const int u = tid + r * NT;
				const int q = u / (8 * L), j = u % (8 * L);
				const uint32_t w[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
				for (int t = 0; t < 4; t++) {
					const int word = 4 * j + t;
					lds[(word % L) * kPlane + q * kLimbStride + word / L] = w[t];
				}
			} else {
				const int u = lane + r * 64;
				const int q = u >> 3, j = u & 7;
				*(uint4*)(plane + q * kLimbStride + 4 * j) = g;
			}
		}
		const size_t next = tile + gridDim.x;
		const bool has_next = PF && next < P.ntiles;  // without PF: one tile per workgroup
		size_t n_outer_v = outer, n_ooff = outer_off;
		int n_coset = coset;
		uint32_t* n_dst = dst;
		const uint32_t* n_src = src;
		if (has_next) {
			geo(next, n_outer_v, n_ooff, n_coset, n_dst, n_src);
			issue(n_src, n_ooff);  // in flight during this tile's stages
		}
		if (IN_COMPACT) {
			// per-(block, limb) 32x32 transposes of this wave's plane
			__syncthreads();
			for (int q = lane; q < kTileBlocks; q += 64) {
				uint32_t* x = plane + q * kLimbStride;
				uint32_t r[32];
#pragma unroll
				for (int i = 0; i < 32; i += 4) *(uint4*)(r + i) = *(const uint4*)(x + i);
				transpose32(r);
#pragma unroll
				for (int i = 0; i < 32; i += 4) *(uint4*)(x + i) = *(const uint4*)(r + i);
			}
		}
		wave_lds_sync();
		unsigned long long t1 = 0;
		if (TR) {
			t1 = ts();
			tr[0] += t1 - t0;
		}

		const int jlow = max(LAST ? 5 : 0, ps.stop_j);
		for (int j = ps.k - 1; j >= jlow; j--) {
			if (!(BS_DBG(P) & 32)) block_stage(j, lane);
			if (BS_DBG(P) & 64)
				asm volatile("" ::: "memory");  // experiment: rely on in-order LDS execution only
			else
				wave_lds_sync();
		}
		if (TR) {
			const unsigned long long t = ts();
			tr[1] += t - t1;
			t1 = t;
		}

		if (LAST) {
			// ---- stages 4..0 (index bits inside the word), lane-private: lane owns blocks qa = lane
			// and qb = lane + 64 for all of them. Per stage both blocks share one multiply: A's
			// v-lanes move down onto the u positions, B's v-lanes stay on the v positions (a pair's
			// twiddle depends only on index bits above s).
			const int qa = lane, qb = qa | (kTileBlocks / 2);
			uint32_t* pa = plane + qa * kLimbStride;
			uint32_t* pb = plane + qb * kLimbStride;
			for (int s = 4; s >= ((BS_DBG(P) & 16) ? 5 : ps.stop_j); s--) {  // bottom pass starts at stage 0: j == s
				// shift count and lane mask as VGPR operands (an SGPR operand halves the issue rate)
				const uint32_t d = vgpr(1u << s);
				const uint32_t um = vgpr(~lane_mask(s));  // u-lanes (bit s clear)
				const uint32_t cb = cu_w[s] ^ tile_tw(s, qb);
				uint32_t W[32], T[32];
#pragma unroll
				for (int i = 0; i < 32; i += 4) {
					const uint4 a = *(const uint4*)(pa + i), b = *(const uint4*)(pb + i);
					T[i] = __builtin_amdgcn_bitop3_b32(a.x >> d, b.x, um, 0xe4);  // (a>>d & um) | (b & ~um)
					T[i + 1] = __builtin_amdgcn_bitop3_b32(a.y >> d, b.y, um, 0xe4);
					T[i + 2] = __builtin_amdgcn_bitop3_b32(a.z >> d, b.z, um, 0xe4);
					T[i + 3] = __builtin_amdgcn_bitop3_b32(a.w >> d, b.w, um, 0xe4);
				}
				// twiddle word i: pattern (bit-lane bits s+1..4) ^ block part, cb on B's lanes and
				// ca = cb ^ twt[s][6] on A's (um) lanes; the host folds the um & twt[s][6] part into pat
#pragma unroll
				for (int i = 0; i < 32; i++) W[i] = ps.pat[s][i] ^ (uint32_t)__builtin_amdgcn_sbfe(cb, i, 1);
				if (BS_DBG(P) & 4) {
#pragma unroll
					for (int i = 0; i < 32; i++) T[i] ^= W[i];
				} else {
					asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // operands complete (see block_stage)
					__builtin_amdgcn_sched_barrier(0);
					mul_tw<FMAX>(ps.field[s], T, W, T);
					__builtin_amdgcn_sched_barrier(0);
				}
#pragma unroll
				for (int i = 0; i < 32; i += 4) {
					uint32_t A[4], Bv[4];
					*(uint4*)A = *(const uint4*)(pa + i);
					*(uint4*)Bv = *(const uint4*)(pb + i);
#pragma unroll
					for (int t = 0; t < 4; t++) {
						// u ^= w*v on the u-lanes, then v ^= u: (x & um) << d == (x << d) & ~um and
						// (x & ~um) >> d == (x >> d) & um for these lane masks
						const uint32_t a = __builtin_amdgcn_bitop3_b32(T[i + t], um, A[t], 0x6a);         // A ^ (T & um)
						const uint32_t b = __builtin_amdgcn_bitop3_b32(T[i + t] >> d, um, Bv[t], 0x6a);  // B ^ ((T >> d) & um)
						A[t] = __builtin_amdgcn_bitop3_b32(a << d, um, a, 0x9a);                          // a ^ ((a << d) & ~um)
						Bv[t] = __builtin_amdgcn_bitop3_b32(b << d, um, b, 0x9a);
					}
					*(uint4*)(pa + i) = *(const uint4*)A;
					*(uint4*)(pb + i) = *(const uint4*)Bv;
				}
			}
			// back to compact words (lane-private)
#pragma unroll
			for (int h = 0; h < 2; h++) {
				uint32_t* x = h ? pb : pa;
				uint32_t r[32];
#pragma unroll
				for (int i = 0; i < 32; i += 4) *(uint4*)(r + i) = *(const uint4*)(x + i);
				transpose32(r);
#pragma unroll
				for (int i = 0; i < 32; i += 4) *(uint4*)(x + i) = *(const uint4*)(r + i);
			}
			if (TR) {
				const unsigned long long t = ts();
				tr[2] += t - t1;
				t1 = t;
			}
		}

		// ---- store tile
		if (LAST) {
			__syncthreads();  // compact elements gather one word from every limb plane
			for (int u = tid; u < kTileBlocks * 8 * L; u += NT) {
				const int q = u / (8 * L), j = u % (8 * L);
				uint32_t w[4];
#pragma unroll
				for (int t = 0; t < 4; t++) {
					const int word = 4 * j + t;
					w[t] = lds[(word % L) * kPlane + q * kLimbStride + word / L];
				}
				if (!(BS_DBG(P) & 2)) st_stream(dst + (outer_off | tile_off(q)) * L + 4 * j, make_uint4(w[0], w[1], w[2], w[3]));
			}
		} else {
#pragma unroll 4
			for (int r = 0; r < kTileBlocks * 8 / 64; r++) {
				const int u = lane + r * 64;
				const int q = u >> 3, j = u & 7;
				const uint4 g = *(const uint4*)(plane + q * kLimbStride + 4 * j);
				if (!(BS_DBG(P) & 2)) st_stream(dst + (outer_off | tile_off(q)) * L + 32 * l + 4 * j, g);
			}
		}
		if (TR) {
			tr[3] += ts() - t1;
			tr[4] += 1;
		}
		if (!PF || !has_next) break;
		tile = next;
		outer = n_outer_v;
		outer_off = n_ooff;
		coset = n_coset;
		dst = n_dst;
		src = n_src;
	}
	if (TR && lane == 0) {
		unsigned long long* o = P.trace + ((size_t)blockIdx.x * (NT / 64) + (tid >> 6)) * 8;
		for (int i = 0; i < 8; i++) o[i] = tr[i];
	}
}

template <int L, int ROLE, int FMAX, bool PF>
__global__ __launch_bounds__(64 * L, 2) void antt_bs_pass(BsParams P) {
	bs_pass_body<L, ROLE, FMAX, PF>(P, blockIdx.x);
}

#ifdef BN_DEV
// ------------------------------------------------------------------------------------
// Experiment (development build only, BN_PERSIST3=1, EXPERIMENTS.md section 5.1): a
// three-pass plan whose passes have at most two tiles per CU (one 2^20 transform: 256 tiles each)
// as ONE launch of the variant-1 pass bodies with a grid-wide barrier between the passes instead of
// kernel boundaries. Every work-group is resident, so the barrier cannot deadlock. Measured 0.157
// ms against 0.0825 ms for the three launches (EXPERIMENTS.md section 5.1, round 5): not used.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned target) {
	__syncthreads();
	if (threadIdx.x == 0) {
		__threadfence();  // agent-scope release of this work-group's stores (other XCDs read them)
		atomicAdd(bar, 1u);
		while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
	}
	__syncthreads();
}

struct BsParams3 {
	BsParams p[3];
};
template <int F0, int F1>
__global__ __launch_bounds__(256, 2) void antt_bs_persist3(BsParams3 Q, unsigned* bar, unsigned base) {
	bs_pass_body<4, ROLE_FIRST, F0, false>(Q.p[0], blockIdx.x);
	grid_barrier(bar, base + gridDim.x);
	bs_pass_body<4, ROLE_MID, F1, false>(Q.p[1], blockIdx.x);
	grid_barrier(bar, base + 2 * gridDim.x);
	bs_pass_body<4, ROLE_LAST, 32, false>(Q.p[2], blockIdx.x);
}

static const void* persist3_kernel(int f0, int f1) {
	if (f0 <= 8) return f1 <= 8 ? (const void*)antt_bs_persist3<8, 8> : (const void*)antt_bs_persist3<8, 32>;
	return f1 <= 8 ? (const void*)antt_bs_persist3<32, 8> : (const void*)antt_bs_persist3<32, 32>;
}
#endif



// ------------------------------------------------------------------------------------
// Lane-split passes (small launches). A pass of T tiles runs 4T waves above; below two tiles per CU
// (one 2^20 transform: 256 tiles, one wave per SIMD) a lone wave issues at half the rate of two
// (DESIGN.md section 5.1). Here each GF(2^32) product of a block pair is split over two waves by the
// tower's top level (v = v0 + v1 X, w = w0 + w1 X over GF(2^16), X^2 = alpha X + 1):
//   wave half 0: (w v)|lo = v0 w0 + v1 w1                 -> words 0..15 of u and v
//   wave half 1: (w v)|hi = v0 w1 + v1 (w0 + alpha w1)    -> words 16..31
// two GF(2^16) products per wave (bsm4, 316 gates: 1264 for the pair against one 1022-gate bsm5)
// and no partial products to exchange. The tile is double-buffered in LDS (a stage reads one copy
// and writes the other), so one work-group barrier per stage orders every access. A work-group is
// 8 waves (4 limbs x 2 halves): two waves per SIMD. Same tiles, tables, HBM layouts and results as
// antt_bs_pass.
// ------------------------------------------------------------------------------------
constexpr int kSplitNT = 512;  // 8 waves
#define BS3_SB() __builtin_amdgcn_sched_barrier(0)
static size_t split_lds_bytes() { return ((size_t)8 * kPlane + (size_t)kMaxStages) * sizeof(uint32_t); }

template <int ROLE>
__global__ __launch_bounds__(kSplitNT, 1) void antt_bs3_pass(BsParams P) {
	extern __shared__ uint32_t lds[];
	constexpr int L = 4;
	constexpr bool IN_COMPACT = ROLE == ROLE_FIRST || ROLE == ROLE_SINGLE;
	constexpr bool LAST = ROLE == ROLE_LAST || ROLE == ROLE_SINGLE;
	const BsPass& ps = P.p;
	const int tid = threadIdx.x;
	const int w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
	// BN_TRACE (development build): per-wave cycles of load, block stages, in-word stages +
	// transposes, store
	const bool TR = BS_TRACE(P);
	unsigned long long tr[6] = {0, 0, 0, 0, 0, 0}, tlast = TR ? __builtin_amdgcn_s_memtime() : 0;
	auto mark = [&](int k) {
		if (!TR) return;
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		const unsigned long long t = __builtin_amdgcn_s_memtime();
		tr[k] += t - tlast;
		tlast = t;
	};
	const int l = w & 3, half = w >> 2;  // limb plane, product half
	uint32_t* const cu_w = lds + 8 * kPlane;  // workgroup-uniform twiddle part per stage
	const size_t n = (size_t)1 << P.log_h;
	auto tile_off = [&](int q) -> size_t {
		size_t off = 0;
#pragma unroll
		for (int m = 0; m < kBlkBits; m++) off |= (size_t)((q >> m) & 1) << ps.bb[m];
		return off;
	};
	const size_t tile = blockIdx.x;
	const size_t outer = tile & (((size_t)1 << ps.n_outer) - 1);
	const size_t rest = tile >> ps.n_outer;
	const int coset = (int)(rest & ((1u << P.log_rate) - 1));
	const size_t batch = rest >> P.log_rate;
	size_t ooff = 0;
	for (int m = 0; m < ps.n_outer; m++) ooff |= ((outer >> m) & 1) << ps.ob[m];
	uint32_t* dst = P.dst + (((batch << P.log_rate) + (size_t)coset) * n) * L;
	const uint32_t* src = IN_COMPACT ? (P.src + batch * n * L) : dst;

	if (tid < ps.k) {
		uint32_t c = 0;
		for (int m = 0; m < ps.n_outer; m++) c ^= ps.two[tid][m] & (0u - (uint32_t)((outer >> m) & 1));
		for (int b = 0; b < P.log_rate; b++) c ^= ps.twc[tid][b] & (0u - (uint32_t)((coset >> b) & 1));
		cu_w[tid] = c;
	}
	// ---- tile into LDS copy 0: 4096 pieces of 16 bytes, 8 per thread, all loads in flight at once
	constexpr int kRounds = (kTileBlocks * 8 * L + kSplitNT - 1) / kSplitNT;
	uint4 g[kRounds];
#pragma unroll
	for (int r = 0; r < kRounds; r++) {
		const int u = tid + r * kSplitNT;
		if (IN_COMPACT) {
			const int q = u / (8 * L), j = u % (8 * L);
			g[r] = ld_stream(src + (ooff | tile_off(q)) * L + 4 * j);
		} else {
			const int pl = u >> 10, rr = u & 1023, q = rr >> 3, j = rr & 7;  // plane, block, 16-B chunk
			g[r] = ld_stream(src + (ooff | tile_off(q)) * L + 32 * pl + 4 * j);
		}
	}
#pragma unroll
	for (int r = 0; r < kRounds; r++) {
		const int u = tid + r * kSplitNT;
		if (IN_COMPACT) {
			const int q = u / (8 * L), j = u % (8 * L);
			const uint32_t wd[4] = {g[r].x, g[r].y, g[r].z, g[r].w};
#pragma unroll
			for (int c = 0; c < 4; c++) {
				const int word = 4 * j + c;
				lds[(word % L) * kPlane + q * kLimbStride + word / L] = wd[c];
			}
		} else {
			const int pl = u >> 10, rr = u & 1023, q = rr >> 3, j = rr & 7;
			*(uint4*)(lds + pl * kPlane + q * kLimbStride + 4 * j) = g[r];
		}
	}
	__syncthreads();
	auto transpose_blocks = [&](uint32_t* base) {
		// 512 per-(block, limb) 32x32 transposes, one per thread
		uint32_t* x = base + (tid >> 7) * kPlane + (tid & 127) * kLimbStride;
		uint32_t r[32];
#pragma unroll
		for (int i = 0; i < 32; i += 4) *(uint4*)(r + i) = *(const uint4*)(x + i);
		transpose32(r);
#pragma unroll
		for (int i = 0; i < 32; i += 4) *(uint4*)(x + i) = *(const uint4*)(r + i);
	};
	if (IN_COMPACT) {
		transpose_blocks(lds);
		__syncthreads();
	}
	// the stages, instantiated per product half H (its words o = 16 H index register arrays, so they
	// must be compile-time constants); returns the LDS copy holding the tile afterwards
	auto stages = [&](auto hc) -> int {
	constexpr int H = decltype(hc)::value;
	constexpr int o = 16 * H;
	int cur = 0;
	// this wave's half of the product w v: V the 32 operand words, W0 / W1 the twiddle's low / high
	// halves as words (bit i of every bit-lane's 16-bit half in word i). Twiddles of a sub-field
	// (the stage's `field`, wave-uniform) leave W1 zero: half h is then V's half h times W0 alone
	auto half_product = [&](int field, const uint32_t* V, const uint32_t* W0, const uint32_t* W1, uint32_t* p) {
		if (field <= 8) {
			BS3_SB();
			bsm3_mul(V + o, W0, p);
			bsm3_mul(V + o + 8, W0, p + 8);
			BS3_SB();
			return;
		}
		if (field <= 16) {
			BS3_SB();
			bsm4_mul(V + o, W0, p);
			BS3_SB();
			return;
		}
		uint32_t a[16], b[16], z[16];
		if (H == 0) {
#pragma unroll
			for (int i = 0; i < 16; i++) a[i] = W0[i], b[i] = W1[i];
		} else {
			uint32_t al[16];
			quad::bs_alpha<4>(W1, al);
#pragma unroll
			for (int i = 0; i < 16; i++) a[i] = W1[i], b[i] = W0[i] ^ al[i];
		}
		BS3_SB();
		bsm4_mul(V, a, p);
		bsm4_mul(V + 16, b, z);
		BS3_SB();
#pragma unroll
		for (int i = 0; i < 16; i++) p[i] ^= z[i];
	};
	auto tile_tw = [&](int j, int q) -> uint32_t {
		uint32_t tw = 0;
#pragma unroll
		for (int m = 0; m < kBlkBits; m++) tw ^= ps.twt[j][m] & (uint32_t)__builtin_amdgcn_sbfe(q, m, 1);
		return tw;
	};

	// ---- tile-bit stages: lane = block pair of limb l, as antt_bs_pass
	const int jlow = max(LAST ? 5 : 0, ps.stop_j);
	for (int j = ps.k - 1; j >= jlow; j--) {
		const int m = ps.stage_m[j];
		const int qu = ((lane >> m) << (m + 1)) | (lane & ((1 << m) - 1));
		const int qv = qu | (1 << m);
		const uint32_t* su = lds + cur * 4 * kPlane + l * kPlane + qu * kLimbStride;
		const uint32_t* sv = lds + cur * 4 * kPlane + l * kPlane + qv * kLimbStride;
		uint32_t* du = lds + (cur ^ 1) * 4 * kPlane + l * kPlane + qu * kLimbStride;
		uint32_t* dv = lds + (cur ^ 1) * 4 * kPlane + l * kPlane + qv * kLimbStride;
		uint32_t V[32], W0[16], W1[16], pr[16];
#pragma unroll
		for (int i = 0; i < 32; i += 4) *(uint4*)(V + i) = *(const uint4*)(sv + i);
		const uint32_t wt = cu_w[j] ^ tile_tw(j, qu);
#pragma unroll
		for (int i = 0; i < 16; i++) {
			W0[i] = (uint32_t)__builtin_amdgcn_sbfe(wt, i, 1);
			W1[i] = (uint32_t)__builtin_amdgcn_sbfe(wt, 16 + i, 1);
		}
		if (TR) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); tr[4] -= __builtin_amdgcn_s_memtime(); }
		half_product(ps.field[j], V, W0, W1, pr);
		if (TR) { uint32_t acc = 0; for (int q = 0; q < 16; q++) acc ^= pr[q]; asm volatile("" ::"v"(acc)); tr[4] += __builtin_amdgcn_s_memtime(); }
#pragma unroll
		for (int i = 0; i < 16; i += 4) {
			uint4 uu = *(const uint4*)(su + o + i);
			uu.x ^= pr[i], uu.y ^= pr[i + 1], uu.z ^= pr[i + 2], uu.w ^= pr[i + 3];
			*(uint4*)(du + o + i) = uu;
			*(uint4*)(dv + o + i) = make_uint4(V[o + i] ^ uu.x, V[o + i + 1] ^ uu.y, V[o + i + 2] ^ uu.z, V[o + i + 3] ^ uu.w);
		}
		__syncthreads();
		cur ^= 1;
	}
	mark(1);

	if (LAST) {
		// ---- stages 4..0 inside the words (antt_bs_pass's packing: lane owns blocks qa = lane and
		// qb = lane + 64 of limb l; A's v-lanes move onto the u positions, B's stay)
		const int qa = lane, qb = qa | (kTileBlocks / 2);
		for (int s = 4; s >= ps.stop_j; s--) {
			const uint32_t d = vgpr(1u << s);
			const uint32_t um = vgpr(~lane_mask(s));
			const uint32_t* sa = lds + cur * 4 * kPlane + l * kPlane + qa * kLimbStride;
			const uint32_t* sb = lds + cur * 4 * kPlane + l * kPlane + qb * kLimbStride;
			uint32_t* da = lds + (cur ^ 1) * 4 * kPlane + l * kPlane + qa * kLimbStride;
			uint32_t* db = lds + (cur ^ 1) * 4 * kPlane + l * kPlane + qb * kLimbStride;
			const uint32_t cb = cu_w[s] ^ tile_tw(s, qb);
			uint32_t T[32], W0[16], W1[16], pr[16];
#pragma unroll
			for (int i = 0; i < 32; i += 4) {
				const uint4 a = *(const uint4*)(sa + i), b = *(const uint4*)(sb + i);
				T[i] = __builtin_amdgcn_bitop3_b32(a.x >> d, b.x, um, 0xe4);
				T[i + 1] = __builtin_amdgcn_bitop3_b32(a.y >> d, b.y, um, 0xe4);
				T[i + 2] = __builtin_amdgcn_bitop3_b32(a.z >> d, b.z, um, 0xe4);
				T[i + 3] = __builtin_amdgcn_bitop3_b32(a.w >> d, b.w, um, 0xe4);
			}
			// twiddle words: the bit-lane pattern plus the block part (antt_bs_pass)
#pragma unroll
			for (int i = 0; i < 16; i++) {
				W0[i] = ps.pat[s][i] ^ (uint32_t)__builtin_amdgcn_sbfe(cb, i, 1);
				W1[i] = ps.pat[s][16 + i] ^ (uint32_t)__builtin_amdgcn_sbfe(cb, 16 + i, 1);
			}
			half_product(ps.field[s], T, W0, W1, pr);
#pragma unroll
			for (int i = 0; i < 16; i += 4) {
				uint32_t A[4], Bv[4];
				*(uint4*)A = *(const uint4*)(sa + o + i);
				*(uint4*)Bv = *(const uint4*)(sb + o + i);
#pragma unroll
				for (int c = 0; c < 4; c++) {
					const uint32_t a = __builtin_amdgcn_bitop3_b32(pr[i + c], um, A[c], 0x6a);
					const uint32_t b = __builtin_amdgcn_bitop3_b32(pr[i + c] >> d, um, Bv[c], 0x6a);
					A[c] = __builtin_amdgcn_bitop3_b32(a << d, um, a, 0x9a);
					Bv[c] = __builtin_amdgcn_bitop3_b32(b << d, um, b, 0x9a);
				}
				*(uint4*)(da + o + i) = *(const uint4*)A;
				*(uint4*)(db + o + i) = *(const uint4*)Bv;
			}
			__syncthreads();
			cur ^= 1;
		}
	}
	return cur;
	};
	mark(0);
	const int cur = half == 0 ? stages(std::integral_constant<int, 0>()) : stages(std::integral_constant<int, 1>());
	mark(2);
	if (LAST) {
		// back to compact words
		uint32_t* const fin = lds + cur * 4 * kPlane;
		transpose_blocks(fin);
		__syncthreads();
		for (int u = tid; u < kTileBlocks * 8 * L; u += kSplitNT) {
			const int q = u / (8 * L), j = u % (8 * L);
			uint32_t wd[4];
#pragma unroll
			for (int c = 0; c < 4; c++) {
				const int word = 4 * j + c;
				wd[c] = fin[(word % L) * kPlane + q * kLimbStride + word / L];
			}
			if (!(BS_DBG(P) & 2)) st_stream(dst + (ooff | tile_off(q)) * L + 4 * j, make_uint4(wd[0], wd[1], wd[2], wd[3]));
		}
	} else {
		const uint32_t* const fin = lds + cur * 4 * kPlane;
		for (int u = tid; u < kTileBlocks * 8 * L; u += kSplitNT) {
			const int pl = u >> 10, r = u & 1023, q = r >> 3, j = r & 7;
			const uint4 g = *(const uint4*)(fin + pl * kPlane + q * kLimbStride + 4 * j);
			if (!(BS_DBG(P) & 2)) st_stream(dst + (ooff | tile_off(q)) * L + 32 * pl + 4 * j, g);
		}
	}
	mark(3);
	if (TR && lane == 0) {
		unsigned long long* o = P.trace + ((size_t)blockIdx.x * (kSplitNT / 64) + w) * 8;
		o[0] = tr[0], o[1] = tr[1], o[2] = tr[2], o[3] = tr[3], o[4] = 1, o[5] = tr[4], o[6] = 0, o[7] = 0;
	}
}

// ------------------------------------------------------------------------------------
// host: pass planning
// ------------------------------------------------------------------------------------
static std::vector<BsPass> plan_passes(const bn_antt_plan* plan) {
	const int log_h = plan->log_h;
	const int width = plan->width;
	auto S = [&](int s, int kk) -> uint32_t {  // s[s][kk], 0 outside the table
		if (kk < 0 || kk >= width - s) return 0u;
		return plan->s_host[(size_t)s * width + kk];
	};
	std::vector<BsPass> passes;
	auto make = [&](int lo, int k, bool bottom) {
		BsPass p{};
		p.lo = lo;
		p.k = k;
		std::vector<int> bits;
		if (bottom) {
			for (int b = 5; b < 5 + kBlkBits; b++) bits.push_back(b);
		} else {
			// stage bits plus the lowest non-word batch bits (adjacent blocks in memory)
			for (int b = 5; (int)bits.size() < kBlkBits - k; b++) bits.push_back(b);
			for (int b = lo; b < lo + k; b++) bits.push_back(b);
		}
		for (int m = 0; m < kBlkBits; m++) p.bb[m] = bits[m];
		p.n_outer = 0;
		for (int b = 5; b < log_h; b++)
			if (std::find(bits.begin(), bits.end(), b) == bits.end()) p.ob[p.n_outer++] = b;
		for (int j = 0; j < k; j++) {
			const int s = lo + j;
			// twiddle of a butterfly block = XOR of s[s][kk] over the set bits kk of
			// (coset << (log_h-1-s)) | (index >> (s+1)); index bit b contributes s[s][b-s-1]
			uint32_t acc = 0;
			for (int kk = 0; kk < width - s; kk++) acc |= S(s, kk);
			p.field[j] = acc < 256u ? 8 : acc < 65536u ? 16 : 32;
			p.stage_m[j] = -1;
			for (int m = 0; m < kBlkBits; m++) {
				if (p.bb[m] == s) p.stage_m[j] = m;
				p.twt[j][m] = S(s, p.bb[m] - s - 1);
			}
			for (int m = 0; m < p.n_outer; m++) p.two[j][m] = S(s, p.ob[m] - s - 1);
			for (int c = 0; c < plan->log_rate; c++) p.twc[j][c] = S(s, log_h - 1 - s + c);
			if (s < 5) {
				// bit-lane p of a word has index bits 0..4 = p: bits s+1..4 contribute per lane
				for (int i = 0; i < 32; i++) {
					uint32_t w = 0;
					for (int b = s + 1; b < 5; b++)
						if ((S(s, b - s - 1) >> i) & 1) w ^= lane_mask(b);
					// A's v-lanes sit on the u positions with twiddle cb ^ twt[s][6] (qa, qb differ in
					// tile bit 6 only): fold that uniform difference in
					if ((p.twt[j][kBlkBits - 1] >> i) & 1) w ^= ~lane_mask(s);
					p.pat[s][i] = w;
				}
			}
		}
		return p;
	};
	// stages of the bottom pass: all 12 of a tile by default. BN_BOTTOM_K=11 (development build,
	// VERDICT r5 item 5) moves its top block stage into the last upper pass (2^24: 7 + 6 + 11)
	int bottom_k = kMinLogH;
#ifdef BN_DEV
	if (const char* e = getenv("BN_BOTTOM_K")) bottom_k = std::max(kMinLogH - 1, std::min(kMinLogH, atoi(e)));
#endif
	if (log_h - bottom_k < 1) bottom_k = kMinLogH;
	const int rest = log_h - bottom_k;
	const int n_up = (rest + kBlkBits - 1) / kBlkBits;
	auto gf8_stage = [&](int s) {
		uint32_t acc = 0;
		for (int kk = 0; kk < width - s; kk++) acc |= S(s, kk);
		return acc < 256u;
	};
	// upper passes, executed first (highest stages first)
	int hi = log_h;
	for (int i = 0; i < n_up; i++) {
		const int remaining_up = n_up - i;
		int k = (hi - bottom_k + remaining_up - 1) / remaining_up;
#ifndef BN_UP_EVEN
		// the first pass takes every top stage whose twiddles lie in GF(2^8) (up to a tile's 7 bits,
		// as long as the later passes still fit): its register-tile kernel runs near the HBM rate with
		// VALU to spare, and each stage it takes leaves the GF(2^32) pass one stage less
		if (i == 0 && remaining_up > 1) {
			int g = 0;
			while (g < kBlkBits && hi - g - 1 >= bottom_k && gf8_stage(hi - g - 1)) g++;
			const int min_first = (hi - bottom_k) - (remaining_up - 1) * kBlkBits;  // the rest must still fit
			if (g > k && g >= min_first) k = g;
		BN_DEV_FIRST_K(k, min_first); }  // development build: BN_FIRST_K=k overrides the first pass's stage count
#endif
		passes.push_back(make(hi - k, k, false));
		hi -= k;
	}
	passes.push_back(make(0, bottom_k, true));
	for (size_t i = 0; i < passes.size(); i++) {
		const bool first = i == 0, last = i + 1 == passes.size();
		passes[i].role = first && last ? ROLE_SINGLE : first ? ROLE_FIRST : last ? ROLE_LAST : ROLE_MID;
	}
	return passes;
}

// kernel instance per (limbs, role, largest stage field); passes whose stages all use GF(2^8)
// twiddles have registers to spare for prefetching the next tile
// next-tile prefetch (BN_PF, persistent grid) is a development-build experiment: the product
// build does not instantiate those kernels
#ifdef BN_DEV
#define BS_KERNEL(R) (pf ? (const void*)antt_bs_pass<L, R, FMAX, true> : (const void*)antt_bs_pass<L, R, FMAX, false>)
#else
#define BS_KERNEL(R) ((void)pf, (const void*)antt_bs_pass<L, R, FMAX, false>)
#endif
template <int L, int FMAX>
static const void* kernel_for_f(int role, bool pf) {
	switch (role) {
		case ROLE_FIRST: return BS_KERNEL(ROLE_FIRST);
		case ROLE_MID: return BS_KERNEL(ROLE_MID);
		case ROLE_LAST: return BS_KERNEL(ROLE_LAST);
		default: return BS_KERNEL(ROLE_SINGLE);
	}
}
#undef BS_KERNEL
static const void* kernel_for(int L, int role, int fmax, bool pf) {
	if (L == 4) return fmax <= 8 ? kernel_for_f<4, 8>(role, pf) : kernel_for_f<4, 32>(role, pf);
	return fmax <= 8 ? kernel_for_f<1, 8>(role, pf) : kernel_for_f<1, 32>(role, pf);
}

static const void* split_kernel_for(int role) {
	switch (role) {
		case ROLE_FIRST: return (const void*)antt_bs3_pass<ROLE_FIRST>;
		case ROLE_MID: return (const void*)antt_bs3_pass<ROLE_MID>;
		case ROLE_LAST: return (const void*)antt_bs3_pass<ROLE_LAST>;
		default: return (const void*)antt_bs3_pass<ROLE_SINGLE>;
	}
}

int pass_fmax(const BsPass& p) {
	int f = 8;
	for (int j = 0; j < p.k; j++) f = std::max(f, p.field[j]);
	return f;
}

// tile + one word per stage and wave for the workgroup-uniform twiddle parts
static size_t lds_bytes(int L) { return ((size_t)L * kPlane + (size_t)L * kMaxStages) * sizeof(uint32_t); }

bool bs_supports(const bn_antt_plan* plan) {
	return plan->log_h >= kMinLogH && plan->log_h - 5 - kBlkBits <= kMaxOuter && plan->log_rate <= kMaxRateBits;
}

int bs_prepare(bn_antt_plan* plan) {
	for (int L : {1, 4})
		for (int role = 0; role < 4; role++)
			for (int f : {8, 32})
				for (int pf = 0; pf < 2; pf++)
					BN_HIP(hipFuncSetAttribute(kernel_for(L, role, f, pf != 0), hipFuncAttributeMaxDynamicSharedMemorySize,
					                           (int)lds_bytes(L)));
	for (int role = 0; role < 4; role++)
		BN_HIP(hipFuncSetAttribute(split_kernel_for(role), hipFuncAttributeMaxDynamicSharedMemorySize, (int)split_lds_bytes()));
#ifdef BN_DEV
	for (int f0 : {8, 32})
		for (int f1 : {8, 32})
			BN_HIP(hipFuncSetAttribute(persist3_kernel(f0, f1), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes(4)));
#endif
	int rc = rr_prepare(plan);
	if (rc != BN_OK) return rc;
	int cus = 0;
	BN_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, plan->device));
	plan->num_cus = std::max(cus, 1);
	plan->variant = 5;  // mixed: register tiles for GF(2^8)-only passes, LDS tiles for the others
	return BN_OK;
}

const BsPass* bs_passes(bn_antt_plan* plan, size_t* n_passes) {
	// the pass tables depend only on the plan: built once and cached in it
	if (plan->bs_passes.empty()) {
		const auto ps = plan_passes(plan);
		plan->bs_passes.resize(ps.size() * sizeof(BsPass));
		memcpy(plan->bs_passes.data(), ps.data(), plan->bs_passes.size());
	}
	*n_passes = plan->bs_passes.size() / sizeof(BsPass);
	return (const BsPass*)plan->bs_passes.data();
}

struct BsDevKnobs {
	int pf_mode = 0, dbg = 0, stop_stage = -1, split = -1, mid_pf = -1, rr_last = -1;
	bool persist = true, trace = false;
	size_t max_passes = ~(size_t)0;
};

static BsDevKnobs dev_knobs() {
	BsDevKnobs k;
#ifdef BN_DEV
	// development build only (make BN_DEV=1): BN_DEBUG_MAX_PASSES=n runs only the first n passes,
	// BN_DEBUG_STOP_STAGE=s runs only stages >= s, BN_DEBUG_FLAGS skips work (see BsParams::dbg),
	// BN_PF=1/2 enables next-tile prefetch for GF(2^8)-only / all passes, BN_PERSIST=0 launches
	// one workgroup per tile, BN_TRACE=1 prints per-wave phase times (cycles)
	if (const char* e = getenv("BN_DEBUG_MAX_PASSES")) k.max_passes = (size_t)atoi(e);
	if (const char* e = getenv("BN_PF")) k.pf_mode = atoi(e);
	if (const char* e = getenv("BN_PERSIST")) k.persist = atoi(e) != 0;
	if (const char* e = getenv("BN_DEBUG_FLAGS")) k.dbg = atoi(e);
	if (const char* e = getenv("BN_DEBUG_STOP_STAGE")) k.stop_stage = atoi(e);
	if (const char* e = getenv("BN_SPLIT")) k.split = atoi(e);  // 0: never lane-split, 1: always
	if (const char* e = getenv("BN_MID_PF")) k.mid_pf = atoi(e);  // 1: middle passes on antt_rr_mid_pf
	if (const char* e = getenv("BN_RR_LAST")) k.rr_last = atoi(e);  // 0: small bottom passes on LDS tiles
	k.trace = getenv("BN_TRACE") != nullptr;
#endif
	return k;
}

// GF(2^16/32) LDS-tile upper passes of fewer tiles than two per CU (one 2^20 transform) run
// lane-split (antt_bs3_pass: two waves per product, two waves per SIMD instead of one). 2^20 A/B
// (EXPERIMENTS.md section 5.1, round 4): upper GF(2^32) pass 0.0139 vs 0.0158 ms, bottom pass 0.0514 vs 0.0496 ms,
// so the bottom pass keeps one wave per limb (EXPERIMENTS.md section 5.1, round 4)
// Development build only (BN_MID_PF=1): GF(2^16/32) middle passes on antt_rr_mid_pf, the
// register-tile kernel that hides the next tile's loads. Measured slower than antt_bs_pass at 2^24
// (pass 1 0.224-0.229 vs 0.189-0.193 ms), so the product never selects it.
static bool use_mid_pf(const bn_antt_plan* plan, const BsPass& pass, size_t ntiles, const BsDevKnobs& kn) {
#ifdef BN_DEV
	if (kn.mid_pf != 1) return false;
	if (plan->variant != 5 || plan->limbs != 4 || pass.role != ROLE_MID || pass_fmax(pass) <= 8) return false;
	RtPass rt;
	if (make_rt(pass, false, &rt) != BN_OK) return false;
	return ntiles >= (size_t)8 * (size_t)plan->num_cus;
#else
	(void)plan, (void)pass, (void)ntiles, (void)kn;
	return false;
#endif
}

static bool use_split(const bn_antt_plan* plan, const BsPass& pass, size_t ntiles, const BsDevKnobs& kn) {
	if (plan->limbs != 4 || pass_fmax(pass) <= 8) return false;
	if (kn.split >= 0) return kn.split != 0;
	if (pass.role == ROLE_LAST || pass.role == ROLE_SINGLE) return false;
	return ntiles < (size_t)2 * (size_t)plan->num_cus;
}

// Bottom pass of a small launch (fewer tiles than two per CU: one wave per SIMD either way) on
// register tiles, compiled without the three-waves bound (antt_rr.hip small_last): C3 (one 2^20
// transform) 0.0800-0.0802 vs 0.0822-0.0824 ms on LDS tiles (round 5, EXPERIMENTS.md section 5.1).
// BN_RR_LAST=0 (development build) keeps it on LDS tiles.
static bool use_rr_last(const bn_antt_plan* plan, const BsPass& pass, size_t ntiles, const BsDevKnobs& kn) {
	if (kn.rr_last == 0 || plan->variant != 5 || plan->limbs != 4 || pass.role != ROLE_LAST) return false;
	return ntiles < (size_t)2 * (size_t)plan->num_cus;
}

static int launch_one(bn_antt_plan* plan, const BsPass& pass, int i, const uint32_t* d_in, uint32_t* d_out,
                      size_t batch, hipStream_t st, const BsDevKnobs& kn) {
	// variant 4: every pass on register tiles; variant 5 (mixed): register tiles for the passes whose
	// twiddles all lie in GF(2^8) (their kernel fits four waves per SIMD), LDS tiles for the others
	if (plan->variant == 4 || (plan->variant == 5 && pass_fmax(pass) <= 8)) return rr_launch_pass(plan, i, d_in, d_out, batch, st);
	if (use_rr_last(plan, pass, (batch << plan->log_rate) << pass.n_outer, kn)) return rr_launch_pass(plan, i, d_in, d_out, batch, st);
	const int L = plan->limbs;
	BsParams prm;
	prm.src = d_in;
	prm.dst = d_out;
	prm.log_h = plan->log_h;
	prm.log_rate = plan->log_rate;
	prm.dbg = kn.dbg;
	prm.p = pass;
	prm.p.stop_j = kn.stop_stage < 0 ? 0 : std::max(0, std::min(prm.p.k, kn.stop_stage - prm.p.lo));
	const size_t ntiles = (batch << plan->log_rate) << pass.n_outer;
#ifdef BN_DEV
	if (use_mid_pf(plan, pass, ntiles, kn)) return rr_launch_mid_pf(plan, i, d_in, d_out, batch, st);
#endif
	if (use_split(plan, pass, ntiles, kn)) {
		prm.ntiles = ntiles;
		prm.trace = nullptr;
		static unsigned long long* strbuf = nullptr;
		if (kn.trace) {
			if (!strbuf) BN_HIP(hipMalloc(&strbuf, (size_t)1 << 26));
			BN_HIP(hipMemset(strbuf, 0, ntiles * 8 * 8 * 8));
			prm.trace = strbuf;
		}
		int rc = timing_begin(plan, i, st);
		if (rc != BN_OK) return rc;
		void* args[] = {&prm};
		BN_HIP(hipLaunchKernel(split_kernel_for(pass.role), dim3((unsigned)ntiles), dim3(kSplitNT), args, split_lds_bytes(), st));
		rc = timing_end(plan, i, st);
		if (rc != BN_OK || !prm.trace) return rc;
		std::vector<unsigned long long> h(ntiles * 8 * 8);
		BN_HIP(hipStreamSynchronize(st));
		BN_HIP(hipMemcpy(h.data(), prm.trace, h.size() * 8, hipMemcpyDeviceToHost));
		double acc[6] = {0};
		for (size_t wv = 0; wv < ntiles * 8; wv++)
			for (int k = 0; k < 6; k++) acc[k] += (double)h[wv * 8 + k];
		const double t = acc[4] > 0 ? acc[4] : 1;
		fprintf(stderr, "trace pass %d (split, %zu waves, cycles per wave): load %.0f  block %.0f [mul %.0f]  inword+tr %.0f  store %.0f\n", i,
		        (size_t)acc[4], acc[0] / t, acc[1] / t, acc[5] / t, acc[2] / t, acc[3] / t);
		return BN_OK;
	}
	// two 74-KB tiles per CU: a persistent grid of two workgroups per CU walks all tiles
	const int fmax = pass_fmax(pass);
	const bool pf = kn.persist && (kn.pf_mode == 2 || (kn.pf_mode == 1 && fmax <= 8));
	const size_t grid = pf ? std::min(ntiles, (size_t)2 * (size_t)plan->num_cus) : ntiles;
	prm.ntiles = ntiles;
	prm.trace = nullptr;
	static unsigned long long* trbuf = nullptr;
	if (kn.trace) {
		if (!trbuf) BN_HIP(hipMalloc(&trbuf, (size_t)1 << 26));
		BN_HIP(hipMemset(trbuf, 0, grid * L * 8 * 8));
		prm.trace = trbuf;
	}
	int rc = timing_begin(plan, i, st);
	if (rc != BN_OK) return rc;
	void* args[] = {&prm};
	BN_HIP(hipLaunchKernel(kernel_for(L, pass.role, fmax, pf), dim3((unsigned)grid), dim3(64 * L), args, lds_bytes(L), st));
	rc = timing_end(plan, i, st);
	if (rc != BN_OK) return rc;
	if (prm.trace) {
		const size_t g = grid * (size_t)L;
		std::vector<unsigned long long> h(g * 8);
		BN_HIP(hipStreamSynchronize(st));
		BN_HIP(hipMemcpy(h.data(), prm.trace, g * 8 * 8, hipMemcpyDeviceToHost));
		double acc[8] = {0};
		for (size_t w = 0; w < g; w++)
			for (int k = 0; k < 8; k++) acc[k] += (double)h[w * 8 + k];
		const double t = acc[4] > 0 ? acc[4] : 1;  // wave-tiles
		fprintf(stderr,
		        "trace pass %d (fmax %d pf %d, %zu wave-tiles, cycles per wave-tile): load %.0f  block %.0f [pre %.0f mul %.0f post %.0f]  inword+tr %.0f  store %.0f\n",
		        i, fmax, (int)pf, (size_t)acc[4], acc[0] / t, acc[1] / t, acc[5] / t, acc[6] / t, acc[7] / t, acc[2] / t, acc[3] / t);
	}
	return BN_OK;
}

// the kernel pass i launches under the plan's variant (variants 1, 4, 5), nullptr otherwise
const void* bs_pass_kernel(bn_antt_plan* plan, int i) {
	size_t n_passes = 0;
	const BsPass* passes = bs_passes(plan, &n_passes);
	if (i < 0 || (size_t)i >= n_passes) return nullptr;
	const BsPass& pass = passes[i];
	const int fmax = pass_fmax(pass);
	if (plan->variant == 4 || (plan->variant == 5 && fmax <= 8)) return rr_pass_kernel(plan, pass);
	if (plan->variant != 1 && plan->variant != 5) return nullptr;
	const BsDevKnobs kn = dev_knobs();
	// the kernel for ONE transform (bench / profiles): a batched launch of the same pass may pick
	// another (the lane-split and prefetching kernels depend on the tile count)
	const size_t ntiles = ((size_t)1 << plan->log_rate) << pass.n_outer;
#ifdef BN_DEV
	if (use_mid_pf(plan, pass, ntiles, kn)) return rr_mid_pf_kernel(pass);
#endif
	if (use_rr_last(plan, pass, ntiles, kn)) return rr_pass_kernel(plan, pass);
	if (use_split(plan, pass, ntiles, kn)) return split_kernel_for(pass.role);
	const bool pf = kn.persist && (kn.pf_mode == 2 || (kn.pf_mode == 1 && fmax <= 8));
	return kernel_for(plan->limbs, pass.role, fmax, pf);
}


#ifdef BN_DEV
static int launch_persist3(bn_antt_plan* plan, const BsPass* passes, const uint32_t* d_in, uint32_t* d_out, size_t batch,
                           hipStream_t st) {
	static unsigned* d_bar = nullptr;
	static unsigned gen = 0;
	if (!d_bar) {
		BN_HIP(hipMalloc(&d_bar, sizeof(unsigned)));
		BN_HIP(hipMemset(d_bar, 0, sizeof(unsigned)));
	}
	BsParams3 q;
	memset(&q, 0, sizeof q);
	size_t ntiles = 0;
	for (int i = 0; i < 3; i++) {
		q.p[i].src = d_in;
		q.p[i].dst = d_out;
		q.p[i].log_h = plan->log_h;
		q.p[i].log_rate = plan->log_rate;
		q.p[i].p = passes[i];
		ntiles = (batch << plan->log_rate) << passes[i].n_outer;
		q.p[i].ntiles = ntiles;
	}
	unsigned base = gen * 2u * (unsigned)ntiles;
	gen++;
	int rc = timing_begin(plan, 0, st);
	if (rc != BN_OK) return rc;
	void* args[] = {&q, &d_bar, &base};
	BN_HIP(hipLaunchKernel(persist3_kernel(pass_fmax(passes[0]), pass_fmax(passes[1])), dim3((unsigned)ntiles), dim3(256), args,
	                       lds_bytes(4), st));
	return timing_end(plan, 0, st);
}
#endif

int launch_bs(bn_antt_plan* plan, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st) {
	size_t n_passes = 0;
	const BsPass* passes = bs_passes(plan, &n_passes);
	const BsDevKnobs kn = dev_knobs();
#ifdef BN_DEV
	if (getenv("BN_PERSIST3") && n_passes == 3 && plan->limbs == 4) {
		bool ok = true;
		for (int i = 0; i < 3; i++) ok = ok && ((batch << plan->log_rate) << passes[i].n_outer) <= (size_t)2 * (size_t)plan->num_cus;
		if (ok) return launch_persist3(plan, passes, d_in, d_out, batch, st);
	}
#endif
	const size_t npass = std::min(n_passes, kn.max_passes);
	for (size_t i = 0; i < npass; i++) {
		int rc = launch_one(plan, passes[i], (int)i, d_in, d_out, batch, st, kn);
		if (rc != BN_OK) return rc;
	}
	return BN_OK;
}

// lane bits that lane coordinate c_k depends on
static const int kCoordDeps[6][2] = {{0, 2}, {1, 2}, {2, -1}, {3, -1}, {4, -1}, {5, -1}};

int make_rt(const BsPass& p, bool bottom, RtPass* out) {
	RtPass r;
	memset(&r, 0, sizeof r);
	r.lo = p.lo;
	r.k = p.k;
	r.role = p.role;
	r.n_outer = p.n_outer;
	memcpy(r.bb, p.bb, sizeof r.bb);
	memcpy(r.ob, p.ob, sizeof r.ob);
	memcpy(r.two, p.two, sizeof r.two);
	memcpy(r.twc, p.twc, sizeof r.twc);
	for (int m = 0; m < kBlkBits; m++) r.jm[m] = -1;
	for (int j = 0; j < p.k; j++)
		if (p.stage_m[j] >= 0) {
			r.jm[p.stage_m[j]] = j;
			r.field_m[p.stage_m[j]] = p.field[j];
		}
	r.mlow = kBlkBits;
	for (int m = 0; m < kBlkBits; m++)
		if (r.jm[m] >= 0) r.mlow = std::min(r.mlow, m);
	// the stage bits must be the top tile bits (stages run from tile bit 6 down)
	for (int m = r.mlow; m < kBlkBits; m++)
		if (r.jm[m] < 0) return BN_ERR_UNSUPPORTED;
	if (bottom && r.mlow != 0) return BN_ERR_UNSUPPORTED;
	auto add_coords = [&](uint32_t* tau, int kmin, const uint32_t* twt) {
		for (int k = kmin; k < 6; k++)
			for (int b : kCoordDeps[k])
				if (b >= 0) tau[b] ^= twt[k + 1];
	};
	for (int m = r.mlow; m < kBlkBits; m++) add_coords(r.tau[m], m, p.twt[r.jm[m]]);
	if (bottom) {
		for (int s = 0; s < 5; s++) {
			const int j = s - p.lo;
			r.field_s[s] = p.field[j];
			r.cb_const[s] = p.twt[j][0];
			add_coords(r.tau_iw[s], 0, p.twt[j]);
			for (int i = 0; i < 32; i++) {
				// p.pat folds the variant-1 block difference (tile bit 6); fold tile bit 0 instead
				uint32_t v = p.pat[s][i];
				if ((p.twt[j][kBlkBits - 1] >> i) & 1) v ^= ~lane_mask(s);
				if ((p.twt[j][0] >> i) & 1) v ^= ~lane_mask(s);
				r.pat[s][i] = v;
			}
		}
	}
	*out = r;
	return BN_OK;
}

// Profiling: each pass launched `reps` times back to back between two hipEvents on `st`
// (steady-state duration per launch, no event between launches). The output buffer holds
// no meaningful values afterwards (passes are re-applied to their own output); the cost of a
// pass does not depend on the values (bitwise arithmetic, no data-dependent control flow).
int bs_time_passes(bn_antt_plan* plan, const uint32_t* d_in, uint32_t* d_out, size_t batch, int reps,
                   hipStream_t st, float* ms, int max_passes, int* n_out) {
	size_t n_passes = 0;
	const BsPass* passes = bs_passes(plan, &n_passes);
	BsDevKnobs kn = dev_knobs();
	kn.trace = false;
	const int saved = plan->timing;
	plan->timing = 0;
	hipEvent_t e0 = nullptr, e1 = nullptr;
	int rc = BN_OK;
	if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) rc = BN_ERR_HIP;
	for (size_t i = 0; rc == BN_OK && i < n_passes; i++) {
		// one untimed launch first: the pass's input is then the steady-state layout
		rc = launch_one(plan, passes[i], (int)i, d_in, d_out, batch, st, kn);
		if (rc == BN_OK && hipEventRecord(e0, st) != hipSuccess) rc = BN_ERR_HIP;
		for (int r = 0; rc == BN_OK && r < reps; r++) rc = launch_one(plan, passes[i], (int)i, d_in, d_out, batch, st, kn);
		if (rc == BN_OK && hipEventRecord(e1, st) != hipSuccess) rc = BN_ERR_HIP;
		float t = 0.f;
		if (rc == BN_OK && (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&t, e0, e1) != hipSuccess))
			rc = BN_ERR_HIP;
		if (rc == BN_OK && (int)i < max_passes) ms[i] = t / (float)reps;
	}
	if (e0) (void)hipEventDestroy(e0);
	if (e1) (void)hipEventDestroy(e1);
	plan->timing = saved;
	if (rc != BN_OK) BN_FAIL(rc, "timing the passes failed");
	*n_out = (int)n_passes;
	return BN_OK;
}

}  // namespace bn
