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
#include <vector>

#include "antt_plan.hpp"
#include "bitsliced.hpp"

namespace bn {

constexpr int kBlkBits = 7;
constexpr int kTileBlocks = 1 << kBlkBits;
constexpr int kLimbStride = 36;  // LDS words per (block, limb): 32 + 4 pad (bank spread)
constexpr int kMinLogH = kBlkBits + 5;
constexpr int kMaxStages = kBlkBits + 5;  // stages per pass
constexpr int kMaxOuter = 32 - 5 - kBlkBits;
constexpr int kMaxRateBits = 8;

enum { ROLE_FIRST = 0, ROLE_MID = 1, ROLE_LAST = 2, ROLE_SINGLE = 3 };

// One pass = k consecutive stages lo..lo+k-1 over every tile. Passed by value as a kernel
// argument (~2.6 KB), so every table read is a scalar load from the kernarg segment.
struct BsPass {
	int lo, k, role, n_outer, stop_j;
	int bb[kBlkBits];                        // index bit of tile block bit m
	int ob[kMaxOuter];                       // fixed (outer) index bits, ascending
	int stage_m[kMaxStages];                 // tile bit of stage lo + j (stages >= 5)
	int field[kMaxStages];                   // 8/16/32: sub-field holding every twiddle of the stage
	uint32_t twt[kMaxStages][kBlkBits];      // twiddle contribution of tile block bit m
	uint32_t two[kMaxStages][kMaxOuter];     // ... of outer bit m
	uint32_t twc[kMaxStages][kMaxRateBits];  // ... of coset bit c
	uint32_t pat[5][32];                     // stages 0..4: bit-lane part of the twiddle words
};

struct BsParams {
	const uint32_t* src;
	uint32_t* dst;
	int log_h, log_rate;
	int dbg;  // timing experiments only (BN_DEBUG_FLAGS): 1 no loads, 2 no stores, 4 no multiplies,
	          // 8 no stage barriers, 16 no in-word stages, 32 no tile-bit stages
	BsPass p;
};

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
// lane's twiddle in word i; `field` (uniform per stage) selects the sub-field circuit.
__device__ __forceinline__ void mul_tw(int field, const uint32_t* x, const uint32_t* W, uint32_t* out) {
	if (field <= 8) {
#pragma unroll
		for (int g = 0; g < 4; g++) bsm3_mul(x + 8 * g, W, out + 8 * g);
	} else if (field <= 16) {
#pragma unroll
		for (int g = 0; g < 2; g++) bsm4_mul(x + 16 * g, W, out + 16 * g);
	} else {
		bsm5_mul(x, W, out);
	}
}

template <int L, int ROLE>
__global__ __launch_bounds__(64 * L, 2) void antt_bs_pass(BsParams P) {
	extern __shared__ uint32_t lds[];
	constexpr int BLK_WORDS = L * kLimbStride;
	constexpr int NT = 64 * L;
	constexpr bool IN_COMPACT = ROLE == ROLE_FIRST || ROLE == ROLE_SINGLE;
	constexpr bool LAST = ROLE == ROLE_LAST || ROLE == ROLE_SINGLE;  // bottom pass, compact out
	uint32_t* cu_lds = lds + kTileBlocks * BLK_WORDS;                // workgroup part of each twiddle
	const BsPass& ps = P.p;
	const int tid = threadIdx.x;
	const size_t n = (size_t)1 << P.log_h;

	// ---- workgroup -> (batch, coset, outer bits)
	const size_t bid = blockIdx.x;
	const size_t outer = bid & (((size_t)1 << ps.n_outer) - 1);
	const size_t rest = bid >> ps.n_outer;
	const int coset = (int)(rest & ((1u << P.log_rate) - 1));
	const size_t batch = rest >> P.log_rate;
	size_t outer_off = 0;
	for (int m = 0; m < ps.n_outer; m++) outer_off |= ((outer >> m) & 1) << ps.ob[m];
	auto tile_off = [&](int q) -> size_t {
		size_t off = 0;
#pragma unroll
		for (int m = 0; m < kBlkBits; m++) off |= (size_t)((q >> m) & 1) << ps.bb[m];
		return off;
	};
	uint32_t* dst = P.dst + (((batch << P.log_rate) + (size_t)coset) * n) * L;
	const uint32_t* src = IN_COMPACT ? (P.src + batch * n * L) : dst;

	// ---- load tile into LDS (coalesced 16-byte loads, all issued before the first LDS write;
	//      compact input is split by limb)
	constexpr int LOADS = kTileBlocks * 8 * L / NT;
	uint4 gbuf[LOADS];
#pragma unroll
	for (int r = 0; r < LOADS; r++) {
		const int u = tid + r * NT;
		const int q = u / (8 * L), j = u % (8 * L);
		if (P.dbg & 1)
			gbuf[r] = make_uint4(u, j, q, tid);
		else
			gbuf[r] = ld_stream(src + (outer_off | tile_off(q)) * L + 4 * j);
	}
	// workgroup-uniform twiddle part of every stage (outer + coset bits), one lane per stage
	if (tid < ps.k) {
		uint32_t c = 0;
		for (int m = 0; m < ps.n_outer; m++) c ^= ps.two[tid][m] & (0u - (uint32_t)((outer >> m) & 1));
		for (int b = 0; b < P.log_rate; b++) c ^= ps.twc[tid][b] & (0u - (uint32_t)((coset >> b) & 1));
		cu_lds[tid] = c;
	}
#pragma unroll
	for (int r = 0; r < LOADS; r++) {
		const int u = tid + r * NT;
		const int q = u / (8 * L), j = u % (8 * L);
		const uint4 g = gbuf[r];
		uint32_t* b = lds + q * BLK_WORDS;
		if (IN_COMPACT) {
			const uint32_t w[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
			for (int t = 0; t < 4; t++) {
				const int word = 4 * j + t;
				b[(word % L) * kLimbStride + word / L] = w[t];
			}
		} else {
			const int l = (4 * j) / 32, i = (4 * j) % 32;
			*(uint4*)(b + l * kLimbStride + i) = g;
		}
	}
	__syncthreads();
	if (IN_COMPACT) {
		for (int u = tid; u < kTileBlocks * L; u += NT) {
			uint32_t* x = lds + (u / L) * BLK_WORDS + (u % L) * kLimbStride;
			uint32_t r[32];
#pragma unroll
			for (int i = 0; i < 32; i += 4) *(uint4*)(r + i) = *(const uint4*)(x + i);
			transpose32(r);
#pragma unroll
			for (int i = 0; i < 32; i += 4) *(uint4*)(x + i) = *(const uint4*)(r + i);
		}
		__syncthreads();
	}

	const int l = tid % L;
	auto tile_tw = [&](int j, int q) -> uint32_t {
		uint32_t w = 0;
#pragma unroll
		for (int m = 0; m < kBlkBits; m++) w ^= ps.twt[j][m] & (0u - (uint32_t)((q >> m) & 1));
		return w;
	};

	// ---- tile-bit stages (index bits >= 5), high to low, through LDS. One thread per
	// (block pair, limb); only V and the twiddle are live during the multiply. Consecutive lanes
	// take consecutive pairs, which keeps the padded LDS rows free of bank conflicts.
	auto block_stage = [&](int j, int pair) {
		const int m = ps.stage_m[j];
		const int qu = ((pair >> m) << (m + 1)) | (pair & ((1 << m) - 1));
		const int qv = qu | (1 << m);
		const uint32_t w = cu_lds[j] ^ tile_tw(j, qu);
		uint32_t* pu = lds + qu * BLK_WORDS + l * kLimbStride;
		uint32_t* pv = lds + qv * BLK_WORDS + l * kLimbStride;
		if constexpr (LAST) {
			// bottom pass: both rows requested up front (measured faster here; in the upper passes
			// the extra live row costs more than the hidden latency)
			uint32_t W[32], V[32], U[32], Pr[32];
#pragma unroll
			for (int i = 0; i < 32; i += 4) {
				*(uint4*)(V + i) = *(const uint4*)(pv + i);
				*(uint4*)(U + i) = *(const uint4*)(pu + i);
			}
#pragma unroll
			for (int i = 0; i < 32; i++) W[i] = 0u - ((w >> i) & 1u);
			__builtin_amdgcn_sched_barrier(0);
			if (P.dbg & 4) {
#pragma unroll
				for (int i = 0; i < 32; i++) Pr[i] = V[i] ^ W[i];
			} else {
				mul_tw(ps.field[j], V, W, Pr);  // sub-field circuits reuse W: Pr must not alias it
			}
			__builtin_amdgcn_sched_barrier(0);
#pragma unroll
			for (int i = 0; i < 32; i += 4) {
				const uint4 u = make_uint4(U[i] ^ Pr[i], U[i + 1] ^ Pr[i + 1], U[i + 2] ^ Pr[i + 2], U[i + 3] ^ Pr[i + 3]);
				*(uint4*)(pu + i) = u;
				*(uint4*)(pv + i) = make_uint4(V[i] ^ u.x, V[i + 1] ^ u.y, V[i + 2] ^ u.z, V[i + 3] ^ u.w);
			}
		} else {
			// only V and the twiddle are live during the multiply; U is read afterwards
			uint32_t W[32], V[32], Pr[32];
#pragma unroll
			for (int i = 0; i < 32; i++) W[i] = 0u - ((w >> i) & 1u);
#pragma unroll
			for (int i = 0; i < 32; i += 4) *(uint4*)(V + i) = *(const uint4*)(pv + i);
			if (P.dbg & 4) {
#pragma unroll
				for (int i = 0; i < 32; i++) Pr[i] = V[i] ^ W[i];
			} else {
				mul_tw(ps.field[j], V, W, Pr);  // sub-field circuits reuse W: Pr must not alias it
			}
#pragma unroll
			for (int i = 0; i < 32; i += 4) {
				uint4 u = *(const uint4*)(pu + i);
				u.x ^= Pr[i];
				u.y ^= Pr[i + 1];
				u.z ^= Pr[i + 2];
				u.w ^= Pr[i + 3];
				*(uint4*)(pu + i) = u;
				*(uint4*)(pv + i) = make_uint4(V[i] ^ u.x, V[i + 1] ^ u.y, V[i + 2] ^ u.z, V[i + 3] ^ u.w);
			}
		}
	};
	const int jlow = max(LAST ? 5 : 0, ps.stop_j);
	for (int j = ps.k - 1; j >= jlow; j--) {
		if (!(P.dbg & 32)) block_stage(j, tid / L);
		if (!(P.dbg & 8)) __syncthreads();
	}

	if (LAST) {
		// ---- stages 4..0 (index bits inside the word), thread-private: thread (pair, limb)
		// owns blocks qa = pair and qb = pair + 64 for all of them, so no barriers. Per stage
		// both blocks share one multiply: A's v-lanes move down onto the u positions, B's
		// v-lanes stay on the v positions (a pair's twiddle depends only on index bits above s).
		const int qa = tid / L, qb = qa | (kTileBlocks / 2);
		uint32_t* pa = lds + qa * BLK_WORDS + l * kLimbStride;
		uint32_t* pb = lds + qb * BLK_WORDS + l * kLimbStride;
		for (int s = 4; s >= ((P.dbg & 16) ? 5 : ps.stop_j); s--) {  // bottom pass starts at stage 0: j == s
			{
				const int d = 1 << s;
				const uint32_t um = ~lane_mask(s);
				const uint32_t ca = cu_lds[s] ^ tile_tw(s, qa), cb = cu_lds[s] ^ tile_tw(s, qb);
				uint32_t W[32], T[32];
#pragma unroll
				for (int i = 0; i < 32; i += 4) {
					const uint4 a = *(const uint4*)(pa + i), b = *(const uint4*)(pb + i);
					T[i] = ((a.x >> d) & um) | (b.x & ~um);
					T[i + 1] = ((a.y >> d) & um) | (b.y & ~um);
					T[i + 2] = ((a.z >> d) & um) | (b.z & ~um);
					T[i + 3] = ((a.w >> d) & um) | (b.w & ~um);
				}
#pragma unroll
				for (int i = 0; i < 32; i++)
					W[i] = ps.pat[s][i] ^ ((0u - ((ca >> i) & 1u)) & um) ^ ((0u - ((cb >> i) & 1u)) & ~um);
				if (P.dbg & 4) {
#pragma unroll
					for (int i = 0; i < 32; i++) T[i] ^= W[i];
				} else {
					mul_tw(ps.field[s], T, W, T);
				}
#pragma unroll
				for (int i = 0; i < 32; i += 4) {
					uint32_t A[4], Bv[4];
					*(uint4*)A = *(const uint4*)(pa + i);
					*(uint4*)Bv = *(const uint4*)(pb + i);
#pragma unroll
					for (int t = 0; t < 4; t++) {
						A[t] ^= T[i + t] & um;
						Bv[t] ^= (T[i + t] & ~um) >> d;
						A[t] ^= (A[t] & um) << d;
						Bv[t] ^= (Bv[t] & um) << d;
					}
					*(uint4*)(pa + i) = *(const uint4*)A;
					*(uint4*)(pb + i) = *(const uint4*)Bv;
				}
			}
		}
		// back to compact (limb-split) words, still thread-private
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
	}
	__syncthreads();

	// ---- store tile
	for (int u = tid; u < kTileBlocks * 8 * L; u += NT) {
		const int q = u / (8 * L), j = u % (8 * L);
		const uint32_t* b = lds + q * BLK_WORDS;
		uint4 g;
		if (LAST) {
			uint32_t w[4];
#pragma unroll
			for (int t = 0; t < 4; t++) {
				const int word = 4 * j + t;
				w[t] = b[(word % L) * kLimbStride + word / L];
			}
			g = make_uint4(w[0], w[1], w[2], w[3]);
		} else {
			const int li = (4 * j) / 32, i = (4 * j) % 32;
			g = *(const uint4*)(b + li * kLimbStride + i);
		}
		if (!(P.dbg & 2)) st_stream(dst + (outer_off | tile_off(q)) * L + 4 * j, g);
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
					p.pat[s][i] = w;
				}
			}
		}
		return p;
	};
	const int rest = log_h - kMinLogH;
	const int n_up = (rest + kBlkBits - 1) / kBlkBits;
	// upper passes, executed first (highest stages first)
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

template <int L>
static const void* kernel_for(int role) {
	switch (role) {
		case ROLE_FIRST: return (const void*)antt_bs_pass<L, ROLE_FIRST>;
		case ROLE_MID: return (const void*)antt_bs_pass<L, ROLE_MID>;
		case ROLE_LAST: return (const void*)antt_bs_pass<L, ROLE_LAST>;
		default: return (const void*)antt_bs_pass<L, ROLE_SINGLE>;
	}
}

// tile + one word per stage for the workgroup-uniform twiddle parts
static size_t lds_bytes(int L) { return ((size_t)kTileBlocks * L * kLimbStride + kMaxStages) * sizeof(uint32_t); }

bool bs_supports(const bn_antt_plan* plan) {
	return plan->log_h >= kMinLogH && plan->log_h - 5 - kBlkBits <= kMaxOuter && plan->log_rate <= kMaxRateBits;
}

int bs_prepare(bn_antt_plan* plan) {
	for (int role = 0; role < 4; role++) {
		BN_HIP(hipFuncSetAttribute(kernel_for<4>(role), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes(4)));
		BN_HIP(hipFuncSetAttribute(kernel_for<1>(role), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes(1)));
	}
	plan->variant = 1;
	return BN_OK;
}

int launch_bs(bn_antt_plan* plan, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st) {
	const auto passes = plan_passes(plan);
	const int L = plan->limbs;
	// debug hooks: BN_DEBUG_MAX_PASSES=n runs only the first n passes,
	// BN_DEBUG_STOP_STAGE=s runs only stages >= s
	size_t npass = passes.size();
	if (const char* e = getenv("BN_DEBUG_MAX_PASSES")) npass = std::min(npass, (size_t)atoi(e));
	for (size_t i = 0; i < npass; i++) {
		BsParams prm;
		prm.src = d_in;
		prm.dst = d_out;
		prm.log_h = plan->log_h;
		prm.log_rate = plan->log_rate;
		prm.dbg = 0;
		if (const char* e = getenv("BN_DEBUG_FLAGS")) prm.dbg = atoi(e);
		prm.p = passes[i];
		prm.p.stop_j = 0;
		if (const char* e = getenv("BN_DEBUG_STOP_STAGE"))
			prm.p.stop_j = std::max(0, std::min(prm.p.k, atoi(e) - prm.p.lo));
		const size_t grid = (batch << plan->log_rate) << passes[i].n_outer;
		int rc = timing_begin(plan, (int)i, st);
		if (rc != BN_OK) return rc;
		void* args[] = {&prm};
		const void* fn = L == 4 ? kernel_for<4>(passes[i].role) : kernel_for<1>(passes[i].role);
		BN_HIP(hipLaunchKernel(fn, dim3((unsigned)grid), dim3(64 * L), args, lds_bytes(L), st));
		rc = timing_end(plan, (int)i, st);
		if (rc != BN_OK) return rc;
	}
	return BN_OK;
}

}  // namespace bn
