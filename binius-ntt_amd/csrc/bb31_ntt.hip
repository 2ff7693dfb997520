// BabyBear (p = 15 * 2^27 + 1) NTT for gfx950: the prime-field sibling of the additive NTT
// (SURVEY.md §8f row 4). Replaces NTT<BB31> of the reference (src/ulvt/ntt/gpuntt.cuh:126-209):
// the reference bit-reverses the input and runs log_n radix-2 stages with bit-reversed
// twiddles, 11 stages per launch; its output is the natural-order DFT
//     X[k] = sum_j x[j] w^(j k),   w = g^(2^(log_group - log_n))
// (checked against the oracle and the reference's MD5 table, tests/golden/bb31_ntt_md5.json).
//
// MI355X design: a mixed-radix "four-step" decomposition with natural order in and out, so
// there is no bit-reversal pass at all. log_n = m_1 + ... + m_L bits (m_i <= 9, L = 1 for
// log_n <= 13). Pass p views the current sub-problem of size M_{p-1} = 2^{m_p} * M_p as
// rows j_p (stride M_p) x columns (the lower digits, contiguous):
//     Y[k_p][c] = DFT_{2^{m_p}} over j_p of Z[j_p][c],   then  Y[k_p][c] *= w_{M_{p-1}}^(c k_p)
// and stores Y in place (row k_p). The last pass takes 32 consecutive k_1 per tile, so both its
// reads (runs of 2^{m_L}) and its writes of the natural-order output X[k_1 + N_1 k_2 + ...]
// (runs of 32 k_1) are coalesced. A tile (2^{m_p} rows x 32 columns, <= 64 KiB) is one
// workgroup; its DFT runs as radix-2 DIF stages in LDS. Values are canonical u32 (< p) in HBM;
// products are Montgomery multiplications by Montgomery-encoded twiddles (risc0_baby_bear.h
// mul, lines 172-180, so w * R is stored). A bit-reversed input (DataOrder::BIT_REVERSED) is
// read through the first pass's addressing: the reads stay runs of 2^{m_1} words.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "common.hpp"

struct bn_bb31_ntt_plan {
	int device = 0;
	int log_n = 0, log_group = 0;
	uint32_t generator = 0;  // canonical
	int L = 0;
	int m[4] = {0, 0, 0, 0};
	uint32_t* wtab = nullptr;  // Montgomery-encoded w^e: lo table [4096] then hi table [2^(log_n-12)] (or one table)
	uint32_t* scratch = nullptr;
	size_t scratch_words = 0;
	hipStream_t own_stream = nullptr;
	uint32_t* h_dev = nullptr;  // host-apply staging (in, out)
};

namespace bn {
namespace {

constexpr uint32_t kP = 2013265921u;    // 15 * 2^27 + 1
constexpr uint32_t kPinv = 0x88000001u;  // p^-1 mod 2^32 (risc0::Fp::M)
constexpr uint32_t kR2 = 1172168163u;    // 2^64 mod p (risc0::Fp::R2)
constexpr int kCols = 32;
constexpr int kMaxM = 9;
constexpr int kThreads = 256;
constexpr int kLoBits = 12;

__host__ __device__ inline uint32_t mont(uint32_t a, uint32_t b) {
	uint64_t o = (uint64_t)a * b;
	const uint32_t red = (0u - (uint32_t)o) * kPinv;
	o += (uint64_t)red * kP;
	const uint32_t r = (uint32_t)(o >> 32);
	return r >= kP ? r - kP : r;
}
__host__ __device__ inline uint32_t bb_add(uint32_t a, uint32_t b) {
	const uint32_t r = a + b;
	return r >= kP ? r - kP : r;
}
__host__ __device__ inline uint32_t bb_sub(uint32_t a, uint32_t b) { return a >= b ? a - b : a + kP - b; }
__host__ __device__ inline uint32_t bb_reduce(uint32_t x) {  // any u32 -> canonical (BB31(r) == r mod p)
	x = x >= kP ? x - kP : x;
	return x >= kP ? x - kP : x;
}
static uint32_t h_mul(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) % kP); }
static uint32_t h_pow(uint32_t x, uint64_t e) {
	uint32_t r = 1;
	while (e) {
		if (e & 1) r = h_mul(r, x);
		x = h_mul(x, x);
		e >>= 1;
	}
	return r;
}

struct BbPass {
	int m;          // digit bits of this pass
	int role;       // 0 first/middle (rows stride Mp, 32-column tiles), 1 last, 2 single (whole array)
	int log_mp;     // log2 M_p (columns of the sub-problem; 0 for the last pass)
	int log_sub;    // log2 M_{p-1} (size of the sub-problem)
	int bitrev_in;  // first pass reading a bit-reversed input
	// last pass: k_1 has m_1 bits; (k_2..k_{L-1}) has gbits bits
	int m1, gbits;
	int log_pos[4], log_out[4], mdig[4];  // digits 2..L-1: position stride, output stride, bits
	int ndig;
};

struct BbArgs {
	const uint32_t* src;
	uint32_t* dst;
	const uint32_t* wtab;
	size_t n;  // words per transform
	int log_n;
	int hi_split;  // 1: wtab = lo[4096] ++ hi[]
	BbPass p;
};

// w^e for e < 2^log_n, Montgomery-encoded
__device__ inline uint32_t wpow(const BbArgs& A, uint32_t e) {
	if (!A.hi_split) return A.wtab[e];
	return mont(A.wtab[e & ((1u << kLoBits) - 1)], A.wtab[(1u << kLoBits) + (e >> kLoBits)]);
}

__device__ inline uint32_t rev_bits(uint32_t v, int bits) { return bits ? __brev(v) >> (32 - bits) : 0u; }

// tile element (row r, column c) <-> words, per role
template <int ROLE>
__global__ __launch_bounds__(kThreads) void bb_pass(BbArgs A) {
	extern __shared__ uint32_t lds[];
	const BbPass& ps = A.p;
	const int m = ps.m;
	const int R = 1 << m;
	const int tid = threadIdx.x;
	const size_t b = blockIdx.y;  // transform of the batch
	const uint32_t* src = A.src + b * A.n;
	uint32_t* dst = A.dst + b * A.n;
	const size_t t = blockIdx.x;
	// tile geometry
	size_t q = 0, cb = 0, g = 0, kb = 0;
	if (ROLE == 0) {
		const size_t ncb = ((size_t)1 << ps.log_mp) / kCols;
		q = t / ncb;
		cb = t % ncb;
	} else if (ROLE == 1) {
		const size_t nkb = ((size_t)1 << ps.m1) / kCols;
		g = t / nkb;
		kb = t % nkb;
	}
	size_t gpos = 0, gout = 0;
	if (ROLE == 1) {
		size_t gg = g;
		for (int i = 0; i < ps.ndig; i++) {
			const size_t d = gg & (((size_t)1 << ps.mdig[i]) - 1);
			gg >>= ps.mdig[i];
			gpos += d << ps.log_pos[i];
			gout += d << ps.log_out[i];
		}
	}
	const int cols = ROLE == 2 ? 1 : kCols;
	const int W = ROLE == 2 ? R : R * kCols;  // words in the tile
	auto src_addr = [&](int r, int c) -> size_t {
		if (ROLE == 0) {
			const size_t j = (q << ps.log_sub) + ((size_t)r << ps.log_mp) + cb * kCols + c;
			return ps.bitrev_in ? (size_t)rev_bits((uint32_t)j, A.log_n) : j;
		}
		if (ROLE == 1) return ((kb * kCols + c) << (A.log_n - ps.m1)) + gpos + r;
		return ps.bitrev_in ? (size_t)rev_bits((uint32_t)r, A.log_n) : (size_t)r;
	};
	// LDS: row r, column c at r * cols + c (a row of 32 words spans half the banks); behind the
	// tile, the tile DFT's twiddles w_R^i (Montgomery-encoded), i < R/2
	uint32_t* twl = lds + W;
	for (int i = tid; i < R / 2; i += kThreads) twl[i] = wpow(A, (uint32_t)i << (A.log_n - m));
	for (int u = tid; u < W; u += kThreads) {
		const int r = u / cols, c = u % cols;
		lds[u] = bb_reduce(src[src_addr(r, c)]);
	}
	__syncthreads();
	// radix-2 DIF stages: natural-order rows in, bit-reversed rows out; stage st uses
	// w_{2 half}^k = w_R^(k R / (2 half))
	const int pairs = (R / 2) * cols;
	for (int st = m - 1; st >= 0; st--) {
		const int half = 1 << st;
		for (int u = tid; u < pairs; u += kThreads) {
			const int c = u % cols, pr = u / cols;
			const int k = pr & (half - 1);
			const int r0 = ((pr >> st) << (st + 1)) | k;
			uint32_t* pu = lds + r0 * cols + c;
			uint32_t* pv = pu + half * cols;
			const uint32_t x = *pu, y = *pv;
			*pu = bb_add(x, y);
			const uint32_t d = bb_sub(x, y);
			*pv = k ? mont(d, twl[k << (m - 1 - st)]) : d;
		}
		__syncthreads();
	}
	// write row k (held at LDS row rev_m(k)). ROLE 0: inter-pass twiddle w_{M_{p-1}}^(c k); a
	// lane keeps its column c and walks rows k = k0, k0 + 8, ... so the twiddle advances by one
	// Montgomery product per element from two table lookups per lane.
	if (ROLE == 0) {
		const int c = tid % kCols, k0 = tid / kCols;  // kThreads / kCols = 8 rows per sweep
		const size_t cf = cb * kCols + c;             // column index inside the sub-problem
		const size_t msk = ((size_t)1 << ps.log_sub) - 1;
		const int sh = A.log_n - ps.log_sub;
		uint32_t tw = wpow(A, (uint32_t)(((cf * (size_t)k0) & msk) << sh));
		const uint32_t step = wpow(A, (uint32_t)(((cf * (size_t)(kThreads / kCols)) & msk) << sh));
		for (int k = k0; k < R; k += kThreads / kCols) {
			const uint32_t v = mont(lds[rev_bits((uint32_t)k, m) * kCols + c], tw);
			dst[(q << ps.log_sub) + ((size_t)k << ps.log_mp) + cf] = v;
			tw = mont(tw, step);
		}
	} else {
		for (int u = tid; u < W; u += kThreads) {
			const int k = u / cols, c = u % cols;
			const uint32_t v = lds[rev_bits((uint32_t)k, m) * cols + c];
			if (ROLE == 1)
				dst[(kb * kCols + c) + gout + ((size_t)k << (A.log_n - m))] = v;
			else
				dst[k] = v;
		}
	}
}

// Register-resident variant for the multi-pass roles (0, 1) and M = m in [6, 9]: the same tile,
// twiddles and output as bb_pass, but a thread holds E = R/8 elements of one column, rows
// t + 8i, so the radix-2 stages with half >= 8 run in registers; one LDS exchange regroups the
// column into runs of 8 rows for the last three stages. LDS traffic per tile: the exchange and the
// output gather, instead of two reads and two writes per element per stage.
template <int ROLE, int M>
__global__ __launch_bounds__(kThreads) void bb_pass_r(BbArgs A) {
	constexpr int R = 1 << M, E = R / 8;
	extern __shared__ uint32_t lds[];
	const BbPass& ps = A.p;
	const int tid = threadIdx.x;
	const size_t b = blockIdx.y;
	const uint32_t* src = A.src + b * A.n;
	uint32_t* dst = A.dst + b * A.n;
	const size_t tile = blockIdx.x;
	size_t q = 0, cb = 0, kb = 0, gpos = 0, gout = 0;
	if (ROLE == 0) {
		const size_t ncb = ((size_t)1 << ps.log_mp) / kCols;
		q = tile / ncb;
		cb = tile % ncb;
	} else {
		const size_t nkb = ((size_t)1 << ps.m1) / kCols;
		size_t g = tile / nkb;
		kb = tile % nkb;
		for (int i = 0; i < ps.ndig; i++) {
			const size_t d = g & (((size_t)1 << ps.mdig[i]) - 1);
			g >>= ps.mdig[i];
			gpos += d << ps.log_pos[i];
			gout += d << ps.log_out[i];
		}
	}
	// ROLE 0 reads rows of 32 contiguous columns (lanes along c); ROLE 1's rows are contiguous,
	// so 8 lanes walk 8 consecutive rows of one column
	const int c = ROLE == 0 ? tid % kCols : tid / 8;
	const int t = ROLE == 0 ? tid / kCols : tid % 8;
	auto src_addr = [&](int r) -> size_t {
		if (ROLE == 0) {
			const size_t j = (q << ps.log_sub) + ((size_t)r << ps.log_mp) + cb * kCols + c;
			return ps.bitrev_in ? (size_t)rev_bits((uint32_t)j, A.log_n) : j;
		}
		return ((kb * kCols + c) << (A.log_n - ps.m1)) + gpos + r;
	};
	uint32_t* twl = lds + R * kCols;
	for (int i = tid; i < R / 2; i += kThreads) twl[i] = wpow(A, (uint32_t)i << (A.log_n - M));
	uint32_t x[E];
#pragma unroll
	for (int i = 0; i < E; i++) x[i] = bb_reduce(src[src_addr(t + 8 * i)]);
	__syncthreads();  // twl
	// stages half = 2^s >= 8: rows t + 8i and t + 8i + half are both in this thread (i + half/8)
#pragma unroll
	for (int s = M - 1; s >= 3; s--) {
		const int hi = 1 << (s - 3);
#pragma unroll
		for (int i = 0; i < E; i++) {
			if (i & hi) continue;
			const uint32_t u = x[i], v = x[i + hi];
			const int k = (t + 8 * i) & ((1 << s) - 1);
			x[i] = bb_add(u, v);
			const uint32_t d = bb_sub(u, v);
			x[i + hi] = k ? mont(d, twl[k << (M - 1 - s)]) : d;
		}
	}
	// regroup: this thread takes rows 8g + j (j < 8) for g = t + 8u
#pragma unroll
	for (int i = 0; i < E; i++) lds[(t + 8 * i) * kCols + c] = x[i];
	__syncthreads();
#pragma unroll
	for (int u = 0; u < E / 8; u++)
#pragma unroll
		for (int j = 0; j < 8; j++) x[8 * u + j] = lds[(8 * (t + 8 * u) + j) * kCols + c];
#pragma unroll
	for (int s = 2; s >= 0; s--) {
		const int half = 1 << s;
#pragma unroll
		for (int i = 0; i < E; i++) {
			const int j = i & 7;
			if (j & half) continue;
			const uint32_t u = x[i], v = x[i + half];
			const int k = j & (half - 1);
			x[i] = bb_add(u, v);
			const uint32_t d = bb_sub(u, v);
			x[i + half] = k ? mont(d, twl[k << (M - 1 - s)]) : d;
		}
	}
#pragma unroll
	for (int u = 0; u < E / 8; u++)
#pragma unroll
		for (int j = 0; j < 8; j++) lds[(8 * (t + 8 * u) + j) * kCols + c] = x[8 * u + j];
	__syncthreads();
	// output: as bb_pass (row k sits at LDS row rev_M(k))
	if (ROLE == 0) {
		const int cc = tid % kCols, k0 = tid / kCols;
		const size_t cf = cb * kCols + cc;
		const size_t msk = ((size_t)1 << ps.log_sub) - 1;
		const int sh = A.log_n - ps.log_sub;
		uint32_t tw = wpow(A, (uint32_t)(((cf * (size_t)k0) & msk) << sh));
		const uint32_t step = wpow(A, (uint32_t)(((cf * (size_t)(kThreads / kCols)) & msk) << sh));
#pragma unroll 4
		for (int k = k0; k < R; k += kThreads / kCols) {
			const uint32_t v = mont(lds[rev_bits((uint32_t)k, M) * kCols + cc], tw);
			dst[(q << ps.log_sub) + ((size_t)k << ps.log_mp) + cf] = v;
			tw = mont(tw, step);
		}
	} else {
#pragma unroll 4
		for (int u = tid; u < R * kCols; u += kThreads) {
			const int k = u / kCols, cc = u % kCols;
			dst[(kb * kCols + cc) + gout + ((size_t)k << (A.log_n - M))] = lds[rev_bits((uint32_t)k, M) * kCols + cc];
		}
	}
}

template <int ROLE>
static const void* pass_fn() {
	return (const void*)bb_pass<ROLE>;
}

static const void* pass_r_fn(int role, int m) {
	static const void* r[2][4] = {
	    {(const void*)bb_pass_r<0, 6>, (const void*)bb_pass_r<0, 7>, (const void*)bb_pass_r<0, 8>, (const void*)bb_pass_r<0, 9>},
	    {(const void*)bb_pass_r<1, 6>, (const void*)bb_pass_r<1, 7>, (const void*)bb_pass_r<1, 8>, (const void*)bb_pass_r<1, 9>}};
	return r[role][m - 6];
}

// the register variant where it applies (roles 0/1, m in 6..9); in the development build BN_BB_LDS=1
// forces bb_pass (A/B)
static const void* pass_fn_for(const BbPass& p) {
#ifdef BN_DEV
	static const bool lds_only = getenv("BN_BB_LDS") != nullptr;
#else
	constexpr bool lds_only = false;
#endif
	if (!lds_only && p.role != 2 && p.m >= 6 && p.m <= 9) return pass_r_fn(p.role, p.m);
	return p.role == 0 ? pass_fn<0>() : p.role == 1 ? pass_fn<1>() : pass_fn<2>();
}

static std::vector<BbPass> bb_passes(const bn_bb31_ntt_plan* P, bool bitrev_in) {
	std::vector<BbPass> v;
	const int n = P->log_n;
	if (P->L == 1) {
		BbPass p{};
		p.m = n;
		p.role = 2;
		p.bitrev_in = bitrev_in;
		v.push_back(p);
		return v;
	}
	int used = 0;
	for (int i = 0; i < P->L; i++) {
		BbPass p{};
		p.m = P->m[i];
		p.log_sub = n - used;
		used += p.m;
		p.log_mp = n - used;
		if (i + 1 < P->L) {
			p.role = 0;
			p.bitrev_in = i == 0 && bitrev_in;
		} else {
			p.role = 1;
			p.m1 = P->m[0];
			// digits 2..L-1: position stride M_i = 2^(n - m_1 - ... - m_i), output stride N_1 ... N_{i-1}
			int pos_used = P->m[0], out_used = P->m[0];
			p.ndig = 0;
			for (int d = 1; d + 1 < P->L; d++) {
				pos_used += P->m[d];
				p.log_pos[p.ndig] = n - pos_used;
				p.log_out[p.ndig] = out_used;
				p.mdig[p.ndig] = P->m[d];
				out_used += P->m[d];
				p.ndig++;
			}
			p.gbits = n - P->m[0] - P->m[P->L - 1];
		}
		v.push_back(p);
	}
	return v;
}

}  // namespace
}  // namespace bn

using namespace bn;

extern "C" int bn_bb31_ntt_plan_create(int device, uint32_t generator, int log_group_order, int log_n,
                                       bn_bb31_ntt_plan** out) {
	BN_CHECK_ARG(out != nullptr, "out is NULL");
	// NTTConfRad2 asserts (src/ulvt/ntt/nttconf.cuh:31-38)
	BN_CHECK_ARG(log_n >= 1 && log_n <= 27, "log_n must be in [1, 27] (got %d)", log_n);
	BN_CHECK_ARG(log_group_order >= log_n && log_group_order <= 27, "log_group_order must be in [log_n, 27]");
	int ndev = 0;
	BN_HIP(hipGetDeviceCount(&ndev));
	BN_CHECK_ARG(device >= 0 && device < ndev, "device %d out of range", device);
	auto* P = new bn_bb31_ntt_plan();
	P->device = device;
	P->log_n = log_n;
	P->log_group = log_group_order;
	P->generator = generator % kP;
	if (log_n <= 13) {
		P->L = 1;
		P->m[0] = log_n;
	} else {
		P->L = (log_n + kMaxM - 1) / kMaxM;
		for (int i = 0; i < P->L; i++) P->m[i] = log_n / P->L + (i < log_n % P->L ? 1 : 0);
	}
	// twiddle tables: w^e * R mod p (Montgomery-encoded), e < 2^log_n
	const uint32_t w = h_pow(P->generator, (uint64_t)1 << (log_group_order - log_n));
	const uint32_t R = (uint32_t)(((uint64_t)1 << 32) % kP);
	std::vector<uint32_t> tab;
	if (log_n <= kLoBits) {
		uint32_t cur = R;
		for (size_t e = 0; e < ((size_t)1 << log_n); e++) {
			tab.push_back(cur);
			cur = h_mul(cur, w);
		}
	} else {
		uint32_t cur = R;
		for (size_t e = 0; e < ((size_t)1 << kLoBits); e++) {
			tab.push_back(cur);
			cur = h_mul(cur, w);
		}
		const uint32_t wh = h_pow(w, (uint64_t)1 << kLoBits);
		cur = R;
		for (size_t e = 0; e < ((size_t)1 << (log_n - kLoBits)); e++) {
			tab.push_back(cur);
			cur = h_mul(cur, wh);
		}
	}
	(void)kR2;
	int prev = 0;
	(void)hipGetDevice(&prev);
	hipError_t e = hipSetDevice(device);
	if (e == hipSuccess) e = hipMalloc(&P->wtab, tab.size() * sizeof(uint32_t));
	if (e == hipSuccess) e = hipMemcpy(P->wtab, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
	if (e == hipSuccess)
		for (const void* f : {pass_fn<0>(), pass_fn<1>(), pass_fn<2>(), pass_r_fn(0, 6), pass_r_fn(0, 7), pass_r_fn(0, 8),
		                      pass_r_fn(0, 9), pass_r_fn(1, 6), pass_r_fn(1, 7), pass_r_fn(1, 8), pass_r_fn(1, 9)})
			if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, ((1 << kMaxM) * kCols + (1 << 12)) * 4);
	(void)hipSetDevice(prev);
	if (e != hipSuccess) {
		bn_bb31_ntt_plan_destroy(P);
		BN_FAIL(BN_ERR_HIP, "bb31 plan allocation failed: %s", hipGetErrorString(e));
	}
	*out = P;
	return BN_OK;
}

extern "C" int bn_bb31_ntt_plan_destroy(bn_bb31_ntt_plan* P) {
	if (!P) return BN_OK;
	int prev = 0;
	(void)hipGetDevice(&prev);
	(void)hipSetDevice(P->device);
	if (P->wtab) (void)hipFree(P->wtab);
	if (P->scratch) (void)hipFree(P->scratch);
	if (P->h_dev) (void)hipFree(P->h_dev);
	if (P->own_stream) (void)hipStreamDestroy(P->own_stream);
	(void)hipSetDevice(prev);
	delete P;
	return BN_OK;
}

static int bb_forward(bn_bb31_ntt_plan* P, const uint32_t* d_in, uint32_t* d_out, size_t batch, int bitrev, hipStream_t st) {
	const size_t n = (size_t)1 << P->log_n;
	const auto passes = bb_passes(P, bitrev != 0);
	// passes 1..L-1 run in place on a scratch buffer (first pass: in -> scratch), the last pass
	// scatters scratch -> out (its reads and writes are different index sets)
	uint32_t* work = d_out;
	if (P->L > 1) {
		if (P->scratch_words < n * batch) {
			if (P->scratch) BN_HIP(hipFree(P->scratch));
			P->scratch = nullptr;
			BN_HIP(hipMalloc(&P->scratch, n * batch * sizeof(uint32_t)));
			P->scratch_words = n * batch;
		}
		work = P->scratch;
	}
	for (size_t i = 0; i < passes.size(); i++) {
		BbArgs A;
		A.src = i == 0 ? d_in : work;
		A.dst = i + 1 == passes.size() ? d_out : work;
		A.wtab = P->wtab;
		A.n = n;
		A.log_n = P->log_n;
		A.hi_split = P->log_n > kLoBits;
		A.p = passes[i];
		const BbPass& p = passes[i];
		size_t tiles;
		int W;
		if (p.role == 2) {
			tiles = 1;
			W = 1 << p.m;
		} else if (p.role == 0) {
			tiles = ((size_t)1 << (P->log_n - p.log_sub)) * (((size_t)1 << p.log_mp) / kCols);
			W = (1 << p.m) * kCols;
		} else {
			tiles = ((size_t)1 << p.gbits) * (((size_t)1 << p.m1) / kCols);
			W = (1 << p.m) * kCols;
		}
		void* args[] = {&A};
		const void* fn = pass_fn_for(p);
		BN_HIP(hipLaunchKernel(fn, dim3((unsigned)tiles, (unsigned)batch), dim3(kThreads), args,
		                       ((size_t)W + ((size_t)1 << p.m) / 2) * 4, st));
	}
	return BN_OK;
}

extern "C" int bn_bb31_ntt_forward_device(bn_bb31_ntt_plan* P, const uint32_t* d_in, uint32_t* d_out, size_t batch,
                                          int in_bit_reversed, void* stream) {
	BN_CHECK_ARG(P != nullptr, "plan is NULL");
	BN_CHECK_ARG(d_in != nullptr && d_out != nullptr, "device buffers must be non-NULL");
	BN_CHECK_ARG(batch >= 1 && batch <= 65535, "batch must be in [1, 65535]");
	const size_t bytes = ((size_t)4 << P->log_n) * batch;
	const char* a = (const char*)d_in;
	const char* b = (const char*)d_out;
	BN_CHECK_ARG(a + bytes <= b || b + bytes <= a, "d_in and d_out must not overlap");
	int prev = 0;
	(void)hipGetDevice(&prev);
	if (prev != P->device) BN_HIP(hipSetDevice(P->device));
	const int rc = bb_forward(P, d_in, d_out, batch, in_bit_reversed, (hipStream_t)stream);
	if (prev != P->device) (void)hipSetDevice(prev);
	return rc;
}

// NTT<BB31>::apply (gpuntt.cuh:150-183): host in -> host out, synchronous; the input order
// flag replaces NTTData::order (BIT_REVERSED input is used as is, IN_ORDER is reversed first).
extern "C" int bn_bb31_ntt_forward_host(bn_bb31_ntt_plan* P, const uint32_t* in, size_t in_elems, uint32_t* out,
                                        int in_bit_reversed) {
	BN_CHECK_ARG(P != nullptr, "plan is NULL");
	BN_CHECK_ARG(in != nullptr && out != nullptr, "host buffers must be non-NULL");
	const size_t n = (size_t)1 << P->log_n;
	BN_CHECK_ARG(in_elems == n, "input has %zu elements, plan expects 2^%d", in_elems, P->log_n);
	int prev = 0;
	(void)hipGetDevice(&prev);
	BN_HIP(hipSetDevice(P->device));
	if (!P->h_dev) BN_HIP(hipMalloc(&P->h_dev, 2 * n * sizeof(uint32_t)));
	if (!P->own_stream) BN_HIP(hipStreamCreateWithFlags(&P->own_stream, hipStreamNonBlocking));
	BN_HIP(hipMemcpyAsync(P->h_dev, in, n * 4, hipMemcpyHostToDevice, P->own_stream));
	int rc = bb_forward(P, P->h_dev, P->h_dev + n, 1, in_bit_reversed, P->own_stream);
	if (rc == BN_OK) {
		BN_HIP(hipMemcpyAsync(out, P->h_dev + n, n * 4, hipMemcpyDeviceToHost, P->own_stream));
		BN_HIP(hipStreamSynchronize(P->own_stream));
	}
	(void)hipSetDevice(prev);
	return rc;
}
