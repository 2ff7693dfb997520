// QM31 sumcheck prover for gfx950: the prime-field sibling of the GF(2^128) sumcheck (SURVEY.md
// §8f row 4). Replaces Sumcheck<NUM_VARS> of src/ulvt/prime_field_sumcheck/sumcheck.cuh:8-96
// (kernels get_round_coefficients / fold_list_halves, core/kernels.cu:5-77): two columns f0, f1
// of 2^N QM31 evaluations; with h = cur / 2 the round messages are
//     points[k] = sum_{x<h} g0(x, k) g1(x, k),  g(x, X) = f(x) + X (f(x+h) - f(x)),  k = 0, 1, 2
// and fold(r): f(x) <- f(x) + r (f(x+h) - f(x)). Field: M31 (p = 2^31 - 1, m31.cuh:6-76),
// CM31 = M31[i]/(i^2+1) (cm31.cuh), QM31 = CM31[u]/(u^2 - (2+i)) (qm31.cuh). A QM31 element is 4
// u32 words (lo.a, lo.b, hi.a, hi.b), the member order of qm31.cuh.
//
// MI355X design: both columns stay resident in HBM for all rounds (the reference allocates and
// copies per round); a round's messages are one streaming pass with 16-byte loads of the four
// rows a lane needs, the per-component sums are exact 64-bit integers (as sum_into_u64) reduced
// through wave shuffles and LDS, one 64-bit atomic per workgroup and value, and read back through
// pinned memory. fold(r) is deferred and fused into the next round's messages pass, so each
// round streams the columns once. Values are canonical (< p) throughout.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "common.hpp"

struct bn_qm31_sumcheck {
	int device = 0;
	int num_vars = 0;
	int round = 0;
	size_t cur = 0;  // evaluations per column still live
	uint32_t* cols = nullptr;  // 2 columns x 2^N x 4 words
	unsigned long long* acc = nullptr;  // 2 x 12 u64 (points 0..2 x 4 components), alternating rounds
	unsigned long long* h_acc = nullptr;  // pinned
	hipStream_t stream = nullptr;
	int cus = 256;
	int wg_per_cu = 8;  // grid cap (BN_QM_WG_PER_CU overrides it in the development build, for tuning)
	int par = 0;  // accumulator set of the next round_messages
	bool pending = false;  // a fold(r) not yet applied to cols (fused into the next round's messages)
	uint4 pend_r = {0, 0, 0, 0};
};

namespace bn {
namespace {

constexpr uint32_t kM = 0x7fffffffu;
constexpr int kT = 256;

struct Cm {
	uint32_t a, b;
};
struct Qm {
	Cm lo, hi;
};

__device__ inline uint32_t m_add(uint32_t a, uint32_t b) {
	const uint32_t s = a + b;
	return s >= kM ? s - kM : s;
}
__device__ inline uint32_t m_sub(uint32_t a, uint32_t b) { return a >= b ? a - b : a + kM - b; }
__device__ inline uint32_t m_mul(uint32_t a, uint32_t b) {
	const uint64_t x = (uint64_t)a * b;  // < 2^62
	uint32_t s = (uint32_t)(x & kM) + (uint32_t)(x >> 31);  // < 2^32
	s = (s & kM) + (s >> 31);
	return s >= kM ? s - kM : s;
}
__device__ inline uint32_t m_red(uint32_t x) {  // any u32 -> canonical
	x = (x & kM) + (x >> 31);
	return x >= kM ? x - kM : x;
}
__device__ inline Cm c_add(Cm x, Cm y) { return {m_add(x.a, y.a), m_add(x.b, y.b)}; }
__device__ inline Cm c_sub(Cm x, Cm y) { return {m_sub(x.a, y.a), m_sub(x.b, y.b)}; }
__device__ inline Cm c_mul(Cm x, Cm y) {
	// Karatsuba: ad + bc = (a + b)(c + d) - ac - bd
	const uint32_t ac = m_mul(x.a, y.a), bd = m_mul(x.b, y.b);
	const uint32_t s = m_mul(m_add(x.a, x.b), m_add(y.a, y.b));
	return {m_sub(ac, bd), m_sub(m_sub(s, ac), bd)};
}
__device__ inline Cm c_mul_r(Cm x) {  // (2 + i)(a + b i) = (2a - b) + (a + 2b) i
	return {m_sub(m_add(x.a, x.a), x.b), m_add(x.a, m_add(x.b, x.b))};
}
__device__ inline Qm q_add(Qm x, Qm y) { return {c_add(x.lo, y.lo), c_add(x.hi, y.hi)}; }
__device__ inline Qm q_sub(Qm x, Qm y) { return {c_sub(x.lo, y.lo), c_sub(x.hi, y.hi)}; }
__device__ inline Qm q_mul(Qm x, Qm y) {
	// (lo + hi u)(lo' + hi' u) = lo lo' + R hi hi' + (lo hi' + hi lo') u, Karatsuba on the u level
	const Cm ll = c_mul(x.lo, y.lo), hh = c_mul(x.hi, y.hi);
	const Cm s = c_mul(c_add(x.lo, x.hi), c_add(y.lo, y.hi));
	return {c_add(ll, c_mul_r(hh)), c_sub(c_sub(s, ll), hh)};
}
__device__ inline Qm q_ld(const uint32_t* p) {
	const uint4 v = *(const uint4*)p;
	return {{v.x, v.y}, {v.z, v.w}};
}
__device__ inline void q_st(uint32_t* p, Qm v) { *(uint4*)p = make_uint4(v.lo.a, v.lo.b, v.hi.a, v.hi.b); }

__global__ __launch_bounds__(kT) void qm_reduce(uint32_t* w, size_t n) {
	for (size_t i = (size_t)blockIdx.x * kT + threadIdx.x; i < n; i += (size_t)gridDim.x * kT) w[i] = m_red(w[i]);
}

__device__ inline void qm_accumulate(unsigned long long (&s)[12], Qm l0, Qm u0, Qm l1, Qm u1) {
	const Qm p[3] = {q_mul(l0, l1), q_mul(u0, u1), q_mul(q_add(q_sub(u0, l0), u0), q_add(q_sub(u1, l1), u1))};
#pragma unroll
	for (int k = 0; k < 3; k++) {
		s[4 * k] += p[k].lo.a;
		s[4 * k + 1] += p[k].lo.b;
		s[4 * k + 2] += p[k].hi.a;
		s[4 * k + 3] += p[k].hi.b;
	}
}

// Block sums -> one device atomic per value. Rounds alternate between two accumulator sets:
// this round's workgroup 0 clears the other set (last read back by the previous round's copy,
// which is ordered before this launch), so no memset is queued per round.
__device__ inline void qm_flush(unsigned long long (&s)[12], unsigned long long* acc, unsigned long long* clr) {
	if (blockIdx.x == 0 && threadIdx.x < 12) clr[threadIdx.x] = 0;
	__shared__ unsigned long long red[kT / 64][12];
#pragma unroll
	for (int i = 0; i < 12; i++) {
		unsigned long long v = s[i];
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
		s[i] = v;
	}
	const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
	if (lane == 0)
#pragma unroll
		for (int i = 0; i < 12; i++) red[wave][i] = s[i];
	__syncthreads();
	if (threadIdx.x < 12) {
		unsigned long long v = 0;
#pragma unroll
		for (int w = 0; w < kT / 64; w++) v += red[w][threadIdx.x];
		if (v) atomicAdd(acc + threadIdx.x, v);
	}
}

// round messages: lanes stride over x < h; exact u64 component sums -> one atomic per value per WG
__global__ __launch_bounds__(kT) void qm_messages(const uint32_t* cols, size_t col_words, size_t h,
                                                  unsigned long long* acc, unsigned long long* clr) {
	unsigned long long s[12];
#pragma unroll
	for (int i = 0; i < 12; i++) s[i] = 0;
	const uint32_t* c1 = cols + col_words;
	for (size_t x = (size_t)blockIdx.x * kT + threadIdx.x; x < h; x += (size_t)gridDim.x * kT) {
		qm_accumulate(s, q_ld(cols + 4 * x), q_ld(cols + 4 * (x + h)), q_ld(c1 + 4 * x), q_ld(c1 + 4 * (x + h)));
	}
	qm_flush(s, acc, clr);
}

// fold(r) of the previous round fused with this round's messages: with the old half H = 2 h,
// lane x < h reads old rows x, x + h, x + H, x + h + H of each column, writes the folded rows x
// and x + h in place (disjoint from every other lane's reads) and accumulates the messages of
// the pair (x, x + h). One pass instead of two: reads 2 x 32 B, writes 2 x 16 B per pair.
__global__ __launch_bounds__(kT) void qm_fold_messages(uint32_t* cols, size_t col_words, size_t h, uint4 r4,
                                                       unsigned long long* acc, unsigned long long* clr) {
	const Qm r = {{r4.x, r4.y}, {r4.z, r4.w}};
	unsigned long long s[12];
#pragma unroll
	for (int i = 0; i < 12; i++) s[i] = 0;
	uint32_t* c1 = cols + col_words;
	const size_t H = 2 * h;
	for (size_t x = (size_t)blockIdx.x * kT + threadIdx.x; x < h; x += (size_t)gridDim.x * kT) {
		Qm l[2], u[2];
#pragma unroll
		for (int j = 0; j < 2; j++) {
			uint32_t* c = j ? c1 : cols;
			const Qm a = q_ld(c + 4 * x), b = q_ld(c + 4 * (x + h));
			const Qm aH = q_ld(c + 4 * (x + H)), bH = q_ld(c + 4 * (x + h + H));
			l[j] = q_add(a, q_mul(q_sub(aH, a), r));
			u[j] = q_add(b, q_mul(q_sub(bH, b), r));
			q_st(c + 4 * x, l[j]);
			q_st(c + 4 * (x + h), u[j]);
		}
		qm_accumulate(s, l[0], u[0], l[1], u[1]);
	}
	qm_flush(s, acc, clr);
}

// fold: f(x) <- f(x) + r (f(x+h) - f(x)) for both columns, x < h
__global__ __launch_bounds__(kT) void qm_fold(uint32_t* cols, size_t col_words, size_t h, uint4 r4) {
	const Qm r = {{r4.x, r4.y}, {r4.z, r4.w}};
	for (size_t i = (size_t)blockIdx.x * kT + threadIdx.x; i < 2 * h; i += (size_t)gridDim.x * kT) {
		const size_t j = i / h, x = i - j * h;
		uint32_t* c = cols + j * col_words;
		const Qm lo = q_ld(c + 4 * x), hi = q_ld(c + 4 * (x + h));
		q_st(c + 4 * x, q_add(lo, q_mul(q_sub(hi, lo), r)));
	}
}

struct DevScope {
	int prev = -1;
	explicit DevScope(int d) {
		if (hipGetDevice(&prev) != hipSuccess) prev = -1;
		if (prev != d) (void)hipSetDevice(d);
	}
	~DevScope() {
		int cur = -1;
		if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
	}
};

static unsigned grid_for(const bn_qm31_sumcheck* S, size_t items) {
	const size_t want = (items + kT - 1) / kT;
	return (unsigned)std::max<size_t>(1, std::min<size_t>(want, (size_t)S->cus * S->wg_per_cu));
}

}  // namespace
}  // namespace bn

using namespace bn;

// Sumcheck(evals, benchmarking) (sumcheck.cuh:24-44): evals = column 0 then column 1, 2^N QM31
// each (the reference restricts NUM_VARS to {1, 20, 24, 28}; any 1 <= N <= 28 is built here).
extern "C" int bn_qm31_sumcheck_create(int device, int num_vars, const uint32_t* evals, bn_qm31_sumcheck** out) {
	BN_CHECK_ARG(out != nullptr && evals != nullptr, "NULL argument");
	BN_CHECK_ARG(num_vars >= 1 && num_vars <= 28, "num_vars must be in [1, 28] (got %d)", num_vars);
	int ndev = 0;
	BN_HIP(hipGetDeviceCount(&ndev));
	BN_CHECK_ARG(device >= 0 && device < ndev, "device %d out of range", device);
	DevScope ds(device);
	auto* S = new bn_qm31_sumcheck();
	S->device = device;
	S->num_vars = num_vars;
	S->cur = (size_t)1 << num_vars;
	const size_t words = 2 * S->cur * 4;
	hipError_t e = hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking);
	if (e == hipSuccess) e = hipMalloc(&S->cols, words * 4);
	if (e == hipSuccess) e = hipMalloc(&S->acc, 24 * sizeof(unsigned long long));
	if (e == hipSuccess) e = hipMemsetAsync(S->acc, 0, 24 * sizeof(unsigned long long), S->stream);
	if (e == hipSuccess) e = hipHostMalloc(&S->h_acc, 12 * sizeof(unsigned long long), hipHostMallocDefault);
	if (e == hipSuccess) e = hipMemcpyAsync(S->cols, evals, words * 4, hipMemcpyHostToDevice, S->stream);
	int cus = 0;
	if (e == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess)
		S->cus = std::max(cus, 1);
#ifdef BN_DEV
	if (const char* v = getenv("BN_QM_WG_PER_CU")) S->wg_per_cu = std::max(1, atoi(v));  // tuning, development build only
#endif
	if (e == hipSuccess) {
		// QM31(uint32_t) assumes values < p; reduce whatever was passed
		hipLaunchKernelGGL(qm_reduce, dim3(grid_for(S, words)), dim3(kT), 0, S->stream, S->cols, words);
		e = hipGetLastError();
	}
	if (e == hipSuccess) e = hipStreamSynchronize(S->stream);
	if (e != hipSuccess) {
		bn_qm31_sumcheck_destroy(S);
		BN_FAIL(BN_ERR_HIP, "qm31 sumcheck setup failed: %s", hipGetErrorString(e));
	}
	*out = S;
	return BN_OK;
}

// A deferred fold not followed by round_messages (fold twice, or the last round) runs alone.
static int apply_pending(bn_qm31_sumcheck* S) {
	if (!S->pending) return BN_OK;
	const size_t h = S->cur, col_words = ((size_t)4) << S->num_vars;  // cur is already the folded size
	hipLaunchKernelGGL(qm_fold, dim3(grid_for(S, 2 * h)), dim3(kT), 0, S->stream, S->cols, col_words, h, S->pend_r);
	BN_HIP(hipGetLastError());
	S->pending = false;
	return BN_OK;
}

// this_round_messages(points) (sumcheck.cuh:46-86): points 0, 1, 2 as 3 x 4 canonical words.
extern "C" int bn_qm31_sumcheck_round_messages(bn_qm31_sumcheck* S, uint32_t* points) {
	BN_CHECK_ARG(S != nullptr && points != nullptr, "NULL argument");
	BN_CHECK_ARG(S->round < S->num_vars, "all %d rounds are done", S->num_vars);
	DevScope ds(S->device);
	const size_t h = S->cur / 2, col_words = ((size_t)4) << S->num_vars;
	unsigned long long* acc = S->acc + 12 * S->par;
	unsigned long long* clr = S->acc + 12 * (1 - S->par);
	if (S->pending) {
		hipLaunchKernelGGL(qm_fold_messages, dim3(grid_for(S, h)), dim3(kT), 0, S->stream, S->cols, col_words, h,
		                   S->pend_r, acc, clr);
		S->pending = false;
	} else {
		hipLaunchKernelGGL(qm_messages, dim3(grid_for(S, h)), dim3(kT), 0, S->stream, S->cols, col_words, h, acc, clr);
	}
	BN_HIP(hipGetLastError());
	BN_HIP(hipMemcpyAsync(S->h_acc, acc, 12 * sizeof(unsigned long long), hipMemcpyDeviceToHost, S->stream));
	S->par ^= 1;
	BN_HIP(hipStreamSynchronize(S->stream));
	// QM31(uint64_t[4]) -> M31(uint64_t) (m31.cuh:21-24): the exact sum, reduced
	for (int i = 0; i < 12; i++) points[i] = (uint32_t)(S->h_acc[i] % 0x7fffffffull);
	return BN_OK;
}

// fold(challenge) (sumcheck.cuh:88-96); the challenge is reduced mod p.
extern "C" int bn_qm31_sumcheck_fold(bn_qm31_sumcheck* S, const uint32_t* challenge) {
	BN_CHECK_ARG(S != nullptr && challenge != nullptr, "NULL argument");
	BN_CHECK_ARG(S->round < S->num_vars, "all %d rounds are done", S->num_vars);
	DevScope ds(S->device);
	const size_t h = S->cur / 2;
	if (int rc = apply_pending(S)) return rc;
	// deferred: the next round_messages fuses it (qm_fold_messages); final_values applies it alone
	S->pend_r = make_uint4(challenge[0] % kM, challenge[1] % kM, challenge[2] % kM, challenge[3] % kM);
	S->pending = true;
	S->cur = h;
	S->round++;
	return BN_OK;
}

// The two remaining values f0(r), f1(r) after all folds (the verifier's final check).
extern "C" int bn_qm31_sumcheck_final_values(bn_qm31_sumcheck* S, uint32_t* out /* 8 words */) {
	BN_CHECK_ARG(S != nullptr && out != nullptr, "NULL argument");
	BN_CHECK_ARG(S->round == S->num_vars, "only after all %d rounds (at round %d)", S->num_vars, S->round);
	DevScope ds(S->device);
	const size_t col_words = ((size_t)4) << S->num_vars;
	if (int rc = apply_pending(S)) return rc;
	BN_HIP(hipMemcpyAsync(out, S->cols, 16, hipMemcpyDeviceToHost, S->stream));
	BN_HIP(hipMemcpyAsync(out + 4, S->cols + col_words, 16, hipMemcpyDeviceToHost, S->stream));
	BN_HIP(hipStreamSynchronize(S->stream));
	return BN_OK;
}

extern "C" int bn_qm31_sumcheck_destroy(bn_qm31_sumcheck* S) {
	if (!S) return BN_OK;
	DevScope ds(S->device);
	if (S->stream) (void)hipStreamSynchronize(S->stream);
	if (S->cols) (void)hipFree(S->cols);
	if (S->acc) (void)hipFree(S->acc);
	if (S->h_acc) (void)hipHostFree(S->h_acc);
	if (S->stream) (void)hipStreamDestroy(S->stream);
	delete S;
	return BN_OK;
}
