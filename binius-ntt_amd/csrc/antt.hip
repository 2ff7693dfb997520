// Additive NTT over GF(2^32) / GF(2^128): plan management, C-ABI entry points and the
// v0 (correctness-first, compact-layout) kernel. The bitsliced fast path lives in
// antt_bs.hip and is selected by bn_antt_forward_device when it supports the plan.
//
// Semantics (src/ulvt/ntt/additive_ntt.cuh): for each coset c < 2^log_rate the input is
// copied and butterflies u += w v ; v += u run for stage = log_h-1 .. 0 over blocks of
// 2^(stage+1) elements, with twiddle w = XOR_k s[stage][k] over the set bits k of
// (c << (log_h-1-stage)) | blk (calculate_twiddle, :59-77). Output is coset-major.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <cxxabi.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "antt_bs.hpp"
#include "field_dev.hpp"
#include "tower.hpp"

namespace bn {

void subspace_evals(int log_h, int log_rate, std::vector<uint32_t>& s) {
	const int width = log_h + log_rate - 1;
	s.assign((size_t)log_h * (size_t)std::max(width, 1), 0u);
	auto at = [&](int i, int j) -> uint32_t& { return s[(size_t)i * (size_t)width + (size_t)j]; };
	std::vector<uint32_t> norm((size_t)std::max(log_h, 1));
	for (int i = 1; i < log_h + log_rate; i++) at(0, i - 1) = 1u << i;
	norm[0] = 1;
	for (int i = 1; i < log_h; i++) {
		const uint64_t np = norm[i - 1];
		const uint64_t p0 = at(i - 1, 0);
		norm[i] = (uint32_t)(tw_square(p0, 5) ^ tw_mul(np, p0, 5));
		for (int j = 1; j < log_h + log_rate - i; j++) {
			const uint64_t sp = at(i - 1, j);
			at(i, j - 1) = (uint32_t)(tw_square(sp, 5) ^ tw_mul(np, sp, 5));
		}
	}
	for (int i = 0; i < log_h; i++) {
		const uint64_t inv = tw_inv(norm[i], 5);
		for (int j = 0; j < log_h + log_rate - i - 1; j++) at(i, j) = (uint32_t)tw_mul(inv, at(i, j), 5);
	}
}

// ------------------------------------------------------------------------------------
// v0 kernel: one launch per group of up to kMaxGroup stages. A workgroup owns a tile of
// 2^(k+c) elements: the k group bits [lo, lo+k) plus the c lowest index bits (so that
// each group of 2^c consecutive elements is read contiguously). Elements are staged in
// LDS; each thread walks its butterflies stage by stage.
// ------------------------------------------------------------------------------------
constexpr int kTileLog = 12;  // 4096 elements; 64 KiB at 16 B/element

struct V0Params {
	const uint32_t* src;  // group input (d_in for the first group: coset copies are implicit)
	uint32_t* dst;        // d_out
	const uint32_t* s;    // subspace table, log_h x width
	int width;
	int log_h;
	int log_rate;
	int lo, k, c;
	int first;  // 1: src is the shared input (same for every coset), else src == dst
};

template <int L>
__global__ __launch_bounds__(256) void antt_v0_group(V0Params p) {
	extern __shared__ uint32_t lds[];
	const int tile_log = p.k + p.c;
	const int tile = 1 << tile_log;
	const int outer_log = p.log_h - tile_log;
	const size_t n = (size_t)1 << p.log_h;
	const int coset = (int)(blockIdx.x >> outer_log);
	const size_t rest = blockIdx.x & (((size_t)1 << outer_log) - 1);
	const int mid_bits = p.lo - p.c;
	const size_t o_mid = rest & (((size_t)1 << mid_bits) - 1);
	const size_t o_hi = rest >> mid_bits;
	auto gidx = [&](int pos) -> size_t {
		const size_t cc = (size_t)pos & (((size_t)1 << p.c) - 1);
		const size_t g = (size_t)pos >> p.c;
		return (o_hi << (p.lo + p.k)) | (g << p.lo) | (o_mid << p.c) | cc;
	};
	const uint32_t* src = p.first ? p.src : (p.dst + (size_t)coset * n * L);
	uint32_t* dst = p.dst + (size_t)coset * n * L;

	uint8_t* tab = (uint8_t*)(lds + (size_t)tile * L);  // GF(2^8) log/exp tables after the tile
	gf8_tables_to_lds(tab);
	for (int pos = threadIdx.x; pos < tile; pos += blockDim.x) {
		const size_t gi = gidx(pos);
#pragma unroll
		for (int l = 0; l < L; l++) lds[pos * L + l] = src[gi * L + l];
	}
	__syncthreads();

	for (int stage = p.lo + p.k - 1; stage >= p.lo; stage--) {
		const int b = stage - p.lo + p.c;
		const int npairs = tile >> 1;
		const uint32_t* srow = p.s + (size_t)stage * p.width;
		const int nbits = p.log_h + p.log_rate - 1 - stage;
		for (int q = threadIdx.x; q < npairs; q += blockDim.x) {
			const int pu = ((q >> b) << (b + 1)) | (q & ((1 << b) - 1));
			const int pv = pu | (1 << b);
			const size_t blk = gidx(pu) >> (stage + 1);
			const uint64_t ind = ((uint64_t)coset << (p.log_h - 1 - stage)) | (uint64_t)blk;
			uint32_t w = 0;
			for (int kk = 0; kk < nbits; kk++)
				if ((ind >> kk) & 1) w ^= srow[kk];
#pragma unroll
			for (int l = 0; l < L; l++) {
				uint32_t u = lds[pu * L + l], v = lds[pv * L + l];
				u ^= (uint32_t)dmul_t<5>(w, v, tab);
				v ^= u;
				lds[pu * L + l] = u;
				lds[pv * L + l] = v;
			}
		}
		__syncthreads();
	}

	for (int pos = threadIdx.x; pos < tile; pos += blockDim.x) {
		const size_t gi = gidx(pos);
#pragma unroll
		for (int l = 0; l < L; l++) dst[gi * L + l] = lds[pos * L + l];
	}
}

// Optional per-launch hipEvent timing (bench.py): events are recorded on the launch stream
// around each kernel and resolved later (timing_resolve), so timing does not serialise the
// passes; `kind` identifies the pass.
static int timing_event(bn_antt_plan* p, hipEvent_t* e) {
	if (!p->ev_pool.empty()) {
		*e = p->ev_pool.back();
		p->ev_pool.pop_back();
		return BN_OK;
	}
	BN_HIP(hipEventCreate(e));
	return BN_OK;
}
int timing_begin(bn_antt_plan* p, int kind, hipStream_t st) {
	if (!p->timing) return BN_OK;
	(void)kind;
	int rc = timing_event(p, &p->cur_begin);
	if (rc != BN_OK) return rc;
	BN_HIP(hipEventRecord(p->cur_begin, st));
	return BN_OK;
}
int timing_end(bn_antt_plan* p, int kind, hipStream_t st) {
	if (!p->timing) return BN_OK;
	hipEvent_t e;
	int rc = timing_event(p, &e);
	if (rc != BN_OK) return rc;
	BN_HIP(hipEventRecord(e, st));
	p->pending.push_back({kind, p->cur_begin, e});
	return BN_OK;
}
static int timing_resolve(bn_antt_plan* p) {
	for (const auto& q : p->pending) {
		BN_HIP(hipEventSynchronize(q.end));
		float ms = 0.f;
		BN_HIP(hipEventElapsedTime(&ms, q.begin, q.end));
		if ((int)p->kind_ms.size() < q.kind + 1) {
			p->kind_ms.resize(q.kind + 1, 0.f);
			p->kind_cnt.resize(q.kind + 1, 0);
		}
		p->kind_ms[q.kind] += ms;
		p->kind_cnt[q.kind] += 1;
		p->ev_pool.push_back(q.begin);
		p->ev_pool.push_back(q.end);
	}
	p->pending.clear();
	return BN_OK;
}

int launch_v0(bn_antt_plan* plan, const uint32_t* d_in, uint32_t* d_out, hipStream_t st) {
	const int log_h = plan->log_h;
	const int L = plan->limbs;
	int hi = log_h;
	bool first = true;
	int kind = 0;
	// balanced passes of <= kTileLog stages (an unbalanced tail would launch 2-point tiles)
	const int passes = (log_h + kTileLog - 1) / kTileLog;
	while (hi > 0) {
		const int k = (hi + (passes - kind) - 1) / (passes - kind);
		const int lo = hi - k;
		const int c = std::min(lo, kTileLog - k);
		V0Params p{d_in, d_out, plan->s_dev, plan->width, log_h, plan->log_rate, lo, k, c, first ? 1 : 0};
		const size_t blocks = ((size_t)1 << (log_h - k - c)) << plan->log_rate;
		const size_t lds = ((size_t)1 << (k + c)) * L * sizeof(uint32_t) + kGf8LdsBytes;
		const void* fn = L == 4 ? (const void*)antt_v0_group<4> : (const void*)antt_v0_group<1>;
		BN_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		int rc = timing_begin(plan, kind, st);
		if (rc != BN_OK) return rc;
		if (L == 4)
			hipLaunchKernelGGL(antt_v0_group<4>, dim3((unsigned)blocks), dim3(256), lds, st, p);
		else
			hipLaunchKernelGGL(antt_v0_group<1>, dim3((unsigned)blocks), dim3(256), lds, st, p);
		BN_HIP(hipGetLastError());
		rc = timing_end(plan, kind, st);
		if (rc != BN_OK) return rc;
		kind++;
		first = false;
		hi = lo;
	}
	return BN_OK;
}

// Bitsliced fast path (antt_bs.hip, antt_rr.hip), used when bs_supports(plan).
int launch_bs(bn_antt_plan* plan, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st);
bool bs_supports(const bn_antt_plan* plan);
int bs_prepare(bn_antt_plan* plan);
int bs_time_passes(bn_antt_plan* plan, const uint32_t* d_in, uint32_t* d_out, size_t batch, int reps,
                   hipStream_t st, float* ms, int max_passes, int* n_out);

// Kernel variants: 0 compact tiles (log_h < 12), 1 bitsliced LDS tiles (antt_bs_pass), 4 bitsliced
// register tiles (antt_rr_pass), 5 = 4 for the passes whose twiddles all lie in GF(2^8) and 1 for
// the others (the default for log_h >= 12).
static bool valid_variant(int v) { return v == 0 || v == 1 || v == 4 || v == 5; }

// development build only (make BN_DEV=1): BN_ANTT_VARIANT overrides the default kernel of new plans
static void dev_variant_override(bn_antt_plan* p) {
#ifdef BN_DEV
	if (const char* e = getenv("BN_ANTT_VARIANT")) {
		const int v = atoi(e);
		if (v != 0 && valid_variant(v)) p->variant = v;
	}
#else
	(void)p;
#endif
}

}  // namespace bn

using namespace bn;

extern "C" int bn_antt_plan_create(int device, int field_bits, int log_h, int log_rate, bn_antt_plan** out) {
	BN_CHECK_ARG(out != nullptr, "plan output pointer is NULL");
	*out = nullptr;
	BN_CHECK_ARG(field_bits == 32 || field_bits == 128, "field_bits must be 32 or 128 (got %d)", field_bits);
	BN_CHECK_ARG(log_h >= 1, "log_h must be >= 1 (got %d)", log_h);
	BN_CHECK_ARG(log_rate >= 0 && log_rate <= 4, "log_rate must be in [0,4] (got %d)", log_rate);
	BN_CHECK_ARG(log_h + log_rate <= field_bits, "log_h + log_rate must be <= %d", field_bits);
	if (log_h + log_rate > 32)
		BN_FAIL(BN_ERR_UNSUPPORTED, "log_h + log_rate > 32 is not built (every twiddle must lie in GF(2^32))");
	int ndev = 0;
	BN_HIP(hipGetDeviceCount(&ndev));
	BN_CHECK_ARG(device >= 0 && device < ndev, "device %d out of range (%d visible)", device, ndev);
	bn_antt_plan* p = new bn_antt_plan();
	p->device = device;
	p->field_bits = field_bits;
	p->log_h = log_h;
	p->log_rate = log_rate;
	p->limbs = field_bits / 32;
	p->width = log_h + log_rate - 1;
	subspace_evals(log_h, log_rate, p->s_host);
	int dev_prev = 0;
	(void)hipGetDevice(&dev_prev);
	hipError_t e = hipSetDevice(device);
	if (e == hipSuccess) e = hipMalloc(&p->s_dev, std::max<size_t>(p->s_host.size(), 1) * sizeof(uint32_t));
	if (e == hipSuccess && !p->s_host.empty())
		e = hipMemcpy(p->s_dev, p->s_host.data(), p->s_host.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
	if (e != hipSuccess) {
		(void)hipSetDevice(dev_prev);
		bn_antt_plan_destroy(p);
		BN_FAIL(BN_ERR_HIP, "plan allocation failed: %s", hipGetErrorString(e));
	}
	p->variant = 0;
	if (bs_supports(p)) {
		int rc = bs_prepare(p);
		if (rc == BN_OK) dev_variant_override(p);
		if (rc != BN_OK) {
			(void)hipSetDevice(dev_prev);
			bn_antt_plan_destroy(p);
			return rc;
		}
	}
	(void)hipSetDevice(dev_prev);
	*out = p;
	return BN_OK;
}

extern "C" int bn_antt_plan_destroy(bn_antt_plan* p) {
	if (!p) return BN_OK;
	int dev_prev = 0;
	(void)hipGetDevice(&dev_prev);
	(void)hipSetDevice(p->device);
	if (p->s_dev) (void)hipFree(p->s_dev);
	if (p->scratch) (void)hipFree(p->scratch);
	if (p->h_dev_in) (void)hipFree(p->h_dev_in);
	if (p->h_dev_out) (void)hipFree(p->h_dev_out);
	for (const auto& q : p->pending) {
		(void)hipEventSynchronize(q.end);
		(void)hipEventDestroy(q.begin);
		(void)hipEventDestroy(q.end);
	}
	for (auto e : p->ev_pool) (void)hipEventDestroy(e);
	if (p->own_stream) (void)hipStreamDestroy(p->own_stream);
	(void)hipSetDevice(dev_prev);
	delete p;
	return BN_OK;
}

static int forward_device_impl(bn_antt_plan* p, const void* d_in, void* d_out, size_t batch, hipStream_t st) {
	const size_t n_in = ((size_t)1 << p->log_h) * p->limbs;
	const size_t n_out = n_in << p->log_rate;
	if (p->variant != 0) return launch_bs(p, (const uint32_t*)d_in, (uint32_t*)d_out, batch, st);
	for (size_t b = 0; b < batch; b++) {
		int rc = launch_v0(p, (const uint32_t*)d_in + b * n_in, (uint32_t*)d_out + b * n_out, st);
		if (rc != BN_OK) return rc;
	}
	return BN_OK;
}

extern "C" int bn_antt_forward_device(bn_antt_plan* p, const void* d_in, void* d_out, size_t batch, void* stream) {
	BN_CHECK_ARG(p != nullptr, "plan is NULL");
	BN_CHECK_ARG(d_in != nullptr && d_out != nullptr, "device buffers must be non-NULL");
	BN_CHECK_ARG(batch >= 1, "batch must be >= 1");
	const size_t in_bytes = ((size_t)1 << p->log_h) * p->limbs * 4 * batch;
	const size_t out_bytes = in_bytes << p->log_rate;
	const char* a = (const char*)d_in;
	const char* b = (const char*)d_out;
	BN_CHECK_ARG(a + in_bytes <= b || b + out_bytes <= a, "d_in and d_out must not overlap");
	int dev_prev = 0;
	(void)hipGetDevice(&dev_prev);
	if (dev_prev != p->device) BN_HIP(hipSetDevice(p->device));
	int rc = forward_device_impl(p, d_in, d_out, batch, (hipStream_t)stream);
	if (dev_prev != p->device) (void)hipSetDevice(dev_prev);
	return rc;
}

// AdditiveNTT::apply (additive_ntt.cuh:201-265): host in -> host out, synchronous.
extern "C" int bn_antt_forward_host(bn_antt_plan* p, const void* in, size_t in_elems, void* out) {
	BN_CHECK_ARG(p != nullptr, "plan is NULL");
	BN_CHECK_ARG(in != nullptr && out != nullptr, "host buffers must be non-NULL");
	BN_CHECK_ARG(in_elems == ((size_t)1 << p->log_h), "input has %zu elements, plan expects 2^%d", in_elems, p->log_h);
	int dev_prev = 0;
	(void)hipGetDevice(&dev_prev);
	BN_HIP(hipSetDevice(p->device));
	const size_t in_bytes = in_elems * p->limbs * 4;
	const size_t out_bytes = in_bytes << p->log_rate;
	if (!p->h_dev_in) {
		BN_HIP(hipMalloc(&p->h_dev_in, in_bytes));
		BN_HIP(hipMalloc(&p->h_dev_out, out_bytes));
	}
	if (!p->own_stream) BN_HIP(hipStreamCreateWithFlags(&p->own_stream, hipStreamNonBlocking));
	BN_HIP(hipMemcpyAsync(p->h_dev_in, in, in_bytes, hipMemcpyHostToDevice, p->own_stream));
	int rc = forward_device_impl(p, p->h_dev_in, p->h_dev_out, 1, p->own_stream);
	if (rc != BN_OK) {
		(void)hipSetDevice(dev_prev);
		return rc;
	}
	BN_HIP(hipMemcpyAsync(out, p->h_dev_out, out_bytes, hipMemcpyDeviceToHost, p->own_stream));
	BN_HIP(hipStreamSynchronize(p->own_stream));
	(void)hipSetDevice(dev_prev);
	return BN_OK;
}

extern "C" int bn_antt_get_subspace_evals(const bn_antt_plan* p, uint32_t* out, size_t out_words) {
	BN_CHECK_ARG(p != nullptr && out != nullptr, "NULL argument");
	BN_CHECK_ARG(out_words >= (size_t)p->log_h * (size_t)p->width, "output too small");
	memcpy(out, p->s_host.data(), (size_t)p->log_h * (size_t)p->width * sizeof(uint32_t));
	return BN_OK;
}

extern "C" int bn_antt_plan_query(const bn_antt_plan* p, int what, int64_t* value) {
	BN_CHECK_ARG(p != nullptr && value != nullptr, "NULL argument");
	switch (what) {
		case 0: *value = p->log_h; break;
		case 1: *value = p->log_rate; break;
		case 2: *value = p->field_bits; break;
		case 3: *value = p->device; break;
		case 4: *value = p->variant; break;
		default: BN_FAIL(BN_ERR_INVALID, "unknown query %d", what);
	}
	return BN_OK;
}

extern "C" int bn_antt_plan_set_variant(bn_antt_plan* p, int variant) {
	BN_CHECK_ARG(p != nullptr, "plan is NULL");
	BN_CHECK_ARG(valid_variant(variant), "variant must be 0, 1, 4 or 5 (got %d)", variant);
	if (variant != 0 && !bs_supports(p)) BN_FAIL(BN_ERR_UNSUPPORTED, "variants 1, 4 and 5 need log_h >= 12");
	if (variant != 0 && p->variant == 0) {
		int prev = 0;
		(void)hipGetDevice(&prev);
		BN_HIP(hipSetDevice(p->device));
		const int rc = bs_prepare(p);
		(void)hipSetDevice(prev);
		if (rc != BN_OK) return rc;
	}
	p->variant = variant;
	return BN_OK;
}

extern "C" int bn_antt_set_event_timing(bn_antt_plan* p, int enable) {
	BN_CHECK_ARG(p != nullptr, "plan is NULL");
	int rc = timing_resolve(p);  // drop what an earlier timing window left
	if (rc != BN_OK) return rc;
	p->timing = enable;
	p->kind_ms.clear();
	p->kind_cnt.clear();
	return BN_OK;
}

extern "C" int bn_antt_time_passes(bn_antt_plan* p, const void* d_in, void* d_out, size_t batch, int reps,
                                   void* stream, float* ms_per_pass, int max_passes, int* n_passes) {
	BN_CHECK_ARG(p != nullptr && d_in != nullptr && d_out != nullptr && ms_per_pass != nullptr && n_passes != nullptr,
	             "NULL argument");
	BN_CHECK_ARG(batch >= 1 && reps >= 1, "batch and reps must be >= 1");
	if (p->variant == 0) BN_FAIL(BN_ERR_UNSUPPORTED, "pass timing is built for kernel variants 1, 4 and 5");
	int dev_prev = 0;
	(void)hipGetDevice(&dev_prev);
	if (dev_prev != p->device) BN_HIP(hipSetDevice(p->device));
	const int rc = bs_time_passes(p, (const uint32_t*)d_in, (uint32_t*)d_out, batch, reps, (hipStream_t)stream,
	                              ms_per_pass, max_passes, n_passes);
	if (dev_prev != p->device) (void)hipSetDevice(dev_prev);
	return rc;
}

extern "C" int bn_antt_pass_kernel_name(bn_antt_plan* p, int pass, char* buf, size_t cap) {
	BN_CHECK_ARG(p != nullptr && buf != nullptr && cap > 0, "NULL argument");
	const void* fn = p->variant != 0 ? bs_pass_kernel(p, pass) : nullptr;
	if (!fn) BN_FAIL(BN_ERR_UNSUPPORTED, "no kernel name for pass %d of variant %d", pass, p->variant);
	const char* mangled = hipKernelNameRefByPtr(fn, nullptr);
	if (!mangled) BN_FAIL(BN_ERR_HIP, "hipKernelNameRefByPtr failed");
	int st = 0;
	char* dem = abi::__cxa_demangle(mangled, nullptr, nullptr, &st);
	snprintf(buf, cap, "%s", (st == 0 && dem) ? dem : mangled);
	free(dem);
	return BN_OK;
}

extern "C" int bn_antt_get_event_timing(bn_antt_plan* p, float* ms, int max_kinds, int* n_kinds) {
	BN_CHECK_ARG(p != nullptr && n_kinds != nullptr, "NULL argument");
	int rc = timing_resolve(p);
	if (rc != BN_OK) return rc;
	*n_kinds = (int)p->kind_ms.size();
	for (int i = 0; i < *n_kinds && i < max_kinds; i++) ms[i] = p->kind_cnt[i] ? p->kind_ms[i] / p->kind_cnt[i] : 0.f;
	return BN_OK;
}
