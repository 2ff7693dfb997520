// Tower-field kernels behind the C-ABI: elementwise compact GF(2^32)/GF(2^128) products,
// compact <-> bitsliced conversion, bitsliced GF(2^128) products and the register-resident
// repeat-loop microbenchmarks (config 2).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.hpp"
#include "field_dev.hpp"
#include "bitsliced.hpp"
#include "quad_mul.hpp"

namespace bn {

// Compact products: Karatsuba down to GF(2^8), whose products are log/exp lookups in LDS.
__global__ __launch_bounds__(256) void k_gf32_mul(const uint32_t* a, const uint32_t* b, uint32_t* o, size_t n) {
	__shared__ uint8_t tab[kGf8LdsBytes];
	gf8_tables_to_lds(tab);
	__syncthreads();
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		o[i] = (uint32_t)dmul_t<5>(a[i], b[i], tab);
}

// Elementwise compact GF(2^128) products (bn_gf128_mul_device) on the quad-lane bitsliced product:
// a wave reads 512 consecutive compact elements of each operand (16-byte coalesced loads) into the
// LDS slots of its 16 quads, element e of quad q's block into word e of rows c (limb c of a) and
// 4 + c (of b). Lane l of the quad then turns rows l and 4 + l into limb planes with one 32x32 bit
// transpose each (bitsliced word i, bit e = bit i of limb l of element e), runs quad_mul, transposes
// the product's row back, and the wave writes 512 compact products. Per product that is ~96
// lane-instructions of transposes on top of the quad product's ~435, against ~1360 for the
// per-lane log/exp Karatsuba of dmul128_t (still the compact repeat microbenchmark, kind 0).
// Every operand of a wave is in LDS before any product is stored: alias-safe (o == a or o == b).
__global__ __launch_bounds__(256, 2) void k_gf128_mul(const uint4* a, const uint4* b, uint4* o, size_t n) {
	extern __shared__ uint32_t lds[];
	const int t = threadIdx.x & 63, w = threadIdx.x >> 6;
	const int l = threadIdx.x & 3, qw = threadIdx.x >> 2;
	const size_t e0 = ((size_t)blockIdx.x * 64 + 16 * w) * 32;  // the wave's first element
	if (e0 >= n) return;                                        // uniform per wave
	uint32_t* const wl = lds + 16 * w * quad::kQuadWords;
	{
		uint4 ga[8], gb[8];
#pragma unroll
		for (int i = 0; i < 8; i++) {
			const size_t e = e0 + 64 * i + t;
			ga[i] = e < n ? a[e] : make_uint4(0, 0, 0, 0);
			gb[i] = e < n ? b[e] : make_uint4(0, 0, 0, 0);
		}
#pragma unroll
		for (int i = 0; i < 8; i++) {
			const int el = 64 * i + t;
			uint32_t* const r = wl + (el >> 5) * quad::kQuadWords + (el & 31);
			r[0] = ga[i].x, r[quad::kRowWords] = ga[i].y, r[2 * quad::kRowWords] = ga[i].z, r[3 * quad::kRowWords] = ga[i].w;
			r[4 * quad::kRowWords] = gb[i].x, r[5 * quad::kRowWords] = gb[i].y;
			r[6 * quad::kRowWords] = gb[i].z, r[7 * quad::kRowWords] = gb[i].w;
		}
	}
	quad::wsync();
	const quad::Slot S{lds + qw * quad::kQuadWords};
	uint32_t x[32];
#pragma unroll
	for (int h = 0; h < 2; h++) {
		quad::sld(x, S, 4 * h + l);
		transpose32(x);
		quad::sst(S, 4 * h + l, x);
	}
	quad::quad_mul<false>(S, nullptr, l);  // row l <- (rows 0..3) * (rows 4..7)
	quad::sld(x, S, l);
	transpose32(x);
	quad::sst(S, l, x);
	quad::wsync();
#pragma unroll
	for (int i = 0; i < 8; i++) {
		const int el = 64 * i + t;
		const size_t e = e0 + el;
		const uint32_t* const r = wl + (el >> 5) * quad::kQuadWords + (el & 31);
		if (e < n) o[e] = make_uint4(r[0], r[quad::kRowWords], r[2 * quad::kRowWords], r[3 * quad::kRowWords]);
	}
}

// Compact <-> bitsliced 128-word blocks (transpose_kernel / untranspose_kernel,
// src/ulvt/utils/bitslicing.cuh:89-105), in place (src == dst) or between disjoint buffers. A wave owns 16 consecutive blocks (8 KiB): it
// reads them with 16-byte coalesced loads into 16 LDS slots of four 32-word rows (row l = limb l of
// the block's 32 elements, or limb plane l), lane l of quad q bit-transposes row l of block q in
// registers (one 32x32 transpose), and the wave writes the 8 KiB back with coalesced stores. Every
// block of a wave is read before any is written. (The one-thread-per-block form held 128 words per
// lane at one wave per SIMD: 1.6-2.2 TB/s.)
constexpr int kBsSlotWords = 4 * quad::kRowWords;  // one block: four padded rows
__global__ __launch_bounds__(256) void k_bitslice(const uint32_t* src, uint32_t* dst, size_t nblk, int untranspose) {
	extern __shared__ uint32_t lds[];
	const int t = threadIdx.x & 63, w = threadIdx.x >> 6, l = threadIdx.x & 3, q = (threadIdx.x >> 2) & 15;
	const size_t b0 = ((size_t)blockIdx.x * 4 + w) * 16;  // the wave's first block
	if (b0 >= nblk) return;                                // uniform per wave
	uint32_t* const wl = lds + w * 16 * kBsSlotWords;
	const uint4* const p = (const uint4*)(src + 128 * b0);
	uint4* const o = (uint4*)(dst + 128 * b0);
	const int nvec = (int)(std::min<size_t>(16, nblk - b0) * 32);  // 16-byte words of the wave's blocks
	constexpr int R = quad::kRowWords;
	uint4 g[8];
#pragma unroll
	for (int i = 0; i < 8; i++) {
		const int idx = 64 * i + t;
		g[i] = idx < nvec ? p[idx] : make_uint4(0, 0, 0, 0);
	}
#pragma unroll
	for (int i = 0; i < 8; i++) {
		const int idx = 64 * i + t, j = idx & 31;
		uint32_t* const sl = wl + (idx >> 5) * kBsSlotWords;
		if (!untranspose) {  // compact: 16-byte word j = element j -> word j of rows 0..3
			sl[j] = g[i].x, sl[R + j] = g[i].y, sl[2 * R + j] = g[i].z, sl[3 * R + j] = g[i].w;
		} else {  // bitsliced: words 4j..4j+3 of the block = row j / 8, words 4 (j % 8) ..
			*(uint4*)(sl + (j >> 3) * R + 4 * (j & 7)) = g[i];
		}
	}
	quad::wsync();
	uint32_t x[32];
	uint32_t* const row = wl + q * kBsSlotWords + l * R;
	quad::ld32(x, row);
	transpose32(x);
	quad::st32(row, x);
	quad::wsync();
#pragma unroll
	for (int i = 0; i < 8; i++) {
		const int idx = 64 * i + t, j = idx & 31;
		const uint32_t* const sl = wl + (idx >> 5) * kBsSlotWords;
		if (idx < nvec)
			o[idx] = untranspose ? make_uint4(sl[j], sl[R + j], sl[2 * R + j], sl[3 * R + j])
			                     : *(const uint4*)(sl + (j >> 3) * R + 4 * (j & 7));
	}
}

// Bitsliced GF(2^128) products o = a * b, 32 per 128-word block (multiply_unrolled<7>,
// circuit_generator/unrolled/binary_tower_unrolled7.cu:6), on the quad-lane product of
// quad_mul.hpp: block b runs on the 4 lanes of one quad (lane l loads limb l of both operands into
// the quad's LDS slot and stores limb l of the product), so no lane holds more than ~4 x 32 words.
// One block per quad and no loop: a persistent grid that prefetched the next block's operands
// kept them live across the product, and the spills (432 B/lane) made it 1.9x slower (3.4e10 vs
// 6.2-6.5e10 products/s). Every operand word is read into the slot before any
// output word is written: alias-safe for o == a or o == b (core.cu:21).
__global__ __launch_bounds__(256, 2) void k_gf128_mul_bs(const uint32_t* a, const uint32_t* b, uint32_t* o, size_t nblk) {
	extern __shared__ uint32_t lds[];
	const int l = threadIdx.x & 3, qw = threadIdx.x >> 2;
	const quad::Slot S{lds + qw * quad::kQuadWords};
	const size_t blk = (size_t)blockIdx.x * 64 + qw;  // uniform per quad
	if (blk >= nblk) return;                          // whole quads leave together
	uint32_t x[32];
	quad::ld32(x, a + 128 * blk + 32 * l);
	quad::sst(S, l, x);
	quad::ld32(x, b + 128 * blk + 32 * l);
	quad::sst(S, 4 + l, x);
	quad::quad_mul<false>(S, nullptr, l);  // row l <- (rows 0..3) * (rows 4..7)
	quad::sld(x, S, l);
	quad::st32(o + 128 * blk + 32 * l, x);
}
static size_t quad_lds_bytes();

// bitsliced_repeat-style microbenchmarks (src/ulvt/finite_fields/tests/profiling/kernels/
// bitsliced_repeat.cu:5-32): `iters` dependent products per lane, operands register-resident.
__global__ __launch_bounds__(256) void k_repeat_compact(uint4* state, const uint4* operand, size_t threads, int iters) {
	__shared__ uint8_t tab[kGf8LdsBytes];
	gf8_tables_to_lds(tab);
	__syncthreads();
	const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
	if (t >= threads) return;
	uint4 x = state[t];
	const uint4 y = operand[t];
	for (int i = 0; i < iters; i++) x = dmul128_t(x, y, tab);
	state[t] = x;
}

__global__ __launch_bounds__(256) void k_repeat_bitsliced(uint32_t* state, const uint32_t* operand, size_t threads, int iters) {
	const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
	if (t >= threads) return;
	uint32_t x[128], y[128];
#pragma unroll
	for (int i = 0; i < 128; i++) {
		x[i] = state[128 * t + i];
		y[i] = operand[128 * t + i];
	}
	for (int it = 0; it < iters; it++) bs_mul128(x, y, x);
#pragma unroll
	for (int i = 0; i < 128; i++) state[128 * t + i] = x[i];
}

// kind 2: the same bitsliced repeat loop on the sumcheck's quad-lane product (quad_mul.hpp): block
// b's 128 words are spread over the 4 lanes of quad b (lane l holds limb l), operands and partial
// products go through the quad's LDS slot, so no lane holds more than ~4 x 32 words of field data.
__global__ __launch_bounds__(256, 2) void k_repeat_quad(uint32_t* state, const uint32_t* operand, size_t blocks, int iters) {
	extern __shared__ uint32_t lds[];
	const int l = threadIdx.x & 3, qw = threadIdx.x >> 2;
	const quad::Slot S{lds + qw * quad::kQuadWords};
	const size_t b = (size_t)blockIdx.x * 64 + qw;
	if (b >= blocks) return;  // whole quads leave together (b is uniform per quad)
	uint32_t x[32], y[32];
	quad::ld32(x, state + 128 * b + 32 * l);
	quad::ld32(y, operand + 128 * b + 32 * l);
	quad::sst(S, l, x);
	for (int it = 0; it < iters; it++) {
		quad::sst(S, 4 + l, y);
		quad::quad_mul<false>(S, nullptr, l);  // row l <- (rows 0..3) * (rows 4..7)
	}
	quad::wsync();
	quad::sld(x, S, l);
	quad::st32(state + 128 * b + 32 * l, x);
}
static size_t quad_lds_bytes() { return (size_t)64 * quad::kQuadWords * sizeof(uint32_t); }

static unsigned grid_for(size_t n, unsigned block) {
	size_t g = (n + block - 1) / block;
	if (g > 65535u * 16u) g = 65535u * 16u;
	return (unsigned)(g ? g : 1);
}

}  // namespace bn

using namespace bn;

extern "C" int bn_gf32_mul_device(const void* a, const void* b, void* o, size_t n, void* stream) {
	BN_CHECK_ARG(a && b && o, "NULL device pointer");
	if (!n) return BN_OK;
	hipLaunchKernelGGL(k_gf32_mul, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, (const uint32_t*)a,
					   (const uint32_t*)b, (uint32_t*)o, n);
	BN_HIP(hipGetLastError());
	return BN_OK;
}


// nblk blocks from src to dst (the same buffer, or disjoint ones); also the sumcheck's compact-input
// constructor, which transposes the caller's columns straight into the prover's storage
int bitslice_launch(const void* src, void* dst, size_t nblk, int untranspose, hipStream_t st) {
	if (!nblk) return BN_OK;
	// 64 blocks per work-group (16 per wave), 36.9 KB of LDS
	const size_t grid = (nblk + 63) / 64;
	BN_CHECK_ARG(grid <= 0x7fffffffu, "too many blocks for one launch");
	hipLaunchKernelGGL(k_bitslice, dim3((unsigned)grid), dim3(256), (size_t)64 * kBsSlotWords * sizeof(uint32_t), st,
	                   (const uint32_t*)src, (uint32_t*)dst, nblk, untranspose);
	BN_HIP(hipGetLastError());
	return BN_OK;
}

extern "C" int bn_bitslice_device(void* buf, size_t nblk, int untranspose, void* stream) {
	BN_CHECK_ARG(buf, "NULL device pointer");
	return bitslice_launch(buf, buf, nblk, untranspose, (hipStream_t)stream);
}

// quad-slot LDS (78 KB) above the 64 KB default: the attribute is set on the current device
// before every launch (cheap, and correct when the caller switches devices)
static int quad_kernel_attr(const void* fn) {
	BN_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)quad_lds_bytes()));
	return BN_OK;
}

extern "C" int bn_gf128_mul_device(const void* a, const void* b, void* o, size_t n, void* stream) {
	BN_CHECK_ARG(a && b && o, "NULL device pointer");
	if (!n) return BN_OK;
	int rc = quad_kernel_attr((const void*)k_gf128_mul);
	if (rc != BN_OK) return rc;
	// 2048 elements per work-group: 64 quads of 32
	const size_t grid = (n + 2047) / 2048;
	BN_CHECK_ARG(grid <= 0x7fffffffu, "too many elements for one launch");
	hipLaunchKernelGGL(k_gf128_mul, dim3((unsigned)grid), dim3(256), quad_lds_bytes(), (hipStream_t)stream, (const uint4*)a,
	                   (const uint4*)b, (uint4*)o, n);
	BN_HIP(hipGetLastError());
	return BN_OK;
}

int gf128_mul_bitsliced_launch(const void* a, const void* b, void* o, size_t nblk, hipStream_t st) {
	if (!nblk) return BN_OK;
	int rc = quad_kernel_attr((const void*)k_gf128_mul_bs);
	if (rc != BN_OK) return rc;
	// 64 blocks per work-group, one per quad
	const size_t grid = (nblk + 63) / 64;
	BN_CHECK_ARG(grid <= 0x7fffffffu, "too many blocks for one launch");
	hipLaunchKernelGGL(k_gf128_mul_bs, dim3((unsigned)grid), dim3(256), quad_lds_bytes(), st, (const uint32_t*)a,
	                   (const uint32_t*)b, (uint32_t*)o, nblk);
	BN_HIP(hipGetLastError());
	return BN_OK;
}

extern "C" int bn_gf128_mul_bitsliced_device(const void* a, const void* b, void* o, size_t nblk, void* stream) {
	BN_CHECK_ARG(a && b && o, "NULL device pointer");
	return gf128_mul_bitsliced_launch(a, b, o, nblk, (hipStream_t)stream);
}

extern "C" int bn_gf128_mul_repeat_device(int kind, void* state, const void* operand, size_t threads, int iters,
										  void* stream) {
	BN_CHECK_ARG(state && operand, "NULL device pointer");
	BN_CHECK_ARG(kind >= 0 && kind <= 2, "kind must be 0 (compact), 1 (bitsliced) or 2 (bitsliced, quad-lane product)");
	BN_CHECK_ARG(iters >= 0, "iters must be >= 0");
	if (!threads) return BN_OK;
	const unsigned grid = (unsigned)((threads + 255) / 256);
	if (kind == 2) {
		int rc = quad_kernel_attr((const void*)k_repeat_quad);
		if (rc != BN_OK) return rc;
		hipLaunchKernelGGL(k_repeat_quad, dim3((unsigned)((threads + 63) / 64)), dim3(256), quad_lds_bytes(),
		                   (hipStream_t)stream, (uint32_t*)state, (const uint32_t*)operand, threads, iters);
	} else if (kind == 0)
		hipLaunchKernelGGL(k_repeat_compact, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint4*)state,
						   (const uint4*)operand, threads, iters);
	else
		hipLaunchKernelGGL(k_repeat_bitsliced, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint32_t*)state,
						   (const uint32_t*)operand, threads, iters);
	BN_HIP(hipGetLastError());
	return BN_OK;
}
