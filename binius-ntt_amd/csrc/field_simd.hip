// Field primitives of the reference's finite_fields surface that sit beside the hot path:
//
//   multiply_unrolled<H>(a, b, dst)      circuit_generator/unrolled/binary_tower_unrolled.cuh:4-5
//       32 bitsliced GF(2^(2^H)) products (2^H words per operand, word i = bit i of the 32
//       elements), alias-safe (the sumcheck core multiplies in place, core.cu:21). Host and
//       device forms share the generated circuits (bitsliced_gen.hpp).
//   mul_binary_tower_32b_simd<H>(a, b)   binary_tower_simd.cuh:77-127
//       a 32-bit word read as 32 / 2^H packed GF(2^(2^H)) elements, multiplied lane by lane.
//   interleave_32b<H>(a, b), xor_adjacent_32b<H>(a)   binary_tower_simd.cuh:129-150
//       the 2^H-bit block shuffles the packed multiply is built from.
//
// The packed multiply here is a lane loop over the compact tower product (tower.hpp); it is a
// primitive for callers and tests, not part of the NTT / sumcheck kernels.
#include <hip/hip_runtime.h>

#include "bitsliced_gen.hpp"
#include "common.hpp"
#include "tower.hpp"

namespace bn {
namespace {

constexpr uint32_t kBlockMask[5] = {0x55555555u, 0x33333333u, 0x0f0f0f0fu, 0x00ff00ffu, 0x0000ffffu};

// Blocks of 2^h bits: c takes a's even blocks and b's even blocks shifted up (a's odd block
// positions); d takes a's odd blocks shifted down and b's odd blocks.
__host__ __device__ inline void interleave_blocks(int h, uint32_t a, uint32_t b, uint32_t* c, uint32_t* d) {
	const uint32_t m = kBlockMask[h];
	const int s = 1 << h;
	const uint32_t t = ((a >> s) ^ b) & m;
	*c = a ^ (t << s);
	*d = b ^ t;
}

// Each pair of adjacent 2^h-bit blocks replaced by their sum in both positions.
__host__ __device__ inline uint32_t xor_adjacent_blocks(int h, uint32_t a) {
	const uint32_t m = kBlockMask[h];
	const int s = 1 << h;
	const uint32_t t = ((a >> s) ^ a) & m;
	return t ^ (t << s);
}

// Lane-wise GF(2^(2^h)) product of two words of packed elements (0 <= h <= 5).
__host__ __device__ inline uint32_t packed_mul(int h, uint32_t a, uint32_t b) {
	const int w = 1 << h;
	const uint32_t m = w == 32 ? ~0u : ((1u << w) - 1u);
	uint32_t r = 0;
	for (int s = 0; s < 32; s += w) r |= (uint32_t)tw_mul((a >> s) & m, (b >> s) & m, h) << s;
	return r;
}

template <int H>
__host__ __device__ inline void unrolled(const uint32_t* a, const uint32_t* b, uint32_t* d) {
	if constexpr (H == 2)
		bsm2_mul(a, b, d);
	else if constexpr (H == 3)
		bsm3_mul(a, b, d);
	else if constexpr (H == 4)
		bsm4_mul(a, b, d);
	else if constexpr (H == 5)
		bsm5_mul(a, b, d);
	else if constexpr (H == 6)
		bsm6_mul(a, b, d);
	else
		bsm7_mul(a, b, d);
}

template <int H>
__global__ __launch_bounds__(256) void k_unrolled(const uint32_t* a, const uint32_t* b, uint32_t* o, size_t nblk) {
	constexpr int W = 1 << H;
	for (size_t blk = blockIdx.x * (size_t)blockDim.x + threadIdx.x; blk < nblk; blk += (size_t)gridDim.x * blockDim.x) {
		uint32_t x[W], y[W], z[W];
#pragma unroll
		for (int i = 0; i < W; i++) {
			x[i] = a[W * blk + i];
			y[i] = b[W * blk + i];
		}
		unrolled<H>(x, y, z);
#pragma unroll
		for (int i = 0; i < W; i++) o[W * blk + i] = z[i];
	}
}

__global__ __launch_bounds__(256) void k_packed(int op, int h, const uint32_t* a, const uint32_t* b, uint32_t* c, uint32_t* d,
                                                size_t n) {
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		if (op == 0) {
			c[i] = packed_mul(h, a[i], b[i]);
		} else if (op == 1) {
			uint32_t x, y;
			interleave_blocks(h, a[i], b[i], &x, &y);
			c[i] = x;
			d[i] = y;
		} else {
			c[i] = xor_adjacent_blocks(h, a[i]);
		}
	}
}

unsigned grid_for(size_t n) {
	size_t g = (n + 255) / 256;
	if (g > 65535u * 16u) g = 65535u * 16u;
	return (unsigned)(g ? g : 1);
}

}  // namespace
}  // namespace bn

using namespace bn;

int gf128_mul_bitsliced_launch(const void* a, const void* b, void* o, size_t nblk, hipStream_t st);  // field.hip

extern "C" int bn_multiply_unrolled(int height, const uint32_t* a, const uint32_t* b, uint32_t* dst) {
	BN_CHECK_ARG(a && b && dst, "NULL argument");
	BN_CHECK_ARG(height >= 2 && height <= 7, "height must be in [2, 7] (got %d)", height);
	switch (height) {
		case 2: unrolled<2>(a, b, dst); break;
		case 3: unrolled<3>(a, b, dst); break;
		case 4: unrolled<4>(a, b, dst); break;
		case 5: unrolled<5>(a, b, dst); break;
		case 6: unrolled<6>(a, b, dst); break;
		default: unrolled<7>(a, b, dst); break;
	}
	return BN_OK;
}

extern "C" int bn_multiply_unrolled_device(int height, const void* a, const void* b, void* dst, size_t nblocks,
                                           void* stream) {
	BN_CHECK_ARG(a && b && dst, "NULL device pointer");
	BN_CHECK_ARG(height >= 2 && height <= 7, "height must be in [2, 7] (got %d)", height);
	if (!nblocks) return BN_OK;
	// <7> (GF(2^128), the sumcheck's product) runs on the quad-lane product, like
	// bn_gf128_mul_bitsliced_device: one lane per 128-word block spills the 9712-gate circuit
	if (height == 7) return gf128_mul_bitsliced_launch(a, b, dst, nblocks, (hipStream_t)stream);
	const void* fns[5] = {(const void*)k_unrolled<2>, (const void*)k_unrolled<3>, (const void*)k_unrolled<4>,
	                      (const void*)k_unrolled<5>, (const void*)k_unrolled<6>};
	void* args[] = {&a, &b, &dst, &nblocks};
	BN_HIP(hipLaunchKernel(fns[height - 2], dim3(grid_for(nblocks)), dim3(256), args, 0, (hipStream_t)stream));
	return BN_OK;
}

extern "C" int bn_mul_binary_tower_32b_simd(int height, uint32_t a, uint32_t b, uint32_t* out) {
	BN_CHECK_ARG(out, "NULL argument");
	BN_CHECK_ARG(height >= 0 && height <= 5, "height must be in [0, 5] (got %d)", height);
	*out = packed_mul(height, a, b);
	return BN_OK;
}

extern "C" int bn_interleave_32b(int height, uint32_t a, uint32_t b, uint32_t* c, uint32_t* d) {
	BN_CHECK_ARG(c && d, "NULL argument");
	BN_CHECK_ARG(height >= 0 && height <= 4, "height must be in [0, 4] (got %d)", height);
	interleave_blocks(height, a, b, c, d);
	return BN_OK;
}

extern "C" int bn_xor_adjacent_32b(int height, uint32_t a, uint32_t* out) {
	BN_CHECK_ARG(out, "NULL argument");
	BN_CHECK_ARG(height >= 0 && height <= 4, "height must be in [0, 4] (got %d)", height);
	*out = xor_adjacent_blocks(height, a);
	return BN_OK;
}

extern "C" int bn_packed32_device(int op, int height, const void* a, const void* b, void* c, void* d, size_t n,
                                  void* stream) {
	BN_CHECK_ARG(op >= 0 && op <= 2, "op must be 0 (multiply), 1 (interleave) or 2 (xor_adjacent)");
	BN_CHECK_ARG(a && c && (op == 2 || b) && (op != 1 || d), "NULL device pointer");
	BN_CHECK_ARG(height >= 0 && height <= (op == 0 ? 5 : 4), "height out of range (got %d)", height);
	if (!n) return BN_OK;
	hipLaunchKernelGGL(k_packed, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, op, height, (const uint32_t*)a,
	                   (const uint32_t*)b, (uint32_t*)c, (uint32_t*)d, n);
	BN_HIP(hipGetLastError());
	return BN_OK;
}
