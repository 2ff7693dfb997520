// Dev microbenchmark: global access patterns for register-resident NTT tiles.
//  A: coalesced 16 B/lane (a wave-instruction covers 1 KiB contiguous)
//  B: lane-private 128 B lines (lane L reads line L of a 8 KiB span in 8 consecutive 16 B loads)
// Each wave copies 16 KiB (16 loads + 16 stores per lane) from src to dst. Not part of the library.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int MODE, int WPB>
__global__ __launch_bounds__(64 * WPB) void kcopy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int spin) {
	const size_t wave = (size_t)blockIdx.x * WPB + (threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	const size_t base = wave * 1024;  // 16 KiB per wave = 1024 x 16 B
	u32x4 r[16];
#pragma unroll
	for (int i = 0; i < 16; i++) {
		size_t idx = MODE == 0 ? base + i * 64 + lane : base + (i >> 3) * 512 + lane * 8 + (i & 7);
		r[i] = __builtin_nontemporal_load(src + idx);
	}
	// fake compute
	for (int s = 0; s < spin; s++) {
#pragma unroll
		for (int i = 0; i < 16; i++) r[i].x = __builtin_amdgcn_bitop3_b32(r[i].x, r[i].y, r[i].z, 0x96);
	}
#pragma unroll
	for (int i = 0; i < 16; i++) {
		size_t idx = MODE == 0 ? base + i * 64 + lane : base + (i >> 3) * 512 + lane * 8 + (i & 7);
		__builtin_nontemporal_store(r[i], dst + idx);
	}
}

int main() {
	const size_t bytes = 256ull << 20;
	u32x4 *a, *b;
	hipMalloc(&a, bytes);
	hipMalloc(&b, bytes);
	hipMemset(a, 1, bytes);
	hipMemset(b, 2, bytes);
	const size_t waves = bytes / 16384;
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	for (int spin : {0, 64, 256}) {
		for (int mode = 0; mode < 2; mode++) {
			auto k = mode == 0 ? kcopy<0, 1> : kcopy<1, 1>;
			hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, 0, a, b, spin);
			hipEventRecord(e0);
			for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, 0, a, b, spin);
			hipEventRecord(e1);
			hipEventSynchronize(e1);
			float ms;
			hipEventElapsedTime(&ms, e0, e1);
			ms /= 5;
			printf("spin %3d mode %s: %.3f ms, %.0f GB/s (read+write)\n", spin, mode == 0 ? "coalesced " : "lane-lines", ms,
			       2.0 * bytes / ms / 1e6);
		}
	}
	return 0;
}
