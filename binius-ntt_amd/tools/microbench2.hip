// Dev microbenchmark: VALU issue rate of dependent vs independent bitop3 chains at 1/2/4 waves
// per SIMD, and the bsm5 circuit at 1/2 waves per SIMD. Not part of the library.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "bitsliced.hpp"

using namespace bn;

template <int CHAINS>
__global__ __launch_bounds__(64) void kchain(uint32_t* data, int iters) {
	uint32_t x[CHAINS];
	const uint32_t y = data[threadIdx.x], z = data[threadIdx.x + 64];
#pragma unroll
	for (int c = 0; c < CHAINS; c++) x[c] = data[threadIdx.x + 128 + c];
	for (int it = 0; it < iters; it++) {
#pragma unroll
		for (int r = 0; r < 64 / CHAINS; r++) {
#pragma unroll
			for (int c = 0; c < CHAINS; c++) x[c] = __builtin_amdgcn_bitop3_b32(x[c], y, z, 0x96);
		}
	}
	uint32_t s = 0;
#pragma unroll
	for (int c = 0; c < CHAINS; c++) s ^= x[c];
	data[blockIdx.x * 64 + threadIdx.x + 4096] = s;
}

template <int OCC>
__global__ __launch_bounds__(256, OCC) void kbsm5(uint32_t* data, int iters) {
	uint32_t V[32], W[32], P[32];
	const size_t t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
	for (int i = 0; i < 32; i++) {
		V[i] = data[(t * 64 + i) & 0xffff];
		W[i] = data[(t * 64 + 32 + i) & 0xffff];
	}
	for (int it = 0; it < iters; it++) {
		bsm5_mul(V, W, P);
#pragma unroll
		for (int i = 0; i < 32; i++) V[i] ^= P[i];
	}
#pragma unroll
	for (int i = 0; i < 32; i++) data[0x10000 + t * 32 + i] = V[i];
}

static float timeit(void (*launch)(uint32_t*), uint32_t* d) {
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	launch(d);
	hipEventRecord(a);
	launch(d);
	hipEventRecord(b);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	return ms;
}

int main() {
	uint32_t* d;
	const size_t words = 64ull << 20;
	hipMalloc(&d, words * 4);
	hipMemset(d, 0x5a, words * 4);
	const int iters = 2000;
	// waves per SIMD = blocks / 1024 (one 64-thread block = one wave)
	for (int wps : {1, 2, 4}) {
		const int blocks = 1024 * wps;
		float t1 = 0, t8 = 0;
		{
			hipEvent_t a, b;
			hipEventCreate(&a);
			hipEventCreate(&b);
			hipLaunchKernelGGL(kchain<1>, dim3(blocks), dim3(64), 0, 0, d, iters);
			hipEventRecord(a);
			hipLaunchKernelGGL(kchain<1>, dim3(blocks), dim3(64), 0, 0, d, iters);
			hipEventRecord(b);
			hipEventSynchronize(b);
			hipEventElapsedTime(&t1, a, b);
			hipLaunchKernelGGL(kchain<8>, dim3(blocks), dim3(64), 0, 0, d, iters);
			hipEventRecord(a);
			hipLaunchKernelGGL(kchain<8>, dim3(blocks), dim3(64), 0, 0, d, iters);
			hipEventRecord(b);
			hipEventSynchronize(b);
			hipEventElapsedTime(&t8, a, b);
		}
		const double instrs = 64.0 * iters;  // per wave
		printf("waves/SIMD %d: dependent chain %.2f cyc/instr/wave, 8 chains %.2f cyc/instr/wave (2.4 GHz)\n", wps,
			   t1 * 1e-3 * 2.4e9 / instrs, t8 * 1e-3 * 2.4e9 / instrs);
	}
	for (int occ : {1, 2}) { // occupancies
		const int blocks = 256 * occ;  // 256 threads = 4 waves = 1 per SIMD per block
		hipEvent_t a, b;
		hipEventCreate(&a);
		hipEventCreate(&b);
		float ms;
		auto k = occ == 1 ? kbsm5<1> : kbsm5<2>;
		hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 100);
		hipEventRecord(a);
		hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 100);
		hipEventRecord(b);
		hipEventSynchronize(b);
		hipEventElapsedTime(&ms, a, b);
		const double instr_per_wave = 100.0 * (1022 + 32);
		printf("bsm5 at %d wave(s)/SIMD: %.2f cyc per circuit-instr per wave; SIMD VALU util %.1f%%\n", occ,
			   ms * 1e-3 * 2.4e9 / instr_per_wave, 100.0 * occ * 2.0 / (ms * 1e-3 * 2.4e9 / instr_per_wave));
	}
	return 0;
}
template __global__ void kbsm5<3>(uint32_t*, int);
template __global__ void kbsm5<4>(uint32_t*, int);
