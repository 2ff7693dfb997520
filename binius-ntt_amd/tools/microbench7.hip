// Dev microbenchmark (not part of the library; VERDICT r3 item 1a, second form): u ^= t v; v ^= u on
// 32 bitsliced GF(2^32) words with a wave-uniform twiddle t, as
//   var: the variable-operand Karatsuba circuit (bsm5_mul, 1022 gates) with t broadcast by v_bfe
//   4R : the GF(2)-linear map of t in hand-written asm (tools/gen_4r_asm.py): 8 tables of the 16
//        XOR combinations of 4 input words (120 VALU), then per output word 8 v_xor_b32 whose src0
//        is chosen by the GPR index mode from a host table (one s_set_gpr_idx_* per term)
// Both run the same dependent butterfly chain over 16 twiddles (cycled); the final states must be
// bit-identical. Prints SIMD-cycles per wave-unit (32 products) at 1..4 waves per SIMD.
// Build: python3 gen_4r_asm.py fourr_asm.hpp && hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../csrc microbench7.hip -o microbench7
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

#include "bitsliced_gen.hpp"
#include "tower.hpp"
#include "fourr_asm.hpp"

using namespace bn;

__global__ __launch_bounds__(256) void k_var(const uint32_t* __restrict__ tws, uint32_t* state, int iters) {
	const int tid = blockIdx.x * 256 + threadIdx.x;
	uint32_t u[32], v[32];
#pragma unroll
	for (int i = 0; i < 32; i++) {
		u[i] = state[(size_t)tid * 64 + i];
		v[i] = state[(size_t)tid * 64 + 32 + i];
	}
#pragma unroll 1
	for (int it = 0; it < iters; it++) {
		const uint32_t t = __builtin_amdgcn_readfirstlane(tws[it & 15]);
		uint32_t W[32], P[32];
#pragma unroll
		for (int i = 0; i < 32; i++) W[i] = (uint32_t)__builtin_amdgcn_sbfe((int)t, i, 1);
		__builtin_amdgcn_sched_barrier(0);
		bsm5_mul(v, W, P);
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int i = 0; i < 32; i++) u[i] ^= P[i];
#pragma unroll
		for (int i = 0; i < 32; i++) v[i] ^= u[i];
	}
#pragma unroll
	for (int i = 0; i < 32; i++) {
		state[(size_t)tid * 64 + i] = u[i];
		state[(size_t)tid * 64 + 32 + i] = v[i];
	}
}

__global__ __launch_bounds__(256) void k_4r(const uint32_t* __restrict__ idx, uint32_t* state, int iters) {
	const int tid = blockIdx.x * 256 + threadIdx.x;
	uint32_t* p = state + (size_t)tid * 64;
	asm volatile(FOURR_ASM_BODY : : "v"(p), "s"(idx), "s"(iters) : FOURR_ASM_CLOBBERS);
}

int main() {
	int cus = 0;
	hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
	uint32_t h_tw[16];
	uint32_t x = 0x12345678u;
	for (int i = 0; i < 16; i++) {
		x ^= x << 13, x ^= x >> 17, x ^= x << 5;
		h_tw[i] = x;
	}
	h_tw[3] = 0;
	h_tw[4] = 1;
	static uint32_t h_idx[16 * 256];
	for (int t = 0; t < 16; t++) {
		uint32_t rows[32] = {0};
		for (int j = 0; j < 32; j++) {
			const uint32_t c = (uint32_t)tw_mul(h_tw[t], 1ull << j, 5);
			for (int i = 0; i < 32; i++) rows[i] |= ((c >> i) & 1u) << j;
		}
		for (int i = 0; i < 32; i++)
			for (int g = 0; g < 8; g++) h_idx[256 * t + 8 * i + g] = 16 * g + ((rows[i] >> (4 * g)) & 15u);
	}
	uint32_t *tws, *idx;
	hipMalloc(&tws, sizeof h_tw);
	hipMemcpy(tws, h_tw, sizeof h_tw, hipMemcpyHostToDevice);
	hipMalloc(&idx, sizeof h_idx);
	hipMemcpy(idx, h_idx, sizeof h_idx, hipMemcpyHostToDevice);
	const size_t max_threads = (size_t)cus * 4 * 256;
	uint32_t *s0, *s1;
	hipMalloc(&s0, max_threads * 256);
	hipMalloc(&s1, max_threads * 256);
	uint32_t* h = (uint32_t*)malloc(max_threads * 256);
	uint32_t* h2 = (uint32_t*)malloc(max_threads * 256);
	uint32_t* h3 = (uint32_t*)malloc(max_threads * 256);
	for (size_t i = 0; i < max_threads * 64; i++) {
		x ^= x << 13, x ^= x >> 17, x ^= x << 5;
		h[i] = x;
	}
	hipMemcpy(s0, h, max_threads * 256, hipMemcpyHostToDevice);
	hipMemcpy(s1, h, max_threads * 256, hipMemcpyHostToDevice);
	hipLaunchKernelGGL(k_var, dim3(cus), dim3(256), 0, 0, tws, s0, 300);
	hipLaunchKernelGGL(k_4r, dim3(cus), dim3(256), 0, 0, idx, s1, 300);
	const hipError_t le = hipGetLastError(), se = hipDeviceSynchronize();
	if (le != hipSuccess || se != hipSuccess) {
		printf("launch error: %s / %s\n", hipGetErrorString(le), hipGetErrorString(se));
		return 1;
	}
	hipMemcpy(h2, s0, (size_t)cus * 256 * 256, hipMemcpyDeviceToHost);
	hipMemcpy(h3, s1, (size_t)cus * 256 * 256, hipMemcpyDeviceToHost);
	size_t diff = 0;
	for (size_t w = 0; w < (size_t)cus * 256 * 64; w++) diff += h2[w] != h3[w];
	printf("parity var vs 4R-asm (300 dependent butterflies, %d lanes): %s (%zu words differ)\n", cus * 256,
	       diff ? "MISMATCH" : "IDENTICAL", diff);
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	const int iters = 2000;
	const char* names[2] = {"var (bsm5_mul + masks)", "4R asm (linear map, GPR index)"};
	for (int mode = 0; mode < 2; mode++) {
		printf("%-32s", names[mode]);
		for (int wps = 1; wps <= 4; wps++) {
			const int grid = cus * wps;
			auto launch = [&]() {
				if (mode == 0) hipLaunchKernelGGL(k_var, dim3(grid), dim3(256), 0, 0, tws, s0, iters);
				else hipLaunchKernelGGL(k_4r, dim3(grid), dim3(256), 0, 0, idx, s1, iters);
			};
			launch();
			hipEventRecord(a);
			launch();
			hipEventRecord(b);
			hipEventSynchronize(b);
			float ms = 0;
			hipEventElapsedTime(&ms, a, b);
			const double wave_prod = (double)grid * 4 * iters;
			printf("  %dw: %5.0f cyc", wps, ms * 1e-3 * 2.4e9 * cus * 4 / wave_prod);
		}
		printf("   (SIMD-cycles per 32-product wave unit @2.4 GHz, 1..4 waves/SIMD)\n");
	}
	return diff ? 1 : 0;
}
