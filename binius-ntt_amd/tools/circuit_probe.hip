// Dev microbenchmark (not part of the library): VALU issue rate of the generated GF(2^32)
// bitsliced multiply (bsm5_mul, 1022 gates / 32 products) with register-resident operands, at
// 1..4 waves per SIMD, one or two independent products interleaved per lane. Prints the achieved
// fraction of the SIMD's issue peak (one wave64 VALU instruction per 2 cycles).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../csrc tools/circuit_probe.hip -o tools/circuit_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "bitsliced_gen.hpp"

using namespace bn;

template <int ILP, int OCC>
__global__ __launch_bounds__(256, OCC) void kmul(uint32_t* d, int iters, unsigned long long* clk) {
	uint32_t V[ILP][32], W[32];
	const int t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
	for (int i = 0; i < 32; i++) {
		W[i] = (uint32_t)__builtin_amdgcn_sbfe(d[t] ^ (i * 0x9e3779b9u), i, 1);
#pragma unroll
		for (int j = 0; j < ILP; j++) V[j][i] = d[t] * (i + 1) + j;
	}
	const unsigned long long t0 = __builtin_amdgcn_s_memtime();
	for (int it = 0; it < iters; it++) {
#pragma unroll
		for (int j = 0; j < ILP; j++) bsm5_mul(V[j], W, V[j]);
		// the twiddle changes every iteration (else the compiler hoists its Karatsuba sums)
#pragma unroll
		for (int i = 0; i < 32; i++) W[i] ^= V[0][(i + 1) & 31];
	}
	const unsigned long long t1 = __builtin_amdgcn_s_memtime();
	uint32_t acc = 0;
#pragma unroll
	for (int i = 0; i < 32; i++)
#pragma unroll
		for (int j = 0; j < ILP; j++) acc ^= V[j][i];
	d[t] = acc;
	if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

int main() {
	int cus = 0;
	(void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
	uint32_t* d;
	unsigned long long* clk;
	(void)hipMalloc(&d, 256 * 4 * 4096);
	(void)hipMalloc(&clk, 8 * 4096);
	(void)hipMemset(d, 1, 256 * 4 * 4096);
	const int iters = 200;
	for (int ilp = 1; ilp <= 2; ilp++)
		for (int wps = 1; wps <= 4; wps++) {
			const int blocks = cus * wps;  // 256-thread blocks: one wave per SIMD each
			hipEvent_t e0, e1;
			(void)hipEventCreate(&e0);
			(void)hipEventCreate(&e1);
			for (int rep = 0; rep < 2; rep++) {
				(void)hipEventRecord(e0);
				const void* fns[2][4] = {{(const void*)kmul<1, 1>, (const void*)kmul<1, 2>, (const void*)kmul<1, 3>, (const void*)kmul<1, 4>},
				                         {(const void*)kmul<2, 1>, (const void*)kmul<2, 2>, (const void*)kmul<2, 3>, (const void*)kmul<2, 4>}};
				int it = iters;
				void* args[] = {&d, &it, &clk};
				(void)hipLaunchKernel(fns[ilp - 1][wps - 1], dim3(blocks), dim3(256), args, 0, 0);
				(void)hipEventRecord(e1);
				(void)hipEventSynchronize(e1);
			}
			float ms = 0;
			(void)hipEventElapsedTime(&ms, e0, e1);
			unsigned long long h[1];
			(void)hipMemcpy(h, clk, 8, hipMemcpyDeviceToHost);
			// wave-instructions: 1022 gates per product (plus loop overhead) per wave
			const double insts = (1022.0 * ilp + 32.0) * iters;
			const double cyc_per_wave_inst = (double)h[0] / insts;  // s_memtime ticks of one wave
			const double simd_frac = wps * 2.0 / cyc_per_wave_inst;  // SIMD issue share used
			printf("ILP %d, %d wave(s)/SIMD: %.2f ticks per VALU instruction per wave -> %.0f%% of SIMD issue peak (kernel %.3f ms)\n",
			       ilp, wps, cyc_per_wave_inst, 100.0 * simd_frac, ms);
		}
	return 0;
}
