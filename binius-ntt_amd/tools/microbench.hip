// Standalone VALU-throughput microbenchmark for the bitsliced multiply circuits (dev tool,
// not part of the library). Each thread keeps 32 words of data + 32 twiddle words in
// registers and applies the circuit `iters` times; reports gates/s and lane-op utilisation.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "bitsliced.hpp"

using namespace bn;

template <int KIND>
__global__ __launch_bounds__(256, 2) void kbench(uint32_t* data, int iters) {
	uint32_t V[32], W[32], P[32];
	const size_t t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
	for (int i = 0; i < 32; i++) {
		V[i] = data[t * 64 + i];
		W[i] = data[t * 64 + 32 + i];
	}
	for (int it = 0; it < iters; it++) {
		if (KIND == 5) bsm5_mul(V, W, P);
		if (KIND == 4) {
			bsm4_mul(V, W, P);
			bsm4_mul(V + 16, W, P + 16);
		}
		if (KIND == 3) {
#pragma unroll
			for (int g = 0; g < 4; g++) bsm3_mul(V + 8 * g, W, P + 8 * g);
		}
#pragma unroll
		for (int i = 0; i < 32; i++) V[i] ^= P[i];
	}
#pragma unroll
	for (int i = 0; i < 32; i++) data[t * 64 + i] = V[i];
}

int main(int argc, char** argv) {
	const int blocks = argc > 1 ? atoi(argv[1]) : 512;
	const int iters = argc > 2 ? atoi(argv[2]) : 200;
	uint32_t* d;
	hipMalloc(&d, (size_t)blocks * 256 * 64 * 4);
	hipMemset(d, 0x5a, (size_t)blocks * 256 * 64 * 4);
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	const int gates[3] = {4 * 93 + 32, 2 * 316 + 32, 1022 + 32};
	for (int kind = 3; kind <= 5; kind++) {
		for (int rep = 0; rep < 2; rep++) {
			hipEventRecord(a);
			if (kind == 3) hipLaunchKernelGGL(kbench<3>, dim3(blocks), dim3(256), 0, 0, d, iters);
			if (kind == 4) hipLaunchKernelGGL(kbench<4>, dim3(blocks), dim3(256), 0, 0, d, iters);
			if (kind == 5) hipLaunchKernelGGL(kbench<5>, dim3(blocks), dim3(256), 0, 0, d, iters);
			hipEventRecord(b);
			hipEventSynchronize(b);
			float ms;
			hipEventElapsedTime(&ms, a, b);
			const double ops = (double)blocks * 256 * iters * gates[kind - 3];
			if (rep) printf("GF(2^%d) twiddle circuit: %.3f ms, %.2f T lane-ops/s (%.1f%% of 78.6T), %.2f G limb-products/s\n",
							1 << kind, ms, ops / ms / 1e9, 100.0 * ops / ms / 1e9 / 78.6,
							(double)blocks * 256 * iters * 32 / ms / 1e6);
		}
	}
	return 0;
}
