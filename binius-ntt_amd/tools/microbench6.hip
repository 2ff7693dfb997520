// Dev microbenchmark (not part of the library): cost of u ^= t * v on 32
// bitsliced GF(2^32) words when the twiddle t is wave-uniform.
//   var : the variable-operand Karatsuba circuit (bsm5_mul, 1022 gates) with the twiddle broadcast
//         into 32 mask words (v_bfe), as the NTT's block stages run it today
//   uni : bsm5_fma_uniform (tools/gen_uniform.py): 9 GF(2^8)-constant products by straight-line
//         code selected per constant with scalar branches + XOR3-fused pre/post sums
// Both run the same dependent butterfly chain (u ^= t v; v ^= u) with the same uniform twiddle
// sequence, so their final states must be bit-identical (checked). Prints lane-products/s and
// cycles per wave-product at 2, 3 and 4 waves per SIMD.
// Build: python3 gen_uniform.py && hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../csrc microbench6.hip -o microbench6
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#pragma clang diagnostic ignored "-Wunused-result"

#include "bitsliced_gen.hpp"
#include "uniform_gen.hpp"
#include "tower.hpp"

using namespace bn;

template <int MODE>
__device__ __forceinline__ uint32_t twiddle_at(const uint32_t* tws, int i) {
	// uniform per wave: every lane reads the same word (a scalar load), rotated per iteration;
	// MODE >= 2: each workgroup starts at its own offset, so co-resident waves take different
	// switch cases (the instruction-cache footprint of the real kernels)
	const int off = MODE >= 2 ? (int)blockIdx.x * 37 : 0;
	return __builtin_amdgcn_readfirstlane(tws[(i + off) & 255]);
}

// MODE 5/6: the product by a wave-uniform t as a GF(2)-linear map: output
// word i = XOR over the 8 input groups g of T_g[(row_i >> 4g) & 15], T_g = the 16 XOR combinations
// of input words 4g..4g+3 (88 XORs), row_i = bit i of t * 2^j over j (host table, scalar loads).
// T_g is a 16-element register array indexed by a uniform value: v_movrels with M0 (or the
// index mode), no scratch.
__device__ __forceinline__ void fourr_fma(const uint32_t* __restrict__ rows, const uint32_t* v, uint32_t* u) {
	uint32_t T0[16], T1[16], T2[16], T3[16], T4[16], T5[16], T6[16], T7[16];
	uint32_t* Ts[8] = {T0, T1, T2, T3, T4, T5, T6, T7};
#pragma unroll
	for (int g = 0; g < 8; g++) {
		uint32_t* T = Ts[g];
		T[0] = 0;
#pragma unroll
		for (int e = 1; e < 16; e++) {
			const int lb = 31 - __builtin_clz(e);  // highest set bit
			T[e] = (e == (1 << lb)) ? v[4 * g + lb] : (T[e & ~(1 << lb)] ^ v[4 * g + lb]);
		}
	}
#pragma unroll
	for (int i = 0; i < 32; i++) {
		const uint32_t r = __builtin_amdgcn_readfirstlane(rows[i]);
		uint32_t acc = 0;
#pragma unroll
		for (int g = 0; g < 8; g++) acc ^= Ts[g][(r >> (4 * g)) & 15u];
		u[i] ^= acc;
	}
}

template <int MODE>
__global__ __launch_bounds__(256) void k_chain(const uint32_t* __restrict__ tws, uint32_t* state, int iters,
                                               const uint32_t* __restrict__ rows = nullptr) {
	const int tid = blockIdx.x * 256 + threadIdx.x;
	uint32_t u[32], v[32];
#pragma unroll
	for (int i = 0; i < 32; i++) {
		u[i] = state[(size_t)tid * 64 + i];
		v[i] = state[(size_t)tid * 64 + 32 + i];
	}
#pragma unroll 1
	for (int it = 0; it < iters; it++) {
		// MODE 4: a per-lane twiddle (the NTT's block stages today): the t-side stays on the VALU
		const uint32_t t = MODE == 4 ? twiddle_at<0>(tws, it) ^ ((uint32_t)threadIdx.x * 0x9E3779B9u) : twiddle_at<MODE>(tws, it);
		if (MODE == 5 || MODE == 6) {
			const int off = MODE == 6 ? (int)blockIdx.x * 37 : 0;
			__builtin_amdgcn_sched_barrier(0);
			fourr_fma(rows + 32 * ((it + off) & 255), v, u);
			__builtin_amdgcn_sched_barrier(0);
		} else if (MODE == 0 || MODE == 2 || MODE == 4) {
			uint32_t W[32], P[32];
#pragma unroll
			for (int i = 0; i < 32; i++) W[i] = (uint32_t)__builtin_amdgcn_sbfe((int)t, i, 1);
			__builtin_amdgcn_sched_barrier(0);
			bsm5_mul(v, W, P);
			__builtin_amdgcn_sched_barrier(0);
#pragma unroll
			for (int i = 0; i < 32; i++) u[i] ^= P[i];
		} else {
			__builtin_amdgcn_sched_barrier(0);
			bsm5_fma_uniform(v, t, u);
			__builtin_amdgcn_sched_barrier(0);
		}
#pragma unroll
		for (int i = 0; i < 32; i++) v[i] ^= u[i];
	}
#pragma unroll
	for (int i = 0; i < 32; i++) {
		state[(size_t)tid * 64 + i] = u[i];
		state[(size_t)tid * 64 + 32 + i] = v[i];
	}
}

int main() {
	int cus = 0;
	hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
	uint32_t h_tw[256];
	uint32_t x = 0x12345678u;
	for (int i = 0; i < 256; i++) {
		x ^= x << 13, x ^= x >> 17, x ^= x << 5;
		h_tw[i] = x;
	}
	h_tw[7] = 0;  // a zero twiddle and a few sub-field ones
	h_tw[8] = 1;
	h_tw[9] = 0x5a;
	uint32_t* tws;
	hipMalloc(&tws, sizeof h_tw);
	hipMemcpy(tws, h_tw, sizeof h_tw, hipMemcpyHostToDevice);
	// the linear map of each twiddle: row i bit j = bit i of t * 2^j
	static uint32_t h_rows[256 * 32];
	for (int t = 0; t < 256; t++)
		for (int j = 0; j < 32; j++) {
			const uint32_t c = (uint32_t)tw_mul(h_tw[t], 1ull << j, 5);
			for (int i = 0; i < 32; i++) h_rows[32 * t + i] |= ((c >> i) & 1u) << j;
		}
	uint32_t* rows;
	hipMalloc(&rows, sizeof h_rows);
	hipMemcpy(rows, h_rows, sizeof h_rows, hipMemcpyHostToDevice);
	const size_t max_threads = (size_t)cus * 4 * 256;
	uint32_t *s0, *s1;
	hipMalloc(&s0, max_threads * 64 * 4);
	hipMalloc(&s1, max_threads * 64 * 4);
	uint32_t* h = (uint32_t*)malloc(max_threads * 64 * 4);
	uint32_t* h2 = (uint32_t*)malloc(max_threads * 64 * 4);
	for (size_t i = 0; i < max_threads * 64; i++) {
		x ^= x << 13, x ^= x >> 17, x ^= x << 5;
		h[i] = x;
	}
	// correctness: same chain, both forms (and the per-workgroup-offset pair)
	for (int pair = 0; pair < 4; pair++) {
		hipMemcpy(s0, h, max_threads * 256, hipMemcpyHostToDevice);
		hipMemcpy(s1, h, max_threads * 256, hipMemcpyHostToDevice);
		if (pair == 0 || pair == 2) {
			hipLaunchKernelGGL(k_chain<0>, dim3(cus), dim3(256), 0, 0, tws, s0, 300, rows);
			if (pair == 0) hipLaunchKernelGGL(k_chain<1>, dim3(cus), dim3(256), 0, 0, tws, s1, 300, rows);
			else hipLaunchKernelGGL(k_chain<5>, dim3(cus), dim3(256), 0, 0, tws, s1, 300, rows);
		} else {
			hipLaunchKernelGGL(k_chain<2>, dim3(cus), dim3(256), 0, 0, tws, s0, 300, rows);
			if (pair == 1) hipLaunchKernelGGL(k_chain<3>, dim3(cus), dim3(256), 0, 0, tws, s1, 300, rows);
			else hipLaunchKernelGGL(k_chain<6>, dim3(cus), dim3(256), 0, 0, tws, s1, 300, rows);
		}
		const hipError_t le = hipGetLastError(), se = hipDeviceSynchronize();
		if (le != hipSuccess || se != hipSuccess) {
			printf("launch error: %s / %s\n", hipGetErrorString(le), hipGetErrorString(se));
			return 1;
		}
		hipMemcpy(h2, s0, (size_t)cus * 256 * 256, hipMemcpyDeviceToHost);
		uint32_t* h3 = (uint32_t*)malloc((size_t)cus * 256 * 256);
		hipMemcpy(h3, s1, (size_t)cus * 256 * 256, hipMemcpyDeviceToHost);
		const bool same = memcmp(h3, h2, (size_t)cus * 256 * 256) == 0;
		if (!same) {
			size_t diff = 0, first = ~(size_t)0;
			for (size_t w = 0; w < (size_t)cus * 256 * 64; w++)
				if (h3[w] != h2[w]) diff++, first = first == ~(size_t)0 ? w : first;
			printf("  %zu of %zu words differ, first at word %zu (%08x vs %08x); unchanged input in the second: %d\n", diff,
			       (size_t)cus * 256 * 64, first, h2[first], h3[first], memcmp(h3, h, (size_t)cus * 256 * 256) == 0);
		}
		free(h3);
		printf("parity var vs %s, %s twiddles (300 dependent butterflies, %d lanes): %s\n", pair < 2 ? "uni" : "4R",
		       (pair & 1) ? "per-workgroup" : "chip-uniform", cus * 256, same ? "IDENTICAL" : "MISMATCH");
	}
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	const int iters = 2000;
	const char* names[7] = {"var (bsm5_mul + masks), same t", "uni (bsm5_fma_uniform), same t",
	                        "var, t per workgroup", "uni, t per workgroup", "var, t per lane (NTT today)",
	                        "4R (linear map, movrels), same t", "4R, t per workgroup"};
	for (int mode = 0; mode < 7; mode++) {
		printf("%-34s", names[mode]);
		for (int wps = 1; wps <= 4; wps++) {
			const int grid = cus * wps;
			auto launch = [&]() {
				if (mode == 0) hipLaunchKernelGGL(k_chain<0>, dim3(grid), dim3(256), 0, 0, tws, s0, iters);
				if (mode == 1) hipLaunchKernelGGL(k_chain<1>, dim3(grid), dim3(256), 0, 0, tws, s0, iters);
				if (mode == 2) hipLaunchKernelGGL(k_chain<2>, dim3(grid), dim3(256), 0, 0, tws, s0, iters);
				if (mode == 3) hipLaunchKernelGGL(k_chain<3>, dim3(grid), dim3(256), 0, 0, tws, s0, iters);
				if (mode == 4) hipLaunchKernelGGL(k_chain<4>, dim3(grid), dim3(256), 0, 0, tws, s0, iters);
				if (mode == 5) hipLaunchKernelGGL(k_chain<5>, dim3(grid), dim3(256), 0, 0, tws, s0, iters, rows);
				if (mode == 6) hipLaunchKernelGGL(k_chain<6>, dim3(grid), dim3(256), 0, 0, tws, s0, iters, rows);
			};
			launch();
			hipEventRecord(a);
			launch();
			hipEventRecord(b);
			hipEventSynchronize(b);
			float ms = 0;
			hipEventElapsedTime(&ms, a, b);
			const double prods = (double)grid * 256 * iters * 32;  // lane-level GF(2^32) products
			const double wave_prod = (double)grid * 4 * iters;      // wave-level 32-product units
			printf("  %dw: %.3g/s %5.0f cyc", wps, prods / (ms * 1e-3), ms * 1e-3 * 2.4e9 * cus * 4 / wave_prod);
		}
		printf("   (lane products/s, SIMD-cycles per wave-unit @2.4 GHz, 1..4 waves/SIMD)\n");
	}
	return 0;
}
