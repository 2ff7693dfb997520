// Dev microbenchmark: VALU issue rate of independent v_bitop3_b32 / v_xor_b32 streams versus the
// VGPR bank of their operands (bank = register index mod 4) at 1-4 waves per SIMD.
// Not part of the library. Build: hipcc -O3 --offload-arch=gfx950 microbench4.hip -o /tmp/mb4
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP16(x) x x x x x x x x x x x x x x x x

// 32 independent instructions per iteration, sources in three different banks (v1, v2, v3),
// destinations cycling over v8..v39
#define B3_DIFF                                                                                   \
	"v_bitop3_b32 v8, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v9, v1, v2, v3 bitop3:0x96\n"         \
	"v_bitop3_b32 v10, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v11, v1, v2, v3 bitop3:0x96\n"
// sources all in bank 0 (v4, v12, v16)
#define B3_SAME                                                                                   \
	"v_bitop3_b32 v8, v4, v12, v16 bitop3:0x96\n v_bitop3_b32 v9, v4, v12, v16 bitop3:0x96\n"     \
	"v_bitop3_b32 v10, v4, v12, v16 bitop3:0x96\n v_bitop3_b32 v11, v4, v12, v16 bitop3:0x96\n"
// two sources in different banks
#define X2_DIFF "v_xor_b32 v8, v1, v2\n v_xor_b32 v9, v1, v2\n v_xor_b32 v10, v1, v2\n v_xor_b32 v11, v1, v2\n"
// dependent chain (each instruction reads the previous result)
#define B3_DEP                                                                                    \
	"v_bitop3_b32 v8, v8, v2, v3 bitop3:0x96\n v_bitop3_b32 v8, v8, v2, v3 bitop3:0x96\n"         \
	"v_bitop3_b32 v8, v8, v2, v3 bitop3:0x96\n v_bitop3_b32 v8, v8, v2, v3 bitop3:0x96\n"
// four independent chains interleaved
#define B3_DEP4                                                                                   \
	"v_bitop3_b32 v8, v8, v2, v3 bitop3:0x96\n v_bitop3_b32 v9, v9, v2, v3 bitop3:0x96\n"         \
	"v_bitop3_b32 v10, v10, v2, v3 bitop3:0x96\n v_bitop3_b32 v11, v11, v2, v3 bitop3:0x96\n"

#define KERNEL(name, body)                                                                        \
	__global__ __launch_bounds__(256) void name(unsigned* out, int iters) {                       \
		for (int i = 0; i < iters; i++) {                                                         \
			asm volatile(REP16(body) ::: "v1", "v2", "v3", "v4", "v8", "v9", "v10", "v11", "v12", "v16"); \
		}                                                                                         \
		if (threadIdx.x == 1000) out[0] = 1;                                                      \
	}

KERNEL(k_b3_diff, B3_DIFF)
KERNEL(k_b3_same, B3_SAME)
KERNEL(k_x2_diff, X2_DIFF)
KERNEL(k_b3_dep, B3_DEP)
KERNEL(k_b3_dep4, B3_DEP4)

int main() {
	unsigned* out;
	hipMalloc(&out, 64);
	int cus = 0;
	hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
	const int iters = 2000;
	const double insts_per_iter = 16 * 4;
	struct K {
		const char* name;
		void (*fn)(unsigned*, int);
	} ks[] = {{"bitop3 3 banks", k_b3_diff}, {"bitop3 same bank", k_b3_same}, {"xor 2 banks", k_x2_diff},
	          {"bitop3 dependent", k_b3_dep}, {"bitop3 4 chains", k_b3_dep4}};
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (auto& k : ks) {
		for (int wps = 1; wps <= 4; wps++) {
			// wps waves per SIMD: work-groups of 4 waves (one per SIMD), wps work-groups per CU
			const int grid = cus * wps;
			hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, out, iters);
			hipEventRecord(a);
			hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, out, iters);
			hipEventRecord(b);
			hipEventSynchronize(b);
			float ms = 0;
			hipEventElapsedTime(&ms, a, b);
			const double waves = (double)grid * 4;
			const double inst = waves * iters * insts_per_iter;
			const double per_simd_cycle = inst / (ms * 1e-3) / (cus * 4.0) / 2.4e9;
			printf("%-18s waves/SIMD %d: %.3f ms, %.3f wave-instr per SIMD-cycle (peak 0.5)\n", k.name, wps, ms, per_simd_cycle);
		}
	}
	return 0;
}
