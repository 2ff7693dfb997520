// Dev microbenchmark (not part of the library): the HBM cost of a 12-stage upper NTT pass over
// 2^24 GF(2^128) elements ("kill-test"). Such a pass owns tiles of 2^12 elements
// that differ in index bits 12..23, i.e. 16-byte elements 64 KiB apart. This copies 256 MiB with
// exactly that tile shape (all of a thread's loads in flight, through a 64 KiB LDS image, two
// work-groups per CU as the pass kernels run) and compares work-group -> tile maps:
//   contig      tile o = 4096 consecutive elements (what the current passes read: the baseline)
//   strided     tile o = elements o + 4096 t, t < 4096; block b takes tile b
//   xcdS        the same tiles, the S tiles of one 16*S-byte run (o = S k + j) on blocks
//               b, b+8, ..., b+8(S-1): one XCD under round-robin placement, dispatched together,
//               so the siblings' 16-byte pieces of a line can meet in that XCD's L2
//   rd-only / wr-only   strided on one side, contiguous on the other
//   pair        tiles of 2 x 4096 elements (index bit 0 plus bits 12..23: 32-byte pieces), 512
//               threads and 128 KiB of LDS, one work-group per CU
// Build: hipcc -O3 --offload-arch=gfx950 strided_copy.hip -o strided_copy
// Run:   ./strided_copy [reps]          (prints one JSON line per variant)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
	do {                                                                        \
		hipError_t e_ = (x);                                                    \
		if (e_ != hipSuccess) {                                                 \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
			exit(1);                                                            \
		}                                                                       \
	} while (0)

constexpr int kLogN = 24;
constexpr size_t kN = (size_t)1 << kLogN;  // elements (16 B each)
constexpr int kTile = 4096;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// tile id of block b under sibling grouping S (S = 1: identity)
__device__ __forceinline__ unsigned tile_of(unsigned b, int S) {
	if (S <= 1) return b;
	const unsigned xcd = b & 7, slot = b >> 3;
	const unsigned j = slot % S, kk = (slot / S) * 8 + xcd;
	return kk * S + j;
}

// MODE 0 contig, 1 strided both, 2 strided read only, 3 strided write only
template <int MODE, int S>
__global__ __launch_bounds__(256, 2) void copy_tile(const u32x4* __restrict__ in, u32x4* __restrict__ out) {
	extern __shared__ u32x4 img[];
	const unsigned o = tile_of(blockIdx.x, S);
	const int tid = threadIdx.x;
	auto addr = [&](int t, bool strided) -> size_t { return strided ? (size_t)o + (size_t)kTile * t : (size_t)o * kTile + t; };
	u32x4 g[16];
#pragma unroll
	for (int r = 0; r < 16; r++) g[r] = __builtin_nontemporal_load(in + addr(tid + 256 * r, MODE == 1 || MODE == 2));
#pragma unroll
	for (int r = 0; r < 16; r++) img[tid + 256 * r] = g[r];
	__syncthreads();
#pragma unroll
	for (int r = 0; r < 16; r++) {
		const int t = tid + 256 * r;
		__builtin_nontemporal_store(img[t], out + addr(t, MODE == 1 || MODE == 3));
	}
}

// pair tiles: index bit 0 and bits 12..23 (2 x 4096 elements), 512 threads, 128 KiB image
template <int S>
__global__ __launch_bounds__(512, 1) void copy_pair(const u32x4* __restrict__ in, u32x4* __restrict__ out) {
	extern __shared__ u32x4 img[];
	const unsigned o = tile_of(blockIdx.x, S);  // pair index: elements 2o, 2o+1 of every 8192-run
	const int tid = threadIdx.x;
	auto addr = [&](int u) -> size_t { return (size_t)2 * o + (u & 1) + (size_t)kTile * (u >> 1); };
	u32x4 g[16];
#pragma unroll
	for (int r = 0; r < 16; r++) g[r] = __builtin_nontemporal_load(in + addr(tid + 512 * r));
#pragma unroll
	for (int r = 0; r < 16; r++) img[tid + 512 * r] = g[r];
	__syncthreads();
#pragma unroll
	for (int r = 0; r < 16; r++) {
		const int u = tid + 512 * r;
		__builtin_nontemporal_store(img[u], out + addr(u));
	}
}

struct V {
	const char* name;
	const void* k;
	int threads;
	size_t lds;
	unsigned grid;
};

int main(int argc, char** argv) {
	const int reps = argc > 1 ? atoi(argv[1]) : 20;
	u32x4 *in, *out;
	CK(hipMalloc(&in, kN * 16));
	CK(hipMalloc(&out, kN * 16));
	CK(hipMemset(in, 1, kN * 16));
	CK(hipMemset(out, 0, kN * 16));
	const size_t lds1 = 72 * 1024, lds2 = 144 * 1024;  // the pass kernels' footprint: 2 / 1 work-groups per CU
	V vs[] = {
	    {"contig", (const void*)copy_tile<0, 1>, 256, lds1, kN / kTile},
	    {"strided", (const void*)copy_tile<1, 1>, 256, lds1, kN / kTile},
	    {"xcd2", (const void*)copy_tile<1, 2>, 256, lds1, kN / kTile},
	    {"xcd4", (const void*)copy_tile<1, 4>, 256, lds1, kN / kTile},
	    {"xcd8", (const void*)copy_tile<1, 8>, 256, lds1, kN / kTile},
	    {"xcd16", (const void*)copy_tile<1, 16>, 256, lds1, kN / kTile},
	    {"rd-only-xcd8", (const void*)copy_tile<2, 8>, 256, lds1, kN / kTile},
	    {"wr-only-xcd8", (const void*)copy_tile<3, 8>, 256, lds1, kN / kTile},
	    {"pair", (const void*)copy_pair<1>, 512, lds2, kN / (2 * kTile)},
	    {"pair-xcd4", (const void*)copy_pair<4>, 512, lds2, kN / (2 * kTile)},
	};
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	for (auto& v : vs) {
		CK(hipFuncSetAttribute(v.k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.lds));
		void* args[] = {&in, &out};
		for (int w = 0; w < 3; w++) CK(hipLaunchKernel(v.k, dim3(v.grid), dim3(v.threads), args, v.lds, 0));
		CK(hipEventRecord(a, 0));
		for (int r = 0; r < reps; r++) CK(hipLaunchKernel(v.k, dim3(v.grid), dim3(v.threads), args, v.lds, 0));
		CK(hipEventRecord(b, 0));
		CK(hipEventSynchronize(b));
		float ms = 0;
		CK(hipEventElapsedTime(&ms, a, b));
		const double t = ms / reps;
		const double bytes = 2.0 * kN * 16;
		printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.0f, \"frac_of_8TBps\": %.3f}\n", v.name, t, bytes / (t * 1e-3) / 1e9,
		       bytes / (t * 1e-3) / 8e12);
		fflush(stdout);
	}
	CK(hipDeviceSynchronize());
	printf("{\"done\": true}\n");
	return 0;
}
