// Dev microbenchmark (not part of the library): LDS cycles per ds_read_b128 / ds_write_b128 wave
// instruction for the per-lane address patterns of the NTT kernels (variant 3's swizzled planes,
// variant 1's padded planes), against the contiguous pattern. Eight waves on one CU each issue
// 64 back-to-back instructions of one pattern (LDS-bound); s_memtime brackets them.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../csrc tools/lds_probe.hip -o tools/lds_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <string>
#include <vector>

constexpr uint32_t kKey[4] = {0x74, 0x2A, 0x52, 0x2F};
static uint32_t par(uint32_t x) { return (uint32_t)__builtin_popcount(x) & 1u; }
static uint32_t sw_key(uint32_t q) {
	return par(q & kKey[0]) | (par(q & kKey[1]) << 1) | (par(q & kKey[2]) << 2) | (par(q & kKey[3]) << 3);
}
static uint32_t blk_byte(uint32_t q) { return 256u * (q >> 1) | 16u * sw_key(q); }
static int gpos(int K, int b) {
	return K == 1 ? (b == 0 ? 2 : b == 1 ? 0 : b == 2 ? 3 : b == 3 ? 1 : b == 4 ? 5 : 4)
	     : K == 2 ? (b == 0 ? 2 : b == 1 ? 0 : b == 2 ? 1 : b == 3 ? 5 : 3)
	              : (b == 0 ? 0 : b == 1 ? 5 : b == 2 ? 2 : 3);
}
static int spos(int K, int b) { return K == 2 ? 4 : (b == 0 ? 1 : 4); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int OP>
__global__ __launch_bounds__(512) void probe(const uint32_t* offs, unsigned long long* out, int reps) {
	__shared__ __attribute__((aligned(16))) uint32_t lds[16384];  // 64 KiB
	const int lane = threadIdx.x & 63;
	const uint32_t off = offs[lane];
	char* p = (char*)lds;
	u32x4 acc = {(unsigned)lane, 1u, 2u, 3u};
	for (int i = threadIdx.x; i < 16384; i += 512) lds[i] = i;
	__syncthreads();
	unsigned long long best = ~0ull;
	for (int rep = 0; rep < reps; rep++) {
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		__syncthreads();
		const unsigned long long t0 = __builtin_amdgcn_s_memtime();
		if (OP == 0) {
#pragma unroll
			for (int i = 0; i < 64; i++) {
				u32x4 v;
				asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(off), "i"((i & 3) * 4096) : "memory");
				acc.x ^= v.x;
			}
		} else {
#pragma unroll
			for (int i = 0; i < 64; i++)
				asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(off), "v"(acc), "i"((i & 3) * 4096) : "memory");
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		__syncthreads();
		const unsigned long long t1 = __builtin_amdgcn_s_memtime();
		if (t1 - t0 < best) best = t1 - t0;
	}
	if (threadIdx.x == 0) {
		out[blockIdx.x * 2] = best;
		out[blockIdx.x * 2 + 1] = acc.x;
	}
}

struct Pat {
	std::string name;
	std::vector<uint32_t> off;
};

int main() {
	std::vector<Pat> pats;
	{
		Pat p{"contiguous lane*16", {}};
		for (int l = 0; l < 64; l++) p.off.push_back(16 * l);
		pats.push_back(p);
		Pat q{"same address", std::vector<uint32_t>(64, 0)};
		pats.push_back(q);
		Pat s{"stride 128 B (8-way)", {}};
		for (int l = 0; l < 64; l++) s.off.push_back(128 * l % 16384);
		pats.push_back(s);
		Pat v1{"v1 padded rows, q = lane", {}};
		for (int l = 0; l < 64; l++) v1.off.push_back(144 * l);
		pats.push_back(v1);
	}
	// variant 3 rounds: every K and contiguous M; register block r = 0, chunk 0
	for (int K = 1; K <= 3; K++)
		for (int a = 0; a + K <= 7; a++) {
			int M[3];
			for (int i = 0; i < K; i++) M[i] = a + i;
			std::vector<int> fr;
			for (int m = 0; m < 7; m++) {
				bool in = false;
				for (int i = 0; i < K; i++) in |= M[i] == m;
				if (!in) fr.push_back(m);
			}
			for (int r : {0, (1 << K) - 1}) {
				Pat p{"v3 K=" + std::to_string(K) + " M0=" + std::to_string(a) + " r=" + std::to_string(r), {}};
				const int nch = (64 >> K) / 4;
				for (int l = 0; l < 64; l++) {
					uint32_t q = 0, s = 0;
					for (int b = 0; b < 7 - K; b++) q |= (uint32_t)((l >> gpos(K, b)) & 1) << fr[b];
					for (int b = 0; b < K - 1; b++) s |= (uint32_t)((l >> spos(K, b)) & 1) << b;
					for (int i = 0; i < K; i++) q |= (uint32_t)((r >> i) & 1) << M[i];
					p.off.push_back(blk_byte(q) ^ (16u * nch * s));
				}
				pats.push_back(p);
			}
		}
	{
		Pat p{"v3 tile load/store (q = u>>3, c = u&7)", {}};
		for (int l = 0; l < 64; l++) p.off.push_back(blk_byte((uint32_t)l >> 3) ^ (16u * (l & 7)));
		pats.push_back(p);
		Pat iw{"v3 in-word (x = lane&15, plane = lane>>4)", {}};
		for (int l = 0; l < 64; l++) iw.off.push_back(12288u * (uint32_t)(l >> 4) + blk_byte((uint32_t)(l & 15)));
		pats.push_back(iw);
	}
	uint32_t* d_off;
	unsigned long long* d_out;
	(void)hipMalloc(&d_off, 64 * 4);
	(void)hipMalloc(&d_out, 2 * 256 * 8);
	for (auto& p : pats) {
		(void)hipMemcpy(d_off, p.off.data(), 64 * 4, hipMemcpyHostToDevice);
		unsigned long long h[2];
		double cyc[2];
		for (int op = 0; op < 2; op++) {
			if (op == 0)
				hipLaunchKernelGGL(probe<0>, dim3(1), dim3(512), 0, 0, d_off, d_out, 8);
			else
				hipLaunchKernelGGL(probe<1>, dim3(1), dim3(512), 0, 0, d_off, d_out, 8);
			(void)hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
			cyc[op] = (double)h[0] / 512.0;
		}
		printf("%-48s read_b128 %6.1f  write_b128 %6.1f  (ticks per wave-instruction, 8 waves)\n", p.name.c_str(), cyc[0], cyc[1]);
	}
	return 0;
}
