// Host-side check of the generated constant-operand circuits: bsm6_fma_w2 (the sumcheck fold's
// lane-pair product, sc_fold_pair in binius-ntt_amd/csrc/sumcheck.hip; 32 bitsliced GF(2^64)
// elements a_e times a constant w = w0 + w1 X, accumulated into out, against the oracle's tower
// product orc_mul(a_e, w, 6), oracle/tower.c), bsm5_fma_tw and bsm5_mul_w (the NTT's per-lane and
// scalar twiddle products). The circuits are __host__ __device__, so the host
// build runs exactly the gate list the kernel runs. Prints "ok" or "FAIL ..." lines.
#include <stdint.h>
#include <stdio.h>

#include "bitsliced_gen.hpp"

extern "C" {
void orc_init(void);
uint64_t orc_mul(uint64_t a, uint64_t b, int h);
}

static uint64_t next(uint64_t& s) {  // splitmix64
	uint64_t z = (s += 0x9E3779B97F4A7C15ull);
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

int main() {
	orc_init();
	uint64_t seed = 12345;
	int fails = 0;
	for (int trial = 0; trial < 64; trial++) {
		uint64_t a[32], o[32];
		for (int e = 0; e < 32; e++) a[e] = next(seed), o[e] = next(seed);
		uint64_t w = next(seed);
		if (trial == 0) w = 0;
		if (trial == 1) w = 1;
		if (trial == 2) w = ~0ull;
		uint32_t abs[64] = {0}, obs[64] = {0};
		for (int i = 0; i < 64; i++)
			for (int e = 0; e < 32; e++) {
				abs[i] |= (uint32_t)((a[e] >> i) & 1u) << e;
				obs[i] |= (uint32_t)((o[e] >> i) & 1u) << e;
			}
		bn::bsm6_fma_w2(abs, (uint32_t)w, (uint32_t)(w >> 32), obs);
		for (int e = 0; e < 32; e++) {
			uint64_t got = 0;
			for (int i = 0; i < 64; i++) got |= (uint64_t)((obs[i] >> e) & 1u) << i;
			const uint64_t want = o[e] ^ orc_mul(a[e], w, 6);
			if (got != want) {
				if (fails++ < 4) printf("FAIL bsm6_fma_w2 trial %d element %d: %016llx != %016llx\n", trial, e,
				                        (unsigned long long)got, (unsigned long long)want);
			}
		}
	}
	if (!fails) printf("ok bsm6_fma_w2 64 trials x 32 elements\n");
	// the NTT's per-lane compact-twiddle product (antt_rr.hip fma_tw): out ^= a * w in GF(2^32)
	int fails5 = 0;
	for (int trial = 0; trial < 64; trial++) {
		uint32_t a[32], o[32];
		for (int e = 0; e < 32; e++) a[e] = (uint32_t)next(seed), o[e] = (uint32_t)next(seed);
		const uint32_t w = trial == 0 ? 0u : trial == 1 ? 1u : (uint32_t)next(seed);
		uint32_t abs[32] = {0}, obs[32] = {0};
		for (int i = 0; i < 32; i++)
			for (int e = 0; e < 32; e++) {
				abs[i] |= ((a[e] >> i) & 1u) << e;
				obs[i] |= ((o[e] >> i) & 1u) << e;
			}
		bn::bsm5_fma_tw(abs, w, obs);
		for (int e = 0; e < 32; e++) {
			uint32_t got = 0;
			for (int i = 0; i < 32; i++) got |= ((obs[i] >> e) & 1u) << i;
			const uint32_t want = o[e] ^ (uint32_t)orc_mul(a[e], w, 5);
			if (got != want && fails5++ < 4) printf("FAIL bsm5_fma_tw trial %d element %d: %08x != %08x\n", trial, e, got, want);
		}
	}
	if (!fails5) printf("ok bsm5_fma_tw 64 trials x 32 elements\n");
	fails += fails5;
	// the bitsliced passes' top tile stage (antt_bs.hip block_stage): out = a * w, w scalar
	int failsw = 0;
	for (int trial = 0; trial < 64; trial++) {
		uint32_t a[32];
		for (int e = 0; e < 32; e++) a[e] = (uint32_t)next(seed);
		const uint32_t w = trial == 0 ? 0u : trial == 1 ? 1u : (uint32_t)next(seed);
		uint32_t abs[32] = {0}, obs[32];
		for (int i = 0; i < 32; i++)
			for (int e = 0; e < 32; e++) abs[i] |= ((a[e] >> i) & 1u) << e;
		bn::bsm5_mul_w(abs, w, obs);
		for (int e = 0; e < 32; e++) {
			uint32_t got = 0;
			for (int i = 0; i < 32; i++) got |= ((obs[i] >> e) & 1u) << i;
			const uint32_t want = (uint32_t)orc_mul(a[e], w, 5);
			if (got != want && failsw++ < 4) printf("FAIL bsm5_mul_w trial %d element %d: %08x != %08x\n", trial, e, got, want);
		}
	}
	if (!failsw) printf("ok bsm5_mul_w 64 trials x 32 elements\n");
	fails += failsw;
	return fails ? 1 : 0;
}
