// GF(2^128) bitsliced product on a quad of lanes (lane l holds limb l), shared by the sumcheck
// kernels (sumcheck.hip) and the bitsliced multiply microbenchmark (field.hip). The design is
// described in sumcheck.hip's header comment.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bitsliced.hpp"

namespace bn {
namespace quad {

constexpr int kRowWords = 36;    // LDS words per 32-word row (padding: bank spread)
constexpr int kQuadWords = 304;  // LDS words per quad slot (8 padded rows + spread)
constexpr int kMaxD = 8;

// compiler ordering for LDS traffic between lanes of one wave (the hardware executes a wave's
// LDS instructions in order)
__device__ __forceinline__ void wsync() {
	asm volatile("" ::: "memory");
	__builtin_amdgcn_wave_barrier();
}

// 16-byte accesses, register arrays filled and drained component-wise: a uint4 store through a
// pointer into a register array takes the array's address, and in some kernels SROA then leaves the
// array in scratch (k_gf128_mul_bs had 272-448 B of private memory per lane from this alone)
__device__ __forceinline__ void ld32(uint32_t* r, const uint32_t* p) {
#pragma unroll
	for (int i = 0; i < 32; i += 4) {
		const uint4 v = *(const uint4*)(p + i);
		r[i] = v.x, r[i + 1] = v.y, r[i + 2] = v.z, r[i + 3] = v.w;
	}
}
__device__ __forceinline__ void st32(uint32_t* p, const uint32_t* r) {
#pragma unroll
	for (int i = 0; i < 32; i += 4) *(uint4*)(p + i) = make_uint4(r[i], r[i + 1], r[i + 2], r[i + 3]);
}

// bitsliced multiply_alpha on GF(2^(2^H)) (binary_tower.cuh multiply_alpha): out may not alias a
template <int H>
__device__ __forceinline__ void bs_alpha(const uint32_t* a, uint32_t* out) {
	if constexpr (H == 0) {
		out[0] = a[0];
	} else {
		constexpr int half = 1 << (H - 1);
		uint32_t t[half];
		bs_alpha<H - 1>(a + half, t);
#pragma unroll
		for (int i = 0; i < half; i++) {
			out[i] = a[half + i];
			out[half + i] = a[i] ^ t[i];
		}
	}
}

// A quad's LDS slot: 8 rows of 32 words, rows padded to 36 words and slots to 304 words. With
// that padding the access patterns of quad_mul (operand rows l and 4+l, product rows 2l and
// 2l+1, the cross-lane reads) are nearly free of bank conflicts for both the 16-lane
// ds_read_b128 groups and the 8-lane ds_write_b128 groups (3328 -> 192 extra cycles per product
// in a lane-group model), while every address stays a base plus an immediate offset.
struct Slot {
	uint32_t* base;
	__device__ __forceinline__ uint32_t* row(int r) const { return base + kRowWords * r; }
};
__device__ __forceinline__ void sld(uint32_t* x, const Slot& S, int r) { ld32(x, S.row(r)); }
__device__ __forceinline__ void sst(const Slot& S, int r, const uint32_t* x) { st32(S.row(r), x); }

// GF(2^128) product on a quad. On entry slot row l holds limb l of the first operand and row 4+l
// limb l of the second — or, with B_SHARED, the second operand is the unswizzled 128-word B
// shared by every quad (the fold's broadcast challenge). On exit row l holds limb l of the product.
// skip_mid (development-build timing experiment only): the third circuit is replaced by its
// operand sum, i.e. 8 instead of 12 circuits per product (wrong results; an upper bound on what a
// 9-circuit Karatsuba top level could save in the kernels that call this).
template <bool B_SHARED>
__device__ __forceinline__ void quad_mul(const Slot& S, const uint32_t* B, int l, bool skip_mid = false) {
	wsync();
	const int ia = l & 1, jb = (l == 1 || l == 2) ? 1 : 0;
	const int ra = 2 * ia, rb = 4 + 2 * jb;  // rows of a0 (a1 = ra + 1) and b0 (b1 = rb + 1)
	auto ldb = [&](uint32_t* x, int h) {
		if constexpr (B_SHARED)
			ld32(x, B + 64 * jb + 32 * h);
		else
			sld(x, S, rb + h);
	};
	uint32_t x[32], y[32], z[32];
	// GF(2^64) Karatsuba: z0 = a0 b0, z2 = a1 b1, z1 = (a0+a1)(b0+b1) + z0 + z2; at most one
	// 32-word value is live across a circuit (the circuits themselves need ~160 VGPRs), the
	// rest is parked in the quad's LDS slot once the operands have been consumed.
	sld(x, S, ra);
	ldb(y, 0);
	bsm5_mul(x, y, z);  // z0
	__builtin_amdgcn_sched_barrier(0);
	wsync();  // also a compiler memory barrier: operands are re-read, never kept live
	sld(x, S, ra + 1);
	ldb(y, 1);
	bsm5_mul(x, y, y);  // z2
	__builtin_amdgcn_sched_barrier(0);
	wsync();
#pragma unroll
	for (int i = 0; i < 32; i++) z[i] ^= y[i];  // lo = z0 + z2
	bs_alpha<5>(y, x);
#pragma unroll
	for (int i = 0; i < 32; i++) y[i] = z[i] ^ x[i];  // lo + alpha(z2)
	uint32_t sa[32], sb[32];
	{
		const uint32_t* A0 = S.row(ra);
		const uint32_t* B0 = B_SHARED ? B + 64 * jb : S.row(rb);
		const int bstep = B_SHARED ? 32 : kRowWords;
#pragma unroll
		for (int i = 0; i < 32; i += 4) {
			const uint4 p = *(const uint4*)(A0 + i), q = *(const uint4*)(A0 + kRowWords + i);
			const uint4 u = *(const uint4*)(B0 + i), v = *(const uint4*)(B0 + bstep + i);
			sa[i] = p.x ^ q.x, sa[i + 1] = p.y ^ q.y, sa[i + 2] = p.z ^ q.z, sa[i + 3] = p.w ^ q.w;
			sb[i] = u.x ^ v.x, sb[i + 1] = u.y ^ v.y, sb[i + 2] = u.z ^ v.z, sb[i + 3] = u.w ^ v.w;
		}
	}
	wsync();  // every lane of the quad has read its operands: the slot is free
	sst(S, 2 * l, z);
	sst(S, 2 * l + 1, y);
	__builtin_amdgcn_sched_barrier(0);
	if (skip_mid) {
#pragma unroll
		for (int i = 0; i < 32; i++) x[i] = sa[i] ^ sb[i];
	} else {
		bsm5_mul(sa, sb, x);  // (a0+a1)(b0+b1)
	}
	__builtin_amdgcn_sched_barrier(0);
	sld(y, S, 2 * l + 1);
#pragma unroll
	for (int i = 0; i < 32; i++) x[i] ^= y[i];  // hi = z1 + alpha(z2)
	sst(S, 2 * l + 1, x);
	wsync();
	// lane q's GF(2^64) product P_q = (lo, hi) sits in rows 2q, 2q+1. Lane l assembles limb l:
	// limbs 0,1 = P00 + P11; limbs 2,3 = P01 + P10 + alpha64(P11), alpha64(P) = (P.hi, P.lo + alpha(P.hi))
	const int e0 = 2 * (l < 2 ? 0 : 2) + (l & 1);
	const uint32_t m2 = (l == 2) ? ~0u : 0u, m3 = (l == 3) ? ~0u : 0u;
	sld(z, S, e0);
	sld(x, S, e0 + 2);
#pragma unroll
	for (int i = 0; i < 32; i++) z[i] ^= x[i];
	sld(x, S, 3);  // P11.hi
	bs_alpha<5>(x, y);
	sld(sa, S, 2);  // P11.lo
#pragma unroll
	for (int i = 0; i < 32; i++) z[i] ^= (x[i] & m2) ^ ((sa[i] ^ y[i]) & m3);
	wsync();
	sst(S, l, z);
	wsync();
}

// Low-latency GF(2^128) product on a group of 16 lanes, for launches too small to fill the GPU
// (the sumcheck's last rounds): the 12 GF(2^32) products of the schoolbook-over-Karatsuba split
// run side by side, one per lane, instead of 3 in sequence per lane of a quad.
//   lane s < 12: q = s / 3 (P_q = A_i B_j as in quad_mul), t = s % 3 (Karatsuba z0, z2, z1)
//   lane s < 8 : P_{s/2} half s%2 (lo = z0 + z2, hi = z1 + z0 + z2 + alpha(z2))
//   lane s < 4 : limb s of the product
// Slot rows: 0-3 operand A, 4-7 operand B (then the P halves), 8-19 the z's, 20-23 alpha(z2).
constexpr int kHexWords = 24 * kRowWords + 16;

template <bool B_SHARED>
__device__ __forceinline__ void hex_mul(const Slot& S, const uint32_t* B, int s) {
	wsync();
	if (s < 12) {
		const int q = s / 3, t = s - 3 * (s / 3);
		const int ia = q & 1, jb = (q == 1 || q == 2) ? 1 : 0;
		const int ra = 2 * ia + (t == 1), rb = 2 * jb + (t == 1);  // z0: (lo, lo), z2: (hi, hi)
		const uint32_t m = t == 2 ? ~0u : 0u;                     // z1: (lo + hi, lo + hi)
		const uint32_t* A0 = S.row(ra);
		const uint32_t* A1 = S.row(2 * ia + 1);
		const uint32_t* B0 = B_SHARED ? B + 32 * rb : S.row(4 + rb);
		const uint32_t* B1 = B_SHARED ? B + 64 * jb + 32 : S.row(4 + 2 * jb + 1);
		uint32_t x[32], y[32], z[32];
#pragma unroll
		for (int i = 0; i < 32; i += 4) {
			const uint4 p = *(const uint4*)(A0 + i), p1 = *(const uint4*)(A1 + i);
			const uint4 u = *(const uint4*)(B0 + i), u1 = *(const uint4*)(B1 + i);
			x[i] = p.x ^ (p1.x & m), x[i + 1] = p.y ^ (p1.y & m), x[i + 2] = p.z ^ (p1.z & m), x[i + 3] = p.w ^ (p1.w & m);
			y[i] = u.x ^ (u1.x & m), y[i + 1] = u.y ^ (u1.y & m), y[i + 2] = u.z ^ (u1.z & m), y[i + 3] = u.w ^ (u1.w & m);
		}
		__builtin_amdgcn_sched_barrier(0);
		bsm5_mul(x, y, z);
		__builtin_amdgcn_sched_barrier(0);
		sst(S, 8 + s, z);
		if (t == 1) {
			bs_alpha<5>(z, x);
			sst(S, 20 + q, x);
		}
	}
	wsync();
	if (s < 8) {  // P_q.lo = z0 + z2, P_q.hi = P_q.lo + z1 + alpha(z2)
		const int q = s >> 1;
		const uint32_t m = (s & 1) ? ~0u : 0u;
		const uint32_t *z0 = S.row(8 + 3 * q), *z2 = S.row(9 + 3 * q), *z1 = S.row(10 + 3 * q), *az = S.row(20 + q);
		uint32_t r[32];
#pragma unroll
		for (int i = 0; i < 32; i++) r[i] = z0[i] ^ z2[i] ^ ((z1[i] ^ az[i]) & m);
		wsync();  // the operand rows are free once every lane has passed the first phase
		sst(S, 4 + s, r);
	}
	wsync();
	if (s < 4) {
		// limb 0 = P0.lo + P1.lo, 1 = P0.hi + P1.hi, 2 = P2.lo + P3.lo + P1.hi,
		// limb 3 = P2.hi + P3.hi + P1.lo + alpha(P1.hi)   (P_q half h in row 4 + 2q + h)
		const int h = s & 1, qa = s < 2 ? 0 : 2;
		const uint32_t m2 = s >= 2 ? ~0u : 0u;
		const uint32_t *pa = S.row(4 + 2 * qa + h), *pb = S.row(6 + 2 * qa + h), *pc = S.row(s == 2 ? 7 : 6);
		uint32_t r[32];
#pragma unroll
		for (int i = 0; i < 32; i++) r[i] = pa[i] ^ pb[i] ^ (pc[i] & m2);
		if (s == 3) {
			uint32_t x[32], y[32];
			sld(x, S, 7);
			bs_alpha<5>(x, y);
#pragma unroll
			for (int i = 0; i < 32; i++) r[i] ^= y[i];
		}
		wsync();
		sst(S, s, r);
	}
	wsync();
}

// Lowest-latency GF(2^128) product on a whole wave, for the sumcheck's smallest launches (a few
// hundred items: one wave per SIMD or less, so latency is all that counts). The GF(2^32)
// products of hex_mul are themselves split by Karatsuba over GF(2^16): 36 bsm4 circuits
// (316 gates) side by side instead of 12 bsm5 circuits (1022), then one more combine phase.
//   lane s < 36: q = s / 9, t = s / 3 % 3 (hex_mul's (q, t)), u = s % 3 (GF(2^16) term: lo, hi, sum)
//   lane s < 12: GF(2^32) product (q, t) = s: lo = z0 + z2, hi = z1 + z0 + z2 + alpha(z2) over its
//                three GF(2^16) products, into hex_mul's z rows (and alpha(z2) for t = 1)
//   then hex_mul's last two phases (P halves, limbs).
// Slot: hex_mul's 24 rows, then 36 GF(2^16) products of 16 words at a 20-word stride.
constexpr int kWideZ16 = 24 * kRowWords;
constexpr int kWideWords = kWideZ16 + 36 * 20 + 16;

template <bool B_SHARED>
__device__ __forceinline__ void wide_mul(const Slot& S, const uint32_t* B, int s) {
	wsync();
	if (s < 36) {
		const int q = s / 9, t = (s / 3) % 3, u = s % 3;
		const int ia = q & 1, jb = (q == 1 || q == 2) ? 1 : 0;
		const int ra = 2 * ia + (t == 1), rb = 2 * jb + (t == 1);
		const uint32_t m = t == 2 ? ~0u : 0u;
		const uint32_t* A0 = S.row(ra);
		const uint32_t* A1 = S.row(2 * ia + 1);
		const uint32_t* B0 = B_SHARED ? B + 32 * rb : S.row(4 + rb);
		const uint32_t* B1 = B_SHARED ? B + 64 * jb + 32 : S.row(4 + 2 * jb + 1);
		// the GF(2^32) operands of (q, t) as in hex_mul, then their GF(2^16) half or half-sum u
		const uint32_t mlo = u == 1 ? 0u : ~0u, mhi = u == 0 ? 0u : ~0u;
		uint32_t x[16], y[16], z[16];
#pragma unroll
		for (int i = 0; i < 16; i += 4) {
			const uint4 p = *(const uint4*)(A0 + i), p1 = *(const uint4*)(A1 + i);
			const uint4 ph = *(const uint4*)(A0 + 16 + i), p1h = *(const uint4*)(A1 + 16 + i);
			const uint4 v = *(const uint4*)(B0 + i), v1 = *(const uint4*)(B1 + i);
			const uint4 vh = *(const uint4*)(B0 + 16 + i), v1h = *(const uint4*)(B1 + 16 + i);
			x[i] = ((p.x ^ (p1.x & m)) & mlo) ^ ((ph.x ^ (p1h.x & m)) & mhi);
			x[i + 1] = ((p.y ^ (p1.y & m)) & mlo) ^ ((ph.y ^ (p1h.y & m)) & mhi);
			x[i + 2] = ((p.z ^ (p1.z & m)) & mlo) ^ ((ph.z ^ (p1h.z & m)) & mhi);
			x[i + 3] = ((p.w ^ (p1.w & m)) & mlo) ^ ((ph.w ^ (p1h.w & m)) & mhi);
			y[i] = ((v.x ^ (v1.x & m)) & mlo) ^ ((vh.x ^ (v1h.x & m)) & mhi);
			y[i + 1] = ((v.y ^ (v1.y & m)) & mlo) ^ ((vh.y ^ (v1h.y & m)) & mhi);
			y[i + 2] = ((v.z ^ (v1.z & m)) & mlo) ^ ((vh.z ^ (v1h.z & m)) & mhi);
			y[i + 3] = ((v.w ^ (v1.w & m)) & mlo) ^ ((vh.w ^ (v1h.w & m)) & mhi);
		}
		__builtin_amdgcn_sched_barrier(0);
		bsm4_mul(x, y, z);
		__builtin_amdgcn_sched_barrier(0);
		uint32_t* zo = S.base + kWideZ16 + 20 * s;
#pragma unroll
		for (int i = 0; i < 16; i += 4) *(uint4*)(zo + i) = make_uint4(z[i], z[i + 1], z[i + 2], z[i + 3]);
	}
	wsync();
	if (s < 12) {
		const int q = s / 3, t = s - 3 * (s / 3);
		const uint32_t* zb = S.base + kWideZ16 + 20 * (3 * s);
		uint32_t z0[16], z2[16], z1[16], al[16], r[32];
#pragma unroll
		for (int i = 0; i < 16; i += 4) {
			*(uint4*)(z0 + i) = *(const uint4*)(zb + i);
			*(uint4*)(z2 + i) = *(const uint4*)(zb + 20 + i);
			*(uint4*)(z1 + i) = *(const uint4*)(zb + 40 + i);
		}
		bs_alpha<4>(z2, al);
#pragma unroll
		for (int i = 0; i < 16; i++) {
			r[i] = z0[i] ^ z2[i];
			r[16 + i] = z1[i] ^ r[i] ^ al[i];
		}
		sst(S, 8 + s, r);
		if (t == 1) {
			uint32_t a[32];
			bs_alpha<5>(r, a);
			sst(S, 20 + q, a);
		}
	}
	wsync();
	if (s < 8) {  // P_q.lo = z0 + z2, P_q.hi = P_q.lo + z1 + alpha(z2)   (as hex_mul)
		const int q = s >> 1;
		const uint32_t m = (s & 1) ? ~0u : 0u;
		const uint32_t *z0 = S.row(8 + 3 * q), *z2 = S.row(9 + 3 * q), *z1 = S.row(10 + 3 * q), *az = S.row(20 + q);
		uint32_t r[32];
#pragma unroll
		for (int i = 0; i < 32; i++) r[i] = z0[i] ^ z2[i] ^ ((z1[i] ^ az[i]) & m);
		wsync();
		sst(S, 4 + s, r);
	}
	wsync();
	if (s < 4) {
		const int h = s & 1, qa = s < 2 ? 0 : 2;
		const uint32_t m2 = s >= 2 ? ~0u : 0u;
		const uint32_t *pa = S.row(4 + 2 * qa + h), *pb = S.row(6 + 2 * qa + h), *pc = S.row(s == 2 ? 7 : 6);
		uint32_t r[32];
#pragma unroll
		for (int i = 0; i < 32; i++) r[i] = pa[i] ^ pb[i] ^ (pc[i] & m2);
		if (s == 3) {
			uint32_t x[32], y[32];
			sld(x, S, 7);
			bs_alpha<5>(x, y);
#pragma unroll
			for (int i = 0; i < 32; i++) r[i] ^= y[i];
		}
		wsync();
		sst(S, s, r);
	}
	wsync();
}

}  // namespace quad
}  // namespace bn
