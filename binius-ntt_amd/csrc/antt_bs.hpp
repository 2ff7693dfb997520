// Shared pass tables of the bitsliced additive-NTT kernels (antt_bs.hip variant 1, antt_rr.hip
// variant 4; variant 5 = both): tiles of 128 bitsliced 32-element blocks, host-tabulated twiddle contributions.
#pragma once

#include <stdint.h>

#include "antt_plan.hpp"

namespace bn {

constexpr int kBlkBits = 7;
constexpr int kTileBlocks = 1 << kBlkBits;
constexpr int kLimbStride = 36;  // LDS words per (block, limb): 32 + 4 pad (bank spread)
constexpr int kMinLogH = kBlkBits + 5;
constexpr int kMaxStages = kBlkBits + 5;  // stages per pass
constexpr int kMaxOuter = 32 - 5 - kBlkBits;
constexpr int kMaxRateBits = 8;

enum { ROLE_FIRST = 0, ROLE_MID = 1, ROLE_LAST = 2, ROLE_SINGLE = 3 };

// One pass = k consecutive stages lo..lo+k-1 over every tile. Passed by value as a kernel
// argument (~2.6 KB), so every table read is a scalar load from the kernarg segment.
struct BsPass {
	int lo, k, role, n_outer, stop_j;
	int bb[kBlkBits];                        // index bit of tile block bit m
	int ob[kMaxOuter];                       // fixed (outer) index bits, ascending
	int stage_m[kMaxStages];                 // tile bit of stage lo + j (stages >= 5)
	int field[kMaxStages];                   // 8/16/32: sub-field holding every twiddle of the stage
	uint32_t twt[kMaxStages][kBlkBits];      // twiddle contribution of tile block bit m
	uint32_t two[kMaxStages][kMaxOuter];     // ... of outer bit m
	uint32_t twc[kMaxStages][kMaxRateBits];  // ... of coset bit c
	uint32_t pat[5][32];                     // stages 0..4: bit-lane part of the twiddle words
};

// Register-tile pass table (variant 4): wave w owns limb plane w of the tile; lane L holds two
// blocks R0, R1; the 7 tile bits are the register index plus six lane coordinates
//   c0 = L0^L2, c1 = L1^L2, c2 = L2, c3 = L3, c4 = L4, c5 = L5
// (partner lanes L ^ 1, 2, 7, 8, 16, 32). Before the stage on tile bit m < 6 the register bit is
// exchanged with coordinate m, so every butterfly is lane-private.
struct RtPass {
	int lo, k, role, n_outer, mlow;
	int bb[kBlkBits];
	int ob[kMaxOuter];
	int jm[kBlkBits];       // stage index (s - lo) of the block stage on tile bit m, -1 if none
	int field_m[kBlkBits];  // its twiddle sub-field
	int field_s[5];         // in-word stages s = 0..4 (bottom pass)
	uint32_t tau[kBlkBits][6];  // block stage on tile bit m: twiddle contribution of lane bit b
	uint32_t tau_iw[5][6];      // in-word stage s: lane-bit contributions to block R1's twiddle
	uint32_t cb_const[5];       // in-word stage s: R1's tile-bit-0 contribution
	uint32_t two[kMaxStages][kMaxOuter];
	uint32_t twc[kMaxStages][kMaxRateBits];
	uint32_t pat[5][32];  // in-word stage s: bit-lane part of the twiddle words (R0/R1 difference folded)
};

// pass tables of a plan (built once, cached in the plan)
const BsPass* bs_passes(bn_antt_plan* plan, size_t* n_passes);
int pass_fmax(const BsPass& p);
// register-tile table of a pass; BN_ERR_UNSUPPORTED when the stage bits are not the top tile bits
int make_rt(const BsPass& p, bool bottom, RtPass* out);
// variant 4 (antt_rr.hip): register-tile kernels over the same passes
int rr_prepare(bn_antt_plan* plan);
int rr_launch_pass(bn_antt_plan* plan, int i, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st);
const void* rr_pass_kernel(bn_antt_plan* plan, const BsPass& pass);
const void* bs_pass_kernel(bn_antt_plan* plan, int i);
// middle passes with the next tile prefetched by LDS-DMA (antt_rr.hip antt_rr_mid_pf)
int rr_launch_mid_pf(bn_antt_plan* plan, int i, const uint32_t* d_in, uint32_t* d_out, size_t batch, hipStream_t st);
const void* rr_mid_pf_kernel(const BsPass& pass);

}  // namespace bn
