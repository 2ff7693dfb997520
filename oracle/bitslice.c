/*
 * CPU ORACLE (test infrastructure only) — compact <-> bitsliced conversion.
 * Restates BitsliceUtils<W> (src/ulvt/utils/bitslicing.cuh:8-87):
 *   transpose32            :14-26  in-place 32x32 bit-matrix transpose
 *   bitslice_transpose     :32-47  element e, limb l (input word 4e+l) -> word 32l+i, bit e
 *   bitslice_untranspose   :49-64  inverse
 * (The reference's *member* bitslice_untranspose() calls the transpose — bitslicing.cuh:78 —
 *  a bug in an unused overload; the static function restated here is the one its callers use.)
 */
#include <string.h>

#include "oracle.h"

/* Square 32x32 bit transpose, recursive-block swap (Hacker's Delight 7-3). */
static void transpose32(uint32_t a[32]) {
	uint32_t m = 0x0000FFFFu;
	for (int j = 16; j != 0; j >>= 1, m ^= (m << j)) {
		for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
			uint32_t t = ((a[k] >> j) ^ a[k + j]) & m;
			a[k] ^= t << j;
			a[k + j] ^= t;
		}
	}
}

void orc_bitslice_transpose32(uint32_t blk[32]) { transpose32(blk); }
void orc_bitslice_untranspose32(uint32_t blk[32]) { transpose32(blk); }

void orc_bitslice_transpose128(uint32_t blk[128]) {
	uint32_t tmp[128];
	memcpy(tmp, blk, sizeof(tmp));
	for (int i = 0; i < 128; i++) blk[32 * (i % 4) + i / 4] = tmp[i];
	for (int c = 0; c < 4; c++) transpose32(blk + 32 * c);
}

void orc_bitslice_untranspose128(uint32_t blk[128]) {
	uint32_t tmp[128];
	memcpy(tmp, blk, sizeof(tmp));
	for (int c = 0; c < 4; c++) transpose32(tmp + 32 * c);
	for (int i = 0; i < 128; i++) blk[4 * (i % 32) + i / 32] = tmp[i];
}

/* Bulk forms (test fixtures at large sizes): n_blocks consecutive 128-word blocks. */
void orc_bitslice_many128(uint32_t* blocks, size_t n_blocks, int untranspose) {
	for (size_t b = 0; b < n_blocks; b++) {
		if (untranspose)
			orc_bitslice_untranspose128(blocks + 128 * b);
		else
			orc_bitslice_transpose128(blocks + 128 * b);
	}
}
