// Verifier helpers of the reference's sumcheck test (src/ulvt/sumcheck/test/verifier.cu) over the
// C-ABI, on __uint128_t values (4 little-endian u32 limbs, bigints.cu:6-13).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../utils/common.hpp"

// evaluate_univariate_given_points (verifier.cu:9-31)
inline __uint128_t evaluate_univariate_given_points(const __uint128_t challenge, const __uint128_t* points,
													const uint32_t num_points) {
	__uint128_t out = 0;
	ulvt::bn_check(bn_sumcheck_interpolate((const uint32_t*)points, (int)num_points, (const uint32_t*)&challenge,
										   (uint32_t*)&out));
	return out;
}

// evaluate_multilinear_composition (verifier.cu:88-107): the columns are compact (the reference's
// call site passes untransposed values, test.cu:80-98); evaluated on the GPU.
inline __uint128_t evaluate_multilinear_composition(const __uint128_t* evals, const __uint128_t* challenges,
													const size_t num_challenges, const size_t num_columns,
													int device = 0) {
	__uint128_t out = 0;
	ulvt::bn_check(bn_multilinear_composition_eval(device, (int)num_challenges, (int)num_columns, 0,
												   (const uint32_t*)evals, (const uint32_t*)challenges,
												   (uint32_t*)&out));
	return out;
}
