// interpolate_at (src/ulvt/prime_field_sumcheck/utils/interpolate.hpp:3-8), host mirror: the
// degree-2 polynomial through (0, evals[0]), (1, evals[1]), (2, evals[2]) evaluated at challenge.
#pragma once

#include "qm31.hpp"

inline const QM31 one_half = QM31((uint32_t)0x40000000);  // 1/2 mod 2^31 - 1

inline QM31 interpolate_at(QM31 challenge, const QM31 evals[3]) {
	return (challenge * (challenge - 1) * evals[2] * one_half) - (challenge * (challenge - 2) * evals[1]) +
		   ((challenge - 1) * (challenge - 2) * evals[0] * one_half);
}
