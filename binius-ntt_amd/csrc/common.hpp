// Shared host-side plumbing for the C-ABI: status codes, thread-local last error,
// HIP error checking that reports instead of aborting.
#pragma once

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include <string>

#include "binius_ntt_amd.h"

namespace bn {

void set_error(const char* fmt, ...);
void clear_error();

}  // namespace bn

#define BN_FAIL(code, ...)             \
	do {                               \
		::bn::set_error(__VA_ARGS__);  \
		return (code);                 \
	} while (0)

#define BN_HIP(call)                                                                                   \
	do {                                                                                               \
		hipError_t e_ = (call);                                                                        \
		if (e_ != hipSuccess) {                                                                        \
			::bn::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_));       \
			return BN_ERR_HIP;                                                                         \
		}                                                                                              \
	} while (0)

#define BN_CHECK_ARG(cond, ...)                      \
	do {                                             \
		if (!(cond)) BN_FAIL(BN_ERR_INVALID, __VA_ARGS__); \
	} while (0)

// Development build only (make BN_DEV=1): BN_FIRST_K=k gives the first upper pass of the bitsliced
// plan k stages (antt_bs.hip plan_passes; round-6 A/B of 6 + 6 + 12, tools/r06_ab4.sh), bounded
// below by what the later passes need. A no-op in the product build.
#ifdef BN_DEV
#define BN_DEV_FIRST_K(k, lo)                                                        \
	do {                                                                             \
		if (const char* e_ = getenv("BN_FIRST_K")) (k) = std::max((lo), std::min(kBlkBits, atoi(e_))); \
	} while (0)
#else
#define BN_DEV_FIRST_K(k, lo) ((void)0)
#endif
