// Host-side C++ mirror of the reference's ulvt utilities (src/ulvt/utils/common.cuh,
// common.cu) over the C-ABI of libbinius_ntt_amd.so. Header-only; link with
// -lbinius_ntt_amd. Nothing here touches the GPU except through include/binius_ntt_amd.h.
#pragma once

#include <stdexcept>
#include <string>

#include "binius_ntt_amd.h"

namespace ulvt {

// Failure of a C-ABI call. The reference prints CUDA errors and carries on (CUDA_CHECK,
// common.cuh:18-29); the mirror throws so that callers cannot miss them.
class BnError : public std::runtime_error {
public:
	BnError(int code, const std::string& what) : std::runtime_error(what), code(code) {}
	int code;
};

inline void bn_check(int rc) {
	if (rc != BN_OK) throw BnError(rc, std::string("binius-ntt-amd: ") + bn_last_error());
}

}  // namespace ulvt

// bool check_gpu_capabilities() (src/ulvt/utils/common.cu:6-43)
inline bool check_gpu_capabilities() { return bn_check_gpu_capabilities() == 1; }
