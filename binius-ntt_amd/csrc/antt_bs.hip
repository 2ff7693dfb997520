// Bitsliced fast path for the additive NTT (placeholder: not yet enabled).
#include "antt_plan.hpp"

namespace bn {

bool bs_supports(const bn_antt_plan*) { return false; }
int bs_prepare(bn_antt_plan*) { return BN_OK; }
int launch_bs(bn_antt_plan*, const uint32_t*, uint32_t*, size_t, hipStream_t) {
	BN_FAIL(BN_ERR_UNSUPPORTED, "bitsliced path not built");
}

}  // namespace bn
