// GF(2^128) sumcheck prover (placeholder until the bitsliced kernels land).
#include "common.hpp"

struct bn_sumcheck {
	int dummy;
};

extern "C" int bn_sumcheck_create(int, int, int, int, const uint32_t*, bn_sumcheck** sc) {
	if (sc) *sc = nullptr;
	BN_FAIL(BN_ERR_UNSUPPORTED, "sumcheck not built yet");
}
extern "C" int bn_sumcheck_create_device(int, int, int, int, void*, int, bn_sumcheck** sc) {
	if (sc) *sc = nullptr;
	BN_FAIL(BN_ERR_UNSUPPORTED, "sumcheck not built yet");
}
extern "C" int bn_sumcheck_round_messages(bn_sumcheck*, uint32_t*, uint32_t*) { BN_FAIL(BN_ERR_UNSUPPORTED, "sumcheck not built yet"); }
extern "C" int bn_sumcheck_move_to_next_round(bn_sumcheck*, const uint32_t*) { BN_FAIL(BN_ERR_UNSUPPORTED, "sumcheck not built yet"); }
extern "C" int bn_sumcheck_round(const bn_sumcheck*, int*) { BN_FAIL(BN_ERR_UNSUPPORTED, "sumcheck not built yet"); }
extern "C" int bn_sumcheck_set_shard(bn_sumcheck*, int, int) { BN_FAIL(BN_ERR_UNSUPPORTED, "sumcheck not built yet"); }
extern "C" int bn_sumcheck_destroy(bn_sumcheck* sc) {
	delete sc;
	return BN_OK;
}
