// Additive-NTT plan: host-side twiddle precomputation and launch bookkeeping.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "common.hpp"

struct bn_antt_plan {
	int device = 0;
	int field_bits = 128;
	int log_h = 0;
	int log_rate = 0;
	int limbs = 4;   // u32 words per element
	int width = 0;   // log_h + log_rate - 1 (columns of the subspace table)
	int variant = 0; // kernel path in use (see antt.hip)
	int num_cus = 0; // compute units of the device (persistent grids)
	std::vector<uint32_t> s_host;  // log_h x width, row-major
	uint32_t* s_dev = nullptr;     // same on the device
	uint32_t* scratch = nullptr;   // pass-intermediate buffer (variant-specific)
	size_t scratch_bytes = 0;
	std::vector<unsigned char> bs_passes;  // variant-1 pass tables (antt_bs.hip), built on first use
	hipStream_t own_stream = nullptr;
	// host-apply staging
	void* h_dev_in = nullptr;
	void* h_dev_out = nullptr;
	// optional per-launch event timing: events are recorded around each pass without any host
	// synchronisation (the passes stay back to back) and resolved by bn_antt_get_event_timing
	int timing = 0;
	struct PendingPass {
		int kind;
		hipEvent_t begin, end;
	};
	std::vector<hipEvent_t> ev_pool;
	std::vector<PendingPass> pending;
	hipEvent_t cur_begin = nullptr;
	std::vector<float> kind_ms;
	std::vector<int> kind_cnt;
};

namespace bn {
// precompute_subspace_evals (src/ulvt/ntt/additive_ntt.cuh:273-309), GF(2^32) values.
void subspace_evals(int log_h, int log_rate, std::vector<uint32_t>& s);
// hipEvent timing around one launch of pass `kind` (no-op unless plan->timing).
int timing_begin(bn_antt_plan* p, int kind, hipStream_t st);
int timing_end(bn_antt_plan* p, int kind, hipStream_t st);
}  // namespace bn
