// Thread-local error reporting and capability check for the C-ABI.
#include "common.hpp"

#include <string.h>

namespace bn {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(g_err, sizeof(g_err), fmt, ap);
	va_end(ap);
}

void clear_error() { g_err[0] = 0; }

}  // namespace bn

extern "C" const char* bn_last_error(void) { return bn::g_err; }

extern "C" const char* bn_version(void) { return "binius-ntt-amd 0.1 (gfx950)"; }

// check_gpu_capabilities (src/ulvt/utils/common.cu:6-43) checked shared memory and
// compute capability; here: a gfx950 device with >= 64 KiB of LDS per workgroup.
extern "C" int bn_check_gpu_capabilities(void) {
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
		bn::set_error("no HIP device visible");
		return 0;
	}
	hipDeviceProp_t p;
	if (hipGetDeviceProperties(&p, 0) != hipSuccess) {
		bn::set_error("hipGetDeviceProperties failed");
		return 0;
	}
	if (strncmp(p.gcnArchName, "gfx950", 6) != 0) {
		bn::set_error("device 0 is %s, this build targets gfx950", p.gcnArchName);
		return 0;
	}
	if (p.sharedMemPerBlock < 65536) {
		bn::set_error("device has only %zu bytes of LDS per workgroup", (size_t)p.sharedMemPerBlock);
		return 0;
	}
	return 1;
}
