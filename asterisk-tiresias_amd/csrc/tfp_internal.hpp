// tfp_internal.hpp — engine entry points shared inside libtiresias_fp.so (not part of the C-ABI).
#pragma once

#include <stdint.h>

#include "../../include/tiresias_fp.h"

extern "C" {
// The search over host samples (query i = lens[i] samples at ptrs[i]), without the engine's
// coalescer: a device group coalesces its callers itself and fans the batch out to its engines.
__attribute__((visibility("hidden"))) int tfp_internal_search_gather(tfp_engine* e, const void* const* ptrs,
                                                                     const int64_t* lens, int32_t nq, bool f32,
                                                                     int32_t sr, const tfp_search_params* P,
                                                                     tfp_result* out);
}
