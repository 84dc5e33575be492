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
// One stream tick without the search: the samples into the ring and, when P is valid, the windows
// full after it fingerprinted into d_db (this engine's device; window i at frames [i F, (i+1) F),
// at most cap_frames) and their channels into act[*nact]. Returns after the values are written:
// a device group copies them to its other shards (tfp_group_stream_push, split channels).
__attribute__((visibility("hidden"))) int tfp_internal_stream_fp(tfp_stream* st, const int16_t* pcm, int32_t T,
                                                                 const tfp_search_params* P, double* d_db,
                                                                 int64_t cap_frames, int32_t* act, int32_t* nact,
                                                                 int64_t* frames_per_window);
}
