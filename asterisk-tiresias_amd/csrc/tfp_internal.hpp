// tfp_internal.hpp — engine entry points shared inside libtiresias_fp.so (not part of the C-ABI).
#pragma once

#include <stdint.h>

#include <mutex>
#include <string>

#include "../../include/tiresias_fp.h"

namespace tfp {
// Last-error messages of a shared handle (engine or device group). The Asterisk module's channel
// threads all call one handle (application_handler.c:180, fp_handler.c:1161-1169), so a message is
// kept per calling thread: a failing call records it in the thread's own slot (with the handle it
// failed on) and, under the handle's lock, in the handle's slot. tfp_*_last_error(h) returns the
// calling thread's message when its last failure was on h (valid until that thread's next failing
// call), else a thread-local copy of the handle's latest message taken under the lock (a device
// group reads its shards' engines' messages from its own threads). Never a pointer into a string
// another thread may rewrite.
struct ErrorSlot {
  std::mutex mu;
  std::string msg;
  void note(const void* h, const char* m);
  const char* read(const void* h);
};
struct ThreadError {
  const void* h = nullptr;
  std::string msg;
};
inline ThreadError& thread_error() {
  thread_local ThreadError te;
  return te;
}
inline void ErrorSlot::note(const void* h, const char* m) {
  ThreadError& te = thread_error();
  te.h = h;
  te.msg = m;
  std::lock_guard<std::mutex> lk(mu);
  msg = m;
}
inline const char* ErrorSlot::read(const void* h) {
  ThreadError& te = thread_error();
  if (te.h == h) return te.msg.c_str();
  thread_local std::string copy;
  std::lock_guard<std::mutex> lk(mu);
  copy = msg;
  return copy.c_str();
}
}  // namespace tfp

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
