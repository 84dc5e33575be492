// tfp_internal.hpp — engine entry points shared inside libtiresias_fp.so (not part of the C-ABI).
#pragma once

#include <stdint.h>

#include <atomic>
#include <mutex>
#include <unordered_map>
#include <string>

#include "../../include/tiresias_fp.h"

namespace tfp {
// Last-error messages of a shared handle (engine or device group). The Asterisk module's channel
// threads all call one handle (application_handler.c:180, fp_handler.c:1161-1169), so a message is
// kept per calling thread as well as per handle; never a pointer into a string another thread may
// rewrite (a device group reads its shards' engines' messages from its own threads).
// Per-handle last-error messages. note() records a failing call's message for the calling thread
// (per handle) and, under the lock, as the handle's latest; read() returns the calling thread's own
// last message for this handle or, if it has none, a copy of the handle's latest. Both live in the
// thread's own per-handle strings, keyed by a serial number that is never reused (a new handle at a
// freed one's address does not inherit its messages), so a returned pointer stays valid until the
// same thread's next failing call or *_last_error read on the same handle, whatever other handles
// and threads do in between.
inline uint64_t error_slot_serial() {
  static std::atomic<uint64_t> n{0};
  return ++n;
}
struct ErrorSlot {
  const uint64_t id = error_slot_serial();
  std::mutex mu;
  std::string msg;
  void note(const void* h, const char* m);
  const char* read(const void* h);
  // this thread's own message for the handle (nullptr: none since clear_own)
  const char* own();
  void clear_own();
};
struct ThreadErrors {
  std::unordered_map<uint64_t, std::string> own, copy;
};
inline ThreadErrors& thread_errors() {
  thread_local ThreadErrors te;
  return te;
}
inline void ErrorSlot::note(const void*, const char* m) {
  thread_errors().own[id] = m;
  std::lock_guard<std::mutex> lk(mu);
  msg = m;
}
inline const char* ErrorSlot::own() {
  ThreadErrors& te = thread_errors();
  auto it = te.own.find(id);
  return it == te.own.end() ? nullptr : it->second.c_str();
}
inline void ErrorSlot::clear_own() { thread_errors().own.erase(id); }
inline const char* ErrorSlot::read(const void*) {
  ThreadErrors& te = thread_errors();
  auto it = te.own.find(id);
  if (it != te.own.end()) return it->second.c_str();
  std::string& c = te.copy[id];
  std::lock_guard<std::mutex> lk(mu);
  c = msg;
  return c.c_str();
}
}  // namespace tfp

extern "C" {
// The calling thread's own last-error message on an engine (nullptr: none since the last clear), and
// its clearing: a device group tells a shard's message for the call it just made from a stale one.
__attribute__((visibility("hidden"))) const char* tfp_internal_engine_own_error(tfp_engine* e);
__attribute__((visibility("hidden"))) void tfp_internal_engine_clear_error(tfp_engine* e);
// Index delta updates that re-sent every main column's tie key (tfp_group_tiebreak_stats).
__attribute__((visibility("hidden"))) int64_t tfp_internal_delta_main_keys(tfp_engine* e);
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
