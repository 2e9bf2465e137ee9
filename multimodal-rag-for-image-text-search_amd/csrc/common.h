// common.h — shared helpers for libmrag (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/mrag.h"

namespace mrag {

// Thread-local error message behind mrag_last_error() (SURVEY.md §8b "Errors").
void set_error(const std::string& msg);
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// RAII device guard: every API call runs on the handle's device.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace mrag

#define MRAG_HIP(call)                                                                    \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) {                                                               \
      (void)hipGetLastError();                                                            \
      return mrag::fail(e_ == hipErrorOutOfMemory ? MRAG_ERR_OOM : MRAG_ERR_HIP,          \
                        "%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
    }                                                                                     \
  } while (0)

#define MRAG_CHECK_LAUNCH() MRAG_HIP(hipGetLastError())

#define MRAG_REQUIRE(cond, ...)                    \
  do {                                             \
    if (!(cond)) return mrag::fail(MRAG_ERR_ARG, __VA_ARGS__); \
  } while (0)

namespace mrag {

// Device-pointer inputs with stream == NULL run on a handle's own non-blocking stream, which
// does not wait for the null stream by itself: order it after everything already queued there
// (torch's default stream), so inputs produced by earlier kernels are complete when read.
inline int wait_null_stream(hipEvent_t ev, hipStream_t s) {
  MRAG_HIP(hipEventRecord(ev, nullptr));
  MRAG_HIP(hipStreamWaitEvent(s, ev, 0));
  return MRAG_OK;
}

// Wait for everything queued on s with the calling thread asleep (an event created with
// hipEventBlockingSync), not spinning: for the multi-millisecond image decode / resize calls,
// whose host threads share the process's CPU quota with the decode pool.
inline int blocking_wait(hipStream_t s) {
  thread_local hipEvent_t ev = nullptr;
  thread_local int ev_dev = -1;
  int dev = 0;
  MRAG_HIP(hipGetDevice(&dev));
  if (ev == nullptr || ev_dev != dev) {
    MRAG_HIP(hipEventCreateWithFlags(&ev, hipEventBlockingSync | hipEventDisableTiming));
    ev_dev = dev;
  }
  MRAG_HIP(hipEventRecord(ev, s));
  MRAG_HIP(hipEventSynchronize(ev));
  return MRAG_OK;
}

// Drains a stream on scope exit unless disarmed: an error return after the first launch must not
// hand buffers that queued kernels still use back to a pool (or drop the lock guarding them).
struct StreamDrain {
  hipStream_t s;
  bool armed = true;
  explicit StreamDrain(hipStream_t st) : s(st) {}
  ~StreamDrain() {
    if (armed) (void)hipStreamSynchronize(s);
  }
};

}  // namespace mrag

// ---------------------------------------------------------------------------
// Device-side helpers
// ---------------------------------------------------------------------------
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace mrag {
// compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N - 1, fully unrolled
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
}  // namespace mrag

// Monotone float -> uint32 map (ascending float == ascending uint).
__device__ __forceinline__ uint32_t mrag_f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float mrag_ord2f(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}
__device__ __forceinline__ uint64_t mrag_d2ord(double d) {
  uint64_t u = (uint64_t)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// "a ranks before b" under the retrieval order (score desc, row asc); rows < 0
// are empty slots and rank last.
__device__ __forceinline__ bool mrag_before(double sa, int64_t ra, double sb, int64_t rb) {
  if (ra < 0) return false;
  if (rb < 0) return true;
  if (sa != sb) return sa > sb;
  return ra < rb;
}
