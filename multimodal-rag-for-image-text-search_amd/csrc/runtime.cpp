// runtime.cpp — error reporting and library-level entry points of libmrag.
#include <cstdarg>
#include <cstring>

#include "common.h"

namespace mrag {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

}  // namespace mrag

extern "C" {

const char* mrag_last_error(void) { return mrag::g_last_error.c_str(); }

const char* mrag_version(void) { return "mrag 0.1.0 (gfx950)"; }

int mrag_get_device_count(int32_t* count) {
  MRAG_REQUIRE(count != nullptr, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *count = 0;
    return mrag::fail(MRAG_ERR_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *count = n;
  return MRAG_OK;
}

}  // extern "C"
