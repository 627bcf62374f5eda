// common.h — error plumbing for the C ABI (thread-local last-error message; no C++
// exception crosses the ABI boundary).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/az_othello.h"

namespace azc {

int set_error(int code, const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace azc

#define AZ_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess)                                                             \
      return azc::set_error(AZ_ERR_HIP, "%s failed: %s (%s:%d)", #call,               \
                            hipGetErrorString(e_), __FILE__, __LINE__);               \
  } while (0)

#define AZ_REQUIRE(cond, code, ...)                                                   \
  do {                                                                                \
    if (!(cond)) return azc::set_error((code), __VA_ARGS__);                          \
  } while (0)

// Wrap an entry point body so no C++ exception (e.g. std::bad_alloc) escapes.
#define AZ_GUARD_BEGIN try {
#define AZ_GUARD_END                                                                  \
  }                                                                                   \
  catch (const std::exception& ex) {                                                  \
    return azc::set_error(AZ_ERR_ARG, "exception: %s", ex.what());                    \
  }                                                                                   \
  catch (...) {                                                                       \
    return azc::set_error(AZ_ERR_ARG, "unknown exception");                           \
  }
