// Internals shared by the translation units of libtpi_hip.so (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

// Sets the thread's tpi_last_error() text; returns -1.
int tpi_fail(const std::string& what);

#define TPI_HIP(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) return tpi_fail(std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)
