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

// SDMA device -> host copies (sdma.cpp).  tpi_sdma_open returns nullptr when the lanes are
// off (TPI_D2H_ENGINE=blit, no HSA runtime to bind, no engine): callers then use
// hipMemcpyAsync.  A lane is one completion signal; a pipeline gives each staging buffer its
// own lane and waits on it (host side) before the buffer is written again.
struct tpi_sdma;
tpi_sdma* tpi_sdma_open(int device, int lanes);
void tpi_sdma_close(tpi_sdma* s);
uint32_t tpi_sdma_engine(const tpi_sdma* s);
int tpi_sdma_d2h(tpi_sdma* s, int lane, void* host_dst, const void* dev_src, size_t n);
// Host -> device lanes on an engine off HIP's own H2D engine and the saves' D2H engine
// (TPI_H2D_ENGINE=sdma<i> pins one); nullptr when none is free.
tpi_sdma* tpi_sdma_open_h2d(int device, int lanes);
int tpi_sdma_h2d(tpi_sdma* s, int lane, void* dev_dst, const void* host_src, size_t n);
int tpi_sdma_wait(tpi_sdma* s, int lane);
int tpi_sdma_wait_all(tpi_sdma* s);
