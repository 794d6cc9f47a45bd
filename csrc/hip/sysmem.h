// Tile metadata that kernels read or write straight in host memory (CRCs, blob sizes, blob
// offsets: engine.hip meta_view) instead of through small per-chunk copies.  Vector loads and
// stores at system scope: neither the GPU's caches nor the host hold a stale copy, whether the
// array is in HBM or in registered host memory.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t tpi_sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t tpi_sys_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void tpi_sys_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
