// A/B for crc_cf.hip: the production kernels (csrc/hip/kernels.hip) compiled into this
// binary, k_crc_tiles timed through tpi_launch_stream_crc(MODE_CRC) on the same random data.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/hip scripts/exp/crc_prod.hip -o scripts/exp/crc_prod
#include "../../csrc/hip/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ void k_fill(uint64_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 8.0;
  const uint64_t tile = 1 << 20;
  const uint64_t n = (uint64_t)(gb * 1e9) / tile * tile;
  tpi_crc_tables* ht = new tpi_crc_tables;
  tpi_crc_tables_init(ht);
  std::vector<uint8_t> img(sizeof(tpi_crc_tables) + TPI_CRC_COLS_WORDS * 4);
  memcpy(img.data(), ht, sizeof(tpi_crc_tables));
  tpi_crc_cols_init(ht, (uint32_t*)(img.data() + sizeof(tpi_crc_tables)));
  tpi_crc_tables* dimg;
  CK(hipMalloc(&dimg, img.size()));
  CK(hipMemcpy(dimg, img.data(), img.size(), hipMemcpyHostToDevice));
  const uint32_t init = tpi_multmodp(tpi_x8nmodp(tile, ht->x2n), 0xFFFFFFFFu);
  uint8_t* d;
  CK(hipMalloc(&d, n));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)d, n / 8);
  uint32_t* dcrc;
  CK(hipMalloc(&dcrc, (n / tile) * 4));
  for (int mode : {2, 2, 2}) {
    auto call = [&] {
      CK(tpi_launch_stream_crc(mode, nullptr, 0, 0, n, d, tile, dimg, dcrc, init, init, nullptr,
                               0, 0));
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    call();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < 10; ++i) call();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("kernels.hip compiled in, mode %d: %7.1f GB/s\n", mode, (double)n * 10 / (ms * 1e-3) / 1e9);
  }
  return 0;
}
