// Host <-> HBM transfer rates the lower-PHY sector group can count on (diagnostic, not shipped): DMA copies
// (hipMemcpyAsync from / to pinned memory, one or several streams, both directions at once) against zero-copy kernels
// that read / write pinned host memory directly, at the transfer sizes of one UL symbol round (142 KB per sector:
// 4 ports x (4096 + 352) complex samples) and one DL slot round. Build: hipcc --offload-arch=gfx950 -O2 -o
// pcie_probe pcie_probe.hip; prints one line per case.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#define CHECK(x)                                                                                                       \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                   \
      std::exit(1);                                                                                                    \
    }                                                                                                                  \
  } while (0)

__global__ void copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst, size_t n)
{
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    dst[i] = src[i];
  }
}

using clk = std::chrono::steady_clock;

double since(clk::time_point t0)
{
  return std::chrono::duration<double>(clk::now() - t0).count();
}

int main()
{
  const size_t sizes[] = {142336, 4 * 142336, 16 * 142336, 2 * 1966080, 8 * 1966080};
  const int    reps    = 200;
  hipStream_t  st[4];
  for (auto& s : st) {
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  const size_t maxb = 8 * 1966080;
  char *       h_def = nullptr, *h_coh = nullptr, *h_out = nullptr, *d_a = nullptr, *d_b = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_def), maxb * 4, hipHostMallocDefault));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_coh), maxb * 4, hipHostMallocCoherent | hipHostMallocMapped));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_out), maxb * 4, hipHostMallocDefault));
  CHECK(hipMalloc(reinterpret_cast<void**>(&d_a), maxb * 4));
  CHECK(hipMalloc(reinterpret_cast<void**>(&d_b), maxb * 4));
  std::memset(h_def, 1, maxb * 4);
  std::memset(h_coh, 1, maxb * 4);
  std::memset(h_out, 1, maxb * 4);
  // CPU side: memcpy into / out of each kind of host memory (what a sector thread does per symbol).
  {
    std::vector<char> src(maxb), dst(maxb);
    std::memset(src.data(), 3, maxb);
    char* plain = static_cast<char*>(std::malloc(maxb));
    std::memset(plain, 0, maxb);
    struct {
      const char* name;
      char*       p;
    } kinds[] = {{"malloc", plain}, {"hipHostMalloc default", h_def}, {"hipHostMalloc coherent|mapped", h_coh}};
    for (auto& k : kinds) {
      for (size_t b : {size_t(142336), size_t(53248)}) {
        auto t0 = clk::now();
        for (int r = 0; r < 2000; ++r) {
          std::memcpy(k.p + (r % 8) * b, src.data() + (r % 8) * b, b);
        }
        double tw = since(t0) / 2000;
        t0        = clk::now();
        for (int r = 0; r < 2000; ++r) {
          std::memcpy(dst.data() + (r % 8) * b, k.p + (r % 8) * b, b);
        }
        double tr = since(t0) / 2000;
        std::printf("cpu %s bytes %zu: write %.1f us (%.1f GB/s), read %.1f us (%.1f GB/s)\n", k.name, b, tw * 1e6,
                    b / tw / 1e9, tr * 1e6, b / tr / 1e9);
      }
    }
    std::free(plain);
  }
  for (size_t b : sizes) {
    // DMA H2D, 1 and 3 streams (each stream its own slice).
    for (int ns : {1, 3}) {
      CHECK(hipDeviceSynchronize());
      auto t0 = clk::now();
      for (int r = 0; r < reps; ++r) {
        const int k = r % ns;
        CHECK(hipMemcpyAsync(d_a + k * maxb, h_def + k * maxb, b, hipMemcpyHostToDevice, st[k]));
      }
      CHECK(hipDeviceSynchronize());
      double t = since(t0);
      std::printf("dma_h2d bytes %zu streams %d: %.2f GB/s, %.1f us per copy\n", b, ns, reps * b / t / 1e9,
                  t / reps * 1e6);
      t0 = clk::now();
      for (int r = 0; r < reps; ++r) {
        const int k = r % ns;
        CHECK(hipMemcpyAsync(h_out + k * maxb, d_a + k * maxb, b, hipMemcpyDeviceToHost, st[k]));
      }
      CHECK(hipDeviceSynchronize());
      t = since(t0);
      std::printf("dma_d2h bytes %zu streams %d: %.2f GB/s, %.1f us per copy\n", b, ns, reps * b / t / 1e9,
                  t / reps * 1e6);
    }
    // Both directions at once: H2D on stream 0, D2H on stream 1.
    {
      CHECK(hipDeviceSynchronize());
      auto t0 = clk::now();
      for (int r = 0; r < reps; ++r) {
        CHECK(hipMemcpyAsync(d_a, h_def, b, hipMemcpyHostToDevice, st[0]));
        CHECK(hipMemcpyAsync(h_out, d_b, b, hipMemcpyDeviceToHost, st[1]));
      }
      CHECK(hipDeviceSynchronize());
      const double t = since(t0);
      std::printf("dma_both bytes %zu: %.2f GB/s each way\n", b, reps * b / t / 1e9);
    }
    // Zero-copy kernels: read pinned host memory into HBM / write HBM into pinned host memory.
    for (int pass = 0; pass < 2; ++pass) {
      char*        src   = pass == 0 ? h_def : h_coh;
      const char*  kind  = pass == 0 ? "default" : "coherent";
      const size_t n4    = b / 16;
      const int    grid  = static_cast<int>(std::min<size_t>(1024, (n4 + 255) / 256));
      CHECK(hipDeviceSynchronize());
      auto t0 = clk::now();
      for (int r = 0; r < reps; ++r) {
        copy_kernel<<<grid, 256, 0, st[0]>>>(reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(d_a), n4);
      }
      CHECK(hipDeviceSynchronize());
      double t = since(t0);
      std::printf("zc_read(%s) bytes %zu: %.2f GB/s, %.1f us per launch\n", kind, b, reps * b / t / 1e9,
                  t / reps * 1e6);
      t0 = clk::now();
      for (int r = 0; r < reps; ++r) {
        copy_kernel<<<grid, 256, 0, st[0]>>>(reinterpret_cast<const float4*>(d_a), reinterpret_cast<float4*>(src), n4);
      }
      CHECK(hipDeviceSynchronize());
      t = since(t0);
      std::printf("zc_write(%s) bytes %zu: %.2f GB/s, %.1f us per launch\n", kind, b, reps * b / t / 1e9,
                  t / reps * 1e6);
    }
  }
  return 0;
}
