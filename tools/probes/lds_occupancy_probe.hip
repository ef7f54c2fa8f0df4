// Calibration probe: how many 384-thread workgroups with a given static LDS size are resident per CU at once.
// Each workgroup touches its LDS, spins ~20 us and records s_memrealtime at start and end; the host reports the
// average concurrency (sum of durations / span) divided by the CU count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int LDS_BYTES>
__global__ __launch_bounds__(1024) void probe(unsigned long long* t, int spin)
{
  __shared__ int buf[LDS_BYTES / 4];
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  buf[threadIdx.x] = threadIdx.x;
  __syncthreads();
  int acc = buf[(threadIdx.x + 1) % blockDim.x];
  unsigned long long s = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - s < static_cast<unsigned long long>(spin)) {
    acc = acc * 3 + 1;
  }
  buf[LDS_BYTES / 4 - 1 - threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    t[2 * blockIdx.x]     = t0;
    t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() + (buf[0] == 12345 ? 1 : 0);
  }
}

template <int LDS_BYTES>
void run(unsigned long long* d, int nblk, int cus, int threads = 384)
{
  probe<LDS_BYTES><<<nblk, threads>>>(d, 2000);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(2 * nblk);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long lo = ~0ull, hi = 0;
  double sum = 0;
  for (int i = 0; i < nblk; ++i) {
    lo = std::min(lo, h[2 * i]);
    hi = std::max(hi, h[2 * i + 1]);
    sum += static_cast<double>(h[2 * i + 1] - h[2 * i]);
  }
  printf("threads %4d lds %6d B: %.2f workgroups/CU resident on average\n", threads, LDS_BYTES,
         sum / static_cast<double>(hi - lo) / cus);
}

int main()
{
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus  = p.multiProcessorCount;
  const int nblk = cus * 16;
  printf("CUs %d, sharedMemPerMultiprocessor %zu, maxSharedMemoryPerMultiProcessor %zu\n", cus, p.sharedMemPerBlock,
         p.maxSharedMemoryPerMultiProcessor);
  unsigned long long* d;
  hipMalloc(&d, 2 * nblk * 4 * 8);
  run<16384>(d, nblk, cus);
  run<32768>(d, nblk, cus);
  run<40960>(d, nblk, cus);
  run<53248>(d, nblk, cus);
  run<60160>(d, nblk, cus);
  run<65536>(d, nblk, cus);
  run<81920>(d, nblk, cus);
  for (int th : {64, 128, 192, 256}) {
    run<1024>(d, nblk * 4, cus, th);
    run<12288>(d, nblk * 4, cus, th);
    run<16384>(d, nblk * 4, cus, th);
    run<26624>(d, nblk * 4, cus, th);
  }
  hipFree(d);
  return 0;
}
