// Calibration probe: LDS instruction throughput per CU for the byte accesses the LDPC decoder uses, 16 waves per CU.
// Patterns: lane-consecutive bytes (stride 1), the decoder's pair layout (stride 2, partner byte ^1), dwords.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ __launch_bounds__(1024) void probe(int* out, int n, unsigned long long* cyc, int stride)
{
  __shared__ __attribute__((aligned(16))) signed char lds[32768];
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) lds[i] = static_cast<signed char>(i * 7);
  __syncthreads();
  const unsigned base = (threadIdx.x % 64) * stride + (threadIdx.x / 64) * 512;
  int acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned a = (base + j * 1024 + k * 64) & 32767u;
      if constexpr (KIND == 0) {
        acc += lds[a];
      } else if constexpr (KIND == 1) {
        lds[a] = static_cast<signed char>(acc + j);
      } else if constexpr (KIND == 2) {
        acc += reinterpret_cast<int*>(lds)[(a & ~3u) / 4];
      } else {
        acc += reinterpret_cast<short*>(lds)[(a & ~1u) / 2];
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  int* out;
  unsigned long long* cyc;
  hipMalloc(&out, 1 << 24);
  hipMalloc(&cyc, 1 << 16);
  const int n = 1024;
  const char* names[] = {"ds_read_i8", "ds_write_b8", "ds_read_b32", "ds_read_i16"};
  for (int kind = 0; kind < 4; ++kind) {
    for (int stride : {1, 2, 4}) {
      for (int waves : {4, 16}) {
        switch (kind) {
          case 0: probe<0><<<cus, 64 * waves>>>(out, n, cyc, stride); break;
          case 1: probe<1><<<cus, 64 * waves>>>(out, n, cyc, stride); break;
          case 2: probe<2><<<cus, 64 * waves>>>(out, n, cyc, stride); break;
          default: probe<3><<<cus, 64 * waves>>>(out, n, cyc, stride); break;
        }
        hipDeviceSynchronize();
        unsigned long long h[1024];
        hipMemcpy(h, cyc, sizeof(unsigned long long) * cus, hipMemcpyDeviceToHost);
        double avg = 0;
        for (int i = 0; i < cus; ++i) avg += static_cast<double>(h[i]);
        avg /= cus;
        printf("%-12s stride %d, %2d waves/CU: %.2f memtime ticks per wave-instruction per CU\n", names[kind], stride,
               waves, avg / (8.0 * n * waves));
      }
    }
  }
  return 0;
}
