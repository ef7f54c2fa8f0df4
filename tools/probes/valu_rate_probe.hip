// Calibration probe: VALU issue rate per SIMD for 32-bit integer and packed 16-bit instructions, as a function of
// the number of waves per SIMD. Each wave runs 8 independent dependency chains of N instructions.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short s16x2 __attribute__((ext_vector_type(2)));

template <int PK, int ILP = 8>
__global__ void probe(unsigned* out, int n, unsigned long long* cyc)
{
  unsigned a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 7u + i;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
#pragma unroll
    for (int r = 0; r < 8 / ILP; ++r)
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      if constexpr (PK) {
        asm volatile("v_pk_add_u16 %0, %0, %0" : "+v"(a[i]));
        asm volatile("v_pk_max_i16 %0, %0, %0" : "+v"(a[i]));
      } else {
        asm volatile("v_add_u32 %0, %0, %0" : "+v"(a[i]));
        asm volatile("v_max_i32 %0, %0, %0" : "+v"(a[i]));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s ^= a[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    cyc[blockIdx.x] = t1 - t0;
  }
}

int main()
{
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  unsigned* out;
  unsigned long long* cyc;
  hipMalloc(&out, 1 << 26);
  hipMalloc(&cyc, 1 << 20);
  const int n = 4096;
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int threads = 64 * 4 * wps;
    if (threads > 1024) {
      continue;
    }
    probe<1, 1><<<cus, threads>>>(out, n, cyc);
    hipDeviceSynchronize();
    {
      unsigned long long h0[1024];
      probe<0, 1><<<cus, threads>>>(out, n, cyc);
      hipDeviceSynchronize();
      hipMemcpy(h0, cyc, sizeof(unsigned long long) * cus, hipMemcpyDeviceToHost);
      double a0 = 0;
      for (int i = 0; i < cus; ++i) {
        a0 += static_cast<double>(h0[i]);
      }
      a0 /= cus;
      printf("dependent v_*_u32 chain waves/SIMD %d: %.2f cycles per VALU instruction per SIMD (%.2f per wave)\n", wps,
             a0 / (16.0 * n * wps), a0 / (16.0 * n));
      probe<1, 1><<<cus, threads>>>(out, n, cyc);
    }
    hipDeviceSynchronize();
    unsigned long long h[1024];
    hipMemcpy(h, cyc, sizeof(unsigned long long) * cus, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < cus; ++i) {
      avg += static_cast<double>(h[i]);
    }
    avg /= cus;
    printf("dependent v_pk chain waves/SIMD %d: %.2f cycles per VALU instruction per SIMD (%.2f per wave)\n", wps,
           avg / (16.0 * n * wps), avg / (16.0 * n));
  }
  for (int pk = 0; pk < 2; ++pk) {
    for (int wps = 1; wps <= 8; wps *= 2) {
      // One block of 4 * wps waves per CU: wps waves on every SIMD.
      const int threads = 64 * 4 * wps;
      if (threads > 1024) {
        continue;
      }
      if (pk) {
        probe<1><<<cus, threads>>>(out, n, cyc);
      } else {
        probe<0><<<cus, threads>>>(out, n, cyc);
      }
      hipDeviceSynchronize();
      unsigned long long h[1024];
      hipMemcpy(h, cyc, sizeof(unsigned long long) * cus, hipMemcpyDeviceToHost);
      double avg = 0;
      for (int i = 0; i < cus; ++i) {
        avg += static_cast<double>(h[i]);
      }
      avg /= cus;
      const double instr_per_simd = 16.0 * n * wps;  // 16 instructions per k per wave
      printf("%s waves/SIMD %d: %.2f cycles per VALU instruction per SIMD (%.2f per wave)\n", pk ? "v_pk_*16" : "v_*_u32 ",
             wps, avg / instr_per_simd, avg / (16.0 * n));
    }
  }
  return 0;
}
