// Calibration probe: throughput of individual VALU opcodes used by the packed LDPC decoder, 4 waves per SIMD,
// 8 independent chains per wave. Prints cycles per instruction per SIMD (2.0 = full rate on a 32-wide SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP_PROBE(NAME, ASM)                                                                                            \
  __global__ void NAME(unsigned* out, int n, unsigned long long* cyc, unsigned s)                                     \
  {                                                                                                                    \
    unsigned a[8];                                                                                                     \
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7u + i;                                                           \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                                       \
    for (int k = 0; k < n; ++k) {                                                                                      \
      _Pragma("unroll") for (int r = 0; r < 2; ++r)                                                                  \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) { asm volatile(ASM : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "s"(s)); } \
    }                                                                                                                  \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                                       \
    unsigned x = 0;                                                                                                    \
    for (int i = 0; i < 8; ++i) x ^= a[i];                                                                             \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                                                    \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                                                   \
  }

OP_PROBE(p_xor, "v_xor_b32 %0, %0, %1")
OP_PROBE(p_pk_add, "v_pk_add_u16 %0, %0, %1")
OP_PROBE(p_pk_mad, "v_pk_mad_u16 %0, %0, %1, %0")
OP_PROBE(p_pk_min, "v_pk_min_u16 %0, %0, %1")
OP_PROBE(p_pk_shl, "v_pk_lshlrev_b16 %0, 5, %0 op_sel_hi:[0,1]")
OP_PROBE(p_perm, "v_perm_b32 %0, %0, %1, %2")
OP_PROBE(p_sdwa_min, "v_min_u16_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1")
OP_PROBE(p_med3, "v_med3_i32 %0, %0, %1, %2")
OP_PROBE(p_bfe, "v_bfe_i32 %0, %0, 3, 1")
OP_PROBE(p_mul_lo, "v_mul_lo_u32 %0, %0, %1")
OP_PROBE(p_mad_u24, "v_mad_u32_u24 %0, %0, %1, %0")
OP_PROBE(p_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")

typedef void (*kern_t)(unsigned*, int, unsigned long long*, unsigned);

int main()
{
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  unsigned* out;
  unsigned long long* cyc;
  hipMalloc(&out, 1 << 24);
  hipMalloc(&cyc, 1 << 16);
  struct {
    const char* name;
    kern_t      k;
  } ops[] = {{"v_xor_b32", p_xor},       {"v_pk_add_u16", p_pk_add},   {"v_pk_mad_u16", p_pk_mad},
             {"v_pk_min_u16", p_pk_min}, {"v_pk_lshlrev_b16", p_pk_shl}, {"v_perm_b32", p_perm},
             {"v_min_u16_sdwa", p_sdwa_min}, {"v_med3_i32", p_med3}, {"v_bfe_i32", p_bfe},
             {"v_mul_lo_u32", p_mul_lo}, {"v_mad_u32_u24", p_mad_u24}, {"v_cndmask_b32", p_cndmask}};
  const int n = 2048;
  for (auto& o : ops) {
    for (int wps : {1, 4}) {
      hipLaunchKernelGGL(o.k, dim3(cus), dim3(256 * wps), 0, 0, out, n, cyc, 0x05040100u);
      hipDeviceSynchronize();
      unsigned long long h[1024];
      hipMemcpy(h, cyc, sizeof(unsigned long long) * cus, hipMemcpyDeviceToHost);
      double avg = 0;
      for (int i = 0; i < cus; ++i) avg += static_cast<double>(h[i]);
      avg /= cus;
      printf("%-18s waves/SIMD %d: %.2f cycles per instruction per SIMD\n", o.name, wps, avg / (16.0 * n * wps));
    }
  }
  return 0;
}
