// Calibration probe: is a long straight-line VALU stream limited by instruction fetch? The same number of independent
// VALU instructions per wave, encoded as 4-byte VOP2 (v_add_u32_e32) or 8-byte VOP3P (v_pk_add_u16), in a straight-line
// body of BODY instructions (larger than a wave's instruction buffer, so every wave streams it from the instruction
// cache; 2 K x 8 B = 16 KB fits the cache, 16 K x 8 B = 128 KB does not) looped to 16 K instructions, on every CU at
// 1..8 waves per SIMD. If the 8-byte stream issues slower than the 4-byte one at equal instruction count, the fetch
// path (not the SIMD) sets the rate.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R4(x) x x x x
#define R16(x) R4(R4(x))
#define R256(x) R16(R16(x))
#define R1K(x) R4(R256(x))
#define R128(x) R4(R16(x)) R4(R16(x))

// -DREPS=n: a body of n x 16 instructions (n = 1, 2, 4, ..., 32) instead of BODY.
#define REP1(x) x
#define REP2(x) x x
#define REP4(x) REP2(x) REP2(x)
#define REP8(x) REP4(x) REP4(x)
#define REP16(x) REP8(x) REP8(x)
#define REP32(x) REP16(x) REP16(x)
#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)
#ifdef REPS
#define BODY CAT(REP, REPS)
#endif
#ifndef BODY
#define BODY R1K
#endif
#ifndef LOOPS_N
#define LOOPS_N 1
#endif

template <int OP, int LOOPS>
__global__ void probe(unsigned* out, unsigned long long* cyc)
{
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < LOOPS; ++it) {
  if constexpr (OP == 0) {
    // 16 K VOP2 instructions (8 independent chains).
    BODY(asm volatile("v_add_u32_e32 %0, %0, %1\n v_add_u32_e32 %2, %2, %3\n v_add_u32_e32 %4, %4, %5\n"
                     " v_add_u32_e32 %6, %6, %7\n v_add_u32_e32 %1, %1, %0\n v_add_u32_e32 %3, %3, %2\n"
                     " v_add_u32_e32 %5, %5, %4\n v_add_u32_e32 %7, %7, %6\n v_add_u32_e32 %0, %0, %1\n"
                     " v_add_u32_e32 %2, %2, %3\n v_add_u32_e32 %4, %4, %5\n v_add_u32_e32 %6, %6, %7\n"
                     " v_add_u32_e32 %1, %1, %0\n v_add_u32_e32 %3, %3, %2\n v_add_u32_e32 %5, %5, %4\n"
                     " v_add_u32_e32 %7, %7, %6"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
  } else {
    // 16 K VOP3P instructions, same dependency structure.
    BODY(asm volatile("v_pk_add_u16 %0, %0, %1\n v_pk_add_u16 %2, %2, %3\n v_pk_add_u16 %4, %4, %5\n"
                     " v_pk_add_u16 %6, %6, %7\n v_pk_add_u16 %1, %1, %0\n v_pk_add_u16 %3, %3, %2\n"
                     " v_pk_add_u16 %5, %5, %4\n v_pk_add_u16 %7, %7, %6\n v_pk_add_u16 %0, %0, %1\n"
                     " v_pk_add_u16 %2, %2, %3\n v_pk_add_u16 %4, %4, %5\n v_pk_add_u16 %6, %6, %7\n"
                     " v_pk_add_u16 %1, %1, %0\n v_pk_add_u16 %3, %3, %2\n v_pk_add_u16 %5, %5, %4\n"
                     " v_pk_add_u16 %7, %7, %6"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
  }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
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
#ifndef NINSTR
#define NINSTR (16.0 * 1024.0)
#endif
  const double ninstr = NINSTR;
  for (int op = 0; op < 2; ++op) {
    for (int wps = 1; wps <= 8; wps *= 2) {
      // One workgroup per CU with 4 x wps waves (wave w on SIMD w mod 4), two workgroups per CU above 1024 threads.
      const int threads = 256 * wps > 1024 ? 1024 : 256 * wps;
      const int blocks  = cus * (256 * wps / threads);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (op == 0) {
          probe<0, LOOPS_N><<<blocks, threads>>>(out, cyc);
        } else {
          probe<1, LOOPS_N><<<blocks, threads>>>(out, cyc);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double waves   = static_cast<double>(blocks) * threads / 64.0;
      const double instr   = waves * ninstr;
      const double per_cu  = instr / cus / (ms * 1e-3);  // wave-instructions per second per CU
      // s_memtime ticks per workgroup (each workgroup spans the launch): ticks / wall time = the counter's rate.
      unsigned long long h[4096];
      hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
      double ticks = 0;
      for (int i = 0; i < blocks; ++i) {
        ticks += static_cast<double>(h[i]);
      }
      ticks /= blocks;
      int clk_khz = 0;
      hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
      printf("%s waves/SIMD %d: %.3f ms, %.2f G wave-instr/s per CU (%.3f per 2.4 GHz cycle); s_memtime %.0f ticks "
             "= %.2f GHz x kernel time; %.2f s_memtime ticks per instruction per SIMD; clock attr %.2f GHz\n",
             op == 0 ? "VOP2  4 B" : "VOP3P 8 B", wps, ms, per_cu / 1e9, per_cu / 2.4e9, ticks,
             ticks / (ms * 1e6), ticks / (ninstr * wps), clk_khz / 1e6);
    }
  }
  return 0;
}
