// Device-side TS 38.211 section 5.2.1 Gold (pseudo-random) sequence at any position, shared by the PDSCH modulator
// (scrambling) and the PUSCH demodulator (descrambling). The x2 LFSR state at n = Nc + 32 w is reached by two GF(2)
// matrix jumps: M^(Nc + 2048 c) for the 2048-bit chunk c = w / 64 (wave-uniform when a wave covers 64 aligned words:
// scalar loads and branches), then M^(32 i), i = w mod 64, one column load per set state bit; x1 does not depend on
// c_init and comes from a table of words. Tables: srsgpu::ensure_gold_tables (capi_pdsch_mod.cpp).
#pragma once

#include "srsgpu_internal.h"

namespace srsgpu {

/// y = M v for a 31x31 GF(2) matrix given by its columns.
__device__ __forceinline__ uint32_t gf2_apply_cols(const uint32_t* __restrict__ cols, uint32_t v)
{
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 31; ++j) {
    r ^= cols[j] & (0u - ((v >> j) & 1u));
  }
  return r;
}

/// Sequence bits c(32 w) .. c(32 w + 31) of initial state c_init, MSB first (bit 31 = c(32 w)). `c_chunk` must be
/// w / 64 (pass it through readfirstlane when it is wave-uniform).
__device__ __forceinline__ uint32_t gold_word(uint32_t c_init,
                                              uint32_t w,
                                              uint32_t c_chunk,
                                              const uint32_t* __restrict__ x1,
                                              const uint32_t* __restrict__ x2_jump,
                                              const uint32_t* __restrict__ x2_lane)
{
  // x2 state (x2(n), ..., x2(n + 30)) at n = Nc + 2048 c, then at n = Nc + 32 w.
  const uint32_t sc = gf2_apply_cols(x2_jump + c_chunk * 31u, c_init);
  const uint32_t i  = w & 63u;
  uint32_t       s  = 0;
#pragma unroll
  for (int j = 0; j < 31; ++j) {
    if ((sc >> j) & 1u) {
      s ^= x2_lane[j * 64 + i];
    }
  }
  // 32 sequence bits: the window plus x2(n + 31) = x2(n + 3) + x2(n + 2) + x2(n + 1) + x2(n).
  const uint32_t x2w = s | (((s ^ (s >> 1) ^ (s >> 2) ^ (s >> 3)) & 1u) << 31);
  return __builtin_bitreverse32(x1[w] ^ x2w);  // LSB-first -> MSB-first
}

} // namespace srsgpu
