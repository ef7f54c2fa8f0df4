// Device-side definitions shared by the LDPC decoder kernels (ldpc_decoder.hip: one lifted check row per lane;
// ldpc_decoder_pk.hip: two rows per lane in packed 16-bit arithmetic).
#pragma once

#include "common.h"
#include "ldpc_base_graphs.h"
#include "srsgpu_internal.h"

namespace srsgpu {
namespace ldpc_dec {

template <int BG>
struct bg_t;

template <>
struct bg_t<1> {
  static constexpr int M  = kBG1_M;
  static constexpr int NF = kBG1_N_FULL;
  static constexpr int K  = kBG1_K;
  static constexpr int NE = kBG1_NUM_EDGES;
  static constexpr int rs(int m) { return kBG1_ROW_START[m]; }
  static constexpr int col(int e) { return kBG1_COL[e]; }
};

template <>
struct bg_t<2> {
  static constexpr int M  = kBG2_M;
  static constexpr int NF = kBG2_N_FULL;
  static constexpr int K  = kBG2_K;
  static constexpr int NE = kBG2_NUM_EDGES;
  static constexpr int rs(int m) { return kBG2_ROW_START[m]; }
  static constexpr int col(int e) { return kBG2_COL[e]; }
};

constexpr int LLR_MAX = 120;
/// Sign bits of the first SIGNS_LO edges of a layer share the state word with min1 (7 b), min2 (7 b), argmin (5 b).
constexpr int SIGNS_LO = 13;
/// Bytes of LDS reduction scratch between the soft-bit image and the shift table.
constexpr int SCRATCH_BYTES = 64 * sizeof(int);

/// Normalisation of a check-node magnitude (0..120). MODE 1: avx2_support.h:71 scale_epi8 (16-bit fixed point,
/// truncating); MODE 0: ldpc_decoder_generic.cpp:70 scale_llr (float, round half away from zero).
template <int MODE>
__device__ __forceinline__ int scale_mag(int m, uint32_t sf16, float sf)
{
  if constexpr (MODE == 1) {
    return static_cast<int>((static_cast<uint32_t>(m) * sf16) >> 16);
  } else {
    return static_cast<int>(roundf(static_cast<float>(m) * sf));
  }
}

/// Lifting shifts are read through the scalar (constant) path: wave-uniform, compile-time offsets -> s_load.
using const_u32_ptr = const __attribute__((address_space(4))) uint32_t*;

/// Scalar-cache warm-up: an s_load of sh[OFF / 4] that the caller consumes (keep_sgpr) only after the work it overlaps.
/// It is an ordinary load, so the compiler's wait-count pass tracks it. An earlier version issued the s_load from
/// inline asm: under register pressure (the __launch_bounds__(192, 8) build) the compiler spilled the asm's destination
/// SGPR with v_writelane and reused it for address arithmetic while the untracked load was still in flight; the load's
/// late return then overwrote a live address register and the kernel faulted ("register-capped fault").
template <int OFF>
__device__ __forceinline__ void scalar_touch(uint32_t& dst, const __attribute__((address_space(4))) uint32_t* sh)
{
  dst = sh[OFF / 4];
}
__device__ __forceinline__ void keep_sgpr(uint32_t v)
{
  asm volatile("" ::"s"(v));
}

/// Unsigned median of three (v_med3_u32).
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c)
{
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

/// Soft bits are kept in LDS in [-LLR_MAX - 1, LLR_MAX + 1]: +/-(LLR_MAX + 1) stands for the reference's +/-infinity
/// (LLR_INFTY = 127). The encoding is exact for inputs in the log_likelihood_ratio domain ([-120, 120] and +/-127,
/// log_likelihood_ratio.h:65) and lets the promotion sum be a single clamp.
constexpr int SOFT_INF = LLR_MAX + 1;
/// Minimum search key: magnitude << 5 | edge. Ties resolve to the lowest edge as in the reference (strict '<').
constexpr uint32_t KEY_INIT = static_cast<uint32_t>(LLR_MAX) << 5;

} // namespace ldpc_dec
} // namespace srsgpu
