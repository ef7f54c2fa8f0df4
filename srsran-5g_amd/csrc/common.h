// Shared device-side helpers for the srsgpu PHY kernels (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>
#include <utility>

namespace srsgpu {

constexpr int WAVE = 64;

/// Compile-time loop: calls f(std::integral_constant<int, I>{}) for I = 0 .. N-1 (fully unrolled, static indices).
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>)
{
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f)
{
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

/// One DPP step of a wave reduction: v ^ (v permuted by CTRL within the enabled rows; 0 elsewhere).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_xor(uint32_t v)
{
  return v ^ static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, ROW_MASK, 0xf, false));
}

/// XOR of v over the 64 lanes (all lanes must be active), returned to every lane. DPP steps: pairs, quads, half-rows,
/// rows (quad_perm / mirrors), then row 0 -> 1 and 2 -> 3 (row_bcast:15) and rows 0-1 -> 2-3 (row_bcast:31): lane 63
/// ends with the total. No LDS round trip (ds_bpermute) on the way.
__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
  v = dpp_xor<0xb1>(v);          // quad_perm [1,0,3,2]
  v = dpp_xor<0x4e>(v);          // quad_perm [2,3,0,1]
  v = dpp_xor<0x141>(v);         // row_half_mirror
  v = dpp_xor<0x140>(v);         // row_mirror
  v = dpp_xor<0x142, 0xa>(v);    // row_bcast:15 into rows 1, 3
  v = dpp_xor<0x143, 0xc>(v);    // row_bcast:31 into rows 2, 3
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

/// One DPP step of an OR reduction.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_or(uint32_t v)
{
  return v | static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, ROW_MASK, 0xf, false));
}

/// OR of v over the 64 lanes (all lanes active), returned to every lane; the steps of wave_xor.
__device__ __forceinline__ uint32_t wave_or(uint32_t v)
{
  v = dpp_or<0xb1>(v);
  v = dpp_or<0x4e>(v);
  v = dpp_or<0x141>(v);
  v = dpp_or<0x140>(v);
  v = dpp_or<0x142, 0xa>(v);
  v = dpp_or<0x143, 0xc>(v);
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

__device__ __forceinline__ int wave_max(int v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int w = __shfl_xor(v, o, WAVE);
    v     = v > w ? v : w;
  }
  return v;
}

/// Integer clamp; lowers to a single v_med3_i32.
__device__ __forceinline__ int clamp_i(int v, int lo, int hi)
{
  return v < lo ? lo : (v > hi ? hi : v);
}

/// (ax + j ay)(bx + j by) with both fused multiply-adds explicit and nothing left to contract, so the rounding does
/// not depend on the compiler's contraction choices in context: the estimator's per-symbol CFO rotation of its
/// estimates and the demodulator's rotation of the compact estimate row must agree bit for bit.
__device__ __forceinline__ void cmul_fused(float ax, float ay, float bx, float by, float& rx, float& ry)
{
#pragma clang fp contract(off)
  const float pyy = ay * by;
  const float pyx = ay * bx;
  rx              = __builtin_fmaf(ax, bx, -pyy);
  ry              = __builtin_fmaf(ax, by, pyx);
}

} // namespace srsgpu
