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

__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v ^= static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), o, WAVE));
  }
  return v;
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

} // namespace srsgpu
