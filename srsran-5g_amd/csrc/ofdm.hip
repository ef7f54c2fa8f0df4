// OFDM slot modulator / demodulator on gfx950: one workgroup per (grid, port, OFDM symbol), a Stockham
// (self-sorting) radix-16 DFT in LDS with the subcarrier mapping, phase compensation, scaling, cyclic prefix and
// bf16 conversion fused into its first and last passes.
//
// Reference (behaviour, not code): lib/phy/lower/modulation/ofdm_modulator_impl.cpp:56 (symbol modulator),
// ofdm_demodulator_impl.cpp:94 (symbol demodulator), phase_compensation_lut.h:50, the unnormalised DFT of
// lib/phy/generic_functions/dft_processor_generic_impl.cpp (sign -1 direct, +1 inverse).
//
// Decomposition for N = 2^n: a first pass of radix 2^(n mod 4) (or 16), then radix-16 passes. N / 16 threads (a
// partial wave below N = 1024), each holding 16 complex values in registers per pass. N = 3 * 2^m (the generic DFT's
// 384 ... 6144, e.g. 1536 / 3072 points at 46.08 / 92.16 Msps): the power-of-two passes of M = 2^m, then one radix-3
// pass; N / 48 threads holding 48 values per pass. A pass a pass reads its butterfly inputs (from HBM in the first pass:
// the grid's subcarriers or the symbol's time samples, coalesced), barriers, twiddles them (exp(-+2 pi i m / N) from
// a 8192-entry table computed in double on the host), runs the in-register radix-R DFT and writes the outputs to LDS —
// or, in the last pass, straight to HBM with the compensation applied: time samples (and the cyclic-prefix copy) or
// bf16 subcarriers. HBM traffic per symbol: the grid row (4 B per subcarrier) and N + CP complex float samples (8 B),
// each touched once.
//
// Sizes above one workgroup's LDS (the generic DFT's 9216 .. 98304 = N2 x M, N2 in {3, 6, 9, 12}, M a power of two
// <= 8192) run as two kernels (a four-step split through an HBM scratch row per symbol): the first computes, for every
// n1 < M, the N2-point DFT of x[n1 + M n2] (n2 < N2) times exp(S 2 pi i n1 k2 / N) into scratch[k2][n1]; the second runs
// the M-point LDS transform of each scratch row k2 and writes output k2 + N2 k1 with the same fused last-pass work.
// X[k2 + N2 k1] = sum_n1 W_M^(n1 k1) W_N^(n1 k2) sum_n2 x[n1 + M n2] W_N2^(n2 k2).
#include <type_traits>
#include "srsgpu_internal.h"

namespace srsgpu {
namespace {


// cos / sin (2 pi k / 16).
__device__ constexpr float kCos16[16] = {1.0f,          0.92387953251f,  0.70710678118f,  0.38268343236f,
                                         0.0f,          -0.38268343236f, -0.70710678118f, -0.92387953251f,
                                         -1.0f,         -0.92387953251f, -0.70710678118f, -0.38268343236f,
                                         0.0f,          0.38268343236f,  0.70710678118f,  0.92387953251f};
__device__ constexpr float kSin16[16] = {0.0f,  0.38268343236f,  0.70710678118f,  0.92387953251f,
                                         1.0f,  0.92387953251f,  0.70710678118f,  0.38268343236f,
                                         0.0f,  -0.38268343236f, -0.70710678118f, -0.92387953251f,
                                         -1.0f, -0.92387953251f, -0.70710678118f, -0.38268343236f};

__device__ __forceinline__ float2 cadd(float2 a, float2 b)
{
  return make_float2(a.x + b.x, a.y + b.y);
}
__device__ __forceinline__ float2 csub(float2 a, float2 b)
{
  return make_float2(a.x - b.x, a.y - b.y);
}
__device__ __forceinline__ float2 cmul(float2 a, float2 b)
{
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

/// In-register DFT of size R (decimation in time, natural order in and out), exponent sign S.
template <int R, int S>
__device__ __forceinline__ void dft_reg(float2* v)
{
  if constexpr (R == 3) {
    // X0 = a + (b + c), X1,2 = a - (b + c) / 2 +- S i sqrt(3) / 2 (b - c).
    const float2 a = v[0], t1 = cadd(v[1], v[2]), t2 = csub(v[1], v[2]);
    const float  h = S * 0.86602540378f;
    const float2 m = make_float2(a.x - 0.5f * t1.x, a.y - 0.5f * t1.y);
    const float2 n = make_float2(-h * t2.y, h * t2.x);
    v[0]           = cadd(a, t1);
    v[1]           = cadd(m, n);
    v[2]           = csub(m, n);
  } else if constexpr (R == 2) {
    const float2 a = v[0], b = v[1];
    v[0]           = cadd(a, b);
    v[1]           = csub(a, b);
  } else if constexpr (R > 2) {
    float2 e[R / 2], o[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      e[i] = v[2 * i];
      o[i] = v[2 * i + 1];
    }
    dft_reg<R / 2, S>(e);
    dft_reg<R / 2, S>(o);
#pragma unroll
    for (int k = 0; k < R / 2; ++k) {
      float2 t;
      if (k == 0) {
        t = o[0];
      } else if (4 * k == R) {  // times S * i
        t = (S > 0) ? make_float2(-o[k].y, o[k].x) : make_float2(o[k].y, -o[k].x);
      } else {
        const int m = k * (16 / R);
        t           = cmul(o[k], make_float2(kCos16[m], S * kSin16[m]));
      }
      v[k]         = cadd(e[k], t);
      v[k + R / 2] = csub(e[k], t);
    }
  }
}

/// Twiddles W^(r k) = exp(S 2 pi i r k / (NS R)), r = 1..R-1, of the butterflies this thread runs in a pass with
/// radix R after passes of total radix NS (k = j mod NS); the table holds exp(-2 pi i m / OFDM_MAX_DFT). Computed at
/// kernel start for every pass, so their L2 latency hides under the first pass's HBM loads.
template <int N, int R, int NS, int S>
__device__ __forceinline__ void load_twiddles(const float2* __restrict__ tw, float2 (&w)[16 / R][R])
{
  constexpr int T   = N / 16;
  const int     tid = static_cast<int>(threadIdx.x);
  if constexpr (R == 16) {
    // W^k from the table (the lanes' k are consecutive, so the gather touches few cache lines; W^(r k) for all r
    // touched up to 64 lines per instruction in the last pass), W^2k, W^4k, W^8k by squaring and the other powers by
    // at most three complex products (relative error < 1e-6).
    const int k  = tid & (NS - 1);
    auto      at = [&](int r) {
      float2 x = tw[(r * k) * static_cast<int>(OFDM_MAX_DFT / (NS * R))];
      if constexpr (S > 0) {
        x.y = -x.y;
      }
      return x;
    };
    float2(&v)[R] = w[0];
    v[1]          = at(1);
    v[2]          = cmul(v[1], v[1]);
    v[4]          = cmul(v[2], v[2]);
    v[8]          = cmul(v[4], v[4]);
    v[3]          = cmul(v[1], v[2]);
    v[5]          = cmul(v[4], v[1]);
    v[6]          = cmul(v[4], v[2]);
    v[7]          = cmul(v[4], v[3]);
#pragma unroll
    for (int r = 9; r < 16; ++r) {
      v[r] = cmul(v[8], v[r - 8]);
    }
    return;
  }
#pragma unroll
  for (int b = 0; b < 16 / R; ++b) {
    const int k = (tid + b * T) & (NS - 1);
#pragma unroll
    for (int r = 1; r < R; ++r) {
      float2 x = tw[(r * k) * static_cast<int>(OFDM_MAX_DFT / (NS * R))];
      if constexpr (S > 0) {
        x.y = -x.y;
      }
      w[b][r] = x;
    }
  }
}

/// W^k = exp(S 2 pi i k / (16 NS)), k = tid mod NS: the base twiddle of this thread's butterfly in a radix-16 pass
/// after passes of total radix NS (the table holds exp(-2 pi i m / OFDM_MAX_DFT)). Loaded at kernel start for every
/// pass (one 8-byte L2 gather each, in flight under the first pass's HBM loads); the powers are expanded in the pass
/// itself (twiddle16), so the transform holds 2 VGPRs per later pass instead of 32.
template <int NS, int S>
__device__ __forceinline__ float2 twiddle_base(const float2* __restrict__ tw)
{
  const int k = static_cast<int>(threadIdx.x) & (NS - 1);
  float2    x = tw[k * static_cast<int>(OFDM_MAX_DFT / (NS * 16))];
  if constexpr (S > 0) {
    x.y = -x.y;
  }
  return x;
}

/// v[r] *= W^r, r = 1..15, from W = w1: W^2, W^4, W^8 by squaring, the other powers by at most three complex products
/// (relative error < 1e-6), each power formed just before its product so that few stay live.
__device__ __forceinline__ void twiddle16(float2 (&v)[16], float2 w1)
{
  const float2 w2 = cmul(w1, w1);
  const float2 w4 = cmul(w2, w2);
  const float2 w8 = cmul(w4, w4);
  const float2 w3 = cmul(w1, w2);
  const float2 w5 = cmul(w4, w1);
  const float2 w6 = cmul(w4, w2);
  const float2 w7 = cmul(w4, w3);
  v[1]            = cmul(v[1], w1);
  v[2]            = cmul(v[2], w2);
  v[3]            = cmul(v[3], w3);
  v[4]            = cmul(v[4], w4);
  v[5]            = cmul(v[5], w5);
  v[6]            = cmul(v[6], w6);
  v[7]            = cmul(v[7], w7);
  v[8]            = cmul(v[8], w8);
  v[9]            = cmul(v[9], cmul(w8, w1));
  v[10]           = cmul(v[10], cmul(w8, w2));
  v[11]           = cmul(v[11], cmul(w8, w3));
  v[12]           = cmul(v[12], cmul(w8, w4));
  v[13]           = cmul(v[13], cmul(w8, w5));
  v[14]           = cmul(v[14], cmul(w8, w6));
  v[15]           = cmul(v[15], cmul(w8, w7));
}

/// One Stockham pass of radix R over N points (NS = product of the previous passes' radices): butterfly j takes
/// x[j + r N / R], twiddles by W^(r k) (k = j mod NS, expanded from the base wb), and writes X[(j - k) R + k + r NS].
/// Twiddled passes are radix 16 (one butterfly per thread); a radix below 16 is the first pass only (NS = 1).
/// SYNC_IN: the inputs come from the LDS buffer the outputs overwrite, so every thread's reads complete first (the
/// first pass reads HBM and needs no barrier before its LDS stores).
template <int N, int R, int NS, int S, bool SYNC_IN, typename Src, typename Dst>
__device__ __forceinline__ void stockham_pass(float2 wb, Src src, Dst dst)
{
  static_assert(R == 16 || NS == 1, "twiddled passes are radix 16");
  constexpr int T = N / 16;
  constexpr int B = 16 / R;
  float2        v[B][R];
  const int     tid = static_cast<int>(threadIdx.x);
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const int j = tid + b * T;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      v[b][r] = src(j + r * (N / R));
    }
  }
  if constexpr (SYNC_IN) {
    __syncthreads();
  }
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const int j = tid + b * T;
    const int k = j & (NS - 1);
    if constexpr (NS > 1) {
      twiddle16(v[b], wb);
    }
    dft_reg<R, S>(v[b]);
    const int base = (j - k) * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      dst(base + r * NS, v[b][r]);
    }
  }
  __syncthreads();
}

constexpr bool is_pow2(int n)
{
  return (n & (n - 1)) == 0;
}
constexpr int ilog2(int n)
{
  return n <= 1 ? 0 : 1 + ilog2(n / 2);
}
/// Threads per workgroup of an N-point transform: 16 values per thread (2^n) or 48 (3 * 2^m, 9 * 2^m).
template <int N>
constexpr int ofdm_threads()
{
  return is_pow2(N) ? N / 16 : N / 48;
}

/// exp(S 2 pi i m / N), 0 <= m < N, of any supported N: the table entry for a power of two, sincospi otherwise
/// (argument 2 m / N rounded once: phase error < 3e-7 rad).
template <int N, int S>
__device__ __forceinline__ float2 twiddle_any(const float2* __restrict__ tw, uint32_t m)
{
  float2 x;
  if constexpr (is_pow2(N)) {
    x = tw[m * (OFDM_MAX_DFT / N)];
    x.y = -x.y;  // the table holds exp(-...)
  } else {
    sincospif(static_cast<float>(2 * m) / static_cast<float>(N), &x.y, &x.x);
  }
  if constexpr (S < 0) {
    x.y = -x.y;
  }
  return x;
}

/// One Stockham pass of the N = 3^a M transform (a = 1, 2; T = N / 48 threads, B = N / (R T) butterflies each). The
/// power-of-two passes come first: their NS divides T, so all butterflies of a thread share k = tid mod NS and the
/// twiddles w of load_twiddles. The radix-3 passes are last (NS = M, then 3 M): twiddles exp(S 2 pi i r k / (3 NS)),
/// k = j mod NS, by sincospi (argument rounded once: phase error < 3e-7 rad).
template <int N, int R, int NS, int S, typename Src, typename Dst>
__device__ __forceinline__ void stockham_pass3(const float2 (&w)[16], Src src, Dst dst)
{
  constexpr int T = N / 48;
  constexpr int B = N / (R * T);
  static_assert(R == 3 || T % NS == 0 || NS == 1, "pass order: powers of two, then radix 3");
  float2    v[B][R];
  const int tid = static_cast<int>(threadIdx.x);
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const int j = tid + b * T;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      v[b][r] = src(j + r * (N / R));
    }
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const int j = tid + b * T;
    const int k = (R == 3) ? j % NS : (j & (NS - 1));
    if constexpr (R == 3) {
#pragma unroll
      for (int r = 1; r < 3; ++r) {
        float2 x;
        sincospif(static_cast<float>(2 * r * k) / static_cast<float>(3 * NS), &x.y, &x.x);
        x.y     = S * x.y;
        v[b][r] = cmul(v[b][r], x);
      }
    } else if constexpr (NS > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) {
        v[b][r] = cmul(v[b][r], w[r]);
      }
    }
    dft_reg<R, S>(v[b]);
    const int base = (j - k) * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      dst(base + r * NS, v[b][r]);
    }
  }
  __syncthreads();
}

/// N = 3^a M: power-of-two passes of M (first radix 2^(m mod 4) or 16, then 16s), then a radix-3 passes.
template <int N, int S, typename Src, typename Dst>
__device__ __forceinline__ void dft_lds3(float2* lds, const float2* __restrict__ tw, Src src_first, Dst dst_last)
{
  constexpr int A3  = (N % 9 == 0) ? 9 : 3;
  constexpr int M   = N / A3;
  constexpr int LM  = ilog2(M);
  constexpr int REM = LM % 4;
  constexpr int R0  = REM ? (1 << REM) : 16;
  constexpr int NP  = LM / 4 + (REM ? 1 : 0);
  static_assert(A3 * M == N && is_pow2(M) && NP >= 2 && NP <= 3, "supported DFT sizes: 3 x (128..2048), 9 x 512");
  auto   ld = [lds](int i) { return lds[i]; };
  auto   st = [lds](int i, float2 v) { lds[i] = v; };
  float2 w0[16] = {}, w1[1][16], w2[1][16];
  load_twiddles<N, 16, R0, S>(tw, w1);
  if constexpr (NP == 3) {
    load_twiddles<N, 16, R0 * 16, S>(tw, w2);
  }
  stockham_pass3<N, R0, 1, S>(w0, src_first, st);
  stockham_pass3<N, 16, R0, S>(w1[0], ld, st);
  if constexpr (NP == 3) {
    stockham_pass3<N, 16, R0 * 16, S>(w2[0], ld, st);
  }
  if constexpr (A3 == 9) {
    stockham_pass3<N, 3, M, S>(w0, ld, st);
    stockham_pass3<N, 3, 3 * M, S>(w0, ld, dst_last);
  } else {
    stockham_pass3<N, 3, M, S>(w0, ld, dst_last);
  }
}

template <int LOG2N, int S, typename Src, typename Dst>
__device__ __forceinline__ void dft_lds(float2* lds, const float2* __restrict__ tw, Src src_first, Dst dst_last)
{
  constexpr int N    = 1 << LOG2N;
  constexpr int REM  = LOG2N % 4;
  constexpr int R0   = REM ? (1 << REM) : 16;
  constexpr int NP   = LOG2N / 4 + (REM ? 1 : 0);
  // The first pass's stores go to j R0 + r: 16 consecutive lanes 16 float2 apart on one bank pair, and 64 % of the
  // 4096-point kernels' LDS cycles are bank-conflict cycles (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE,
  // profiles/r5_lds_counters.txt). An XOR swizzle (i ^ ((i >> 4) & 15), or of bits 1-3 only, pairs kept) removed every
  // conflict (LDS-array cycles 5.0M -> 1.4M, LDS issue stalls 5.7M -> 0.4M per modulator launch), but the
  // runtime XOR splits the merged ds_write_b128 / ds_read2st64_b64 into single b64 accesses (2x the LDS instructions,
  // +9 % VALU) and the bench gets slower: modulator stage 45.6 -> 68-73 us per step, demodulator unchanged, headline
  // 144.2k -> 142.6k (profiles/r5_ofdm_swizzle_ab.txt). The LDS conflicts do not bound these kernels: plain layout.
  auto ld = [lds](int i) { return lds[i]; };
  auto st = [lds](int i, float2 v) { lds[i] = v; };
  static_assert(NP >= 2 && NP <= 4, "supported DFT sizes: 128..8192");
  const float2 b1 = twiddle_base<R0, S>(tw);
  const float2 b2 = NP >= 3 ? twiddle_base<R0 * 16, S>(tw) : float2{};
  const float2 b3 = NP == 4 ? twiddle_base<R0 * 256, S>(tw) : float2{};
  stockham_pass<N, R0, 1, S, false>(float2{}, src_first, st);  // NS = 1: no twiddles
  if constexpr (NP == 2) {
    stockham_pass<N, 16, R0, S, true>(b1, ld, dst_last);
  } else if constexpr (NP == 3) {
    stockham_pass<N, 16, R0, S, true>(b1, ld, st);
    stockham_pass<N, 16, R0 * 16, S, true>(b2, ld, dst_last);
  } else {
    stockham_pass<N, 16, R0, S, true>(b1, ld, st);
    stockham_pass<N, 16, R0 * 16, S, true>(b2, ld, st);
    stockham_pass<N, 16, R0 * 256, S, true>(b3, ld, dst_last);
  }
}

/// 4096 points on two waves (128 threads, two radix-16 butterflies per thread and pass, j0 = tid and j1 = tid + 128)
/// through a 16 KB LDS buffer. The one-butterfly transform holds the 4096-point block in 32 KB of LDS and at 92 VGPRs
/// runs 5 four-wave workgroups per CU: 5 symbols in flight per CU, and each waits out its HBM loads, barriers and
/// stores in lockstep with the others. Here a symbol takes two waves and 16 KB, so 8 symbols are in flight per CU
/// (4 waves per SIMD), each thread with two independent butterflies. The Stockham index maps put butterfly j0's outputs
/// of passes 1 and 2 into the first half of the 4096 points and j1's into the second, and each pass reads inputs
/// j + 256 r, r < 8 from the first half and r >= 8 from the second: every exchange runs as write half A, read the A
/// inputs, write half B, read the B inputs, with the same 2048-entry buffer.
template <int S, typename Src, typename Dst>
__device__ __forceinline__ void dft4096_two_waves(float2* lds, const float2* __restrict__ tw, Src src_first, Dst dst_last)
{
  constexpr int T = 128, H = 2048;
  const int     tid = static_cast<int>(threadIdx.x);
  // Pass bases: NS = 16 (k = j mod 16, the same for both butterflies), NS = 256 (k = j: j1's base loaded apart).
  const float2 b1  = twiddle_base<16, S>(tw);
  const float2 b2a = twiddle_base<256, S>(tw);
  float2       b2b = tw[(tid + T) * static_cast<int>(OFDM_MAX_DFT / (256 * 16))];
  if constexpr (S > 0) {
    b2b.y = -b2b.y;
  }
  // a: butterfly j0's values, c: j1's. Each exchange frees one set before the reads that refill it, so that at most
  // 32 complex values are live: write j0's outputs (half A), read every butterfly's inputs r < 8 into a (j0's into
  // a[0..7], j1's into a[8..15]), then compute / write j1's (half B) and read the inputs r >= 8 into c likewise;
  // the next pass's butterflies are {a[0..7], c[0..7]} and {a[8..15], c[8..15]}, regrouped by renaming.
  float2 a[16], c[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    a[r] = src_first(tid + r * 256);
  }
  auto regroup = [&]() {
    float2 t[16];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      t[r]     = a[8 + r];
      t[8 + r] = c[8 + r];
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      a[8 + r] = c[r];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      c[r] = t[r];
    }
  };
  // One pass with its exchange: twiddles (pass 2), DFT and half-A write of j0, reads r < 8, DFT and half-B write of
  // j1, reads r >= 8; dst_index(b, r) is the pass's output position of butterfly j_b's value r.
  auto pass_exchange = [&](auto twiddle0, auto twiddle1, auto dst_index, auto fetch1) {
    twiddle0(a);
    dft_reg<16, S>(a);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      lds[dst_index(0, r)] = a[r];
    }
    fetch1();  // pass 1: j1's HBM inputs, in flight across the half-A exchange
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      a[r]     = lds[tid + r * 256];
      a[8 + r] = lds[tid + T + r * 256];
    }
    __syncthreads();
    twiddle1(c);
    dft_reg<16, S>(c);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      lds[dst_index(1, r) - H] = c[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      c[r]     = lds[tid + r * 256];
      c[8 + r] = lds[tid + T + r * 256];
    }
    regroup();
  };
  auto none = [](float2 (&)[16]) {};
  // Pass 1 (radix 16, no twiddles): butterfly j takes x[j + 256 r] and writes X[16 j + r].
  pass_exchange(none, none, [&](int b, int r) { return (tid + b * T) * 16 + r; }, [&]() {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      c[r] = src_first(tid + T + r * 256);
    }
  });
  // Pass 2 (NS = 16): butterfly j, k = j mod 16, writes X[(j - k) 16 + k + 16 r] = X[256 (j / 16) + k + 16 r].
  __syncthreads();  // the previous exchange's B reads are done before the buffer is written again
  auto tw1 = [&](float2 (&v)[16]) { twiddle16(v, b1); };
  pass_exchange(
      tw1, tw1,
      [&](int b, int r) {
        const int j = tid + b * T;
        return (j >> 4) * 256 + (j & 15) + 16 * r;
      },
      []() {});
  // Pass 3 (NS = 256): butterfly j (k = j) writes X[j + 256 r] to HBM. An opaque copy of the thread index keeps the
  // output addressing here (hoisted to the kernel start, it spilled). One point per lane and store: two consecutive
  // points per lane (a DPP lane-pair swap, 16-byte stores) measured the same within +-0.6 us in three A/Bs, for 32
  // DPP moves and ~130 selects more (profiles/r6za_ofdm_modulator_ab.txt).
  int tid3 = tid;
  asm volatile("" : "+v"(tid3));
  twiddle16(a, b2a);
  dft_reg<16, S>(a);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    dst_last(tid3 + 256 * r, a[r]);
  }
  twiddle16(c, b2b);
  dft_reg<16, S>(c);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    dst_last(tid3 + T + 256 * r, c[r]);
  }
}

/// Threads per workgroup of the N-point kernels of exponent sign S (the two-wave 4096-point transform, used by the
/// modulator, 128; the 4096-point demodulator keeps four waves: two measured the bench equal and the isolated
/// launch 10 % slower, profiles/r6n_ofdm_demod_waves_ab.txt).
template <int N>
constexpr int ofdm_kernel_threads(int S)
{
  return (N == 4096 && S > 0) ? 128 : ofdm_threads<N>();
}

/// Minimum waves per SIMD the N-point kernels of sign S are compiled for (the two-wave 4096-point one: 8 workgroups
/// per CU, at most 128 VGPRs; the others: the compiler's choice).
template <int N>
constexpr int ofdm_min_waves(int S)
{
  return (N == 4096 && S > 0) ? 4 : 1;
}

/// Any supported N: the power-of-two or the 3 x 2^m decomposition (the modulator's 4096 points: dft4096_two_waves).
template <int N, int S, typename Src, typename Dst>
__device__ __forceinline__ void dft_any(float2* lds, const float2* __restrict__ tw, Src src_first, Dst dst_last)
{
  if constexpr (is_pow2(N)) {
    dft_lds<ilog2(N), S>(lds, tw, src_first, dst_last);
  } else {
    dft_lds3<N, S>(lds, tw, src_first, dst_last);
  }
}

__device__ __forceinline__ uint32_t bf16_bits(float v)
{
  const uint32_t u = __float_as_uint(v);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

/// One job of a launch resolved to its buffers: the grid row, the first sample of the symbol's cyclic prefix, the
/// prefix length and the phase compensation times the scaling.
struct job_ref {
  uint32_t* grid;
  float2*   samples;
  uint32_t  cp;
  float2    coef;
  uint32_t* grid_copy;  ///< demodulation: a second destination row (nullptr: none)
};

/// Jobs as offsets into one grid buffer and one sample buffer (plans and srsgpu_ofdm_jobs_execute).
struct offset_jobs {
  const ofdm_job* jobs;
  uint32_t*       grid;
  float2*         samples;
  uint32_t*       twin = nullptr;  ///< modulation: the grid's HBM twin (same layout), read first (nullptr: none)
  __device__ __forceinline__ job_ref get(unsigned b) const
  {
    // The job is the workgroup's (b = blockIdx.x): its offsets in SGPRs, so that every grid load and sample store
    // addresses the kernel-argument base plus a 32-bit offset (the compiler cannot prove the loaded fields uniform).
    const ofdm_job j    = jobs[b];
    const uint32_t goff = __builtin_amdgcn_readfirstlane(j.grid_offset);
    const uint32_t soff = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(j.sample_offset));
    return {grid + goff, samples + soff, static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(j.cp_len)),
            make_float2(__uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(j.coef_re))),
                        __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(j.coef_im)))),
            twin != nullptr ? twin + goff : nullptr};
  }
};

/// Jobs with absolute device addresses (srsgpu_ofdm_jobs_execute_direct).
struct direct_jobs {
  const srsgpu_ofdm_direct_job* jobs;
  __device__ __forceinline__ job_ref get(unsigned b) const
  {
    const srsgpu_ofdm_direct_job j = jobs[b];
    return {reinterpret_cast<uint32_t*>(j.grid), reinterpret_cast<float2*>(j.samples), j.cp_len,
            make_float2(j.coef_re, j.coef_im), reinterpret_cast<uint32_t*>(j.grid_copy)};
  }
};

/// TWIN: every RE comes from the job's twin row (jb.grid_copy, the PDSCH batch's HBM grid) unless that holds the
/// sentinel 0xffffffff, then from its grid row (the REs the host wrote).
template <int N, typename JS, bool TWIN = false>
__global__ __launch_bounds__(ofdm_kernel_threads<N>(+1), ofdm_min_waves<N>(+1)) void ofdm_modulate_kernel(JS js,
                                                                                              uint32_t nsc,
                                                                                              const float2* __restrict__ tw)
{
  __shared__ float2   lds[N == 4096 ? N / 2 : N];
  const job_ref       jb   = js.get(blockIdx.x);
  const int           half = static_cast<int>(nsc / 2);
  const uint32_t*     row  = jb.grid;
  const uint32_t*     trow = jb.grid_copy;
  // Bin b < rg/2 carries subcarrier rg/2 + b, bin b >= N - rg/2 subcarrier b - (N - rg/2), the rest are zero. The
  // guard bins load subcarrier 0 and discard it (no branch per load; unsigned offsets from the row's SGPR base).
  auto src = [row, trow, half](int b) {
    const uint32_t ub    = static_cast<uint32_t>(b);
    const bool     lower = ub < static_cast<uint32_t>(half);
    const bool     upper = ub >= static_cast<uint32_t>(N - half);
    const uint32_t sc    = lower ? ub + static_cast<uint32_t>(half) : (upper ? ub - static_cast<uint32_t>(N - half) : 0u);
    uint32_t u;
    if constexpr (TWIN) {
      u = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(trow) + sc * 4u);
      if (u == 0xffffffffu) {
        u = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(row) + sc * 4u);
      }
    } else {
      u = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(row) + sc * 4u);
    }
    u = (lower || upper) ? u : 0u;
    return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
  };
  const float2 coef = jb.coef;
  float2*      sym  = jb.samples;
  const int    cp   = static_cast<int>(jb.cp);
  // Unsigned 32-bit byte offsets from the symbol's SGPR base.
  auto dst = [sym, coef, cp](int n, float2 v) {
    const float2 y    = cmul(v, coef);
    char*        base = reinterpret_cast<char*>(sym);
    *reinterpret_cast<float2*>(base + static_cast<uint32_t>(cp + n) * 8u) = y;
    if (n >= N - cp) {
      *reinterpret_cast<float2*>(base + static_cast<uint32_t>(n - (N - cp)) * 8u) = y;
    }
  };
  if constexpr (N == 4096) {
    dft4096_two_waves<+1>(lds, tw, src, dst);
  } else {
    dft_any<N, +1>(lds, tw, src, dst);
  }
}

template <int N, typename JS>
__global__ __launch_bounds__(ofdm_kernel_threads<N>(-1), ofdm_min_waves<N>(-1)) void ofdm_demodulate_kernel(JS js,
                                                                                                uint32_t nsc,
                                                                                                uint32_t window_offset,
                                                                                                const float2* __restrict__ tw)
{
  __shared__ float2 lds[N];  // (the two-wave 4096-point demodulation measured 10 % slower in isolation)
  const job_ref     jb   = js.get(blockIdx.x);
  const int         half = static_cast<int>(nsc / 2);
  // Unsigned 32-bit byte offsets from the job's SGPR bases (no 64-bit address arithmetic per access).
  const char*       x    = reinterpret_cast<const char*>(jb.samples + jb.cp - window_offset);
  auto              src  = [x](int n) { return *reinterpret_cast<const float2*>(x + static_cast<uint32_t>(n) * 8u); };
  const float2      coef = jb.coef;
  char*             row  = reinterpret_cast<char*>(jb.grid);
  char*             row2 = reinterpret_cast<char*>(jb.grid_copy);
  auto dst = [row, row2, coef, half, tw, window_offset](int b, float2 v) {
    const uint32_t ub    = static_cast<uint32_t>(b);
    const bool     lower = ub < static_cast<uint32_t>(half);
    const bool     upper = ub >= static_cast<uint32_t>(N - half);
    const uint32_t sc    = lower ? ub + static_cast<uint32_t>(half) : ub - static_cast<uint32_t>(N - half);
    float2         y     = cmul(v, coef);
    if (window_offset != 0) {  // times exp(+j 2 pi offset b / N)
      y = cmul(y, twiddle_any<N, +1>(tw, (window_offset * ub) % N));
    }
    const uint32_t w = bf16_bits(y.x) | (bf16_bits(y.y) << 16);
    if (lower || upper) {  // guard bins are not stored
      *reinterpret_cast<uint32_t*>(row + sc * 4u) = w;
      if (row2 != nullptr) {
        *reinterpret_cast<uint32_t*>(row2 + sc * 4u) = w;
      }
    }
  };
  dft_any<N, -1>(lds, tw, src, dst);
}

/// Bin b of an N-point transform -> subcarrier of a grid of 2 half subcarriers (-1: a guard bin).
template <int N>
__device__ __forceinline__ int bin_subcarrier(int b, int half)
{
  return (b < half) ? half + b : (b >= N - half ? b - (N - half) : -1);
}

/// Split transform, first kernel: one thread per n1 < M of one job (blockIdx.y), 256 threads per workgroup.
template <int N2, int M, int S, bool MOD>
__global__ __launch_bounds__(256) void ofdm_split_first_kernel(const ofdm_job* __restrict__ jobs,
                                                               uint32_t nsc,
                                                               uint32_t window_offset,
                                                               const uint32_t* __restrict__ grid,
                                                               const float2* __restrict__ in,
                                                               float2* __restrict__ scratch)
{
  constexpr int N  = N2 * M;
  const int     n1 = static_cast<int>(blockIdx.x * 256u + threadIdx.x);
  if (n1 >= M) {
    return;
  }
  const ofdm_job jb = jobs[blockIdx.y];
  float2         x[N2];
  if constexpr (MOD) {
    const uint32_t* row  = grid + jb.grid_offset;
    const int       half = static_cast<int>(nsc / 2);
#pragma unroll
    for (int n2 = 0; n2 < N2; ++n2) {
      const int sc = bin_subcarrier<N>(n1 + M * n2, half);
      if (sc < 0) {
        x[n2] = make_float2(0.f, 0.f);
      } else {
        const uint32_t u = row[sc];
        x[n2]            = make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
      }
    }
  } else {
    const float2* src = in + jb.sample_offset + jb.cp_len - window_offset;
#pragma unroll
    for (int n2 = 0; n2 < N2; ++n2) {
      x[n2] = src[n1 + M * n2];
    }
  }
  // exp(S 2 pi i m / N2), m < N2 (argument rounded once).
  float2 w2[N2];
#pragma unroll
  for (int m = 0; m < N2; ++m) {
    sincospif(static_cast<float>(2 * m) / static_cast<float>(N2), &w2[m].y, &w2[m].x);
    w2[m].y = S * w2[m].y;
  }
  float2* out = scratch + static_cast<size_t>(blockIdx.y) * N + n1;
#pragma unroll
  for (int k2 = 0; k2 < N2; ++k2) {
    float2 acc = x[0];
#pragma unroll
    for (int n2 = 1; n2 < N2; ++n2) {
      const float2 t = cmul(x[n2], w2[(n2 * k2) % N2]);
      acc            = cadd(acc, t);
    }
    if (k2 != 0) {
      float2 w;
      sincospif(static_cast<float>(2 * ((n1 * k2) % N)) / static_cast<float>(N), &w.y, &w.x);
      w.y = S * w.y;
      acc = cmul(acc, w);
    }
    out[k2 * M] = acc;
  }
}

/// Split transform, second kernel: workgroup (job, k2) runs the M-point LDS transform of scratch row k2 and writes
/// outputs k2 + N2 k1 (time samples with coefficient and cyclic prefix, or bf16 subcarriers).
template <int N2, int M, int S, bool MOD>
__global__ __launch_bounds__(M / 16) void ofdm_split_second_kernel(const ofdm_job* __restrict__ jobs,
                                                                   uint32_t nsc,
                                                                   uint32_t window_offset,
                                                                   const float2* __restrict__ tw,
                                                                   const float2* __restrict__ scratch,
                                                                   uint32_t* __restrict__ grid,
                                                                   float2* __restrict__ out)
{
  constexpr int     N   = N2 * M;
  __shared__ float2 lds[M];
  const uint32_t    job = blockIdx.x / N2, k2 = blockIdx.x % N2;
  const ofdm_job    jb  = jobs[job];
  const float2*     row = scratch + static_cast<size_t>(job) * N + static_cast<size_t>(k2) * M;
  auto              src = [row](int n) { return row[n]; };
  const float2      coef = make_float2(jb.coef_re, jb.coef_im);
  if constexpr (MOD) {
    float2*   sym = out + jb.sample_offset;
    const int cp  = static_cast<int>(jb.cp_len);
    auto dst = [sym, coef, cp, k2](int k1, float2 v) {
      const int    n = static_cast<int>(k2) + N2 * k1;
      const float2 y = cmul(v, coef);
      sym[cp + n]    = y;
      if (n >= N - cp) {
        sym[n - (N - cp)] = y;
      }
    };
    dft_lds<ilog2(M), S>(lds, tw, src, dst);
  } else {
    uint32_t* grow = grid + jb.grid_offset;
    const int half = static_cast<int>(nsc / 2);
    auto dst = [grow, coef, half, tw, window_offset, k2](int k1, float2 v) {
      const int b  = static_cast<int>(k2) + N2 * k1;
      const int sc = bin_subcarrier<N>(b, half);
      if (sc < 0) {
        return;
      }
      float2 y = cmul(v, coef);
      if (window_offset != 0) {  // times exp(+j 2 pi offset b / N)
        y = cmul(y, twiddle_any<N, +1>(tw, (window_offset * static_cast<uint32_t>(b)) % N));
      }
      grow[sc] = bf16_bits(y.x) | (bf16_bits(y.y) << 16);
    };
    dft_lds<ilog2(M), S>(lds, tw, src, dst);
  }
}

template <int N2, int M>
void launch_split(bool            inverse,
                  const ofdm_job* jobs,
                  int             nof_jobs,
                  uint32_t        nsc,
                  uint32_t        window_offset,
                  const float2*   tw,
                  const uint32_t* grid_in,
                  uint32_t*       grid_out,
                  const float2*   samples_in,
                  float2*         samples_out,
                  float2*         scratch,
                  hipStream_t     stream)
{
  const dim3 g1((M + 255) / 256, static_cast<unsigned>(nof_jobs)), b1(256);
  const dim3 g2(static_cast<unsigned>(nof_jobs) * N2), b2(M / 16);
  if (inverse) {
    hipLaunchKernelGGL((ofdm_split_first_kernel<N2, M, +1, true>), g1, b1, 0, stream, jobs, nsc, 0u, grid_in,
                       nullptr, scratch);
    hipLaunchKernelGGL((ofdm_split_second_kernel<N2, M, +1, true>), g2, b2, 0, stream, jobs, nsc, 0u, tw, scratch,
                       nullptr, samples_out);
  } else {
    hipLaunchKernelGGL((ofdm_split_first_kernel<N2, M, -1, false>), g1, b1, 0, stream, jobs, nsc, window_offset,
                       nullptr, samples_in, scratch);
    hipLaunchKernelGGL((ofdm_split_second_kernel<N2, M, -1, false>), g2, b2, 0, stream, jobs, nsc, window_offset, tw,
                       scratch, grid_out, nullptr);
  }
}

template <int N, typename JS>
void launch_one(bool inverse, JS js, int nof_jobs, uint32_t nsc, uint32_t window_offset, const float2* tw,
                hipStream_t stream)
{
  const int threads = ofdm_kernel_threads<N>(inverse ? 1 : -1);  // every thread takes part in the passes' barriers
  if (inverse) {
    if constexpr (std::is_same_v<JS, offset_jobs>) {
      if (js.twin != nullptr) {
        hipLaunchKernelGGL((ofdm_modulate_kernel<N, JS, true>), dim3(static_cast<unsigned>(nof_jobs)), dim3(threads), 0,
                           stream, js, nsc, tw);
        return;
      }
    }
    hipLaunchKernelGGL((ofdm_modulate_kernel<N, JS>), dim3(static_cast<unsigned>(nof_jobs)), dim3(threads), 0, stream,
                       js, nsc, tw);
  } else {
    hipLaunchKernelGGL((ofdm_demodulate_kernel<N, JS>), dim3(static_cast<unsigned>(nof_jobs)), dim3(threads), 0,
                       stream, js, nsc, window_offset, tw);
  }
}

/// Every non-split DFT size: its launch over the job source.
template <typename JS>
bool launch_sizes(bool inverse, uint32_t dft_size, JS js, int nof_jobs, uint32_t nsc, uint32_t window_offset,
                  const float2* tw, hipStream_t stream)
{
  switch (dft_size) {
    case 128: launch_one<128>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 256: launch_one<256>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 512: launch_one<512>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 1024: launch_one<1024>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 2048: launch_one<2048>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 4096: launch_one<4096>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 8192: launch_one<8192>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 384: launch_one<384>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 768: launch_one<768>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 1536: launch_one<1536>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 3072: launch_one<3072>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 4608: launch_one<4608>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    case 6144: launch_one<6144>(inverse, js, nof_jobs, nsc, window_offset, tw, stream); return true;
    default: return false;
  }
}

} // namespace

void launch_ofdm(bool            inverse,
                 uint32_t        dft_size,
                 const ofdm_job* d_jobs,
                 int             nof_jobs,
                 uint32_t        nsc,
                 uint32_t        window_offset,
                 const float*    d_twiddles,
                 const uint32_t* d_grid_in,
                 uint32_t*       d_grid_out,
                 const float*    d_samples_in,
                 float*          d_samples_out,
                 float*          d_scratch,
                 hipStream_t     stream,
                 const uint32_t* d_twin)
{
  if (nof_jobs <= 0) {
    return;
  }
  const auto* tw  = reinterpret_cast<const float2*>(d_twiddles);
  const auto* sin = reinterpret_cast<const float2*>(d_samples_in);
  auto*       so  = reinterpret_cast<float2*>(d_samples_out);
  // The kernels only read the input buffer of their direction.
  const offset_jobs js{d_jobs, inverse ? const_cast<uint32_t*>(d_grid_in) : d_grid_out,
                       inverse ? so : const_cast<float2*>(sin), inverse ? const_cast<uint32_t*>(d_twin) : nullptr};
  if (launch_sizes(inverse, dft_size, js, nof_jobs, nsc, window_offset, tw, stream)) {
    return;
  }
  auto* sc = reinterpret_cast<float2*>(d_scratch);
  switch (dft_size) {
    case 9216: launch_split<9, 1024>(inverse, d_jobs, nof_jobs, nsc, window_offset, tw, d_grid_in, d_grid_out, sin, so, sc, stream); break;
    case 12288: launch_split<3, 4096>(inverse, d_jobs, nof_jobs, nsc, window_offset, tw, d_grid_in, d_grid_out, sin, so, sc, stream); break;
    case 18432: launch_split<9, 2048>(inverse, d_jobs, nof_jobs, nsc, window_offset, tw, d_grid_in, d_grid_out, sin, so, sc, stream); break;
    case 24576: launch_split<3, 8192>(inverse, d_jobs, nof_jobs, nsc, window_offset, tw, d_grid_in, d_grid_out, sin, so, sc, stream); break;
    case 36864: launch_split<9, 4096>(inverse, d_jobs, nof_jobs, nsc, window_offset, tw, d_grid_in, d_grid_out, sin, so, sc, stream); break;
    case 49152: launch_split<6, 8192>(inverse, d_jobs, nof_jobs, nsc, window_offset, tw, d_grid_in, d_grid_out, sin, so, sc, stream); break;
    case 98304: launch_split<12, 8192>(inverse, d_jobs, nof_jobs, nsc, window_offset, tw, d_grid_in, d_grid_out, sin, so, sc, stream); break;
    default: break;
  }
}

bool launch_ofdm_direct(bool                          inverse,
                        uint32_t                      dft_size,
                        const srsgpu_ofdm_direct_job* d_jobs,
                        int                           nof_jobs,
                        uint32_t                      nsc,
                        uint32_t                      window_offset,
                        const float*                  d_twiddles,
                        hipStream_t                   stream)
{
  if (nof_jobs <= 0) {
    return true;
  }
  return launch_sizes(inverse, dft_size, direct_jobs{d_jobs}, nof_jobs, nsc, window_offset,
                      reinterpret_cast<const float2*>(d_twiddles), stream);
}

} // namespace srsgpu
