// LDPC rate dematching with HARQ soft combining for 5G NR (TS 38.212 §5.4.2), batched over codeblocks, for gfx950.
//
// Drop-in semantics of srsran::ldpc_rate_dematcher_impl::rate_dematch (reference lib/phy/upper/channel_coding/ldpc/
// ldpc_rate_dematcher_impl.cpp:46): bit de-interleaving (:203), circular-buffer allotment starting at k0 with filler
// skipping (:128), copy on the first pass for new data and saturated LLR combining afterwards (generic :116 or SIMD
// ldpc_rate_dematcher_avx2_impl.cpp:29), filler LLRs = +infinity, and the reference's exact treatment of positions the
// first pass does not reach (zeroed / left as they were, including the limited-buffer tail zeroing of :198).
//
// The reference walks the circular buffer sequentially; here every output position k is computed independently:
// its valid-position index v(k) (fillers removed) maps to the input indices n = ((v - v0) mod V) + p*V, p = 0, 1, ...,
// which are combined in increasing n exactly like the sequential walk. The formulation is validated against the CPU
// oracle (tests/test_pusch_gpu.py) on random configurations, including LBRM and inputs ending in the first pass.
#include "common.h"
#include "srsgpu_internal.h"

namespace srsgpu {
namespace {

constexpr int LLR_MAX = 120;

template <int MODE>
__device__ __forceinline__ int llr_combine(int a, int b)
{
  if constexpr (MODE == 1) {
    // avx2 combine: int8 saturating add, clamp to +/-LLR_MAX.
    return clamp_i(a + b, -LLR_MAX, LLR_MAX);
  } else {
    // log_likelihood_ratio operator+ (log_likelihood_ratio.cpp:40): a == -b -> 0; infinities absorb; else saturate.
    if (a == -b) {
      return 0;
    }
    if (a > LLR_MAX || a < -LLR_MAX) {
      return a;
    }
    if (b > LLR_MAX || b < -LLR_MAX) {
      return b;
    }
    return clamp_i(a + b, -LLR_MAX, LLR_MAX);
  }
}

/// Value of HARQ buffer position k after rate dematching (the per-position formulation above).
template <int MODE>
__device__ __forceinline__ int dematch_position(const dm_desc& d, const int8_t* __restrict__ in, int k, int old,
                                                int zero_from)
{
  const int E = static_cast<int>(d.E), Qm = d.Qm, R = E / Qm;
  const int Ncb = static_cast<int>(d.Ncb);
  const int nsys = static_cast<int>(d.nsys), F = d.nof_filler, ninfo = nsys - F;
  const int V  = Ncb - F;
  const int v0 = static_cast<int>(d.v0);
  // Input index of circular-buffer visit n: bit n / R of symbol n % R (bit interleaver, :203), division by the
  // host-computed magic number (exact for n < 2^20).
  auto in_index = [&](int n) {
    const int q = static_cast<int>((static_cast<uint64_t>(static_cast<uint32_t>(n)) * d.r_magic) >> 40);
    return (n - q * R) * Qm + q;
  };
  int val = old;
  if (k < Ncb) {
    if (k >= ninfo && k < nsys) {
      val = d.new_data ? 127 : val;  // filler bits: +infinity (:172)
    } else {
      const int v  = k < ninfo ? k : k - F;
      int       n0 = v - v0;
      n0           = n0 < 0 ? n0 + V : n0;
      int n        = n0;
      if (d.new_data) {
        if (v >= v0) {
          if (n0 < E) {
            val = in[in_index(n0)];  // first pass: copy
            n   = n0 + V;
          } else {
            n = E;  // not reached: keep (or zeroed below)
          }
        } else {
          val = (k < ninfo) ? 0 : val;  // before k0: systematic zeroed, parity keeps its content
        }
      }
      for (; n < E; n += V) {
        val = llr_combine<MODE>(val, in[in_index(n)]);
      }
    }
  }
  return (k >= zero_from) ? 0 : val;
}

/// Any transmission, position by position (dword read-modify-write where aligned).
template <int MODE>
__device__ __forceinline__ void dematch_general(const dm_desc& d, const int8_t* __restrict__ llrs,
                                                int8_t* __restrict__ buf)
{
  const int8_t* in  = llrs + d.llr_offset;
  const int     E = static_cast<int>(d.E);
  const int     N = static_cast<int>(d.N), Ncb = static_cast<int>(d.Ncb);
  const int     nsys = static_cast<int>(d.nsys), F = d.nof_filler, ninfo = nsys - F;
  const int     V  = Ncb - F;
  const int     v0 = static_cast<int>(d.v0);
  // Walk end of an incomplete first pass (E < V - v0): allot_llrs zeroes the last (Ncb - k_end) LLRs of the buffer.
  const bool incomplete = d.new_data && (E < V - v0);
  int        zero_from  = N;
  if (incomplete) {
    const int vend = v0 + E;
    int       kend = vend < ninfo ? vend : vend + F;
    kend           = kend < nsys ? nsys : kend;
    kend           = kend % Ncb;
    if (kend != 0) {
      zero_from = N - (Ncb - kend);
    }
  }
  if (((static_cast<uint32_t>(reinterpret_cast<uintptr_t>(buf)) | static_cast<uint32_t>(N)) & 3u) == 0u) {
    // Dword read-modify-write of four consecutive positions per lane.
    auto* buf32 = reinterpret_cast<uint32_t*>(buf);
    for (int k4 = threadIdx.x; k4 < N / 4; k4 += blockDim.x) {
      const uint32_t old = buf32[k4];
      uint32_t       w   = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int v = dematch_position<MODE>(d, in, 4 * k4 + b, static_cast<int8_t>(old >> (8 * b)), zero_from);
        w |= (static_cast<uint32_t>(v) & 0xffu) << (8 * b);
      }
      buf32[k4] = w;
    }
  } else {
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
      buf[k] = static_cast<int8_t>(dematch_position<MODE>(d, in, k, buf[k], zero_from));
    }
  }
}

/// First transmissions without repetition (new data, E <= V): the positions visited by the first pass before the
/// circular buffer wraps are plain copies of the de-interleaved input. They are written symbol-major: lane r reads
/// the Qm LLRs of symbol r (contiguous) and stores bit j at visit n = j R + r, so every store instruction of a wave
/// covers consecutive buffer bytes. Every other position (fillers, wrapped visits, positions not reached, the
/// limited-buffer tail) takes the per-position path, skipped a whole 16-position vector at a time when it holds only
/// copy positions. The two phases write disjoint bytes.
template <int MODE>
__device__ __forceinline__ void dematch_new_data(const dm_desc& d, const int8_t* __restrict__ llrs,
                                                 int8_t* __restrict__ buf)
{
  const int8_t* in  = llrs + d.llr_offset;
  const int     E = static_cast<int>(d.E), Qm = d.Qm, R = E / Qm;
  const int     N = static_cast<int>(d.N), Ncb = static_cast<int>(d.Ncb);
  const int     nsys = static_cast<int>(d.nsys), F = d.nof_filler, ninfo = nsys - F;
  const int     V  = Ncb - F;
  const int     v0 = static_cast<int>(d.v0);
  const int     nc = (V - v0 < E) ? V - v0 : E;  // visits before the wrap: copies of positions v0 .. v0 + nc - 1
  int           zero_from = N;
  if (E < V - v0) {
    const int vend = v0 + E;
    int       kend = vend < ninfo ? vend : vend + F;
    kend           = kend < nsys ? nsys : kend;
    kend           = kend % Ncb;
    if (kend != 0) {
      zero_from = N - (Ncb - kend);
    }
  }
  // Phase 1: copies, symbol-major.
  // 256QAM symbols 8-byte aligned (codewords are whole symbols from an aligned offset): one 8-byte load each.
  const bool q8 = Qm == 8 && ((d.llr_offset & 7u) == 0u);
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    int8_t sym[8];
    if (q8) {
      const uint2 v = *reinterpret_cast<const uint2*>(in + 8 * r);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sym[j] = static_cast<int8_t>(((j < 4) ? v.x : v.y) >> (8 * (j & 3)));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sym[j] = (j < Qm) ? in[r * Qm + j] : 0;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = j * R + r;
      if (j < Qm && n < nc) {
        const int v = v0 + n;
        const int k = v < ninfo ? v : v + F;
        if (k < zero_from) {
          buf[k] = sym[j];
        }
      }
    }
  }
  // Phase 2: every non-copy position, 16 positions per lane and step.
  auto is_copy = [&](int k) {
    if (k >= Ncb || (k >= ninfo && k < nsys) || k >= zero_from) {
      return false;
    }
    const int v = k < ninfo ? k : k - F;
    return v >= v0 && v - v0 < nc;
  };
  for (int k0 = 16 * static_cast<int>(threadIdx.x); k0 < N; k0 += 16 * static_cast<int>(blockDim.x)) {
    // Copy positions form one or two k-intervals: a vector entirely inside is skipped.
    if (k0 + 15 < N && is_copy(k0) && is_copy(k0 + 15) &&
        !(k0 < ninfo && k0 + 15 >= ninfo)) {
      continue;
    }
    if (k0 >= zero_from && k0 + 15 < N && ((reinterpret_cast<uintptr_t>(buf) + static_cast<uint32_t>(k0)) & 15u) == 0u) {
      *reinterpret_cast<uint4*>(buf + k0) = make_uint4(0u, 0u, 0u, 0u);  // limited-buffer / walk-end zero tail
      continue;
    }
    for (int b = 0; b < 16 && k0 + b < N; ++b) {
      const int k = k0 + b;
      if (!is_copy(k)) {
        // The previous content only matters where the reference leaves it (not zeroed, not a filler).
        const bool keeps = k < zero_from && !(k >= ninfo && k < nsys);
        buf[k]           = static_cast<int8_t>(dematch_position<MODE>(d, in, k, keeps ? buf[k] : 0, zero_from));
      }
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void rate_dematch_kernel(const dm_desc* __restrict__ descs,
                                                           const int8_t* __restrict__ llrs,
                                                           int8_t* __restrict__ harq,
                                                           int8_t* const* __restrict__ harq_cbs,
                                                           uint8_t* __restrict__ cb_crc_ok)
{
  const dm_desc d = descs[blockIdx.x];
  // The codeblock's soft buffer: at its offset in the batch HARQ buffer, or wherever harq_cbs[cb] points (a slot of a
  // persistent rx-buffer arena, srsgpu_pusch_decoder_plan_execute_arena).
  int8_t* const buf = (harq_cbs != nullptr) ? harq_cbs[d.cb_index] : harq + d.harq_offset;
  // New data invalidates the codeblock CRC flags of the HARQ context (pusch_decoder_impl.cpp:132).
  if (d.new_data && cb_crc_ok != nullptr && threadIdx.x == 0) {
    cb_crc_ok[d.cb_index] = 0;
  }
  const int V = static_cast<int>(d.Ncb) - d.nof_filler;
  if (d.new_data && static_cast<int>(d.E) <= V && d.Qm <= 8) {
    dematch_new_data<MODE>(d, llrs, buf);
  } else {
    dematch_general<MODE>(d, llrs, buf);
  }
}

} // namespace

void launch_rate_dematch(int           mode,
                         const dm_desc* d_desc,
                         int           nof_cbs,
                         const int8_t* d_llrs,
                         int8_t*       d_harq,
                         uint8_t*      d_cb_crc_ok,
                         hipStream_t   stream,
                         int8_t* const* d_harq_cbs)
{
  if (nof_cbs <= 0) {
    return;
  }
  if (mode == 1) {
    rate_dematch_kernel<1><<<nof_cbs, 256, 0, stream>>>(d_desc, d_llrs, d_harq, d_harq_cbs, d_cb_crc_ok);
  } else {
    rate_dematch_kernel<0><<<nof_cbs, 256, 0, stream>>>(d_desc, d_llrs, d_harq, d_harq_cbs, d_cb_crc_ok);
  }
}

} // namespace srsgpu
