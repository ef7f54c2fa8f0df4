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

template <int MODE>
__global__ __launch_bounds__(256) void rate_dematch_kernel(const dm_desc* __restrict__ descs,
                                                           const int8_t* __restrict__ llrs,
                                                           int8_t* __restrict__ harq,
                                                           uint8_t* __restrict__ cb_crc_ok)
{
  const dm_desc d = descs[blockIdx.x];
  // New data invalidates the codeblock CRC flags of the HARQ context (pusch_decoder_impl.cpp:132).
  if (d.new_data && cb_crc_ok != nullptr && threadIdx.x == 0) {
    cb_crc_ok[d.cb_index] = 0;
  }
  const int8_t* in  = llrs + d.llr_offset;
  int8_t*       buf = harq + d.harq_offset;
  const int     E = static_cast<int>(d.E), Qm = d.Qm, R = E / Qm;
  const int     N = static_cast<int>(d.N), Ncb = static_cast<int>(d.Ncb);
  const int     nsys = static_cast<int>(d.nsys), F = d.nof_filler, ninfo = nsys - F;
  const int     V  = Ncb - F;
  const int     v0 = static_cast<int>(d.v0);
  const bool    new_data = d.new_data != 0;
  // Walk end of an incomplete first pass (E < V - v0): allot_llrs zeroes the last (Ncb - k_end) LLRs of the buffer.
  const bool incomplete = new_data && (E < V - v0);
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
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    int val = buf[k];
    if (k < Ncb) {
      if (k >= ninfo && k < nsys) {
        val = new_data ? 127 : val;  // filler bits: +infinity (:172)
      } else {
        const int v  = k < ninfo ? k : k - F;
        int       n0 = v - v0;
        n0           = n0 < 0 ? n0 + V : n0;
        int n        = n0;
        if (new_data) {
          if (v >= v0) {
            if (n0 < E) {
              val = in[(n0 % R) * Qm + n0 / R];  // first pass: copy
              n   = n0 + V;
            } else {
              n = E;  // not reached: keep (or zeroed below)
            }
          } else {
            val = (k < ninfo) ? 0 : val;  // before k0: systematic zeroed, parity keeps its content
          }
        }
        for (; n < E; n += V) {
          val = llr_combine<MODE>(val, in[(n % R) * Qm + n / R]);
        }
      }
    }
    if (k >= zero_from) {
      val = 0;
    }
    buf[k] = static_cast<int8_t>(val);
  }
}

} // namespace

void launch_rate_dematch(int           mode,
                         const dm_desc* d_desc,
                         int           nof_cbs,
                         const int8_t* d_llrs,
                         int8_t*       d_harq,
                         uint8_t*      d_cb_crc_ok,
                         hipStream_t   stream)
{
  if (nof_cbs <= 0) {
    return;
  }
  if (mode == 1) {
    rate_dematch_kernel<1><<<nof_cbs, 256, 0, stream>>>(d_desc, d_llrs, d_harq, d_cb_crc_ok);
  } else {
    rate_dematch_kernel<0><<<nof_cbs, 256, 0, stream>>>(d_desc, d_llrs, d_harq, d_cb_crc_ok);
  }
}

} // namespace srsgpu
