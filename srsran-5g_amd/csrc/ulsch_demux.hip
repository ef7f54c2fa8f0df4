// UL-SCH demultiplexer (UCI on PUSCH) on gfx950: one lane per RE routes the RE's layers x Qm demodulated LLRs to the
// UL-SCH data stream and / or a UCI stream (HARQ-ACK, CSI Part 1, CSI Part 2) by the plan's per-RE table, applying the
// 1- / 2-bit UCI placeholder sign fixes with the transmission's scrambling sequence (plan-resident Gold words).
//
// Reference (behaviour, not code): lib/phy/upper/channel_processors/pusch/ulsch_demultiplex_impl.cpp:455
// (demux_current_ofdm_symbol), :91 (on_uci_placeholder_1bit), :131 (on_uci_placeholder_2bit). Byte traffic: every
// codeword LLR read once and written once (HBM-bound, tiny next to the demodulator that produced it).
#include "srsgpu_internal.h"

namespace srsgpu {
namespace {

constexpr int DEMUX_THREADS = 256;

__global__ __launch_bounds__(DEMUX_THREADS) void ulsch_demux_kernel(const ulsch_demux_desc* __restrict__ descs,
                                                                   const ulsch_demux_route* __restrict__ routes,
                                                                   const mod_chunk* __restrict__ chunks,
                                                                   const int8_t* __restrict__ llrs,
                                                                   int8_t* __restrict__ sch,
                                                                   int8_t* __restrict__ harq,
                                                                   int8_t* __restrict__ csi1,
                                                                   int8_t* __restrict__ csi2,
                                                                   const uint32_t* __restrict__ gseq)
{
  const mod_chunk         ch = chunks[blockIdx.x];
  const ulsch_demux_desc& d  = descs[ch.tx];
  const uint32_t          r  = ch.re_begin + threadIdx.x;
  if (r >= ch.re_end) {
    return;
  }
  const ulsch_demux_route rt  = routes[d.route + r];
  const uint32_t          lq  = d.lq;
  const int8_t*           src = llrs + d.llr_offset + r * lq;
  int8_t                  v[32];
  for (uint32_t j = 0; j < lq; ++j) {
    v[j] = src[j];
  }
  const uint32_t kind = rt.uci >> 30;
  if (kind != 0) {
    int8_t* const  out[3] = {harq, csi1, csi2};
    int8_t*        dst    = out[kind - 1] + d.uci_offset[kind - 1] + (rt.uci & 0x3fffffffu) * lq;
    const uint32_t ph     = d.placeholder[kind - 1];
    if (ph != 0) {
      // Scrambling bits of the RE's LLRs (MSB-first words): per modulation symbol, "y" (1 bit: the second LLR takes the
      // first one's scrambling) and "x" (LLRs 2..Qm-1 unscrambled).
      const uint32_t nwords = (d.nof_llrs + 31u) >> 5;
      const uint32_t pos    = r * lq;
      const uint32_t wi     = pos >> 5;
      const uint64_t w0     = gseq[d.seq_word_offset + wi];
      const uint64_t w1     = (wi + 1 < nwords) ? gseq[d.seq_word_offset + wi + 1] : 0u;
      const uint64_t sb     = ((w0 << 32) | w1) << (pos & 31u);
      for (uint32_t j = 0; j < lq; ++j) {
        const uint32_t b   = static_cast<uint32_t>(sb >> (63 - j)) & 1u;
        const uint32_t k   = j % d.qm;
        bool           neg = false;
        if (k == 1 && ph == 1) {
          neg = (b ^ (static_cast<uint32_t>(sb >> (64 - j)) & 1u)) != 0;
        } else if (k >= 2) {
          neg = b != 0;
        }
        dst[j] = static_cast<int8_t>(neg ? -v[j] : v[j]);
      }
    } else {
      for (uint32_t j = 0; j < lq; ++j) {
        dst[j] = v[j];
      }
    }
  }
  if (rt.sch != DEMUX_NONE) {
    // A HARQ-ACK RE of <= 2 bits stays in the UL-SCH set with zeroed LLRs.
    const bool zero = kind == 1;
    int8_t*    dst  = sch + d.sch_offset + rt.sch * lq;
    for (uint32_t j = 0; j < lq; ++j) {
      dst[j] = zero ? int8_t(0) : v[j];
    }
  }
  if (rt.csi2 != DEMUX_NONE) {
    // CSI Part 2 on a reserved RE punctured by HARQ-ACK of <= 2 bits: it reads the zeroed LLRs.
    int8_t* dst = csi2 + d.uci_offset[2] + rt.csi2 * lq;
    for (uint32_t j = 0; j < lq; ++j) {
      dst[j] = 0;
    }
  }
}

} // namespace

void launch_ulsch_demux(const ulsch_demux_desc*  d_desc,
                        const ulsch_demux_route* d_routes,
                        const mod_chunk*         d_chunks,
                        int                      nof_chunks,
                        const int8_t*            d_llrs,
                        int8_t*                  d_sch,
                        int8_t*                  d_harq,
                        int8_t*                  d_csi1,
                        int8_t*                  d_csi2,
                        const uint32_t*          d_seq,
                        hipStream_t              stream)
{
  if (nof_chunks <= 0) {
    return;
  }
  hipLaunchKernelGGL(ulsch_demux_kernel, dim3(static_cast<unsigned>(nof_chunks)), dim3(DEMUX_THREADS), 0, stream,
                     d_desc, d_routes, d_chunks, d_llrs, d_sch, d_harq, d_csi1, d_csi2, d_seq);
}

} // namespace srsgpu
