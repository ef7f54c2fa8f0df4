// Host side of the UL-SCH demultiplexer C ABI (include/srsgpu_phy.h): the per-OFDM-symbol RE sets of TS 38.212
// section 6.2.7 as ulsch_demultiplex_impl::configure_current_ofdm_symbol (ulsch_demultiplex_impl.cpp:316) builds them,
// flattened into one routing entry per codeword RE, plus the scrambling sequences for the placeholders.
#include "capi_internal.h"
#include <algorithm>
#include <array>
#include <vector>

using namespace srsgpu;

static_assert(sizeof(srsgpu_ulsch_demux_config) == 64, "srsgpu_ulsch_demux_config layout (mirrored by srsgpu)");

struct srsgpu_ulsch_demux_plan {
  srsgpu_context*                    ctx        = nullptr;
  ulsch_demux_desc*                  d_desc     = nullptr;
  ulsch_demux_route*                 d_routes   = nullptr;
  mod_chunk*                         d_chunks   = nullptr;
  uint32_t*                          d_seq      = nullptr;
  int                                nof_chunks = 0;
  std::vector<std::array<uint32_t, 5>> nof_llrs;  ///< Per transmission: codeword, UL-SCH, HARQ-ACK, CSI-1, CSI-2.
  std::vector<std::array<std::array<uint32_t, 14>, 5>> symbol_llrs;  ///< The same per OFDM symbol.
};

namespace {

/// re_set_select (:68): from the available RE indices (ascending) every d-th one, count of them.
std::vector<uint32_t> re_select(const std::vector<uint32_t>& avail, uint32_t d, uint32_t count)
{
  std::vector<uint32_t> out;
  for (size_t i = 0; i < avail.size() && out.size() < count; i += d) {
    out.push_back(avail[i]);
  }
  return out;
}

std::vector<uint32_t> indices(const std::vector<uint8_t>& set)
{
  std::vector<uint32_t> out;
  for (uint32_t i = 0; i < set.size(); ++i) {
    if (set[i]) {
      out.push_back(i);
    }
  }
  return out;
}

/// (d, m_re_count) of every step: all M available REs, or every (M / remainder)-th one, remainder of them.
void pick(uint32_t m, uint32_t remainder, uint32_t& d, uint32_t& n)
{
  d = 1;
  n = m;
  if (remainder < m) {
    d = m / remainder;
    n = remainder;
  }
}

} // namespace

extern "C" {

int srsgpu_ulsch_demux_plan_create(srsgpu_context*                  ctx,
                                   const srsgpu_ulsch_demux_config* cfgs,
                                   uint32_t                         nof_tx,
                                   srsgpu_ulsch_demux_plan**        plan_out)
{
  if (ctx == nullptr || plan_out == nullptr || (cfgs == nullptr && nof_tx > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  std::vector<ulsch_demux_desc>     descs(nof_tx);
  std::vector<ulsch_demux_route>    routes;
  std::vector<mod_chunk>            chunks;
  std::vector<std::array<uint32_t, 5>> counts(nof_tx);
  std::vector<std::array<std::array<uint32_t, 14>, 5>> sym_counts(nof_tx);
  std::vector<uint32_t>             c_inits(nof_tx), nwords(nof_tx);
  for (uint32_t t = 0; t < nof_tx; ++t) {
    const srsgpu_ulsch_demux_config& c  = cfgs[t];
    const uint32_t                   qm = c.modulation_order, L = c.nof_layers;
    if ((qm != 2 && qm != 4 && qm != 6 && qm != 8) || L < 1 || L > 4 || c.nof_prb < 1 || c.nof_prb > 275 ||
        c.nof_symbols < 1 || c.start_symbol + c.nof_symbols > 14 || (c.dmrs_type != 1 && c.dmrs_type != 2) ||
        c.nof_cdm_groups_without_data < 1 || c.nof_cdm_groups_without_data > (c.dmrs_type == 1 ? 2 : 3) ||
        (c.dmrs_symbol_mask & 0x3fffu) == 0 || (c.dmrs_symbol_mask & 0x3fffu) == 0x3fffu || c.n_id >= (1u << 15)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid modulation, layers, allocation or DM-RS", t);
    }
    const uint32_t lq   = qm * L;
    const uint32_t mask = c.dmrs_symbol_mask;
    auto           dm   = [&](unsigned l) { return ((mask >> l) & 1u) != 0; };
    // l1: first symbol without DM-RS after the first DM-RS symbol (:29); l1_csi: first symbol without DM-RS (:45).
    unsigned first_dmrs = 0;
    while (!dm(first_dmrs)) {
      ++first_dmrs;
    }
    unsigned l1 = first_dmrs;
    while (l1 < 14 && dm(l1)) {
      ++l1;
    }
    unsigned l1_csi = 0;
    while (dm(l1_csi)) {
      ++l1_csi;
    }
    const uint32_t re_dmrs = (12u - (c.dmrs_type == 2 ? 4u : 6u) * c.nof_cdm_groups_without_data) * c.nof_prb;
    uint32_t       m_rvd = 0, m_harq = 0, m_csi1 = 0, m_csi2 = 0;
    uint32_t       n_sch = 0, n_uci[3] = {0, 0, 0}, n_re = 0;
    ulsch_demux_desc& d  = descs[t];
    d.route              = static_cast<uint32_t>(routes.size());
    for (unsigned l = c.start_symbol; l < static_cast<unsigned>(c.start_symbol + c.nof_symbols); ++l) {
      const uint32_t       M = dm(l) ? re_dmrs : 12u * c.nof_prb;
      std::vector<uint8_t> ulsch(M, 1), uci(M, dm(l) ? 0 : 1);
      std::vector<uint32_t> rvd, harq, csi1, csi2;
      uint32_t              M_uci = dm(l) ? 0u : M;
      uint32_t              dd, nn;
      // Step 1: reserved REs for HARQ-ACK.
      const uint32_t rem_rvd = (c.nof_harq_ack_rvd - std::min(m_rvd, c.nof_harq_ack_rvd)) / lq;
      if (l >= l1 && M_uci > 0 && rem_rvd > 0) {
        pick(M_uci, rem_rvd, dd, nn);
        rvd = re_select(indices(ulsch), dd, nn);
        m_rvd += nn * lq;
      }
      // Step 2: HARQ-ACK of more than two bits.
      const uint32_t rem_harq = (c.nof_enc_harq_ack_bits - std::min(m_harq, c.nof_enc_harq_ack_bits)) / lq;
      if (l >= l1 && M_uci > 0 && c.nof_harq_ack_bits > 2 && rem_harq > 0) {
        pick(M_uci, rem_harq, dd, nn);
        harq = re_select(indices(uci), dd, nn);
        for (uint32_t i : harq) {
          ulsch[i] = uci[i] = 0;
        }
        M_uci = static_cast<uint32_t>(indices(uci).size());
        m_harq += nn * lq;
      }
      // Step 3: CSI Part 1 outside the reserved REs.
      const uint32_t rem_csi1 = (c.nof_enc_csi_part1_bits - std::min(m_csi1, c.nof_enc_csi_part1_bits)) / lq;
      const uint32_t M_r      = static_cast<uint32_t>(rvd.size());
      if (l >= l1_csi && M_uci > M_r && rem_csi1 > 0) {
        std::vector<uint8_t> avail = uci;
        for (uint32_t i : rvd) {
          avail[i] = 0;
        }
        pick(M_uci - M_r, rem_csi1, dd, nn);
        csi1 = re_select(indices(avail), dd, nn);
        for (uint32_t i : csi1) {
          ulsch[i] = uci[i] = 0;
        }
        m_csi1 += nn * lq;
      }
      // Step 3bis: CSI Part 2.
      M_uci                   = static_cast<uint32_t>(indices(uci).size());
      const uint32_t rem_csi2 = (c.nof_enc_csi_part2_bits - std::min(m_csi2, c.nof_enc_csi_part2_bits)) / lq;
      if (l >= l1_csi && l >= c.csi2_first_symbol && M_uci > 0 && rem_csi2 > 0) {
        pick(M_uci, rem_csi2, dd, nn);
        csi2 = re_select(indices(uci), dd, nn);
        for (uint32_t i : csi2) {
          ulsch[i] = uci[i] = 0;
        }
        m_csi2 += nn * lq;
      }
      // Step 5: HARQ-ACK of up to two bits on the reserved REs (they stay in the UL-SCH set).
      if (M_r > 0 && c.nof_harq_ack_bits <= 2 && rem_harq > 0) {
        pick(M_r, rem_harq, dd, nn);
        harq = re_select(rvd, dd, nn);
        m_harq += nn * lq;
      }
      // Routing entries of the symbol's REs: UCI streams in the order the reference feeds their buffers (RE order
      // within the symbol), the UL-SCH stream in RE order.
      // CSI Part 2 may be mapped onto reserved REs that HARQ-ACK of <= 2 bits then punctures: those REs feed both.
      std::vector<ulsch_demux_route> sym(M, ulsch_demux_route{DEMUX_NONE, 0, DEMUX_NONE});
      const std::vector<uint32_t>* sets[3] = {&harq, &csi1, &csi2};
      for (uint32_t k = 0; k < 3; ++k) {
        for (uint32_t i : *sets[k]) {
          if (k == 2 && (sym[i].uci >> 30) == 1) {
            sym[i].csi2 = n_uci[2]++;
          } else {
            sym[i].uci = ((k + 1) << 30) | n_uci[k]++;
          }
        }
      }
      const uint32_t n_sch0 = n_sch;
      for (uint32_t i = 0; i < M; ++i) {
        if (ulsch[i]) {
          sym[i].sch = n_sch++;
        }
      }
      sym_counts[t][0][l] = M * lq;
      sym_counts[t][1][l] = (n_sch - n_sch0) * lq;
      sym_counts[t][2][l] = static_cast<uint32_t>(harq.size()) * lq;
      sym_counts[t][3][l] = static_cast<uint32_t>(csi1.size()) * lq;
      sym_counts[t][4][l] = static_cast<uint32_t>(csi2.size()) * lq;
      routes.insert(routes.end(), sym.begin(), sym.end());
      n_re += M;
    }
    // ulsch_demultiplex_impl::on_end_codeword asserts every UCI field complete.
    if (m_harq != c.nof_enc_harq_ack_bits || m_csi1 != c.nof_enc_csi_part1_bits || m_csi2 != c.nof_enc_csi_part2_bits) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: UCI does not fit the allocation (HARQ-ACK %u/%u, CSI-1 %u/%u, CSI-2 "
                  "%u/%u bits placed)", t, m_harq, c.nof_enc_harq_ack_bits, m_csi1, c.nof_enc_csi_part1_bits, m_csi2,
                  c.nof_enc_csi_part2_bits);
    }
    d.llr_offset    = c.llr_offset;
    d.sch_offset    = c.sch_offset;
    d.uci_offset[0] = c.harq_offset;
    d.uci_offset[1] = c.csi1_offset;
    d.uci_offset[2] = c.csi2_offset;
    d.nof_llrs      = n_re * lq;
    d.qm            = static_cast<uint8_t>(qm);
    d.lq            = static_cast<uint8_t>(lq);
    const uint32_t bits[3] = {c.nof_harq_ack_bits, c.nof_csi_part1_bits, c.nof_csi_part2_bits};
    for (int k = 0; k < 3; ++k) {
      d.placeholder[k] = (bits[k] == 1 || bits[k] == 2) ? static_cast<uint8_t>(bits[k]) : 0;
    }
    counts[t]  = {n_re * lq, n_sch * lq, n_uci[0] * lq, n_uci[1] * lq, n_uci[2] * lq};
    c_inits[t] = (static_cast<uint32_t>(c.rnti) << 15) + c.n_id;
    nwords[t]  = (n_re * lq + 31u) / 32u;
    for (uint32_t r0 = 0; r0 < n_re; r0 += 256) {
      chunks.push_back(mod_chunk{t, 0, r0, std::min(n_re, r0 + 256)});
    }
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  int r = ensure_gold_tables(ctx);
  if (r != SRSGPU_OK) {
    return r;
  }
  const std::vector<uint32_t> seq_off = gold_sequence_offsets(nwords);
  for (uint32_t t = 0; t < nof_tx; ++t) {
    descs[t].seq_word_offset = seq_off[t];
  }
  auto* plan       = new srsgpu_ulsch_demux_plan();
  plan->ctx        = ctx;
  plan->nof_chunks = static_cast<int>(chunks.size());
  plan->nof_llrs   = std::move(counts);
  plan->symbol_llrs = std::move(sym_counts);
  if (!chunks.empty()) {
    if (build_gold_sequences(ctx, c_inits, nwords, seq_off, &plan->d_seq) != SRSGPU_OK) {
      srsgpu_ulsch_demux_plan_destroy(plan);
      return SRSGPU_ERR_HIP;
    }
    const bool ok =
        hipMalloc(&plan->d_desc, descs.size() * sizeof(ulsch_demux_desc)) == hipSuccess &&
        hipMemcpy(plan->d_desc, descs.data(), descs.size() * sizeof(ulsch_demux_desc), hipMemcpyHostToDevice) ==
            hipSuccess &&
        hipMalloc(&plan->d_routes, routes.size() * sizeof(ulsch_demux_route)) == hipSuccess &&
        hipMemcpy(plan->d_routes, routes.data(), routes.size() * sizeof(ulsch_demux_route), hipMemcpyHostToDevice) ==
            hipSuccess &&
        hipMalloc(&plan->d_chunks, chunks.size() * sizeof(mod_chunk)) == hipSuccess &&
        hipMemcpy(plan->d_chunks, chunks.data(), chunks.size() * sizeof(mod_chunk), hipMemcpyHostToDevice) ==
            hipSuccess;
    if (!ok) {
      srsgpu_ulsch_demux_plan_destroy(plan);
      return fail(SRSGPU_ERR_HIP, "failed to upload the demultiplexer routing");
    }
  }
  *plan_out = plan;
  return SRSGPU_OK;
}

uint32_t srsgpu_ulsch_demux_plan_nof_llrs(const srsgpu_ulsch_demux_plan* plan, uint32_t tx, uint32_t stream)
{
  return (plan == nullptr || tx >= plan->nof_llrs.size() || stream > 4) ? 0u : plan->nof_llrs[tx][stream];
}

int srsgpu_ulsch_demux_plan_symbol_llrs(const srsgpu_ulsch_demux_plan* plan, uint32_t tx, uint32_t stream,
                                        uint32_t counts[14])
{
  if (plan == nullptr || counts == nullptr || tx >= plan->symbol_llrs.size() || stream > 4) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid plan, transmission or stream");
  }
  std::copy(plan->symbol_llrs[tx][stream].begin(), plan->symbol_llrs[tx][stream].end(), counts);
  return SRSGPU_OK;
}

int srsgpu_ulsch_demux_plan_execute(const srsgpu_ulsch_demux_plan* plan,
                                    const int8_t*                  d_llrs,
                                    int8_t*                        d_sch,
                                    int8_t*                        d_harq,
                                    int8_t*                        d_csi1,
                                    int8_t*                        d_csi2,
                                    void*                          stream)
{
  if (plan == nullptr || d_llrs == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  for (const auto& n : plan->nof_llrs) {
    if ((n[1] > 0 && d_sch == nullptr) || (n[2] > 0 && d_harq == nullptr) || (n[3] > 0 && d_csi1 == nullptr) ||
        (n[4] > 0 && d_csi2 == nullptr)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "an output stream the plan writes is NULL");
    }
  }
  launch_ulsch_demux(plan->d_desc, plan->d_routes, plan->d_chunks, plan->nof_chunks, d_llrs, d_sch, d_harq, d_csi1,
                     d_csi2, plan->d_seq, static_cast<hipStream_t>(stream));
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

void srsgpu_ulsch_demux_plan_destroy(srsgpu_ulsch_demux_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  for (void* p : {static_cast<void*>(plan->d_desc), static_cast<void*>(plan->d_routes),
                  static_cast<void*>(plan->d_chunks), static_cast<void*>(plan->d_seq)}) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  delete plan;
}

} // extern "C"
