// Host side of the PUSCH demodulator C ABI (include/srsgpu_phy.h): validation (the equalizer and demapper
// combinations, allocation inside the grid), the max-log demapper interval tables (derived from the Gray PAM, like the
// reference's demodulation_mapper_qam64.cpp / _qam256.cpp tables) and per-transmission descriptors / 8192-LLR chunks.
#include "capi_internal.h"
#include <algorithm>
#include <cmath>
#include <vector>

using namespace srsgpu;

static_assert(sizeof(srsgpu_pusch_demod_config) == 32, "srsgpu_pusch_demod_config layout (mirrored by srsgpu)");
static_assert(SRSGPU_DEMOD_STATS == DEMOD_STATS_PER_TX, "statistics row layout");

struct srsgpu_pusch_demodulator_plan {
  srsgpu_context*       ctx        = nullptr;
  demod_desc*           d_desc     = nullptr;
  mod_chunk*            d_chunks   = nullptr;
  demod_tp_job*         d_tp_jobs  = nullptr;  ///< Transform-precoded (transmission, symbol) work items.
  demap_pair_table*     d_tables   = nullptr;
  uint32_t*             d_seq      = nullptr;  ///< Descrambling sequences of the transmissions (plan lifetime).
  uint16_t*             d_crbs     = nullptr;  ///< Allocated CRB lists of the CRB-mask transmissions.
  float*                d_acc      = nullptr;  ///< Statistics accumulators (zero between executes).
  int                   nof_chunks = 0;
  int                   chunk_threads = 256;  ///< Lanes per chunk workgroup (launch_pusch_demodulate).
  int                   nof_tp_jobs = 0;
  int                   nof_tx     = 0;
  std::vector<uint32_t> nof_llrs;
  std::vector<uint32_t> seq_off;  ///< First sequence word of each transmission in d_seq.
};

namespace {

/// TS 38.211 section 6.3.1.4: transform precoding needs M_RB = 2^a 3^b 5^c (transform_precoding_helpers.h).
bool tp_valid_nof_prb(unsigned n)
{
  if (n == 0) {
    return false;
  }
  for (unsigned f : {2u, 3u, 5u}) {
    while (n % f == 0) {
      n /= f;
    }
  }
  return n == 1;
}

} // namespace

namespace {

/// Max-log (slope, intercept) pieces of one bit pair of a Gray PAM with 2^(qm/2) levels: for stream bit 2k, the
/// levels (odd integers, units of a = 1 / sqrt(average power)) carrying 0 and 1 as modulation_mapper_lut_impl.cpp:39
/// builds them; LLR(y) = (min_{x1} (y - x1)^2 - min_{x0} (y - x0)^2) / nv is linear between consecutive even
/// integers: slope 2 (x0 - x1) a, intercept (x1^2 - x0^2) a^2. Pieces are merged pairwise when every pair is equal
/// (the reference's 4a-wide tables).
demap_pair_table pair_table(unsigned qm, unsigned k)
{
  const int      half = static_cast<int>(qm / 2);
  const int      L    = 1 << half;
  std::vector<int> x0s, x1s;
  for (unsigned idx = 0; idx < (1u << qm); ++idx) {
    int real = 0, off = -1;
    for (int j = 0; j < half; ++j) {
      real += off;
      off *= 2;
      real *= ((idx >> (2 * j + 1)) & 1u) ? 1 : -1;
    }
    const unsigned bit = (idx >> (qm - 1 - 2 * k)) & 1u;
    (bit ? x1s : x0s).push_back(real);
  }
  auto nearest = [](const std::vector<int>& xs, int y) {
    int best = xs[0];
    for (int x : xs) {
      if (std::abs(y - x) < std::abs(y - best)) {
        best = x;
      }
    }
    return best;
  };
  std::vector<int> slopes(static_cast<size_t>(L)), inters(static_cast<size_t>(L));
  for (int i = 0; i < L; ++i) {
    const int y  = 2 * (i - L / 2) + 1;
    const int x0 = nearest(x0s, y), x1 = nearest(x1s, y);
    slopes[static_cast<size_t>(i)] = 2 * (x0 - x1);
    inters[static_cast<size_t>(i)] = (x1 * x1 - x0 * x0) / 2;
  }
  bool mergeable = true;
  for (int i = 0; i < L / 2; ++i) {
    mergeable &= slopes[2 * i] == slopes[2 * i + 1] && inters[2 * i] == inters[2 * i + 1];
  }
  const int   avg = 2 * (L * L - 1) / 3;  // average power of the integer constellation
  const float a   = 1.0F / std::sqrt(static_cast<float>(avg));
  const int   step = mergeable ? 2 : 1;
  demap_pair_table t{};
  // INTERVAL_WIDTH = 2 (or 4) * M_SQRT1_42 / M_SQRT1_170 as a float; the SIMD demappers scale by its reciprocal.
  t.inv_width = 1.0F / static_cast<float>(2.0 * step / std::sqrt(static_cast<double>(avg)));
  t.count = static_cast<uint32_t>(L / step);
  for (int i = 0; i < L / step; ++i) {
    t.piece[i][0] = static_cast<float>(slopes[static_cast<size_t>(i * step)]) * a;
    t.piece[i][1] = static_cast<float>(inters[static_cast<size_t>(i * step)]) / static_cast<float>(avg / 2);
  }
  return t;
}

} // namespace

extern "C" {

int srsgpu_pusch_demodulator_plan_create(srsgpu_context*                  ctx,
                                         const srsgpu_pusch_demod_config* cfgs,
                                         uint32_t                         nof_tx,
                                         uint32_t                         grid_nof_prb,
                                         uint32_t                         grid_nof_ports,
                                         srsgpu_pusch_demodulator_plan**  plan_out)
{
  return srsgpu_pusch_demodulator_plan_create_ex(ctx, cfgs, nullptr, nof_tx, grid_nof_prb, grid_nof_ports, plan_out);
}

int srsgpu_pusch_demodulator_plan_create_ex(srsgpu_context*                  ctx,
                                            const srsgpu_pusch_demod_config* cfgs,
                                            const srsgpu_alloc_ext*          exts,
                                            uint32_t                         nof_tx,
                                            uint32_t                         grid_nof_prb,
                                            uint32_t                         grid_nof_ports,
                                            srsgpu_pusch_demodulator_plan**  plan_out)
{
  if (ctx == nullptr || plan_out == nullptr || (cfgs == nullptr && nof_tx > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  if (grid_nof_prb == 0 || grid_nof_prb > 275 || grid_nof_ports == 0 || grid_nof_ports > 4) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid grid geometry (%u PRB, %u ports)", grid_nof_prb, grid_nof_ports);
  }
  const uint32_t          nsc = 12u * grid_nof_prb;
  std::vector<demod_desc>   descs(nof_tx);
  std::vector<mod_chunk>    chunks;
  std::vector<demod_tp_job> tp_jobs;
  std::vector<uint16_t>     crb_lists;
  std::vector<uint32_t>     nllr(nof_tx);
  uint32_t                  total_words = 0, max_lq = 0;
  for (uint32_t t = 0; t < nof_tx; ++t) {
    const srsgpu_pusch_demod_config& c  = cfgs[t];
    const srsgpu_alloc_ext*          x  = (exts != nullptr) ? &exts[t] : nullptr;
    if (x != nullptr && (x->nof_reserved > 0 || x->prg_size > 0)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: the PUSCH demodulator takes a CRB mask only", t);
    }
    // Allocated CRBs: the mask's, or the contiguous [rb_start, rb_start + nof_rb).
    std::vector<uint16_t> crbs;
    const bool            masked = x != nullptr && x->crb_mask != nullptr;
    if (masked) {
      for (uint32_t rb = 0; rb < grid_nof_prb; ++rb) {
        if (x->crb_mask[rb] != 0) {
          crbs.push_back(static_cast<uint16_t>(rb));
        }
      }
    }
    const uint32_t nof_alloc_rb = masked ? static_cast<uint32_t>(crbs.size()) : c.nof_rb;
    const unsigned                   qm = c.modulation_order;
    const unsigned                   L  = c.nof_tx_layers, P = c.nof_rx_ports;
    if (qm != 2 && qm != 4 && qm != 6 && qm != 8) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid modulation order %u", t, qm);
    }
    // channel_equalizer_generic_impl.cpp:247 is_supported: 1, 2 or 4 ports... (any 1..4 for one layer), layers <= ports.
    if (L < 1 || L > 4 || P < L || P > grid_nof_ports || c.equalizer > SRSGPU_EQ_MMSE) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid layers / ports / equalizer (%u, %u, %u)", t, L, P,
                  c.equalizer);
    }
    if (L == 2 && c.equalizer == SRSGPU_EQ_ZF && P != 2 && P != 4) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: ZF with two layers needs two or four ports", t);
    }
    if (c.nof_symbols < 1 || c.start_symbol + c.nof_symbols > 14 || (c.dmrs_type != 1 && c.dmrs_type != 2) ||
        c.nof_cdm_groups_without_data < 1 || c.nof_cdm_groups_without_data > (c.dmrs_type == 1 ? 2 : 3) ||
        c.n_id > 1023 || nof_alloc_rb < 1 || (!masked && c.rb_start + c.nof_rb > grid_nof_prb) ||
        c.estimate_layout > SRSGPU_CE_COMPACT || c.cfo_compensated > 1 || c.numerology > 4 ||
        c.transform_precoding > 1) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid time / frequency allocation or DM-RS configuration", t);
    }
    demod_desc d{};
    unsigned   nd = 0;
    for (unsigned k = 0; k < 12; ++k) {
      const unsigned group = (c.dmrs_type == 2) ? (k % 6) / 2 : k % 2;
      if (group >= c.nof_cdm_groups_without_data) {
        d.dmrs_lut |= static_cast<uint64_t>(k) << (4 * nd);
        ++nd;
      }
    }
    uint32_t nre = 0;
    for (unsigned l = 0; l < 14; ++l) {
      d.sym_cum[l] = static_cast<uint16_t>(nre);
      if (l >= c.start_symbol && l < static_cast<unsigned>(c.start_symbol + c.nof_symbols)) {
        const uint32_t m = (((c.dmrs_symbol_mask >> l) & 1u) ? nd : 12u) * nof_alloc_rb;
        if (c.transform_precoding && m > 0) {
          // pusch_demodulator_impl.cpp:347 (one layer), transform_precoder_dft_impl.cpp (M_sc % 12, valid M_RB).
          if (L != 1 || m % 12 != 0 || !tp_valid_nof_prb(m / 12) || m > 3240) {
            return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: transform precoding needs one layer and 12 x 2^a 3^b 5^c data "
                        "REs per symbol (symbol %u has %u)", t, l, m);
          }
          tp_jobs.push_back(demod_tp_job{t, l});
        }
        nre += m;
      }
    }
    d.sym_cum[14] = d.sym_cum[15] = static_cast<uint16_t>(nre);
    const uint32_t Lq = L * qm;
    if (static_cast<uint64_t>(nre) * Lq > MOD_MAX_BITS) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: codeword too long", t);
    }
    const uint64_t slot_elems = static_cast<uint64_t>(grid_nof_ports) * 14u * nsc;
    if ((static_cast<uint64_t>(c.grid_index) + 1) * slot_elems * 4u >= (1ull << 32)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: grid index beyond 32-bit element offsets", t);
    }
    const uint32_t first_sc = masked ? 0u : c.rb_start * 12u;  // CRB lists address absolute subcarriers
    d.grid_base       = static_cast<uint32_t>(c.grid_index * slot_elems) + first_sc;
    d.port_stride     = 14u * nsc;
    d.nsc             = nsc;
    d.ce_layer_stride = static_cast<uint32_t>(slot_elems);
    d.ce_base         = static_cast<uint32_t>(c.grid_index * slot_elems * 4u) + first_sc;
    d.crb_list        = masked ? static_cast<uint32_t>(crb_lists.size()) : DEMOD_CONTIGUOUS;
    crb_lists.insert(crb_lists.end(), crbs.begin(), crbs.end());
    d.transform_precoding = c.transform_precoding;
    d.cfo_sc              = masked ? static_cast<uint16_t>(crbs.front() * 12u) : 0u;
    d.ce_compact      = c.estimate_layout == SRSGPU_CE_COMPACT ? 1 : 0;
    if (d.ce_compact) {
      d.ce_base += c.start_symbol * nsc;  // the estimator's single row (srsgpu_pusch_chest_config::estimate_layout)
    }
    // Compact + CFO compensation (>= 2 DM-RS symbols: the estimator has a CFO): per-symbol rotation in the kernel.
    d.ce_cfo = (d.ce_compact && c.cfo_compensated && __builtin_popcount(c.dmrs_symbol_mask) >= 2) ? 1u : 0u;
    symbol_start_epochs(c.numerology, d.epochs);
    d.llr_offset      = c.llr_offset;
    d.nof_llrs        = nre * Lq;
    d.c_init          = (static_cast<uint32_t>(c.rnti) << 15) + c.n_id;  // pusch_demodulator_impl.cpp:279
    d.tx              = t;
    d.dmrs_mask       = c.dmrs_symbol_mask;
    d.qm              = static_cast<uint8_t>(qm);
    d.L               = static_cast<uint8_t>(L);
    d.P               = static_cast<uint8_t>(P);
    d.nd_dmrs         = static_cast<uint8_t>(nd);
    d.eq              = (L >= 3 || c.equalizer == SRSGPU_EQ_MMSE) ? DEMOD_EQ_MMSE : DEMOD_EQ_ZF;
    descs[t]          = d;
    nllr[t]           = d.nof_llrs;
    const uint32_t nwords = c.transform_precoding ? 0u : (d.nof_llrs + 31) / 32;  // TP: per-symbol jobs instead
    total_words += nwords;
    max_lq = std::max(max_lq, Lq);
  }
  // Chunk size: DEMOD_CHUNK_WORDS codeword words per workgroup; a plan too small to fill the GPU that way (a one-PDU
  // slot: 38 chunks of 1 024 REs for 273 PRB, each lane of a chunk walking 4 REs) takes chunks of about 256 REs on
  // 256 lanes instead, so the latency of the launch is about one RE per lane.
  uint32_t chunk_words = DEMOD_CHUNK_WORDS;
  bool     small_plan  = false;
  if (total_words < 256u * DEMOD_CHUNK_WORDS) {
    small_plan  = true;
    chunk_words = std::min<uint32_t>(DEMOD_CHUNK_WORDS, std::max<uint32_t>(8u, 8u * max_lq));
  }
  for (uint32_t t = 0; t < nof_tx; ++t) {
    const demod_desc& d      = descs[t];
    const uint32_t    Lq     = static_cast<uint32_t>(d.L) * d.qm;
    const uint32_t    nre    = d.nof_llrs / Lq;
    const uint32_t    nwords = cfgs[t].transform_precoding ? 0u : (d.nof_llrs + 31) / 32;
    for (uint32_t w0 = 0; w0 < nwords; w0 += chunk_words) {
      const uint32_t b0 = w0 * 32, b1 = b0 + chunk_words * 32;
      mod_chunk      ch{t, w0, (b0 + Lq - 1) / Lq, std::min(nre, (b1 + Lq - 1) / Lq)};
      if (ch.re_end > ch.re_begin) {
        chunks.push_back(ch);
      }
    }
  }
  std::vector<demap_pair_table> tables;
  for (unsigned k = 0; k < 3; ++k) {
    tables.push_back(pair_table(6, k));
  }
  for (unsigned k = 0; k < 4; ++k) {
    tables.push_back(pair_table(8, k));
  }
  // The kernel shares one interval index among all bit pairs but the last (pusch_demodulator.hip demap).
  for (unsigned first : {0u, 3u}) {
    const unsigned np = first == 0 ? 3 : 4;
    for (unsigned k = 1; k + 1 < np; ++k) {
      if (tables[first + k].inv_width != tables[first].inv_width || tables[first + k].count != tables[first].count) {
        return fail(SRSGPU_ERR_INVALID_ARG, "internal: demapper interval tables do not share their width");
      }
    }
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  int r = ensure_gold_tables(ctx);
  if (r != SRSGPU_OK) {
    return r;
  }
  std::vector<uint32_t> c_inits(descs.size()), nwords(descs.size());
  for (size_t t = 0; t < descs.size(); ++t) {
    c_inits[t] = descs[t].c_init;
    nwords[t]  = (descs[t].nof_llrs + 31u) / 32u;
  }
  const std::vector<uint32_t> seq_off = gold_sequence_offsets(nwords);
  for (size_t t = 0; t < descs.size(); ++t) {
    descs[t].seq_word_offset = seq_off[t];
  }
  auto* plan        = new srsgpu_pusch_demodulator_plan();
  plan->ctx         = ctx;
  plan->nof_chunks  = static_cast<int>(chunks.size());
  plan->nof_tp_jobs = static_cast<int>(tp_jobs.size());
  plan->nof_tx      = static_cast<int>(nof_tx);
  plan->nof_llrs    = std::move(nllr);
  plan->seq_off     = seq_off;
  const bool work   = !chunks.empty() || !tp_jobs.empty();
  if (work && build_gold_sequences(ctx, c_inits, nwords, seq_off, &plan->d_seq) != SRSGPU_OK) {
    srsgpu_pusch_demodulator_plan_destroy(plan);
    return SRSGPU_ERR_HIP;
  }
  bool ok = hipMalloc(&plan->d_tables, tables.size() * sizeof(demap_pair_table)) == hipSuccess &&
            hipMemcpy(plan->d_tables, tables.data(), tables.size() * sizeof(demap_pair_table),
                      hipMemcpyHostToDevice) == hipSuccess;
  if (ok && work) {
    ok = hipMalloc(&plan->d_desc, descs.size() * sizeof(demod_desc)) == hipSuccess &&
         hipMemcpy(plan->d_desc, descs.data(), descs.size() * sizeof(demod_desc), hipMemcpyHostToDevice) ==
             hipSuccess;
  }
  if (!chunks.empty()) {
    // Lanes per chunk from its REs: a few-PRB transmission's chunk is a few hundred REs, which 256 lanes finish in two
    // or three trips after paying the workgroup's descriptor -> sequence staging -> first-load latency chain; 128 lanes
    // take ~5 REs each (headline bench 139.0k -> 141.2k slots/s, demodulator stage 47 -> 40 us per step,
    // profiles/r4_demod_threads_ab.txt), 64 for chunks of at most 384 REs.
    uint32_t most = 0;
    for (const mod_chunk& ch : chunks) {
      most = std::max(most, ch.re_end - ch.re_begin);
    }
    plan->chunk_threads = small_plan ? 256 : (most <= 384 ? 64 : (most <= 768 ? 128 : 256));
  }
  if (ok && !chunks.empty()) {
    ok = hipMalloc(&plan->d_chunks, chunks.size() * sizeof(mod_chunk)) == hipSuccess &&
         hipMemcpy(plan->d_chunks, chunks.data(), chunks.size() * sizeof(mod_chunk), hipMemcpyHostToDevice) ==
             hipSuccess;
  }
  if (ok && !tp_jobs.empty()) {
    ok = hipMalloc(&plan->d_tp_jobs, tp_jobs.size() * sizeof(demod_tp_job)) == hipSuccess &&
         hipMemcpy(plan->d_tp_jobs, tp_jobs.data(), tp_jobs.size() * sizeof(demod_tp_job), hipMemcpyHostToDevice) ==
             hipSuccess;
  }
  if (ok && !crb_lists.empty()) {
    ok = hipMalloc(&plan->d_crbs, crb_lists.size() * sizeof(uint16_t)) == hipSuccess &&
         hipMemcpy(plan->d_crbs, crb_lists.data(), crb_lists.size() * sizeof(uint16_t), hipMemcpyHostToDevice) ==
             hipSuccess;
  }
  if (ok && nof_tx > 0) {
    const size_t acc_bytes = static_cast<size_t>(nof_tx) * DEMOD_ACC_PER_TX * sizeof(float);
    ok = hipMalloc(&plan->d_acc, acc_bytes) == hipSuccess && hipMemset(plan->d_acc, 0, acc_bytes) == hipSuccess;
  }
  if (!ok) {
    srsgpu_pusch_demodulator_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload demodulator descriptors");
  }
  *plan_out = plan;
  return SRSGPU_OK;
}

uint32_t srsgpu_pusch_demodulator_plan_nof_llrs(const srsgpu_pusch_demodulator_plan* plan, uint32_t tx)
{
  return (plan == nullptr || tx >= plan->nof_llrs.size()) ? 0u : plan->nof_llrs[tx];
}

int srsgpu_pusch_demodulator_plan_execute(const srsgpu_pusch_demodulator_plan* plan,
                                          const uint32_t*                      d_grids,
                                          const uint32_t*                      d_ch_estimates,
                                          const float*                         d_noise_var,
                                          int8_t*                              d_llrs,
                                          void*                                stream)
{
  if (plan == nullptr || d_grids == nullptr || d_ch_estimates == nullptr || d_noise_var == nullptr ||
      d_llrs == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  return srsgpu_pusch_demodulator_plan_execute_ex(plan, d_grids, d_ch_estimates, d_noise_var, d_llrs, nullptr, stream);
}

int srsgpu_pusch_demodulator_plan_execute_ex(const srsgpu_pusch_demodulator_plan* plan,
                                             const uint32_t*                      d_grids,
                                             const uint32_t*                      d_ch_estimates,
                                             const float*                         d_noise_var,
                                             int8_t*                              d_llrs,
                                             float*                               d_stats,
                                             void*                                stream)
{
  if (plan == nullptr || d_grids == nullptr || d_ch_estimates == nullptr || d_noise_var == nullptr ||
      d_llrs == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  const hipStream_t s   = static_cast<hipStream_t>(stream);
  float*            acc = d_stats != nullptr ? plan->d_acc : nullptr;
  launch_pusch_demodulate(plan->d_desc, plan->d_chunks, plan->nof_chunks, plan->chunk_threads, plan->d_tables,
                          d_grids, d_ch_estimates, d_noise_var, d_llrs, plan->d_seq, plan->d_crbs, acc, s);
  launch_pusch_demodulate_tp(plan->d_desc, plan->d_tp_jobs, plan->nof_tp_jobs, plan->d_tables, d_grids,
                             d_ch_estimates, d_noise_var, d_llrs, plan->d_seq, plan->d_crbs, acc, s);
  if (d_stats != nullptr) {
    launch_pusch_demod_stats(plan->d_acc, d_stats, plan->nof_tx, s);
  }
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

void srsgpu_pusch_demodulator_plan_destroy(srsgpu_pusch_demodulator_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  for (void* p : {static_cast<void*>(plan->d_desc), static_cast<void*>(plan->d_chunks),
                  static_cast<void*>(plan->d_tp_jobs), static_cast<void*>(plan->d_tables),
                  static_cast<void*>(plan->d_seq), static_cast<void*>(plan->d_crbs), static_cast<void*>(plan->d_acc)}) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  delete plan;
}

} // extern "C"

extern "C" int srsgpu_pusch_demodulator_plan_scrambling(const srsgpu_pusch_demodulator_plan* plan,
                                                        uint32_t                             tx,
                                                        uint32_t*                            d_words,
                                                        void*                                stream)
{
  if (plan == nullptr || d_words == nullptr || tx >= static_cast<uint32_t>(plan->nof_tx)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument or transmission index out of range");
  }
  const size_t nwords = (plan->nof_llrs[tx] + 31u) / 32u;
  if (nwords == 0) {
    return SRSGPU_OK;
  }
  HIP_TRY(hipMemcpyAsync(d_words, plan->d_seq + plan->seq_off[tx], nwords * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                         static_cast<hipStream_t>(stream)));
  return SRSGPU_OK;
}
