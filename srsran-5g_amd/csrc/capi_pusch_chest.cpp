// Host side of the PUSCH DM-RS channel estimator C ABI (include/srsgpu_phy.h): validation, the per-symbol DM-RS
// sequence initial states (dmrs_pusch_estimator_impl.cpp:69), the resampled raised-cosine smoothing filter
// (port_channel_estimator_helpers.cpp filter_type, taps generated from the raised-cosine formula) and one job per
// (transmission, rx port, CDM group).
#include "capi_internal.h"
#include "low_papr_tables.h"
#include <algorithm>
#include <cmath>
#include <vector>

using namespace srsgpu;

static_assert(sizeof(srsgpu_pusch_chest_config) == 32, "srsgpu_pusch_chest_config layout (mirrored by srsgpu)");

struct srsgpu_pusch_chest_plan {
  srsgpu_context* ctx        = nullptr;
  chest_job*      d_jobs     = nullptr;
  int             nof_jobs   = 0;
  chest_geom      geom       = {};  ///< Plan-wide maxima (LDS sizing).
  uint32_t*       d_seq      = nullptr;  ///< DM-RS sequence words of every job (plan lifetime).
  uint16_t*       d_crbs     = nullptr;  ///< CRB lists of the CRB-mask transmissions (relative to their first CRB).
  float2*         d_lp       = nullptr;  ///< Low-PAPR DM-RS sequences of the transform-precoded transmissions.
};

namespace {

/// Raised cosine, roll-off 0.2, 10 samples per symbol, n = 0..30 (t = (n - 15) / 10), as the reference tabulates it
/// (port_channel_estimator_helpers.cpp:51 RC_FILTER): normalised to unit energy and quantised to 7 decimals, so that
/// the float taps the estimator derives from it are the reference's bit for bit. The reference's table holds
/// 0.3235207 at n = 14 and 16, one unit of the last decimal below the rounded prototype value (0.32352076).
double rc_tap(int n)
{
  const double pi   = 3.14159265358979323846;
  const double beta = 0.2;
  auto         raw  = [&](int i) {
    const double t    = (i - 15) / 10.0;
    const double sinc = (t == 0) ? 1.0 : std::sin(pi * t) / (pi * t);
    return sinc * std::cos(pi * beta * t) / (1 - (2 * beta * t) * (2 * beta * t));  // |2 beta t| < 1 for i = 0..30
  };
  double energy = 0;
  for (int i = 0; i != 31; ++i) {
    energy += raw(i) * raw(i);
  }
  double q = std::nearbyint(raw(n) / std::sqrt(energy) * 1e7);
  if (n == 14 || n == 16) {
    q -= 1;
  }
  return q / 1e7;
}

/// time_alignment_estimator_dft_impl::get_idft (:216): guard-scaled size, next power of two, 128..4096.
unsigned ta_dft_size(unsigned nof_re)
{
  const unsigned n    = nof_re * 4096u / 3300u;
  unsigned       size = 1;
  while (size < n) {
    size <<= 1;
  }
  return std::max(128u, size);
}

/// TS 38.211 section 5.2.2 low-PAPR base sequence of group u (v = 0, alpha = 0) and length m, as
/// low_papr_sequence_generator_impl.cpp builds it: the phase tables for m = 6..24, the length-30 formula, and
/// Zadoff-Chu of the largest prime N_ZC < m for m >= 36 with q = (int)(q_hat + 0.5), q_hat = (float) N_ZC (u + 1) / 31.
/// Returns false for a length the specification does not define.
bool low_papr_sequence(unsigned u, unsigned m, std::vector<float2>& out)
{
  std::vector<int> arg(m);
  unsigned         nzc = 4;
  const int8_t*    phi = m == 6 ? kLowPaprPhi6[u] : m == 12 ? kLowPaprPhi12[u] : m == 18 ? kLowPaprPhi18[u]
                                                                  : m == 24 ? kLowPaprPhi24[u] : nullptr;
  if (phi != nullptr) {
    for (unsigned n = 0; n < m; ++n) {
      arg[n] = phi[n];  // units of pi / 4 = pi / N_ZC with N_ZC = 4
    }
  } else if (m == 30) {
    nzc = 31;
    for (unsigned n = 0; n < m; ++n) {
      arg[n] = -static_cast<int>(((u + 1ull) * (n + 1ull) * (n + 2ull)) % 62u);
    }
  } else if (m >= 36) {
    nzc = m - 1;
    auto prime = [](unsigned x) {
      for (unsigned d = 2; d * d <= x; ++d) {
        if (x % d == 0) {
          return false;
        }
      }
      return x > 1;
    };
    while (!prime(nzc)) {
      --nzc;
    }
    const float   q_hat = static_cast<float>(nzc) * static_cast<float>(u + 1) / 31.f;
    const int64_t q     = static_cast<int64_t>(static_cast<float>(static_cast<double>(q_hat) + 0.5));
    for (unsigned n = 0; n < m; ++n) {
      const int64_t mm = n % nzc;
      arg[n]           = -static_cast<int>((q * mm * (mm + 1)) % (2 * nzc));
    }
  } else {
    return false;
  }
  for (unsigned n = 0; n < m; ++n) {
    const double a = 3.14159265358979323846 * static_cast<double>(arg[n]) / static_cast<double>(nzc);
    out.push_back(make_float2(static_cast<float>(std::cos(a)), static_cast<float>(std::sin(a))));
  }
  return true;
}

} // namespace

extern "C" {

int srsgpu_pusch_chest_plan_create(srsgpu_context*                  ctx,
                                   const srsgpu_pusch_chest_config* cfgs,
                                   uint32_t                         nof_tx,
                                   uint32_t                         grid_nof_prb,
                                   uint32_t                         grid_nof_ports,
                                   srsgpu_pusch_chest_plan**        plan_out)
{
  return srsgpu_pusch_chest_plan_create_ex(ctx, cfgs, nullptr, nof_tx, grid_nof_prb, grid_nof_ports, plan_out);
}

int srsgpu_pusch_chest_plan_create_ex(srsgpu_context*                  ctx,
                                      const srsgpu_pusch_chest_config* cfgs,
                                      const srsgpu_alloc_ext*          exts,
                                      uint32_t                         nof_tx,
                                      uint32_t                         grid_nof_prb,
                                      uint32_t                         grid_nof_ports,
                                      srsgpu_pusch_chest_plan**        plan_out)
{
  if (ctx == nullptr || plan_out == nullptr || (cfgs == nullptr && nof_tx > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  if (grid_nof_prb == 0 || grid_nof_prb > 275 || grid_nof_ports == 0 || grid_nof_ports > 4) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid grid geometry (%u PRB, %u ports)", grid_nof_prb, grid_nof_ports);
  }
  const uint32_t         nsc        = 12u * grid_nof_prb;
  const uint64_t         slot_elems = static_cast<uint64_t>(grid_nof_ports) * 14u * nsc;
  std::vector<chest_job> jobs;
  std::vector<uint16_t>  crb_lists;
  std::vector<float2>    lp_table;
  for (uint32_t t = 0; t < nof_tx; ++t) {
    srsgpu_pusch_chest_config c = cfgs[t];
    const unsigned            L = c.nof_tx_layers, P = c.nof_rx_ports;
    const srsgpu_alloc_ext*   x = (exts != nullptr) ? &exts[t] : nullptr;
    if (x != nullptr && (x->nof_reserved > 0 || x->prg_size > 0)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: the PUSCH estimator takes a CRB mask only", t);
    }
    // CRB mask (configuration::rb_mask): a contiguous mask is the plain allocation; otherwise the allocated CRBs
    // relative to the first one drive the pilot, sequence and estimate positions.
    std::vector<uint16_t> rel;
    if (x != nullptr && x->crb_mask != nullptr) {
      std::vector<uint16_t> crbs;
      for (uint32_t rb = 0; rb < grid_nof_prb; ++rb) {
        if (x->crb_mask[rb] != 0) {
          crbs.push_back(static_cast<uint16_t>(rb));
        }
      }
      if (crbs.empty()) {
        return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: empty CRB mask", t);
      }
      c.rb_start = crbs.front();
      c.nof_rb   = static_cast<uint16_t>(crbs.size());
      if (crbs.back() - crbs.front() + 1u != crbs.size()) {
        for (uint16_t rb : crbs) {
          rel.push_back(static_cast<uint16_t>(rb - crbs.front()));
        }
      }
    }
    const bool     masked  = !rel.empty();
    const unsigned span_rb = masked ? rel.back() + 1u : c.nof_rb;
    // Transform precoding: the low-PAPR sequence of group n_RS_ID mod 30 over the allocation's pilots (type 1, one
    // layer: dmrs_pusch_estimator.h get_dmrs_type / get_nof_tx_layers for low_papr_sequence_configuration).
    uint32_t lp_base = CHEST_CONTIGUOUS;
    if (c.dmrs_sequence > SRSGPU_DMRS_LOW_PAPR) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid DM-RS sequence kind %u", t, c.dmrs_sequence);
    }
    if (c.dmrs_sequence == SRSGPU_DMRS_LOW_PAPR) {
      if (L != 1 || c.dmrs_type != 1 || c.scrambling_id > 1007) {
        return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: low-PAPR DM-RS takes one layer, type 1 and n_RS_ID <= 1007", t);
      }
      lp_base = static_cast<uint32_t>(lp_table.size());
      if (!low_papr_sequence(c.scrambling_id % 30u, c.nof_rb * 6u, lp_table)) {
        return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: no low-PAPR sequence of length %u", t, c.nof_rb * 6u);
      }
    }
    if (L < 1 || L > 4 || P < 1 || P > grid_nof_ports || (c.dmrs_type != 1 && c.dmrs_type != 2) || c.n_scid > 1) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid layers / ports / DM-RS type", t);
    }
    if (c.nof_symbols < 1 || c.start_symbol + c.nof_symbols > 14 || c.nof_rb < 1 ||
        c.rb_start + c.nof_rb > grid_nof_prb || !(c.scaling > 0.f) || c.fd_smoothing > SRSGPU_CHEST_FD_FILTER ||
        c.estimate_layout > SRSGPU_CE_COMPACT || c.td_strategy > SRSGPU_CHEST_TD_INTERPOLATE ||
        c.compensate_cfo > 1 || c.numerology > 4) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid allocation, scaling, strategy or numerology", t);
    }
    if (c.estimate_layout == SRSGPU_CE_COMPACT && c.td_strategy == SRSGPU_CHEST_TD_INTERPOLATE) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: the interpolate strategy needs the per-symbol layout", t);
    }
    std::vector<unsigned> dmrs;
    for (unsigned l = 0; l < 14; ++l) {
      if ((c.dmrs_symbol_mask >> l) & 1u) {
        if (l < c.start_symbol || l >= static_cast<unsigned>(c.start_symbol + c.nof_symbols)) {
          return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: DM-RS symbol %u outside the allocation", t, l);
        }
        dmrs.push_back(l);
      }
    }
    if (dmrs.empty()) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: no DM-RS symbols", t);
    }
    if ((static_cast<uint64_t>(c.grid_index) + 1) * slot_elems * 4u >= (1ull << 32)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: grid index beyond 32-bit element offsets", t);
    }
    const bool     t2     = c.dmrs_type == 2;
    const unsigned per_rb = t2 ? 4 : 6;
    const unsigned stride = t2 ? 1 : 2;  // configure_interpolator of the group's RE pattern
    // Smoothing filter (filter_type): min(nof_rb, 3) RBs of the 31-tap prototype resampled at the pilot stride.
    const unsigned nrb3  = std::min<unsigned>(c.nof_rb, 3);
    const unsigned half  = (nrb3 * 10 + 1) / 2 / stride;
    const unsigned first = 15 - half * stride;
    const unsigned ntaps = 2 * half + 1;
    float          taps[32] = {};
    float          total    = 0;
    for (unsigned i = 0; i < ntaps; ++i) {
      taps[i] = static_cast<float>(rc_tap(static_cast<int>(first + i * stride)));
      total += taps[i];
    }
    const float rcp_total = 1 / total;
    for (unsigned i = 0; i < ntaps; ++i) {
      taps[i] *= rcp_total;
    }
    unsigned nof_v = std::min<unsigned>(12, ntaps / 2);
    if (c.nof_rb == 1) {
      nof_v = per_rb;
    }
    const unsigned ngroups = (L + 1) / 2;
    // Symbol epochs and the "interpolate" plane table (apply_td_domain_strategy, :509): for symbol l the planes of the
    // DM-RS symbols around it (or the first / last two), and the weight of the second.
    float          epochs[14];
    symbol_start_epochs(c.numerology, epochs);
    int8_t         q0[14] = {}, q1[14] = {};
    float          wq[14] = {};
    const int      s_first = c.start_symbol, s_last = c.start_symbol + c.nof_symbols;
    auto           dm    = [&](int l) { return l >= 0 && l < 14 && ((c.dmrs_symbol_mask >> l) & 1u); };
    auto           count = [&](int a, int b) { int n = 0; for (int l = a; l < b; ++l) n += dm(l); return n; };
    for (int l = s_first; l < s_last; ++l) {
      int before = -1, after = -1;
      for (int x = s_first; x < l; ++x) if (dm(x)) before = x;
      for (int x = s_last - 1; x >= l; --x) if (dm(x)) after = x;
      bool copied = false;
      if (before == -1) {
        int second = -1;
        for (int x = s_last - 1; x >= after + 1; --x) if (dm(x)) second = x;
        if (second == -1) {
          q0[l] = q1[l] = 0;
          copied = true;
        } else {
          before = after;
          after  = second;
        }
      }
      if (!copied && after == -1) {
        int second_last = -1;
        for (int x = s_first; x < before; ++x) if (dm(x)) second_last = x;
        if (second_last == -1) {
          q0[l] = q1[l] = static_cast<int8_t>(dmrs.size() - 1);
          copied = true;
        } else {
          after  = before;
          before = second_last;
        }
      }
      if (!copied) {
        const int i = count(s_first, before);
        q0[l]       = static_cast<int8_t>(i);
        q1[l]       = static_cast<int8_t>(i + 1);
        wq[l]       = static_cast<float>(l - before) / static_cast<float>(after - before);
      }
    }
    // Time alignment (estimate_time_alignment, port_channel_estimator_helpers.cpp:246): type 1 patterns are the stride-2
    // PUSCH patterns (pilots in the first bins); others take the RE-mask path (pilots at their subcarrier offsets).
    // A non-contiguous mask takes the RE-mask path for both types (pilot span of the re_mask = rb_mask kron pattern).
    const unsigned khz      = 15u << c.numerology;
    const unsigned ta_re    = (t2 || masked) ? (span_rb - 1u) * 12u + (t2 ? 7u : 10u) + 1u : c.nof_rb * per_rb;
    const unsigned ta_dft   = ta_dft_size(ta_re);
    const unsigned ta_strd  = (t2 || masked) ? 1u : 2u;
    const double   ta_fs    = static_cast<double>(static_cast<uint64_t>(ta_dft) * khz * 1000u * ta_strd);
    const double   half_cp  = static_cast<double>(144u * 64u / (1u << (c.numerology + 1))) * T_C;
    const unsigned ta_max   = static_cast<unsigned>(std::floor(half_cp * ta_fs));
    unsigned       ta_log2  = 0;
    while ((1u << ta_log2) < ta_dft) {
      ++ta_log2;
    }
    for (unsigned p = 0; p < P; ++p) {
      for (unsigned g = 0; g < ngroups; ++g) {
        chest_job jb{};
        jb.grid_base       = static_cast<uint32_t>(c.grid_index * slot_elems) + p * 14u * nsc + c.rb_start * 12u;
        jb.ce_layer_stride = static_cast<uint32_t>(slot_elems);
        jb.ce_base = static_cast<uint32_t>(c.grid_index * slot_elems * 4u + 2u * g * slot_elems) + p * 14u * nsc +
                     c.rb_start * 12u;
        jb.nsc        = nsc;
        jb.seq_offset = c.rb_start * per_rb;
        for (size_t s = 0; s < dmrs.size(); ++s) {
          // c_init = ((14 n_slot + l + 1)(2 N_ID + 1) 2^17 + 2 N_ID + n_SCID) mod 2^31 (dmrs_pusch_estimator_impl.cpp:83)
          const uint64_t nid = c.scrambling_id;
          jb.c_init[s]       = static_cast<uint32_t>(
              ((14ull * c.slot_index + dmrs[s] + 1) * (2 * nid + 1) * (1ull << 17) + 2 * nid + c.n_scid) % (1ull << 31));
          jb.dmrs_symbols[s] = static_cast<uint8_t>(dmrs[s]);
        }
        jb.pattern = 0;
        for (unsigned j = 0; j < per_rb; ++j) {
          const unsigned k = t2 ? (2 * g + (j & 1) + 6 * (j >> 1)) : (g + 2 * j);
          jb.pattern |= k << (4 * j);
        }
        jb.noise_slot    = 4 * t + p;
        jb.beta          = c.scaling;
        std::copy(taps, taps + 32, jb.taps);
        jb.nof_pilots    = static_cast<uint16_t>(c.nof_rb * per_rb);
        jb.nof_rb        = c.nof_rb;
        jb.nof_dmrs      = static_cast<uint8_t>(dmrs.size());
        jb.group_layers  = static_cast<uint8_t>(std::min<unsigned>(2, L - 2 * g));
        jb.group         = static_cast<uint8_t>(g);
        jb.pilots_per_rb = static_cast<uint8_t>(per_rb);
        jb.fd            = c.fd_smoothing;
        jb.ntaps         = static_cast<uint8_t>(ntaps);
        jb.nof_v_pilots  = static_cast<uint8_t>(nof_v);
        jb.interp_offset = static_cast<uint8_t>(t2 ? 2 * g : g);
        jb.interp_stride = static_cast<uint8_t>(stride);
        jb.first_symbol  = c.start_symbol;
        jb.nof_symbols   = c.nof_symbols;
        jb.nof_out_symbols = c.estimate_layout == SRSGPU_CE_COMPACT ? 1 : c.nof_symbols;  // compact: start_symbol's row
        jb.td_interp       = c.td_strategy == SRSGPU_CHEST_TD_INTERPOLATE;
        jb.compensate_cfo  = c.compensate_cfo;
        jb.compact_cfo     = c.estimate_layout == SRSGPU_CE_COMPACT && c.compensate_cfo && dmrs.size() >= 2;
        std::copy(epochs, epochs + 14, jb.epochs);
        std::copy(q0, q0 + 14, jb.td_q0);
        std::copy(q1, q1 + 14, jb.td_q1);
        std::copy(wq, wq + 14, jb.td_w);
        jb.scs_hz       = static_cast<float>(khz * 1000u);
        jb.ta_fs        = ta_fs;
        jb.ta_dft       = static_cast<uint16_t>(ta_dft);
        jb.ta_max       = static_cast<uint16_t>(ta_max);
        jb.ta_log2      = static_cast<uint8_t>(ta_log2);
        jb.ta_positions = (t2 || masked) ? 1 : 0;
        jb.crb_list     = masked ? static_cast<uint32_t>(crb_lists.size()) : CHEST_CONTIGUOUS;
        jb.span_pilots  = static_cast<uint16_t>(span_rb * per_rb);
        jb.lp_base      = lp_base;
        jobs.push_back(jb);
      }
    }
    crb_lists.insert(crb_lists.end(), rel.begin(), rel.end());
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  int r = ensure_gold_tables(ctx);
  if (r != SRSGPU_OK) {
    return r;
  }
  auto* plan     = new srsgpu_pusch_chest_plan();
  plan->ctx      = ctx;
  plan->nof_jobs = static_cast<int>(jobs.size());
  chest_geom& g = plan->geom;
  g             = {1, 1, 1, 1, 1, 128};
  for (const chest_job& jb : jobs) {
    g.max_pilots = std::max<int>(g.max_pilots, jb.nof_pilots);
    g.max_dmrs   = std::max<int>(g.max_dmrs, jb.nof_dmrs);
    g.max_words  = std::max<int>(g.max_words, static_cast<int>(((2 * jb.seq_offset) % 32 + 2 * jb.span_pilots + 31) / 32));
    g.max_planes = std::max<int>(g.max_planes, jb.td_interp ? jb.nof_dmrs : 1);
    g.max_gl     = std::max<int>(g.max_gl, jb.group_layers);
    g.max_dft    = std::max<int>(g.max_dft, jb.ta_dft);
  }
  if (pusch_chest_lds_bytes(g) > 160 * 1024) {
    delete plan;
    return fail(SRSGPU_ERR_INVALID_ARG, "channel estimation job too large for the LDS");
  }
  // DM-RS sequences, resident: per job and DM-RS symbol the words the kernel stages (from the allocation's first
  // sequence word), filled once.
  std::vector<uint32_t> c_inits, nwords, offsets, wstart;
  uint32_t              base = 0;
  for (chest_job& jb : jobs) {
    const uint32_t n0 = 2u * jb.seq_offset;
    const uint32_t nw = ((n0 & 31u) + 2u * jb.span_pilots + 31u) >> 5;
    jb.gseq_base      = base;
    for (unsigned s = 0; s < jb.nof_dmrs; ++s) {
      c_inits.push_back(jb.c_init[s]);
      nwords.push_back(nw);
      offsets.push_back(base + s * nw);
      wstart.push_back(n0 >> 5);
    }
    base += jb.nof_dmrs * nw;
  }
  if (build_gold_sequences(ctx, c_inits, nwords, offsets, &plan->d_seq, &wstart) != SRSGPU_OK) {
    srsgpu_pusch_chest_plan_destroy(plan);
    return SRSGPU_ERR_HIP;
  }
  if (!lp_table.empty() &&
      (hipMalloc(&plan->d_lp, lp_table.size() * sizeof(float2)) != hipSuccess ||
       hipMemcpy(plan->d_lp, lp_table.data(), lp_table.size() * sizeof(float2), hipMemcpyHostToDevice) !=
           hipSuccess)) {
    srsgpu_pusch_chest_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload low-PAPR sequences");
  }
  if (!crb_lists.empty() &&
      (hipMalloc(&plan->d_crbs, crb_lists.size() * sizeof(uint16_t)) != hipSuccess ||
       hipMemcpy(plan->d_crbs, crb_lists.data(), crb_lists.size() * sizeof(uint16_t), hipMemcpyHostToDevice) !=
           hipSuccess)) {
    srsgpu_pusch_chest_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload CRB lists");
  }
  if (!jobs.empty() && (hipMalloc(&plan->d_jobs, jobs.size() * sizeof(chest_job)) != hipSuccess ||
                        hipMemcpy(plan->d_jobs, jobs.data(), jobs.size() * sizeof(chest_job), hipMemcpyHostToDevice) !=
                            hipSuccess)) {
    srsgpu_pusch_chest_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload channel estimation jobs");
  }
  *plan_out = plan;
  return SRSGPU_OK;
}

int srsgpu_pusch_chest_plan_execute(const srsgpu_pusch_chest_plan* plan,
                                    const uint32_t*                d_grids,
                                    uint32_t*                      d_ch_estimates,
                                    float*                         d_noise_var,
                                    float*                         d_metrics,
                                    void*                          stream)
{
  if (plan == nullptr || d_grids == nullptr || d_ch_estimates == nullptr || d_noise_var == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  launch_pusch_chest(plan->d_lp, plan->d_crbs, plan->d_jobs, plan->nof_jobs, plan->geom, d_grids, d_ch_estimates, d_noise_var, d_metrics,
                     plan->d_seq, static_cast<hipStream_t>(stream));
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

int srsgpu_pusch_chest_plan_execute_copy(const srsgpu_pusch_chest_plan* plan,
                                         const uint32_t*                d_grids,
                                         uint32_t*                      d_ch_estimates,
                                         float*                         d_noise_var,
                                         float*                         d_metrics,
                                         const srsgpu_copy_span*        d_spans,
                                         uint32_t                       nof_spans,
                                         uint64_t                       max_bytes,
                                         void*                          stream)
{
  if (plan == nullptr || d_grids == nullptr || d_ch_estimates == nullptr || d_noise_var == nullptr ||
      (d_spans == nullptr && nof_spans > 0) || nof_spans > 65536 || (max_bytes & 15u) != 0 ||
      max_bytes > (uint64_t{1} << 32)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid argument (max_bytes a multiple of 16)");
  }
  if (plan->nof_jobs <= 0) {
    return srsgpu_copy_spans(d_spans, nof_spans, max_bytes, stream);
  }
  launch_pusch_chest(plan->d_lp, plan->d_crbs, plan->d_jobs, plan->nof_jobs, plan->geom, d_grids, d_ch_estimates,
                     d_noise_var, d_metrics, plan->d_seq, static_cast<hipStream_t>(stream), d_spans,
                     static_cast<int>(nof_spans), max_bytes);
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

void srsgpu_pusch_chest_plan_destroy(srsgpu_pusch_chest_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  if (plan->d_jobs != nullptr) {
    (void)hipFree(plan->d_jobs);
  }
  if (plan->d_seq != nullptr) {
    (void)hipFree(plan->d_seq);
  }
  if (plan->d_crbs != nullptr) {
    (void)hipFree(plan->d_crbs);
  }
  if (plan->d_lp != nullptr) {
    (void)hipFree(plan->d_lp);
  }
  delete plan;
}

} // extern "C"
