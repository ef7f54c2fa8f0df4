// Conversions between the reference's per-transmission configurations and the srsgpu C-ABI descriptors, shared by
// the one-transmission bindings (pusch_chain_gpu.cpp, pdsch_chain_gpu.cpp) and the slot-batched processors
// (upper_phy_gpu.cpp), so both describe a transmission to the kernels identically:
//   * dmrs_pusch_estimator::configuration -> srsgpu_pusch_chest_config (+ CRB mask),
//   * pusch_demodulator::configuration    -> srsgpu_pusch_demod_config (+ CRB mask),
//   * pdsch_modulator::config_t           -> srsgpu_pdsch_mod_config (+ CRB mask, reserved RE patterns, PRG weights),
//   * dmrs_pdsch_processor::config_t      -> srsgpu_pdsch_dmrs_config (+ CRB mask),
// plus the results in the other direction: the estimator's metrics into a channel_estimate, the demodulator's LLRs,
// scrambling sequence and statistics into a pusch_codeword_buffer / pusch_demodulator_notifier in the reference's
// block order, and sentinel-scratch grid rows into a resource_grid_writer.
#pragma once

#include "gpu_staging.h"
#include "signal_chain_gpu.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran/phy/upper/channel_estimation.h"
#include "srsran/phy/upper/channel_processors/pdsch/pdsch_modulator.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_codeword_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_demodulator.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_demodulator_notifier.h"
#include "srsran/phy/upper/signal_processors/dmrs_pdsch_processor.h"
#include "srsran/phy/upper/signal_processors/dmrs_pusch_estimator.h"
#include "srsran/srsvec/bit.h"

#include <cmath>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

namespace srsran {
namespace gpu {

/// Value of an RE no mapper wrote in a sentinel scratch grid (a bf16 NaN pair, never produced from finite inputs).
constexpr uint32_t GRID_SENTINEL = 0xffffffffu;

/// CRB allocation of an rb_mask restricted to a grid of grid_prb PRBs: first CRB, count, and the one-byte-per-CRB mask
/// when it is not contiguous (empty otherwise).
struct crb_alloc {
  unsigned             rb_start = 0;
  unsigned             nof_rb   = 0;
  unsigned             span_end = 0;  ///< Last allocated CRB + 1.
  std::vector<uint8_t> mask;
};

inline crb_alloc make_crb_alloc(const crb_bitmap& rb_mask, unsigned grid_prb, const char* who)
{
  crb_alloc a;
  const int lo = rb_mask.find_lowest();
  const int hi = rb_mask.find_highest();
  if (lo < 0 || hi < lo || static_cast<unsigned>(hi) >= grid_prb) {
    throw std::invalid_argument(std::string(who) + ": RB mask empty or beyond the resource grid");
  }
  a.rb_start = static_cast<unsigned>(lo);
  a.nof_rb   = static_cast<unsigned>(rb_mask.count());
  a.span_end = static_cast<unsigned>(hi) + 1;
  if (a.span_end - a.rb_start != a.nof_rb) {
    a.mask.assign(grid_prb, 0);
    for (unsigned rb = a.rb_start; rb != a.span_end; ++rb) {
      a.mask[rb] = rb_mask.test(rb) ? 1 : 0;
    }
  }
  return a;
}

inline uint16_t symbol_mask_bits(const bounded_bitset<MAX_NSYMB_PER_SLOT>& m)
{
  uint16_t bits = 0;
  for (unsigned l = 0; l != std::min<unsigned>(m.size(), 14); ++l) {
    bits |= m.test(l) ? (1u << l) : 0u;
  }
  return bits;
}

/// Grid CRB mask (one byte per CRB) of a crb_bitmap.
inline std::vector<uint8_t> crb_bytes(const crb_bitmap& m, unsigned grid_prb)
{
  std::vector<uint8_t> out(grid_prb, 0);
  for (unsigned rb = 0; rb != std::min<unsigned>(grid_prb, m.size()); ++rb) {
    out[rb] = m.test(rb) ? 1 : 0;
  }
  return out;
}

/// Wideband precoding weights [port][layer] of PRG 0.
inline void wideband_weights(const precoding_configuration& pc, float (&w)[4][4][2])
{
  std::memset(w, 0, sizeof(w));
  for (unsigned p = 0; p != pc.get_nof_ports(); ++p) {
    for (unsigned ly = 0; ly != pc.get_nof_layers(); ++ly) {
      const cf_t c = pc.get_coefficient(ly, p, 0);
      w[p][ly][0]  = c.real();
      w[p][ly][1]  = c.imag();
    }
  }
}

/// Copies the non-sentinel REs of scratch rows (row (p, l) at scratch + (p * 14 + l) * nsc; symbols [l0, l0 + nsym) of
/// ports 0..P-1) into the grid; a port that received any RE is marked non-empty (resource_grid_writer_impl clears the
/// empty flag on put(), which the OFDM modulator checks, ofdm_modulator_impl.cpp:77).
inline void store_written_res(resource_grid_writer& grid, const uint32_t* scratch, unsigned P, unsigned nsc,
                              unsigned l0, unsigned nsym)
{
  for (unsigned p = 0; p != P; ++p) {
    int      first_k = -1;
    unsigned first_l = 0;
    cbf16_t  first_v;
    for (unsigned l = l0; l != l0 + nsym; ++l) {
      const uint32_t* src = scratch + (static_cast<size_t>(p) * 14 + l) * nsc;
      span<cbf16_t>   dst = grid.get_view(p, l);
      for (unsigned k = 0; k != nsc; ++k) {
        if (src[k] != GRID_SENTINEL) {
          std::memcpy(&dst[k], &src[k], sizeof(uint32_t));
          if (first_k < 0) {
            first_k = static_cast<int>(k);
            first_l = l;
            first_v = dst[k];
          }
        }
      }
    }
    if (first_k >= 0) {
      grid.put(p, first_l, static_cast<unsigned>(first_k), 1, span<const cbf16_t>(&first_v, 1));
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------------
// PUSCH
// ---------------------------------------------------------------------------------------------------------------------

/// A PUSCH DM-RS estimation as srsgpu describes it: descriptor, allocation and plan-cache key bytes.
struct pusch_chest_desc {
  srsgpu_pusch_chest_config c;
  crb_alloc                 alloc;
  unsigned                  nof_ports  = 0;
  unsigned                  nof_layers = 0;

  srsgpu_alloc_ext ext() const
  {
    srsgpu_alloc_ext e;
    std::memset(&e, 0, sizeof(e));
    e.crb_mask = alloc.mask.empty() ? nullptr : alloc.mask.data();
    return e;
  }
  void append_key(std::vector<uint8_t>& key) const
  {
    key_append(key, c);
    key.insert(key.end(), alloc.mask.begin(), alloc.mask.end());
  }
};

inline pusch_chest_desc make_pusch_chest_desc(const dmrs_pusch_estimator::configuration& config, unsigned grid_prb,
                                              const pusch_estimator_options& opts, uint8_t estimate_layout,
                                              const char* who)
{
  pusch_chest_desc d;
  d.nof_ports  = config.rx_ports.size();
  d.nof_layers = config.get_nof_tx_layers();
  if (d.nof_ports == 0 || d.nof_ports > 4 || d.nof_layers == 0 || d.nof_layers > 4 ||
      config.c_prefix != cyclic_prefix::NORMAL) {
    throw std::invalid_argument(std::string(who) + ": 1..4 rx ports and layers and a normal cyclic prefix");
  }
  d.alloc                      = make_crb_alloc(config.rb_mask, grid_prb, who);
  srsgpu_pusch_chest_config& c = d.c;
  std::memset(&c, 0, sizeof(c));
  if (std::holds_alternative<dmrs_pusch_estimator::low_papr_sequence_configuration>(config.sequence_config)) {
    c.dmrs_sequence = SRSGPU_DMRS_LOW_PAPR;
    c.scrambling_id = static_cast<uint16_t>(
        std::get<dmrs_pusch_estimator::low_papr_sequence_configuration>(config.sequence_config).n_rs_id);
    c.dmrs_type = 1;
  } else {
    const auto& s   = std::get<dmrs_pusch_estimator::pseudo_random_sequence_configuration>(config.sequence_config);
    c.dmrs_sequence = SRSGPU_DMRS_PSEUDO_RANDOM;
    c.scrambling_id = static_cast<uint16_t>(s.scrambling_id);
    c.n_scid        = s.n_scid ? 1 : 0;
    c.dmrs_type     = (s.type == dmrs_type::TYPE1) ? 1 : 2;
  }
  c.nof_tx_layers    = static_cast<uint8_t>(d.nof_layers);
  c.nof_rx_ports     = static_cast<uint8_t>(d.nof_ports);
  c.start_symbol     = static_cast<uint8_t>(config.first_symbol);
  c.nof_symbols      = static_cast<uint8_t>(config.nof_symbols);
  c.dmrs_symbol_mask = symbol_mask_bits(config.symbols_mask);
  c.rb_start         = static_cast<uint16_t>(d.alloc.rb_start);
  c.nof_rb           = static_cast<uint16_t>(d.alloc.nof_rb);
  c.slot_index       = static_cast<uint16_t>(config.slot.slot_index());
  c.numerology       = static_cast<uint8_t>(config.slot.numerology());
  c.fd_smoothing     = opts.fd_smoothing;
  c.td_strategy      = opts.td_strategy;
  c.compensate_cfo   = opts.compensate_cfo ? 1 : 0;
  c.estimate_layout  = estimate_layout;
  c.scaling          = config.scaling;
  c.grid_index       = 0;
  return d;
}

/// The estimator's per-port results into a channel_estimate, as port_channel_estimator_average_impl.cpp:140-151 sets
/// them: nv = noise variances [port], m = metrics [port][SRSGPU_CHEST_METRICS] (RSRP, EPRE, nv, SNR, TA s, CFO Hz).
inline void write_chest_metrics(channel_estimate& estimate, const float* nv, const float* m, unsigned P, unsigned L)
{
  for (unsigned p = 0; p != P; ++p) {
    const float* mp = m + SRSGPU_CHEST_METRICS * p;
    estimate.set_noise_variance(nv[p], p);
    estimate.set_epre(mp[1], p);
    estimate.set_snr(mp[3], p);
    for (unsigned ly = 0; ly != L; ++ly) {
      estimate.set_rsrp(mp[0], p, ly);
      estimate.set_time_alignment(phy_time_unit::from_seconds(mp[4]), p, ly);
      estimate.set_cfo_Hz(std::isnan(mp[5]) ? std::optional<float>() : std::optional<float>(mp[5]), p, ly);
    }
  }
}

/// A PUSCH demodulation as srsgpu describes it.
struct pusch_demod_desc {
  srsgpu_pusch_demod_config c;
  crb_alloc                 alloc;
  unsigned                  nof_ports  = 0;
  unsigned                  nof_layers = 0;
  unsigned                  qm         = 0;

  srsgpu_alloc_ext ext() const
  {
    srsgpu_alloc_ext e;
    std::memset(&e, 0, sizeof(e));
    e.crb_mask = alloc.mask.empty() ? nullptr : alloc.mask.data();
    return e;
  }
  void append_key(std::vector<uint8_t>& key) const
  {
    key_append(key, c);
    key.insert(key.end(), alloc.mask.begin(), alloc.mask.end());
  }
};

inline pusch_demod_desc make_pusch_demod_desc(const pusch_demodulator::configuration& config, unsigned grid_prb,
                                              const pusch_demodulator_options& opts, uint8_t estimate_layout,
                                              const char* who)
{
  pusch_demod_desc d;
  d.nof_ports  = config.rx_ports.size();
  d.nof_layers = config.nof_tx_layers;
  d.qm         = get_bits_per_symbol(config.modulation);
  if (d.nof_ports == 0 || d.nof_ports > 4 || d.nof_layers == 0 || d.nof_layers > 4) {
    throw std::invalid_argument(std::string(who) + ": 1..4 rx ports and layers");
  }
  d.alloc                      = make_crb_alloc(config.rb_mask, grid_prb, who);
  srsgpu_pusch_demod_config& c = d.c;
  std::memset(&c, 0, sizeof(c));
  c.rnti                        = config.rnti;
  c.n_id                        = static_cast<uint16_t>(config.n_id);
  c.modulation_order            = static_cast<uint8_t>(d.qm);
  c.nof_tx_layers               = static_cast<uint8_t>(d.nof_layers);
  c.nof_rx_ports                = static_cast<uint8_t>(d.nof_ports);
  c.start_symbol                = static_cast<uint8_t>(config.start_symbol_index);
  c.nof_symbols                 = static_cast<uint8_t>(config.nof_symbols);
  c.dmrs_type                   = (config.dmrs_config_type == dmrs_type::TYPE1) ? 1 : 2;
  c.nof_cdm_groups_without_data = static_cast<uint8_t>(config.nof_cdm_groups_without_data);
  c.equalizer                   = opts.equalizer;
  c.dmrs_symbol_mask            = symbol_mask_bits(config.dmrs_symb_pos);
  c.rb_start                    = static_cast<uint16_t>(d.alloc.rb_start);
  c.nof_rb                      = static_cast<uint16_t>(d.alloc.nof_rb);
  c.estimate_layout             = estimate_layout;
  c.transform_precoding         = config.enable_transform_precoding ? 1 : 0;
  return d;
}

/// demodulation_stats of one (SINR dB, EVM) row: the SINR is reported always (+inf without the post-equalisation
/// SINR, as pusch_demodulator_impl.cpp:400 does with no accumulated noise), the EVM with the EVM calculator only.
inline pusch_demodulator_notifier::demodulation_stats demod_stats_of(const float* row, const pusch_demodulator_options& o)
{
  pusch_demodulator_notifier::demodulation_stats out;
  out.sinr_dB.emplace(o.enable_post_eq_sinr ? row[0] : std::numeric_limits<float>::infinity());
  if (o.enable_evm && !std::isnan(row[1])) {
    out.evm.emplace(row[1]);
  }
  return out;
}

/// Feeds a demodulated codeword to the reference's codeword buffer in pusch_demodulator_impl's order
/// (pusch_demodulator_impl.cpp:272-443): per OFDM symbol with data, the buffer's block views filled with the
/// descrambled LLRs and their scrambling bits, the symbol's provisional statistics before its last block, the end
/// statistics after the last symbol, then on_end_codeword. seq_words: the descrambling sequence, bit 31 of word w =
/// c(32 w); stats: SRSGPU_DEMOD_STATS floats. seq_bytes / block_seq: the caller's scratch.
inline void feed_codeword(pusch_codeword_buffer&                  codeword_buffer,
                          pusch_demodulator_notifier&             notifier,
                          const pusch_demodulator::configuration& config,
                          unsigned                                nof_rb,
                          const int8_t*                           llrs,
                          const uint32_t*                         seq_words,
                          unsigned                                nof_llrs,
                          const float*                            stats,
                          const pusch_demodulator_options&        opts,
                          std::vector<uint8_t>&                   seq_bytes,
                          dynamic_bit_buffer&                     block_seq,
                          const char*                             who)
{
  const size_t nwords = (nof_llrs + 31) / 32;
  seq_bytes.resize(nwords * 4);
  for (size_t w = 0; w != nwords; ++w) {
    seq_bytes[4 * w]     = static_cast<uint8_t>(seq_words[w] >> 24);
    seq_bytes[4 * w + 1] = static_cast<uint8_t>(seq_words[w] >> 16);
    seq_bytes[4 * w + 2] = static_cast<uint8_t>(seq_words[w] >> 8);
    seq_bytes[4 * w + 3] = static_cast<uint8_t>(seq_words[w]);
  }
  const bit_buffer seq             = bit_buffer::from_bytes(span<uint8_t>(seq_bytes)).first(nof_llrs);
  const unsigned   nof_bits_per_re = config.nof_tx_layers * get_bits_per_symbol(config.modulation);
  const unsigned   dmrs_re_per_prb =
      config.nof_cdm_groups_without_data * (config.dmrs_config_type == dmrs_type::TYPE1 ? 6 : 4);
  const unsigned l0  = config.start_symbol_index;
  unsigned       pos = 0;
  for (unsigned l = l0; l != l0 + config.nof_symbols; ++l) {
    const unsigned nof_re_symbol = nof_rb * (config.dmrs_symb_pos.test(l) ? NRE - dmrs_re_per_prb : NRE);
    if (nof_re_symbol == 0) {
      continue;
    }
    unsigned count = 0;
    while (count != nof_re_symbol) {
      span<log_likelihood_ratio> block = codeword_buffer.get_next_block_view((nof_re_symbol - count) * nof_bits_per_re);
      if (block.size() % nof_bits_per_re != 0 || pos + block.size() > nof_llrs) {
        throw std::logic_error(std::string(who) + ": codeword buffer block not aligned to the REs");
      }
      std::memcpy(block.data(), llrs + pos, block.size());
      block_seq.resize(block.size());
      srsvec::copy_offset(block_seq, 0, seq, pos, block.size());
      count += block.size() / nof_bits_per_re;
      pos += block.size();
      if (count == nof_re_symbol) {
        notifier.on_provisional_stats(l, demod_stats_of(stats + 2 * l, opts));
      }
      codeword_buffer.on_new_block(block, block_seq);
    }
  }
  notifier.on_end_stats(demod_stats_of(stats + 2 * 14, opts));
  codeword_buffer.on_end_codeword();
}

// ---------------------------------------------------------------------------------------------------------------------
// PDSCH
// ---------------------------------------------------------------------------------------------------------------------

/// A PDSCH modulation as srsgpu describes it, owning the storage its srsgpu_alloc_ext points into.
struct pdsch_mod_desc {
  srsgpu_pdsch_mod_config           c;
  std::vector<uint8_t>              crb_mask;
  std::vector<std::vector<uint8_t>> res_crbs;
  std::vector<srsgpu_re_pattern>    res;
  std::vector<float>                prg_w;
  unsigned                          prg_size = 0;
  unsigned                          nof_prg  = 0;

  /// The extension; valid while this object lives and is not moved.
  srsgpu_alloc_ext ext()
  {
    for (size_t i = 0; i != res.size(); ++i) {
      res[i].crb_mask = res_crbs[i].data();
    }
    srsgpu_alloc_ext e;
    std::memset(&e, 0, sizeof(e));
    e.crb_mask     = crb_mask.data();
    e.reserved     = res.empty() ? nullptr : res.data();
    e.nof_reserved = static_cast<uint32_t>(res.size());
    if (!prg_w.empty()) {
      e.prg_size    = static_cast<uint16_t>(prg_size);
      e.nof_prg     = static_cast<uint16_t>(nof_prg);
      e.prg_weights = prg_w.data();
    }
    return e;
  }
  void append_key(std::vector<uint8_t>& key) const
  {
    key_append(key, c);
    key.insert(key.end(), crb_mask.begin(), crb_mask.end());
    for (size_t i = 0; i != res.size(); ++i) {
      key_append(key, res[i].re_mask);
      key_append(key, res[i].symbol_mask);
      key.insert(key.end(), res_crbs[i].begin(), res_crbs[i].end());
    }
    key_append(key, prg_size);
    const auto* pw = reinterpret_cast<const uint8_t*>(prg_w.data());
    key.insert(key.end(), pw, pw + prg_w.size() * sizeof(float));
  }
};

inline pdsch_mod_desc make_pdsch_mod_desc(const pdsch_modulator::config_t& config, unsigned nof_bits, unsigned grid_prb,
                                          unsigned grid_ports, const char* who)
{
  const precoding_configuration& pc = config.precoding;
  const unsigned                 L  = pc.get_nof_layers();
  const unsigned                 P  = pc.get_nof_ports();
  if (L == 0 || L > 4 || P < L || P > 4 || P > grid_ports) {
    throw std::invalid_argument(std::string(who) + ": one codeword, 1..4 layers on 1..4 ports");
  }
  pdsch_mod_desc   d;
  const crb_bitmap crbs = config.freq_allocation.get_crb_mask(config.bwp_start_rb, config.bwp_size_rb);
  d.crb_mask            = crb_bytes(crbs, grid_prb);
  srsgpu_pdsch_mod_config& c = d.c;
  std::memset(&c, 0, sizeof(c));
  c.rnti                        = config.rnti;
  c.n_id                        = static_cast<uint16_t>(config.n_id);
  c.modulation_order            = static_cast<uint8_t>(get_bits_per_symbol(config.modulation1));
  c.nof_layers                  = static_cast<uint8_t>(L);
  c.nof_ports                   = static_cast<uint8_t>(P);
  c.start_symbol                = static_cast<uint8_t>(config.start_symbol_index);
  c.nof_symbols                 = static_cast<uint8_t>(config.nof_symbols);
  c.dmrs_type                   = (config.dmrs_config_type == dmrs_type::TYPE1) ? 1 : 2;
  c.nof_cdm_groups_without_data = static_cast<uint8_t>(config.nof_cdm_groups_without_data);
  c.dmrs_symbol_mask            = symbol_mask_bits(config.dmrs_symb_pos);
  c.bwp_start_rb                = static_cast<uint16_t>(config.bwp_start_rb);
  c.bwp_size_rb                 = static_cast<uint16_t>(config.bwp_size_rb);
  c.rb_start                    = static_cast<uint16_t>(std::max(crbs.find_lowest(), 0));
  c.nof_rb                      = static_cast<uint16_t>(crbs.count());
  c.scaling                     = config.scaling;
  wideband_weights(pc, c.precoding);
  c.cw_offset  = 0;
  c.nof_bits   = nof_bits;
  c.grid_index = 0;
  for (const re_pattern& r : config.reserved.get_re_patterns()) {
    d.res_crbs.push_back(crb_bytes(r.crb_mask, grid_prb));
    srsgpu_re_pattern x;
    std::memset(&x, 0, sizeof(x));
    for (unsigned k = 0; k != NRE; ++k) {
      x.re_mask |= r.re_mask.test(k) ? (1u << k) : 0u;
    }
    for (unsigned l = 0; l != 14; ++l) {
      x.symbol_mask |= r.symbols.test(l) ? (1u << l) : 0u;
    }
    d.res.push_back(x);
  }
  d.prg_size = pc.get_prg_size();
  if (pc.get_nof_prg() > 1) {
    d.nof_prg = pc.get_nof_prg();
    for (unsigned g = 0; g != pc.get_nof_prg(); ++g) {
      for (unsigned p = 0; p != P; ++p) {
        for (unsigned ly = 0; ly != L; ++ly) {
          const cf_t w = pc.get_coefficient(ly, p, g);
          d.prg_w.push_back(w.real());
          d.prg_w.push_back(w.imag());
        }
      }
    }
  }
  return d;
}

/// A PDSCH DM-RS mapping as srsgpu describes it.
struct pdsch_dmrs_desc {
  srsgpu_pdsch_dmrs_config c;
  std::vector<uint8_t>     crb_mask;

  srsgpu_alloc_ext ext() const
  {
    srsgpu_alloc_ext e;
    std::memset(&e, 0, sizeof(e));
    e.crb_mask = crb_mask.data();
    return e;
  }
  void append_key(std::vector<uint8_t>& key) const
  {
    key_append(key, c);
    key.insert(key.end(), crb_mask.begin(), crb_mask.end());
  }
};

inline pdsch_dmrs_desc make_pdsch_dmrs_desc(const dmrs_pdsch_processor::config_t& config, unsigned grid_prb,
                                            unsigned grid_ports, const char* who)
{
  const precoding_configuration& pc = config.precoding;
  const unsigned                 L  = pc.get_nof_layers();
  const unsigned                 P  = pc.get_nof_ports();
  if (L == 0 || L > 4 || P < L || P > 4 || P > grid_ports) {
    throw std::invalid_argument(std::string(who) + ": 1..4 layers on 1..4 ports");
  }
  pdsch_dmrs_desc d;
  d.crb_mask                  = crb_bytes(config.rb_mask, grid_prb);
  srsgpu_pdsch_dmrs_config& c = d.c;
  std::memset(&c, 0, sizeof(c));
  c.slot_index           = static_cast<uint16_t>(config.slot.slot_index());
  c.scrambling_id        = static_cast<uint16_t>(config.scrambling_id);
  c.n_scid               = config.n_scid ? 1 : 0;
  c.dmrs_type            = (config.type == dmrs_type::TYPE1) ? 1 : 2;
  c.nof_layers           = static_cast<uint8_t>(L);
  c.nof_ports            = static_cast<uint8_t>(P);
  c.dmrs_symbol_mask     = symbol_mask_bits(config.symbols_mask);
  c.reference_point_k_rb = static_cast<uint16_t>(config.reference_point_k_rb);
  c.rb_start             = static_cast<uint16_t>(std::max(config.rb_mask.find_lowest(), 0));
  c.nof_rb               = static_cast<uint16_t>(config.rb_mask.count());
  c.amplitude            = config.amplitude;
  wideband_weights(pc, c.precoding);
  c.grid_index = 0;
  return d;
}

} // namespace gpu
} // namespace srsran
