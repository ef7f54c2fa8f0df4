// Reference-side bindings of the PUSCH signal chain (the files a srsRAN maintainer adds next to
// lib/phy/upper/signal_processors/ and lib/phy/upper/channel_processors/pusch/): srsran::dmrs_pusch_estimator
// (include/srsran/phy/upper/signal_processors/dmrs_pusch_estimator.h:100) and srsran::pusch_demodulator
// (include/srsran/phy/upper/channel_processors/pusch/pusch_demodulator.h:95) over the srsgpu C ABI, created by
// dmrs_pusch_estimator_factory / pusch_demodulator_factory implementations, so that the reference's own
// pusch_processor_impl (pusch_processor_impl.cpp:217 estimate, :335 demodulate), wired by upper_phy_factories.cpp:432-609,
// runs its channel estimation and demodulation on an MI355X.
//
// Data path per call: the rows the kernel reads are staged from the caller's resource grid / channel estimate (host
// objects of the reference: resource_grid_reader::get_view, channel_estimate::get_symbol_ch_estimate) through pinned
// memory into HBM, the cached plan runs on the binding's stream, and the results come back into the reference's
// objects: the estimator writes the allocated REs of every symbol / port / layer of the channel_estimate and its
// noise variance, RSRP, EPRE, SNR, time alignment and CFO (dmrs_pusch_estimator_impl.cpp:45 resize, port_channel_
// estimator_average_impl.cpp:140-151); the demodulator feeds the codeword buffer block by block with the descrambled
// LLRs and the scrambling sequence, and notifies the per-symbol and end statistics in the reference's order
// (pusch_demodulator_impl.cpp:272-443).
#include "signal_chain_gpu.h"

#include "gpu_staging.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_codeword_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_demodulator_notifier.h"
#include "srsran/srsvec/bit.h"

#include <cmath>
#include <limits>
#include <stdexcept>
#include <string>

namespace srsran {

namespace {

/// CRB allocation of an rb_mask restricted to a grid of grid_prb PRBs: first CRB, count, and the one-byte-per-CRB mask
/// when it is not contiguous (empty otherwise).
struct crb_alloc {
  unsigned             rb_start = 0;
  unsigned             nof_rb   = 0;
  unsigned             span_end = 0;  ///< Last allocated CRB + 1.
  std::vector<uint8_t> mask;
};

crb_alloc make_crb_alloc(const crb_bitmap& rb_mask, unsigned grid_prb, const char* who)
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

uint16_t symbol_mask_bits(const bounded_bitset<MAX_NSYMB_PER_SLOT>& m)
{
  uint16_t bits = 0;
  for (unsigned l = 0; l != std::min<unsigned>(m.size(), 14); ++l) {
    bits |= m.test(l) ? (1u << l) : 0u;
  }
  return bits;
}

// --------------------------------------------------------------------------------------------------------------------
// DM-RS PUSCH channel estimator
// --------------------------------------------------------------------------------------------------------------------

class dmrs_pusch_estimator_gpu : public dmrs_pusch_estimator
{
  static constexpr const char* WHO = "dmrs_pusch_estimator_gpu";

public:
  dmrs_pusch_estimator_gpu(std::shared_ptr<srsgpu_context> owner_, const gpu::pusch_estimator_options& opts_) :
    owner(std::move(owner_)),
    ctx(owner.get()),
    opts(opts_),
    stream(ctx, WHO),
    plans(srsgpu_pusch_chest_plan_destroy),
    grid_buf(WHO),
    ce_buf(WHO),
    stat_buf(WHO)
  {
  }

  void estimate(channel_estimate& estimate, const resource_grid_reader& grid, const configuration& config) override
  {
    gpu::device_scope dev_scope(ctx, WHO);
    const unsigned P = config.rx_ports.size();
    const unsigned L = config.get_nof_tx_layers();
    if (P == 0 || P > 4 || L == 0 || L > 4 || config.c_prefix != cyclic_prefix::NORMAL) {
      throw std::invalid_argument(std::string(WHO) + ": 1..4 rx ports and layers and a normal cyclic prefix");
    }
    const unsigned nsc      = grid.get_nof_subc();
    const unsigned grid_prb = nsc / NRE;
    const crb_alloc a       = make_crb_alloc(config.rb_mask, grid_prb, WHO);

    srsgpu_pusch_chest_config c;
    std::memset(&c, 0, sizeof(c));
    if (std::holds_alternative<low_papr_sequence_configuration>(config.sequence_config)) {
      c.dmrs_sequence = SRSGPU_DMRS_LOW_PAPR;
      c.scrambling_id = static_cast<uint16_t>(std::get<low_papr_sequence_configuration>(config.sequence_config).n_rs_id);
      c.dmrs_type     = 1;
    } else {
      const auto& s   = std::get<pseudo_random_sequence_configuration>(config.sequence_config);
      c.dmrs_sequence = SRSGPU_DMRS_PSEUDO_RANDOM;
      c.scrambling_id = static_cast<uint16_t>(s.scrambling_id);
      c.n_scid        = s.n_scid ? 1 : 0;
      c.dmrs_type     = (s.type == dmrs_type::TYPE1) ? 1 : 2;
    }
    c.nof_tx_layers    = static_cast<uint8_t>(L);
    c.nof_rx_ports     = static_cast<uint8_t>(P);
    c.start_symbol     = static_cast<uint8_t>(config.first_symbol);
    c.nof_symbols      = static_cast<uint8_t>(config.nof_symbols);
    c.dmrs_symbol_mask = symbol_mask_bits(config.symbols_mask);
    c.rb_start         = static_cast<uint16_t>(a.rb_start);
    c.nof_rb           = static_cast<uint16_t>(a.nof_rb);
    c.slot_index       = static_cast<uint16_t>(config.slot.slot_index());
    c.numerology       = static_cast<uint8_t>(config.slot.numerology());
    c.fd_smoothing     = opts.fd_smoothing;
    c.td_strategy      = opts.td_strategy;
    c.compensate_cfo   = opts.compensate_cfo ? 1 : 0;
    c.estimate_layout  = SRSGPU_CE_PER_SYMBOL;
    c.scaling          = config.scaling;
    c.grid_index       = 0;

    std::vector<uint8_t> key;
    gpu::key_append(key, c);
    gpu::key_append(key, grid_prb);
    key.insert(key.end(), a.mask.begin(), a.mask.end());
    srsgpu_pusch_chest_plan* plan = plans.get(key, [&] {
      srsgpu_alloc_ext ext;
      std::memset(&ext, 0, sizeof(ext));
      ext.crb_mask                  = a.mask.empty() ? nullptr : a.mask.data();
      srsgpu_pusch_chest_plan* p    = nullptr;
      gpu::srsgpu_check(srsgpu_pusch_chest_plan_create_ex(ctx, &c, &ext, 1, grid_prb, P, &p), WHO);
      return p;
    });

    // Rx grid: the DM-RS symbols of every rx port, [port][symbol][subcarrier] (the plan's grid layout).
    const size_t row = static_cast<size_t>(nsc) * sizeof(uint32_t);
    grid_buf.reserve(P * 14 * row);
    hipStream_t s = stream.get();
    for (unsigned p = 0; p != P; ++p) {
      for (unsigned l = 0; l != 14; ++l) {
        if ((c.dmrs_symbol_mask >> l) & 1u) {
          span<const cbf16_t> v = grid.get_view(config.rx_ports[p], l);
          std::memcpy(grid_buf.host((p * 14 + l) * row), v.data(), row);
          grid_buf.upload((p * 14 + l) * row, row, s);
        }
      }
    }
    // Estimates [layer][port][symbol][subcarrier], noise variances [port], metrics [port][SRSGPU_CHEST_METRICS].
    const size_t ce_bytes = static_cast<size_t>(L) * P * 14 * row;
    ce_buf.reserve(static_cast<size_t>(4) * P * 14 * row);
    stat_buf.reserve(sizeof(float) * (4 + 4 * SRSGPU_CHEST_METRICS));
    gpu::srsgpu_check(srsgpu_pusch_chest_plan_execute(plan, grid_buf.dev<uint32_t>(), ce_buf.dev<uint32_t>(),
                                                      stat_buf.dev<float>(), stat_buf.dev<float>(4 * sizeof(float)),
                                                      s),
                      WHO);
    // The allocated subcarriers of every row (one 2D copy), and the statistics.
    const size_t col0 = static_cast<size_t>(a.rb_start) * NRE * sizeof(uint32_t);
    const size_t cols = static_cast<size_t>(a.span_end - a.rb_start) * NRE * sizeof(uint32_t);
    gpu::hip_check(hipMemcpy2DAsync(ce_buf.host(col0), row, ce_buf.dev(col0), row, cols, ce_bytes / row,
                                    hipMemcpyDeviceToHost, s),
                   WHO, "estimate download");
    stat_buf.download(0, sizeof(float) * (4 + 4 * SRSGPU_CHEST_METRICS), s);
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");

    // Into the reference's channel estimate (dimensions as dmrs_pusch_estimator_impl.cpp:45 sets them).
    estimate.resize({static_cast<unsigned>(config.rb_mask.size()), config.first_symbol + config.nof_symbols, P, L});
    const float* nv = stat_buf.host<float>();
    const float* m  = stat_buf.host<float>(4 * sizeof(float));
    for (unsigned ly = 0; ly != L; ++ly) {
      for (unsigned p = 0; p != P; ++p) {
        for (unsigned l = config.first_symbol; l != config.first_symbol + config.nof_symbols; ++l) {
          span<cbf16_t> dst   = estimate.get_symbol_ch_estimate(l, p, ly);
          const size_t  k0    = static_cast<size_t>(a.rb_start) * NRE;
          const size_t  n     = std::min<size_t>(dst.size(), static_cast<size_t>(a.span_end) * NRE) - k0;
          const auto*   src   = ce_buf.host<uint32_t>(((static_cast<size_t>(ly) * P + p) * 14 + l) * row);
          if (a.mask.empty()) {
            std::memcpy(dst.data() + k0, src + k0, n * sizeof(uint32_t));
          } else {
            for (unsigned rb = a.rb_start; rb != a.span_end; ++rb) {
              if (a.mask[rb] != 0 && (rb + 1) * NRE <= dst.size()) {
                std::memcpy(dst.data() + rb * NRE, src + rb * NRE, NRE * sizeof(uint32_t));
              }
            }
          }
        }
      }
    }
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

private:
  std::shared_ptr<srsgpu_context>           owner;
  srsgpu_context*                           ctx;
  gpu::pusch_estimator_options              opts;
  gpu::owned_stream                         stream;
  gpu::plan_cache<srsgpu_pusch_chest_plan>  plans;
  gpu::staged_buffer                        grid_buf;
  gpu::staged_buffer                        ce_buf;
  gpu::staged_buffer                        stat_buf;
};

class dmrs_pusch_estimator_factory_gpu : public dmrs_pusch_estimator_factory
{
public:
  dmrs_pusch_estimator_factory_gpu(int device, const gpu::pusch_estimator_options& opts_) :
    ctx(gpu::shared_context(device)), opts(opts_)
  {
  }
  std::unique_ptr<dmrs_pusch_estimator> create() override
  {
    return std::make_unique<dmrs_pusch_estimator_gpu>(ctx, opts);
  }

private:
  std::shared_ptr<srsgpu_context> ctx;
  gpu::pusch_estimator_options    opts;
};

// --------------------------------------------------------------------------------------------------------------------
// PUSCH demodulator
// --------------------------------------------------------------------------------------------------------------------

class pusch_demodulator_gpu : public pusch_demodulator
{
  static constexpr const char* WHO = "pusch_demodulator_gpu";

public:
  pusch_demodulator_gpu(std::shared_ptr<srsgpu_context> owner_, const gpu::pusch_demodulator_options& opts_) :
    owner(std::move(owner_)),
    ctx(owner.get()),
    opts(opts_),
    stream(ctx, WHO),
    plans(srsgpu_pusch_demodulator_plan_destroy),
    grid_buf(WHO),
    ce_buf(WHO),
    out_buf(WHO)
  {
  }

  void demodulate(pusch_codeword_buffer&      codeword_buffer,
                  pusch_demodulator_notifier& notifier,
                  const resource_grid_reader& grid,
                  const channel_estimate&     estimates,
                  const configuration&        config) override
  {
    gpu::device_scope dev_scope(ctx, WHO);
    const unsigned P  = config.rx_ports.size();
    const unsigned L  = config.nof_tx_layers;
    const unsigned Qm = get_bits_per_symbol(config.modulation);
    if (P == 0 || P > 4 || L == 0 || L > 4) {
      throw std::invalid_argument(std::string(WHO) + ": 1..4 rx ports and layers");
    }
    const unsigned  nsc      = grid.get_nof_subc();
    const unsigned  grid_prb = nsc / NRE;
    const crb_alloc a        = make_crb_alloc(config.rb_mask, grid_prb, WHO);

    srsgpu_pusch_demod_config c;
    std::memset(&c, 0, sizeof(c));
    c.rnti                        = config.rnti;
    c.n_id                        = static_cast<uint16_t>(config.n_id);
    c.modulation_order            = static_cast<uint8_t>(Qm);
    c.nof_tx_layers               = static_cast<uint8_t>(L);
    c.nof_rx_ports                = static_cast<uint8_t>(P);
    c.start_symbol                = static_cast<uint8_t>(config.start_symbol_index);
    c.nof_symbols                 = static_cast<uint8_t>(config.nof_symbols);
    c.dmrs_type                   = (config.dmrs_config_type == dmrs_type::TYPE1) ? 1 : 2;
    c.nof_cdm_groups_without_data = static_cast<uint8_t>(config.nof_cdm_groups_without_data);
    c.equalizer                   = opts.equalizer;
    c.dmrs_symbol_mask            = symbol_mask_bits(config.dmrs_symb_pos);
    c.rb_start                    = static_cast<uint16_t>(a.rb_start);
    c.nof_rb                      = static_cast<uint16_t>(a.nof_rb);
    c.estimate_layout             = SRSGPU_CE_PER_SYMBOL;
    c.transform_precoding         = config.enable_transform_precoding ? 1 : 0;

    std::vector<uint8_t> key;
    gpu::key_append(key, c);
    gpu::key_append(key, grid_prb);
    key.insert(key.end(), a.mask.begin(), a.mask.end());
    srsgpu_pusch_demodulator_plan* plan = plans.get(key, [&] {
      srsgpu_alloc_ext ext;
      std::memset(&ext, 0, sizeof(ext));
      ext.crb_mask                     = a.mask.empty() ? nullptr : a.mask.data();
      srsgpu_pusch_demodulator_plan* p = nullptr;
      gpu::srsgpu_check(srsgpu_pusch_demodulator_plan_create_ex(ctx, &c, &ext, 1, grid_prb, P, &p), WHO);
      return p;
    });
    const uint32_t nof_llrs = srsgpu_pusch_demodulator_plan_nof_llrs(plan, 0);

    // Rx grid rows of the allocated symbols, [port][symbol][subcarrier].
    hipStream_t    s     = stream.get();
    const size_t   row   = static_cast<size_t>(nsc) * sizeof(uint32_t);
    const unsigned l0    = config.start_symbol_index;
    const unsigned nsym  = config.nof_symbols;
    grid_buf.reserve(P * 14 * row);
    for (unsigned p = 0; p != P; ++p) {
      for (unsigned l = l0; l != l0 + nsym; ++l) {
        std::memcpy(grid_buf.host((p * 14 + l) * row), grid.get_view(config.rx_ports[p], l).data(), row);
      }
      grid_buf.upload((p * 14 + l0) * row, nsym * row, s);
    }
    // Channel estimates [layer][port][symbol][subcarrier] (channel_estimate rows are CRB-indexed like the grid) and
    // the noise variances at [4 tx + port].
    const size_t ce_slot = static_cast<size_t>(P) * 14 * row;
    ce_buf.reserve(4 * ce_slot + 4 * sizeof(float));
    for (unsigned ly = 0; ly != L; ++ly) {
      for (unsigned p = 0; p != P; ++p) {
        const size_t base = ly * ce_slot + static_cast<size_t>(p) * 14 * row;
        for (unsigned l = l0; l != l0 + nsym; ++l) {
          span<const cbf16_t> v = estimates.get_symbol_ch_estimate(l, p, ly);
          const size_t        n = std::min<size_t>(v.size(), nsc) * sizeof(uint32_t);
          std::memcpy(ce_buf.host(base + l * row), v.data(), n);
          if (n < row) {
            std::memset(ce_buf.host(base + l * row + n), 0, row - n);
          }
        }
        ce_buf.upload(base + l0 * row, nsym * row, s);
      }
    }
    float* nv = ce_buf.host<float>(4 * ce_slot);
    for (unsigned p = 0; p != 4; ++p) {
      nv[p] = p < P ? estimates.get_noise_variance(p) : 0.0F;
    }
    ce_buf.upload(4 * ce_slot, 4 * sizeof(float), s);

    // LLRs, statistics and the descrambling sequence.
    const size_t seq_words = (nof_llrs + 31) / 32;
    const size_t stats_off = (nof_llrs + 15) / 16 * 16;
    const size_t seq_off   = stats_off + SRSGPU_DEMOD_STATS * sizeof(float);
    out_buf.reserve(seq_off + seq_words * 4);
    gpu::srsgpu_check(srsgpu_pusch_demodulator_plan_execute_ex(plan, grid_buf.dev<uint32_t>(), ce_buf.dev<uint32_t>(),
                                                               ce_buf.dev<float>(4 * ce_slot), out_buf.dev<int8_t>(),
                                                               out_buf.dev<float>(stats_off), s),
                      WHO);
    gpu::srsgpu_check(srsgpu_pusch_demodulator_plan_scrambling(plan, 0, out_buf.dev<uint32_t>(seq_off), s), WHO);
    out_buf.download(0, seq_off + seq_words * 4, s);
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");

    // The sequence words (bit 31 of word w = c(32 w)) as an MSB-first byte stream (srsran::bit_buffer packing).
    seq_bytes.resize(seq_words * 4);
    const uint32_t* words = out_buf.host<uint32_t>(seq_off);
    for (size_t w = 0; w != seq_words; ++w) {
      seq_bytes[4 * w]     = static_cast<uint8_t>(words[w] >> 24);
      seq_bytes[4 * w + 1] = static_cast<uint8_t>(words[w] >> 16);
      seq_bytes[4 * w + 2] = static_cast<uint8_t>(words[w] >> 8);
      seq_bytes[4 * w + 3] = static_cast<uint8_t>(words[w]);
    }
    const bit_buffer seq = bit_buffer::from_bytes(span<uint8_t>(seq_bytes)).first(nof_llrs);

    // Blocks in the reference's order: per OFDM symbol with data, the codeword buffer's block views, the symbol's
    // provisional statistics before its last block, the end statistics after the last symbol.
    const int8_t*  llrs            = out_buf.host<int8_t>();
    const float*   st              = out_buf.host<float>(stats_off);
    const unsigned nof_bits_per_re = L * Qm;
    const unsigned dmrs_re_per_prb =
        config.nof_cdm_groups_without_data * (config.dmrs_config_type == dmrs_type::TYPE1 ? 6 : 4);
    unsigned pos = 0;
    for (unsigned l = l0; l != l0 + nsym; ++l) {
      const unsigned nof_re_symbol = a.nof_rb * (config.dmrs_symb_pos.test(l) ? NRE - dmrs_re_per_prb : NRE);
      if (nof_re_symbol == 0) {
        continue;
      }
      unsigned count = 0;
      while (count != nof_re_symbol) {
        span<log_likelihood_ratio> block = codeword_buffer.get_next_block_view((nof_re_symbol - count) * nof_bits_per_re);
        if (block.size() % nof_bits_per_re != 0 || pos + block.size() > nof_llrs) {
          throw std::logic_error(std::string(WHO) + ": codeword buffer block not aligned to the REs");
        }
        std::memcpy(block.data(), llrs + pos, block.size());
        block_seq.resize(block.size());
        srsvec::copy_offset(block_seq, 0, seq, pos, block.size());
        count += block.size() / nof_bits_per_re;
        pos += block.size();
        if (count == nof_re_symbol) {
          notifier.on_provisional_stats(l, stats_of(st + 2 * l));
        }
        codeword_buffer.on_new_block(block, block_seq);
      }
    }
    notifier.on_end_stats(stats_of(st + 2 * 14));
    codeword_buffer.on_end_codeword();
  }

private:
  /// demodulation_stats of one (SINR dB, EVM) row: the SINR is reported always (+inf without the post-equalisation
  /// SINR, as pusch_demodulator_impl.cpp:400 does with no accumulated noise), the EVM with the EVM calculator only.
  pusch_demodulator_notifier::demodulation_stats stats_of(const float* row) const
  {
    pusch_demodulator_notifier::demodulation_stats out;
    out.sinr_dB.emplace(opts.enable_post_eq_sinr ? row[0] : std::numeric_limits<float>::infinity());
    if (opts.enable_evm && !std::isnan(row[1])) {
      out.evm.emplace(row[1]);
    }
    return out;
  }

  std::shared_ptr<srsgpu_context>                owner;
  srsgpu_context*                                ctx;
  gpu::pusch_demodulator_options                 opts;
  gpu::owned_stream                              stream;
  gpu::plan_cache<srsgpu_pusch_demodulator_plan> plans;
  gpu::staged_buffer                             grid_buf;
  gpu::staged_buffer                             ce_buf;
  gpu::staged_buffer                             out_buf;
  std::vector<uint8_t>                           seq_bytes;
  dynamic_bit_buffer                             block_seq;
};

class pusch_demodulator_factory_gpu : public pusch_demodulator_factory
{
public:
  pusch_demodulator_factory_gpu(int device, const gpu::pusch_demodulator_options& opts_) :
    ctx(gpu::shared_context(device)), opts(opts_)
  {
  }
  std::unique_ptr<pusch_demodulator> create() override { return std::make_unique<pusch_demodulator_gpu>(ctx, opts); }

private:
  std::shared_ptr<srsgpu_context> ctx;
  gpu::pusch_demodulator_options  opts;
};

} // namespace

std::shared_ptr<dmrs_pusch_estimator_factory>
create_dmrs_pusch_estimator_factory_gpu(int device, const gpu::pusch_estimator_options& opts)
{
  return std::make_shared<dmrs_pusch_estimator_factory_gpu>(device, opts);
}

std::shared_ptr<pusch_demodulator_factory> create_pusch_demodulator_factory_gpu(int                                   device,
                                                                                const gpu::pusch_demodulator_options& opts)
{
  return std::make_shared<pusch_demodulator_factory_gpu>(device, opts);
}

} // namespace srsran
