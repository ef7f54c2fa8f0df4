// TEST INFRASTRUCTURE ONLY: timed slot-level runs of the reference's own PHY stages (built from its sources into
// oracle/_ref/libsrsref.so) for bench.py's cpu_baseline leg: the DL stages after the encoder (PDSCH DM-RS + PDSCH
// modulator of every UE into one grid, OFDM modulation of every port) and the UL stages before the decoder (OFDM
// demodulation of every port, then per UE DM-RS channel estimation and PUSCH demodulation). The open-source reference
// estimates at most one layer per PUSCH (port_channel_estimator_average_impl.cpp:83), so the UL stages run
// single-layer UEs (ZF 1 x N). Every reference object is thread_local: bench.py runs one slot loop per host core.
#include "srsran/phy/support/precoding_configuration.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/upper/channel_estimation.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_codeword_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_demodulator_notifier.h"
#include "srsran/srsvec/bit.h"

#include "lib/phy/generic_functions/dft_processor_generic_impl.h"
#include "lib/phy/generic_functions/precoding/channel_precoder_generic.h"
#include "lib/phy/lower/modulation/ofdm_demodulator_impl.h"
#include "lib/phy/lower/modulation/ofdm_modulator_impl.h"
#include "lib/phy/support/interpolator/interpolator_linear_impl.h"
#include "lib/phy/support/resource_grid_impl.h"
#include "lib/phy/support/resource_grid_mapper_impl.h"
#include "lib/phy/support/time_alignment_estimator/time_alignment_estimator_dft_impl.h"
#include "lib/phy/upper/channel_modulation/demodulation_mapper_impl.h"
#include "lib/phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_modulator_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_demodulator_impl.h"
#include "lib/phy/upper/equalization/channel_equalizer_generic_impl.h"
#include "lib/phy/upper/sequence_generators/low_papr_sequence_generator_impl.h"
#include "lib/phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "lib/phy/upper/signal_processors/dmrs_pdsch_processor_impl.h"
#include "lib/phy/upper/signal_processors/dmrs_pusch_estimator_impl.h"
#include "lib/phy/upper/signal_processors/port_channel_estimator_average_impl.h"

#include <chrono>
#include <cstring>
#include <memory>
#include <vector>

using namespace srsran;

namespace {

using clk = std::chrono::steady_clock;

long long ns_since(clk::time_point t0)
{
  return std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count();
}

class sink_buffer : public pusch_codeword_buffer
{
public:
  explicit sink_buffer(unsigned n) : data(n) {}
  span<log_likelihood_ratio> get_next_block_view(unsigned block_size) override
  {
    return span<log_likelihood_ratio>(data).subspan(pos, std::min<unsigned>(block_size, data.size() - pos));
  }
  void on_new_block(span<const log_likelihood_ratio> b, const bit_buffer&) override { pos += b.size(); }
  void on_end_codeword() override {}
  std::vector<log_likelihood_ratio> data;
  unsigned                          pos = 0;
};

class null_notifier : public pusch_demodulator_notifier
{
public:
  void on_provisional_stats(unsigned, const demodulation_stats&) override {}
  void on_end_stats(const demodulation_stats&) override {}
};

precoding_configuration identity(unsigned L, unsigned P)
{
  precoding_configuration p(L, P, 1, MAX_NOF_PRBS);
  for (unsigned port = 0; port != P; ++port) {
    for (unsigned l = 0; l != L; ++l) {
      p.set_coefficient(cf_t(port == l ? 1.0F : 0.0F, 0.0F), l, port, 0);
    }
  }
  return p;
}

} // namespace

extern "C" {

/// One DL slot after the encoder: per UE PDSCH DM-RS + PDSCH modulation (identity precoding, DM-RS symbols
/// dmrs_mask, type 1, 2 CDM groups without data) into a 273-PRB 4-port grid, then OFDM modulation of the 4 ports
/// (4096-point DFT, generic). Returns the elapsed nanoseconds of those stages; out_ofdm_ns gets the OFDM part.
long long ref_dl_slot_timed(int            nof_ues,
                            const int*     rb_start,
                            const int*     nof_rb,
                            int            qm,
                            int            nof_layers,
                            unsigned       dmrs_mask,
                            const uint8_t* codewords,
                            const int*     cw_byte_offset,
                            long long*     out_ofdm_ns)
{
  static thread_local pdsch_modulator_impl modulator(
      std::make_unique<modulation_mapper_lut_impl>(), std::make_unique<pseudo_random_generator_impl>(),
      std::make_unique<resource_grid_mapper_impl>(std::make_unique<channel_precoder_generic>()));
  static thread_local dmrs_pdsch_processor_impl dmrs(
      std::make_unique<pseudo_random_generator_impl>(),
      std::make_unique<resource_grid_mapper_impl>(std::make_unique<channel_precoder_generic>()));
  static thread_local resource_grid_impl grid(4, 14, 273 * 12);
  static thread_local std::unique_ptr<ofdm_slot_modulator_impl> ofdm;
  static thread_local std::vector<cf_t>                          samples;
  if (!ofdm) {
    ofdm_modulator_common_configuration common;
    common.dft = std::make_unique<dft_processor_generic_impl>(
        dft_processor::configuration{4096, dft_processor::direction::INVERSE});
    ofdm = std::make_unique<ofdm_slot_modulator_impl>(
        common, ofdm_modulator_configuration{1, 273, 4096, cyclic_prefix::NORMAL, 1.0F / 64, 3.5e9});
    samples.resize(ofdm->get_slot_size(0));
  }
  const modulation_scheme mod = qm == 8 ? modulation_scheme::QAM256
                                        : (qm == 6 ? modulation_scheme::QAM64
                                                   : (qm == 4 ? modulation_scheme::QAM16 : modulation_scheme::QPSK));
  const int                       nof_dmrs = __builtin_popcount(dmrs_mask);
  symbol_slot_mask                dmrs_pos(14);
  for (unsigned l = 0; l != 14; ++l) {
    dmrs_pos.set(l, ((dmrs_mask >> l) & 1U) != 0);
  }
  std::vector<dynamic_bit_buffer> cws(static_cast<size_t>(nof_ues));
  for (int u = 0; u < nof_ues; ++u) {
    const unsigned nbits = static_cast<unsigned>(nof_rb[u] * 12 * (14 - nof_dmrs) * nof_layers * qm);
    cws[u].resize(nbits);
    srsvec::copy_offset(cws[u], span<const uint8_t>(codewords + cw_byte_offset[u], (nbits + 7) / 8), 0);
  }
  auto t0 = clk::now();
  for (int u = 0; u < nof_ues; ++u) {
    dmrs_pdsch_processor::config_t dc;
    dc.slot                 = slot_point(subcarrier_spacing::kHz30, 0);
    dc.reference_point_k_rb = 0;
    dc.type                 = dmrs_type::TYPE1;
    dc.scrambling_id        = 500;
    dc.n_scid               = false;
    dc.amplitude            = 1.4125375F;
    dc.symbols_mask         = dmrs_pos;
    dc.rb_mask = crb_bitmap(273);
    dc.rb_mask.fill(rb_start[u], rb_start[u] + nof_rb[u]);
    dc.precoding = identity(nof_layers, 4);
    dmrs.map(grid.get_writer(), dc);

    pdsch_modulator::config_t mc;
    mc.rnti                        = static_cast<uint16_t>(0x4601 + u);
    mc.bwp_size_rb                 = 273;
    mc.bwp_start_rb                = 0;
    mc.modulation1                 = mod;
    mc.modulation2                 = mod;
    mc.freq_allocation             = rb_allocation::make_type1(rb_start[u], nof_rb[u]);
    mc.start_symbol_index          = 0;
    mc.nof_symbols                 = 14;
    mc.dmrs_symb_pos               = dc.symbols_mask;
    mc.dmrs_config_type            = dmrs_type::TYPE1;
    mc.nof_cdm_groups_without_data = 2;
    mc.n_id                        = 500;
    mc.scaling                     = 1.0F;
    mc.precoding                   = identity(nof_layers, 4);
    const bit_buffer cw[1]         = {cws[u]};
    modulator.modulate(grid.get_writer(), span<const bit_buffer>(cw, 1), mc);
  }
  auto t1 = clk::now();
  for (unsigned p = 0; p != 4; ++p) {
    ofdm->modulate(samples, grid.get_reader(), p, 0);
  }
  *out_ofdm_ns = ns_since(t1);
  return ns_since(t0);
}

/// One UL slot before the decoder: OFDM demodulation of 4 ports (4096-point generic DFT), then per UE single-layer
/// DM-RS channel estimation (filter / average, CFO compensation when compensate_cfo: du_low's defaults) on the DM-RS
/// symbols of dmrs_mask and PUSCH demodulation (ZF 1 x 4) of its RBs, for slot slot_index of the frame (DM-RS c_init;
/// the OFDM phase compensation of the slot within the subframe). Returns the elapsed nanoseconds; out_ofdm_ns /
/// out_chest_ns get the OFDM and estimation parts. llr_out (optional): the LLRs of every UE, concatenated.
long long ref_ul_slot_timed_at(int          nof_ues,
                               const int*   rb_start,
                               const int*   nof_rb,
                               int          qm,
                               unsigned     dmrs_mask,
                               int          compensate_cfo,
                               int          slot_index,
                               const float* samples_in,
                               int8_t*      llr_out,
                               long long*   out_ofdm_ns,
                               long long*   out_chest_ns)
{
  static thread_local resource_grid_impl                          grid(4, 14, 273 * 12);
  static thread_local std::unique_ptr<ofdm_slot_demodulator_impl> ofdm;
  static thread_local std::unique_ptr<dmrs_pusch_estimator_impl>  ests[2];
  static thread_local std::unique_ptr<pusch_demodulator_impl>     demod;
  static thread_local unsigned                                    slot_size = 0;
  if (!ofdm) {
    ofdm_demodulator_common_configuration common;
    common.dft = std::make_unique<dft_processor_generic_impl>(
        dft_processor::configuration{4096, dft_processor::direction::DIRECT});
    ofdm = std::make_unique<ofdm_slot_demodulator_impl>(
        common, ofdm_demodulator_configuration{1, 273, 4096, cyclic_prefix::NORMAL, 0, 1.0F / 64, 3.5e9});
    slot_size = ofdm->get_slot_size(0);
    for (int c = 0; c != 2; ++c) {
      time_alignment_estimator_dft_impl::collection_dft_processors dfts;
      for (unsigned n = time_alignment_estimator_dft_impl::min_dft_size;
           n <= time_alignment_estimator_dft_impl::max_dft_size;
           n *= 2) {
        dfts.emplace(n, std::make_unique<dft_processor_generic_impl>(
                            dft_processor::configuration{n, time_alignment_estimator_dft_impl::dft_direction}));
      }
      ests[c] = std::make_unique<dmrs_pusch_estimator_impl>(
          std::make_unique<pseudo_random_generator_impl>(), std::make_unique<low_papr_sequence_generator_impl>(),
          std::make_unique<port_channel_estimator_average_impl>(
              std::make_unique<interpolator_linear_impl>(),
              std::make_unique<time_alignment_estimator_dft_impl>(std::move(dfts)),
              port_channel_estimator_fd_smoothing_strategy::filter,
              port_channel_estimator_td_interpolation_strategy::average,
              c == 1));
    }
    demod = std::make_unique<pusch_demodulator_impl>(
        std::make_unique<channel_equalizer_generic_impl>(channel_equalizer_algorithm_type::zf),
        nullptr,
        std::make_unique<demodulation_mapper_impl>(),
        nullptr,
        std::make_unique<pseudo_random_generator_impl>(),
        273,
        true);
  }
  const modulation_scheme mod = qm == 8 ? modulation_scheme::QAM256
                                        : (qm == 6 ? modulation_scheme::QAM64
                                                   : (qm == 4 ? modulation_scheme::QAM16 : modulation_scheme::QPSK));
  dmrs_pusch_estimator_impl& est      = *ests[compensate_cfo ? 1 : 0];
  const int                  nof_dmrs = __builtin_popcount(dmrs_mask);
  symbol_slot_mask           dmrs_pos(14);
  for (unsigned l = 0; l != 14; ++l) {
    dmrs_pos.set(l, ((dmrs_mask >> l) & 1U) != 0);
  }
  std::vector<cf_t> buf(slot_size);
  size_t            llr_pos = 0;
  auto              t0      = clk::now();
  for (unsigned p = 0; p != 4; ++p) {
    std::copy(reinterpret_cast<const cf_t*>(samples_in) + p * slot_size,
              reinterpret_cast<const cf_t*>(samples_in) + (p + 1) * slot_size,
              buf.begin());
    ofdm->demodulate(grid.get_writer(), buf, p, static_cast<unsigned>(slot_index) % 2u);
  }
  *out_ofdm_ns   = ns_since(t0);
  long long chest = 0;
  channel_estimate ce({273, 14, 4, 1});
  null_notifier    notifier;
  for (int u = 0; u < nof_ues; ++u) {
    dmrs_pusch_estimator::configuration cfg;
    cfg.slot = slot_point(subcarrier_spacing::kHz30, static_cast<unsigned>(slot_index));
    dmrs_pusch_estimator::pseudo_random_sequence_configuration seq;
    seq.type          = dmrs_type::TYPE1;
    seq.nof_tx_layers = 1;
    seq.scrambling_id = 500;
    seq.n_scid        = false;
    cfg.sequence_config = seq;
    cfg.scaling         = 1.4125375F;
    cfg.c_prefix        = cyclic_prefix::NORMAL;
    cfg.symbols_mask    = dmrs_pos;
    cfg.rb_mask = crb_bitmap(273);
    cfg.rb_mask.fill(rb_start[u], rb_start[u] + nof_rb[u]);
    cfg.first_symbol = 0;
    cfg.nof_symbols  = 14;
    for (uint8_t p = 0; p != 4; ++p) {
      cfg.rx_ports.push_back(p);
    }
    auto t1 = clk::now();
    est.estimate(ce, grid.get_reader(), cfg);
    chest += ns_since(t1);

    pusch_demodulator::configuration dcfg;
    dcfg.rnti               = static_cast<uint16_t>(0x4601 + u);
    dcfg.rb_mask            = cfg.rb_mask;
    dcfg.modulation         = mod;
    dcfg.start_symbol_index = 0;
    dcfg.nof_symbols        = 14;
    dcfg.dmrs_symb_pos      = dmrs_pos;
    dcfg.dmrs_config_type            = dmrs_type::TYPE1;
    dcfg.nof_cdm_groups_without_data = 2;
    dcfg.n_id                        = 500;
    dcfg.nof_tx_layers               = 1;
    dcfg.enable_transform_precoding  = false;
    for (uint8_t p = 0; p != 4; ++p) {
      dcfg.rx_ports.push_back(p);
    }
    sink_buffer cw(static_cast<unsigned>(nof_rb[u] * 12 * (14 - nof_dmrs) * qm));
    demod->demodulate(cw, notifier, grid.get_reader(), ce, dcfg);
    if (llr_out != nullptr) {
      std::memcpy(llr_out + llr_pos, cw.data.data(), cw.data.size());
      llr_pos += cw.data.size();
    }
  }
  *out_chest_ns = chest;
  return ns_since(t0);
}

/// ref_ul_slot_timed_at of slot 0 of the frame.
long long ref_ul_slot_timed(int          nof_ues,
                            const int*   rb_start,
                            const int*   nof_rb,
                            int          qm,
                            unsigned     dmrs_mask,
                            int          compensate_cfo,
                            const float* samples_in,
                            int8_t*      llr_out,
                            long long*   out_ofdm_ns,
                            long long*   out_chest_ns)
{
  return ref_ul_slot_timed_at(nof_ues, rb_start, nof_rb, qm, dmrs_mask, compensate_cfo, 0, samples_in, llr_out,
                              out_ofdm_ns, out_chest_ns);
}

} // extern "C"
