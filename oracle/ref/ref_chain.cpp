// TEST INFRASTRUCTURE ONLY: the reference's own PUSCH and PDSCH processors (pusch_processor_impl, pdsch_processor_impl,
// compiled from their sources by oracle/build_chain.sh) assembled twice - once from the reference's CPU components, once
// with the signal-chain bindings of integration/ (GPU DM-RS estimator, PUSCH demodulator, PDSCH modulator, PDSCH DM-RS,
// and the HAL accelerators) plugged in through the same interfaces - plus the lower-PHY OFDM slot transforms both ways,
// so tests/test_chain_gpu.py can compare the two on the same inputs. The wiring mirrors the reference's factories
// (pusch/factories.cpp, pdsch/factories.cpp, upper_phy_factories.cpp:432-1014): estimator filter / average / CFO
// compensation (du_low defaults), ZF equalizer with EVM and post-equalisation SINR, the UL-SCH demultiplexer and the UCI
// decoder of the reference, LDPC with early stop.
//
// A UE transmitter (chain_ue_tx) built from the reference's PDSCH encoder, modulator and DM-RS processor makes the
// test's PUSCH: the PUSCH scrambling (c_init = rnti 2^15 + n_id), modulation, layer mapping and DM-RS sequences are the
// PDSCH ones (TS 38.211 6.3.1.1 / 7.3.1.1, 6.4.1.1.1 / 7.4.1.1.1).
#include "hw_accelerator_pusch_dec_gpu.h"
#include "gpu_staging.h"
#include "signal_chain_gpu.h"
#include "upper_phy_gpu.h"

#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_processor_result_notifier.h"
#include "srsran/phy/upper/unique_rx_buffer.h"
#include "srsran/ran/sch/sch_dmrs_power.h"
#include "srsran/srsvec/bit.h"

#include "lib/phy/generic_functions/dft_processor_generic_impl.h"
#include "lib/phy/generic_functions/precoding/channel_precoder_generic.h"
#include "lib/phy/lower/modulation/ofdm_demodulator_impl.h"
#include "lib/phy/lower/modulation/ofdm_modulator_impl.h"
#include "lib/phy/support/interpolator/interpolator_linear_impl.h"
#include "lib/phy/support/resource_grid_impl.h"
#include "lib/phy/support/resource_grid_mapper_impl.h"
#include "lib/phy/support/time_alignment_estimator/time_alignment_estimator_dft_impl.h"
#include "lib/phy/upper/channel_coding/crc_calculator_generic_impl.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_decoder_avx2.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_decoder_avx512.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_encoder_avx2.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_avx2_impl.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_rate_matcher_impl.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_segmenter_rx_impl.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_segmenter_tx_impl.h"
#include "lib/phy/upper/channel_coding/polar/polar_code_impl.h"
#include "lib/phy/upper/channel_coding/polar/polar_deallocator_impl.h"
#include "lib/phy/upper/channel_coding/polar/polar_decoder_impl.h"
#include "lib/phy/upper/channel_coding/polar/polar_encoder_impl.h"
#include "lib/phy/upper/channel_coding/polar/polar_rate_dematcher_impl.h"
#include "lib/phy/upper/channel_coding/short/short_block_detector_impl.h"
#include "lib/phy/upper/channel_modulation/demodulation_mapper_impl.h"
#include "lib/phy/upper/channel_modulation/evm_calculator_generic_impl.h"
#include "lib/phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_encoder_hw_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_modulator_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_processor_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_codeblock_decoder.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_decoder_hw_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_decoder_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_demodulator_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_processor_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_processor_validator_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_processor_validator_impl.h"
#include "lib/phy/upper/channel_processors/pusch/ulsch_demultiplex_impl.h"
#include "lib/phy/upper/channel_processors/uci/uci_decoder_impl.h"
#include "lib/phy/upper/equalization/channel_equalizer_generic_impl.h"
#include "lib/phy/upper/sequence_generators/low_papr_sequence_generator_impl.h"
#include "lib/phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "lib/phy/upper/signal_processors/dmrs_pdsch_processor_impl.h"
#include "lib/phy/upper/signal_processors/dmrs_pusch_estimator_impl.h"
#include "lib/phy/upper/signal_processors/port_channel_estimator_average_impl.h"
#include "lib/phy/upper/signal_processors/ptrs/ptrs_pdsch_generator_impl.h"
#include "lib/phy/upper/downlink_processor_single_executor_impl.h"
#include "lib/phy/upper/uplink_processor_impl.h"
#include "srsran/gateways/baseband/buffer/baseband_gateway_buffer_reader.h"
#include "srsran/phy/lower/lower_phy_rx_symbol_context.h"
#include "srsran/gateways/baseband/buffer/baseband_gateway_buffer_writer.h"
#include "srsran/phy/lower/processors/downlink/pdxch/pdxch_processor.h"
#include "srsran/phy/lower/processors/downlink/pdxch/pdxch_processor_baseband.h"
#include "srsran/phy/lower/processors/downlink/pdxch/pdxch_processor_notifier.h"
#include "srsran/phy/lower/processors/downlink/pdxch/pdxch_processor_request_handler.h"
#include "srsran/phy/lower/processors/uplink/puxch/puxch_processor.h"
#include "srsran/phy/lower/processors/uplink/puxch/puxch_processor_baseband.h"
#include "srsran/phy/lower/processors/uplink/puxch/puxch_processor_notifier.h"
#include "srsran/phy/lower/processors/uplink/puxch/puxch_processor_request_handler.h"
#include "srsran/phy/upper/rx_buffer_pool.h"
#include "srsran/phy/upper/uplink_pdu_validator.h"
#include "srsran/phy/upper/upper_phy_rg_gateway.h"
#include "srsran/phy/upper/upper_phy_rx_results_notifier.h"
#include "srsran/phy/upper/channel_processors/pdcch/pdcch_processor.h"
#include "srsran/phy/upper/channel_processors/ssb/ssb_processor.h"
#include "srsran/phy/upper/signal_processors/nzp_csi_rs_generator.h"
#include "srsran/phy/upper/signal_processors/prs/prs_generator.h"
#include "srsran/srslog/srslog.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <exception>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <random>
#include <sys/prctl.h>
#include <thread>
#include <memory>
#include <vector>

using namespace srsran;

namespace {

constexpr unsigned CB_IDS_PER_HARQ = 160;

/// Test PUSCH / PDSCH parameters (mirrored by tests/chain_harness.py).
struct chain_params {
  int32_t slot;              ///< Slot index within the frame (30 kHz SCS).
  int32_t rnti;
  int32_t n_id;
  int32_t qm;                ///< Modulation order.
  float   target_code_rate;  ///< R x 1024.
  int32_t rv;
  int32_t base_graph;
  int32_t new_data;
  int32_t harq_id;
  int32_t nof_layers;
  int32_t nof_ports;         ///< Rx ports (PUSCH) or precoding ports (PDSCH).
  int32_t dmrs_mask;
  int32_t dmrs_type2;
  int32_t scrambling_id;
  int32_t n_scid;
  int32_t cdm_groups;        ///< CDM groups without data.
  int32_t rb_start;          ///< VRB allocation start within the BWP.
  int32_t nof_rb;
  int32_t bwp_start;
  int32_t bwp_size;
  int32_t start_symbol;
  int32_t nof_symbols;
  int32_t nof_harq_ack;
  int32_t nof_csi_part1;
  int32_t dc_position;       ///< -1: none.
  int32_t tbs_lbrm_bytes;
  int32_t grid_prb;
  int32_t max_iterations;
  int32_t csi2_size0;        ///< CSI Part 2 bits (0: no CSI Part 2) when bit 0 of CSI Part 1 is 0 (or always, when
  int32_t csi2_size1;        ///< csi2_size1 == 0) / when it is 1 (uci_part2_size_description, one 1-bit parameter)
};

symbol_slot_mask symbol_mask(int bits)
{
  symbol_slot_mask m(14);
  for (unsigned l = 0; l != 14; ++l) {
    m.set(l, ((bits >> l) & 1) != 0);
  }
  return m;
}

modulation_scheme to_mod(int qm)
{
  return static_cast<modulation_scheme>(qm);
}

std::unique_ptr<crc_calculator> crc(crc_generator_poly p)
{
  return std::make_unique<crc_calculator_generic_impl>(p);
}

template <typename S>
S sch_crc()
{
  S s;
  s.crc16  = crc(crc_generator_poly::CRC16);
  s.crc24A = crc(crc_generator_poly::CRC24A);
  s.crc24B = crc(crc_generator_poly::CRC24B);
  return s;
}

std::unique_ptr<ldpc_decoder> cpu_ldpc_decoder()
{
  if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw")) {
    return std::make_unique<ldpc_decoder_avx512>();
  }
  return std::make_unique<ldpc_decoder_avx2>();
}

std::unique_ptr<time_alignment_estimator_dft_impl> ta_estimator()
{
  time_alignment_estimator_dft_impl::collection_dft_processors dfts;
  for (unsigned n = time_alignment_estimator_dft_impl::min_dft_size; n <= time_alignment_estimator_dft_impl::max_dft_size;
       n *= 2) {
    dfts.emplace(n, std::make_unique<dft_processor_generic_impl>(
                        dft_processor::configuration{n, time_alignment_estimator_dft_impl::dft_direction}));
  }
  return std::make_unique<time_alignment_estimator_dft_impl>(std::move(dfts));
}

std::unique_ptr<uci_decoder> cpu_uci_decoder()
{
  return std::make_unique<uci_decoder_impl>(std::make_unique<short_block_detector_impl>(),
                                            std::make_unique<polar_code_impl>(),
                                            std::make_unique<polar_rate_dematcher_impl>(),
                                            std::make_unique<polar_decoder_impl>(std::make_unique<polar_encoder_impl>(),
                                                                                 polar_code::NMAX_LOG),
                                            std::make_unique<polar_deallocator_impl>(),
                                            crc(crc_generator_poly::CRC6),
                                            crc(crc_generator_poly::CRC11));
}

std::unique_ptr<resource_grid_mapper> cpu_mapper()
{
  return std::make_unique<resource_grid_mapper_impl>(std::make_unique<channel_precoder_generic>());
}

/// Minimal unique_rx_buffer::callback (as oracle/ref/ref_hal.cpp): per codeblock soft bits, data bits, CRC flags.
class test_rx_buffer : public unique_rx_buffer::callback
{
public:
  test_rx_buffer(unsigned nof_cbs, unsigned first_abs_id) :
    crcs(nof_cbs, 0), soft(nof_cbs, std::vector<log_likelihood_ratio>(66 * 384)),
    data(nof_cbs, std::vector<uint8_t>(22 * 384 / 8)), abs0(first_abs_id)
  {
  }
  unsigned   get_nof_codeblocks() const override { return static_cast<unsigned>(crcs.size()); }
  void       reset_codeblocks_crc() override { std::fill(crcs.begin(), crcs.end(), 0); }
  span<bool> get_codeblocks_crc() override { return span<bool>(reinterpret_cast<bool*>(crcs.data()), crcs.size()); }
  unsigned   get_absolute_codeblock_id(unsigned cb) const override { return abs0 + cb; }
  span<log_likelihood_ratio> get_codeblock_soft_bits(unsigned cb, unsigned size) override
  {
    return span<log_likelihood_ratio>(soft[cb]).first(size);
  }
  bit_buffer get_codeblock_data_bits(unsigned cb, unsigned size) override
  {
    return bit_buffer::from_bytes(data[cb]).first(size);
  }
  bool try_lock() override { return true; }
  void unlock() override {}
  void release() override { reset_codeblocks_crc(); }

private:
  std::vector<char>                              crcs;
  std::vector<std::vector<log_likelihood_ratio>> soft;
  std::vector<std::vector<uint8_t>>              data;
  unsigned                                       abs0;
};

class result_capture : public pusch_processor_result_notifier
{
public:
  void on_uci(const pusch_processor_result_control& r) override
  {
    uci      = r;
    have_uci = true;
  }
  void on_sch(const pusch_processor_result_data& r) override
  {
    sch      = r;
    have_sch = true;
  }
  pusch_processor_result_control uci;
  pusch_processor_result_data    sch;
  bool                           have_uci = false;
  bool                           have_sch = false;
};

class pdsch_done : public pdsch_processor_notifier
{
public:
  void on_finish_processing() override { done = true; }
  bool done = false;
};

/// A pusch_processor_impl over the given estimator / demodulator / decoder (one processing thread).
std::unique_ptr<pusch_processor> make_pusch_processor(std::unique_ptr<dmrs_pusch_estimator> est,
                                                      std::unique_ptr<pusch_demodulator>    demod,
                                                      std::unique_ptr<pusch_decoder>        dec,
                                                      unsigned                              max_iter)
{
  std::vector<std::unique_ptr<pusch_processor_impl::concurrent_dependencies>> deps;
  deps.push_back(std::make_unique<pusch_processor_impl::concurrent_dependencies>(
      std::move(est),
      std::move(demod),
      std::make_unique<ulsch_demultiplex_impl>(),
      cpu_uci_decoder(),
      channel_estimate::channel_estimate_dimensions{MAX_RB, MAX_NSYMB_PER_SLOT, 4, 4}));
  pusch_processor_impl::configuration cfg;
  cfg.thread_local_dependencies_pool =
      std::make_shared<pusch_processor_impl::concurrent_dependencies_pool_type>(std::move(deps));
  cfg.decoder               = std::move(dec);
  cfg.dec_nof_iterations    = max_iter;
  cfg.dec_enable_early_stop = true;
  cfg.csi_sinr_calc_method  = channel_state_information::sinr_type::post_equalization;
  return std::make_unique<pusch_processor_impl>(cfg);
}

std::unique_ptr<pusch_decoder> cpu_pusch_decoder()
{
  std::vector<std::unique_ptr<pusch_codeblock_decoder>> cbs;
  auto                                                  cb_crc = sch_crc<pusch_codeblock_decoder::sch_crc>();
  cbs.push_back(std::make_unique<pusch_codeblock_decoder>(
      std::make_unique<ldpc_rate_dematcher_avx2_impl>(), cpu_ldpc_decoder(), cb_crc));
  auto pool = std::make_shared<pusch_decoder_impl::codeblock_decoder_pool>(std::move(cbs));
  return std::make_unique<pusch_decoder_impl>(
      std::make_unique<ldpc_segmenter_rx_impl>(), pool, sch_crc<pusch_decoder_impl::sch_crc>(), nullptr, MAX_RB, 4);
}

std::unique_ptr<pdsch_encoder> cpu_pdsch_encoder()
{
  auto seg_crc = sch_crc<ldpc_segmenter_tx_impl::sch_crc>();
  return std::make_unique<pdsch_encoder_impl>(
      std::make_unique<ldpc_segmenter_tx_impl>(seg_crc),
      std::make_unique<ldpc_encoder_avx2>(),
      std::make_unique<ldpc_rate_matcher_impl>());
}

std::unique_ptr<pdsch_modulator> cpu_pdsch_modulator()
{
  return std::make_unique<pdsch_modulator_impl>(
      std::make_unique<modulation_mapper_lut_impl>(), std::make_unique<pseudo_random_generator_impl>(), cpu_mapper());
}

std::unique_ptr<dmrs_pdsch_processor> cpu_dmrs_pdsch()
{
  return std::make_unique<dmrs_pdsch_processor_impl>(std::make_unique<pseudo_random_generator_impl>(), cpu_mapper());
}

std::unique_ptr<pdsch_processor> make_pdsch_processor(std::unique_ptr<pdsch_encoder>        enc,
                                                      std::unique_ptr<pdsch_modulator>      mod,
                                                      std::unique_ptr<dmrs_pdsch_processor> dmrs)
{
  return std::make_unique<pdsch_processor_impl>(
      std::move(enc),
      std::move(mod),
      std::move(dmrs),
      std::make_unique<ptrs_pdsch_generator_generic_impl>(std::make_unique<pseudo_random_generator_impl>(),
                                                          cpu_mapper()));
}

/// A PUSCH processor of mode 0 (reference CPU components), 1 (GPU estimator + demodulator, reference CPU decoder) or
/// 2 (GPU estimator + demodulator, pusch_decoder_hw_impl over `hw_pool`'s GPU accelerators). Estimator: filter
/// smoothing, CFO compensation and the given time strategy; ZF with post-equalisation SINR; EVM when `evm`.
std::unique_ptr<pusch_processor> new_pusch_processor(int                                                     device,
                                                     int                                                     mode,
                                                     port_channel_estimator_td_interpolation_strategy        td,
                                                     unsigned                                                max_iter,
                                                     bool                                                    evm,
                                                     const std::shared_ptr<pusch_decoder_hw_impl::hw_decoder_pool>& hw_pool)
{
  if (mode == 0) {
    auto est = std::make_unique<dmrs_pusch_estimator_impl>(
        std::make_unique<pseudo_random_generator_impl>(),
        std::make_unique<low_papr_sequence_generator_impl>(),
        std::make_unique<port_channel_estimator_average_impl>(std::make_unique<interpolator_linear_impl>(),
                                                              ta_estimator(),
                                                              port_channel_estimator_fd_smoothing_strategy::filter,
                                                              td,
                                                              true));
    auto demod = std::make_unique<pusch_demodulator_impl>(
        std::make_unique<channel_equalizer_generic_impl>(channel_equalizer_algorithm_type::zf),
        nullptr,
        std::make_unique<demodulation_mapper_impl>(),
        evm ? std::make_unique<evm_calculator_generic_impl>(std::make_unique<modulation_mapper_lut_impl>()) : nullptr,
        std::make_unique<pseudo_random_generator_impl>(),
        MAX_RB,
        true);
    return make_pusch_processor(std::move(est), std::move(demod), cpu_pusch_decoder(), max_iter);
  }
  // GPU signal chain behind the same interfaces; factories dropped right after create() like the reference's.
  const gpu::pusch_estimator_options est_opts =
      gpu::make_pusch_estimator_options(port_channel_estimator_fd_smoothing_strategy::filter, td, true);
  gpu::pusch_demodulator_options demod_opts;
  demod_opts.enable_evm = evm;
  std::unique_ptr<pusch_decoder> dec;
  if (mode == 1) {
    dec = cpu_pusch_decoder();
  } else {
    auto crcs = sch_crc<pusch_decoder_hw_impl::sch_crc>();
    dec       = std::make_unique<pusch_decoder_hw_impl>(std::make_unique<ldpc_segmenter_rx_impl>(), crcs, hw_pool, nullptr);
  }
  return make_pusch_processor(create_dmrs_pusch_estimator_factory_gpu(device, est_opts)->create(),
                              create_pusch_demodulator_factory_gpu(device, demod_opts)->create(),
                              std::move(dec),
                              max_iter);
}

/// A PDSCH processor of mode 0 (reference CPU components) or 1 (pdsch_encoder_hw_impl over the GPU accelerator, GPU
/// modulator, GPU DM-RS).
std::unique_ptr<pdsch_processor> new_pdsch_processor(int device, int mode)
{
  if (mode == 0) {
    return make_pdsch_processor(cpu_pdsch_encoder(), cpu_pdsch_modulator(), cpu_dmrs_pdsch());
  }
  auto seg_crc = sch_crc<ldpc_segmenter_tx_impl::sch_crc>();
  auto crcs    = sch_crc<pdsch_encoder_hw_impl::sch_crc>();
  auto enc     = std::make_unique<pdsch_encoder_hw_impl>(
      crcs, std::make_unique<ldpc_segmenter_tx_impl>(seg_crc), hal::create_hw_accelerator_pdsch_enc_factory_gpu(device)->create());
  return make_pdsch_processor(
      std::move(enc), create_pdsch_modulator_factory_gpu(device)->create(), create_dmrs_pdsch_processor_factory_gpu(device)->create());
}

pusch_processor::pdu_t make_pusch_pdu(const chain_params& cc)
{
  const chain_params* c = &cc;
  const unsigned      P = c->nof_ports;
  pusch_processor::pdu_t pdu;
  pdu.slot                  = slot_point(subcarrier_spacing::kHz30, static_cast<unsigned>(c->slot));
  pdu.rnti                  = static_cast<uint16_t>(c->rnti);
  pdu.bwp_size_rb           = c->bwp_size;
  pdu.bwp_start_rb          = c->bwp_start;
  pdu.cp                    = cyclic_prefix::NORMAL;
  pdu.mcs_descr             = {to_mod(c->qm), c->target_code_rate};
  pdu.codeword              = pusch_processor::codeword_description{
      static_cast<unsigned>(c->rv), c->base_graph == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2,
      c->new_data != 0};
  pdu.uci.nof_harq_ack          = c->nof_harq_ack;
  pdu.uci.nof_csi_part1         = c->nof_csi_part1;
  pdu.uci.alpha_scaling         = 1.0F;
  pdu.uci.beta_offset_harq_ack  = 20.0F;
  pdu.uci.beta_offset_csi_part1 = 6.25F;
  pdu.uci.beta_offset_csi_part2 = 6.25F;
  if (c->csi2_size0 > 0 && c->csi2_size1 <= 0) {
    pdu.uci.csi_part2_size = uci_part2_size_description(static_cast<unsigned>(c->csi2_size0));
  } else if (c->csi2_size0 > 0 || c->csi2_size1 > 0) {
    uci_part2_size_description::entry& entry = pdu.uci.csi_part2_size.entries.emplace_back();
    entry.parameters.push_back({0, 1});
    entry.map.push_back(static_cast<uint16_t>(c->csi2_size0));
    entry.map.push_back(static_cast<uint16_t>(c->csi2_size1));
  }
  pdu.n_id                      = c->n_id;
  pdu.nof_tx_layers             = c->nof_layers;
  for (unsigned i = 0; i != P; ++i) {
    pdu.rx_ports.push_back(static_cast<uint8_t>(i));
  }
  pdu.dmrs_symbol_mask   = symbol_mask(c->dmrs_mask);
  pdu.dmrs               = pusch_processor::dmrs_configuration{c->dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1,
                                                 static_cast<unsigned>(c->scrambling_id),
                                                 c->n_scid != 0,
                                                 static_cast<unsigned>(c->cdm_groups)};
  pdu.freq_alloc         = rb_allocation::make_type1(c->rb_start, c->nof_rb);
  pdu.start_symbol_index = c->start_symbol;
  pdu.nof_symbols        = c->nof_symbols;
  pdu.tbs_lbrm           = units::bytes(static_cast<unsigned>(c->tbs_lbrm_bytes));
  if (c->dc_position >= 0) {
    pdu.dc_position = static_cast<unsigned>(c->dc_position);
  }

  return pdu;
}

pdsch_processor::pdu_t make_pdsch_pdu(const chain_params& cc, const float* weights)
{
  const chain_params* c = &cc;
  const unsigned      P = c->nof_ports;
  const unsigned      L = c->nof_layers;
  pdsch_processor::pdu_t pdu;
  pdu.slot         = slot_point(subcarrier_spacing::kHz30, static_cast<unsigned>(c->slot));
  pdu.rnti         = static_cast<uint16_t>(c->rnti);
  pdu.bwp_size_rb  = c->bwp_size;
  pdu.bwp_start_rb = c->bwp_start;
  pdu.cp           = cyclic_prefix::NORMAL;
  pdu.codewords.push_back({to_mod(c->qm), static_cast<unsigned>(c->rv)});
  pdu.n_id                        = c->n_id;
  pdu.ref_point                   = pdsch_processor::pdu_t::CRB0;
  pdu.dmrs_symbol_mask            = symbol_mask(c->dmrs_mask);
  pdu.dmrs                        = c->dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  pdu.scrambling_id               = c->scrambling_id;
  pdu.n_scid                      = c->n_scid != 0;
  pdu.nof_cdm_groups_without_data = c->cdm_groups;
  pdu.freq_alloc                  = rb_allocation::make_type1(c->rb_start, c->nof_rb);
  pdu.start_symbol_index          = c->start_symbol;
  pdu.nof_symbols                 = c->nof_symbols;
  pdu.ldpc_base_graph             = c->base_graph == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  pdu.tbs_lbrm                    = units::bytes(static_cast<unsigned>(c->tbs_lbrm_bytes));
  pdu.ratio_pdsch_dmrs_to_sss_dB  = get_sch_to_dmrs_ratio_dB(c->cdm_groups);
  pdu.ratio_pdsch_data_to_sss_dB  = 0.0F;
  pdu.precoding                   = precoding_configuration(L, P, 1, MAX_NOF_PRBS);
  for (unsigned port = 0; port != P; ++port) {
    for (unsigned l = 0; l != L; ++l) {
      pdu.precoding.set_coefficient(cf_t(weights[2 * (port * L + l)], weights[2 * (port * L + l) + 1]), l, port, 0);
    }
  }
  return pdu;
}

/// A persistent thread running posted jobs (the processors' thread-local pools bind one instance per thread, so the
/// benchmark's threads must live across repetitions, like the reference benchmark's unique_threads within a case).
class bench_worker
{
public:
  bench_worker() : th([this] { loop(); }) {}
  ~bench_worker()
  {
    {
      std::lock_guard<std::mutex> lock(mtx);
      quit = true;
    }
    cv.notify_all();
    th.join();
  }
  void post(std::function<void()> f)
  {
    std::lock_guard<std::mutex> lock(mtx);
    job  = std::move(f);
    done = false;
    cv.notify_all();
  }
  void wait()
  {
    std::unique_lock<std::mutex> lock(mtx);
    cv.wait(lock, [this] { return done; });
  }

private:
  void loop()
  {
    std::unique_lock<std::mutex> lock(mtx);
    for (;;) {
      cv.wait(lock, [this] { return quit || job; });
      if (quit) {
        return;
      }
      std::function<void()> f = std::move(job);
      job                      = nullptr;
      lock.unlock();
      f();
      lock.lock();
      done = true;
      cv.notify_all();
    }
  }
  std::mutex              mtx;
  std::condition_variable cv;
  std::function<void()>   job;
  bool                    done = true;
  bool                    quit = false;
  std::thread             th;
};

struct chain_harness {
  // PUSCH: 0 CPU reference, 1 GPU estimator + demodulator + CPU decoder, 2 GPU estimator + demodulator + HW decoder.
  std::unique_ptr<pusch_processor>                                     pusch[3];
  // PDSCH: 0 CPU reference, 1 HW encoder (GPU) + GPU modulator + GPU DM-RS.
  std::unique_ptr<pdsch_processor>                                     pdsch[2];
  std::map<std::pair<int, int>, std::unique_ptr<test_rx_buffer>>       rx;
  std::shared_ptr<ofdm_modulator_factory>                              ofdm_mod_gpu;
  std::shared_ptr<ofdm_demodulator_factory>                            ofdm_demod_gpu;
  // UE transmitter (reference CPU components).
  std::unique_ptr<pdsch_encoder>        tx_enc  = cpu_pdsch_encoder();
  std::unique_ptr<pdsch_modulator>      tx_mod  = cpu_pdsch_modulator();
  std::unique_ptr<dmrs_pdsch_processor> tx_dmrs = cpu_dmrs_pdsch();
};

/// Copies a (P, 14, nsc) bf16-pair array into the grid (all ports, all symbols).
void load_grid(resource_grid& g, const uint16_t* in, unsigned P, unsigned nsc)
{
  std::vector<cbf16_t> row(nsc);
  for (unsigned p = 0; p != P; ++p) {
    for (unsigned l = 0; l != 14; ++l) {
      std::memcpy(row.data(), in + 2 * (static_cast<size_t>(p) * 14 + l) * nsc, nsc * sizeof(cbf16_t));
      g.get_writer().put(p, l, 0, 1, row);
    }
  }
}

void store_grid(const resource_grid& g, uint16_t* out, unsigned P, unsigned nsc)
{
  for (unsigned p = 0; p != P; ++p) {
    for (unsigned l = 0; l != 14; ++l) {
      span<const cbf16_t> v = g.get_reader().get_view(p, l);
      std::memcpy(out + 2 * (static_cast<size_t>(p) * 14 + l) * nsc, v.data(), nsc * sizeof(cbf16_t));
    }
  }
}

precoding_configuration identity(unsigned L, unsigned P)
{
  precoding_configuration pc(L, P, 1, MAX_NOF_PRBS);
  for (unsigned p = 0; p != P; ++p) {
    for (unsigned l = 0; l != L; ++l) {
      pc.set_coefficient(cf_t(p == l ? 1.0F : 0.0F, 0.0F), l, p, 0);
    }
  }
  return pc;
}

unsigned nof_data_re(const chain_params& c)
{
  const unsigned dmrs_re = c.cdm_groups * (c.dmrs_type2 ? 4 : 6);
  unsigned       n       = 0;
  for (int l = c.start_symbol; l != c.start_symbol + c.nof_symbols; ++l) {
    n += ((c.dmrs_mask >> l) & 1) ? NRE - dmrs_re : NRE;
  }
  return n * c.nof_rb;
}

/// Runs a harness entry point, turning a C++ exception (a binding's configuration or HIP error) into an error code
/// the Python side reports, instead of terminating the test process.
template <typename F>
int guarded(const char* name, F&& f)
{
  try {
    return f();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s: %s\n", name, e.what());
    return -100;
  }
}

} // namespace

extern "C" {

/// Builds the CPU and GPU processors (GPU `device`): see the file comment.
static void* chain_create_impl(int device, unsigned max_cb_ids)
{
  auto* h = new chain_harness();
  for (int mode = 0; mode <= 2; ++mode) {
    std::shared_ptr<pusch_decoder_hw_impl::hw_decoder_pool> hw_pool;
    if (mode == 2) {
      std::vector<std::unique_ptr<hal::hw_accelerator_pusch_dec>> accs;
      accs.push_back(hal::create_hw_accelerator_pusch_dec_factory_gpu(device, max_cb_ids)->create());
      hw_pool = std::make_shared<pusch_decoder_hw_impl::hw_decoder_pool>(std::move(accs));
    }
    h->pusch[mode] =
        new_pusch_processor(device, mode, port_channel_estimator_td_interpolation_strategy::average, 6, true, hw_pool);
  }
  h->pdsch[0] = new_pdsch_processor(device, 0);
  h->pdsch[1] = new_pdsch_processor(device, 1);
  h->ofdm_mod_gpu   = create_ofdm_modulator_factory_gpu(device);
  h->ofdm_demod_gpu = create_ofdm_demodulator_factory_gpu(device);
  return h;
}

void chain_destroy(void* p)
{
  delete static_cast<chain_harness*>(p);
}

/// UE transmitter: the TB encoded (reference pdsch_encoder_impl), scrambled, modulated and layer-mapped
/// (pdsch_modulator_impl, identity precoding: layer l on port l) and the DM-RS of ports 0..L-1 with the PUSCH
/// DM-RS-to-data amplitude (dmrs_pdsch_processor_impl), into grid_out (L, 14, 12 grid_prb) bf16 pairs. Returns the
/// number of codeword bits.
static int chain_ue_tx_impl(void* p, const chain_params* c, const uint8_t* tb, unsigned tb_bytes, uint16_t* grid_out)
{
  auto*          h   = static_cast<chain_harness*>(p);
  const unsigned L   = c->nof_layers;
  const unsigned nsc = 12 * c->grid_prb;
  const unsigned G   = nof_data_re(*c) * L * c->qm;
  resource_grid_impl grid(L, 14, nsc);
  grid.set_all_zero();

  std::vector<uint8_t> cw(G);
  pdsch_encoder::configuration ec;
  ec.base_graph     = c->base_graph == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  ec.rv             = c->rv;
  ec.mod            = to_mod(c->qm);
  ec.Nref           = 0;
  ec.nof_layers     = L;
  ec.nof_ch_symbols = G / c->qm;
  h->tx_enc->encode(cw, span<const uint8_t>(tb, tb_bytes), ec);
  dynamic_bit_buffer packed(G);
  srsvec::bit_pack(packed, cw);

  pdsch_modulator::config_t mc;
  mc.rnti                        = static_cast<uint16_t>(c->rnti);
  mc.bwp_size_rb                 = c->bwp_size;
  mc.bwp_start_rb                = c->bwp_start;
  mc.modulation1                 = to_mod(c->qm);
  mc.modulation2                 = to_mod(c->qm);
  mc.freq_allocation             = rb_allocation::make_type1(c->rb_start, c->nof_rb);
  mc.start_symbol_index          = c->start_symbol;
  mc.nof_symbols                 = c->nof_symbols;
  mc.dmrs_symb_pos               = symbol_mask(c->dmrs_mask);
  mc.dmrs_config_type            = c->dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  mc.nof_cdm_groups_without_data = c->cdm_groups;
  mc.n_id                        = c->n_id;
  mc.scaling                     = 1.0F;
  mc.precoding                   = identity(L, L);
  const bit_buffer cws[1]        = {packed};
  h->tx_mod->modulate(grid.get_writer(), span<const bit_buffer>(cws, 1), mc);

  dmrs_pdsch_processor::config_t dc;
  dc.slot                 = slot_point(subcarrier_spacing::kHz30, static_cast<unsigned>(c->slot));
  dc.reference_point_k_rb = 0;
  dc.type                 = c->dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  dc.scrambling_id        = c->scrambling_id;
  dc.n_scid               = c->n_scid != 0;
  dc.amplitude            = convert_dB_to_amplitude(-get_sch_to_dmrs_ratio_dB(c->cdm_groups));
  dc.symbols_mask         = symbol_mask(c->dmrs_mask);
  dc.rb_mask              = rb_allocation::make_type1(c->rb_start, c->nof_rb).get_crb_mask(c->bwp_start, c->bwp_size);
  dc.precoding            = identity(L, L);
  h->tx_dmrs->map(grid.get_writer(), dc);
  store_grid(grid, grid_out, L, nsc);
  return static_cast<int>(G);
}

/// pusch_processor_impl::process in mode 0 / 1 / 2 on the received grid (nof_ports, 14, 12 grid_prb) bf16 pairs.
/// out[]: 0 SCH notified, 1 TB CRC ok, 2 codeblocks, 3 LDPC observations, 4 min / 5 max / 6 mean iterations,
/// 7 SINR dB, 8 EVM, 9 TA (s), 10 CFO (Hz), 11 EPRE dB, 12 RSRP dB (NaN when absent), 13 UCI notified,
/// 14 HARQ-ACK status, 15 HARQ-ACK bits (bit i = payload[i]), 16 CSI Part 1 status, 17 CSI Part 1 bits.
static int chain_pusch_process_impl(void* p, int mode, const chain_params* c, const uint16_t* grid_in, uint8_t* tb,
                        unsigned tb_bytes, double* out)
{
  auto*          h   = static_cast<chain_harness*>(p);
  const unsigned P   = c->nof_ports;
  const unsigned nsc = 12 * c->grid_prb;
  resource_grid_impl grid(P, 14, nsc);
  load_grid(grid, grid_in, P, nsc);

  const pusch_processor::pdu_t pdu = make_pusch_pdu(*c);

  auto key = std::make_pair(mode == 0 ? 0 : mode, c->harq_id);
  const unsigned nof_cbs =
      ldpc::compute_nof_codeblocks(units::bytes(tb_bytes).to_bits(),
                                   c->base_graph == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2);
  auto it = h->rx.find(key);
  if (it == h->rx.end() || it->second->get_nof_codeblocks() != nof_cbs) {
    h->rx[key] = std::make_unique<test_rx_buffer>(nof_cbs, static_cast<unsigned>(c->harq_id) * CB_IDS_PER_HARQ);
  }
  result_capture notifier;
  h->pusch[mode]->process(span<uint8_t>(tb, tb_bytes), unique_rx_buffer(*h->rx[key]), notifier, grid.get_reader(), pdu);

  for (int i = 0; i != 18; ++i) {
    out[i] = std::nan("");
  }
  out[0] = notifier.have_sch ? 1 : 0;
  out[13] = notifier.have_uci ? 1 : 0;
  if (notifier.have_sch) {
    const auto& d = notifier.sch.data;
    out[1]        = d.tb_crc_ok ? 1 : 0;
    out[2]        = d.nof_codeblocks_total;
    out[3]        = d.ldpc_decoder_stats.get_nof_observations();
    if (d.ldpc_decoder_stats.get_nof_observations() != 0) {
      out[4] = d.ldpc_decoder_stats.get_min();
      out[5] = d.ldpc_decoder_stats.get_max();
      out[6] = d.ldpc_decoder_stats.get_mean();
    }
    const channel_state_information& csi = notifier.sch.csi;
    auto opt = [](std::optional<float> v) { return v.has_value() ? static_cast<double>(*v) : std::nan(""); };
    out[7]   = opt(csi.get_sinr_dB());
    out[8]   = opt(csi.get_total_evm());
    out[9]   = csi.get_time_alignment().has_value() ? csi.get_time_alignment()->to_seconds() : std::nan("");
    out[10]  = opt(csi.get_cfo_Hz());
    out[11]  = opt(csi.get_epre_dB());
    out[12]  = opt(csi.get_rsrp_dB());
  }
  if (notifier.have_uci) {
    auto bits = [](const pusch_uci_field& f) {
      double v = 0;
      for (unsigned i = 0; i != f.payload.size(); ++i) {
        v += f.payload.test(i) ? std::ldexp(1.0, static_cast<int>(i)) : 0.0;
      }
      return v;
    };
    out[14] = static_cast<double>(notifier.uci.harq_ack.status);
    out[15] = bits(notifier.uci.harq_ack);
    out[16] = static_cast<double>(notifier.uci.csi_part1.status);
    out[17] = bits(notifier.uci.csi_part1);
  }
  return 0;
}

/// pdsch_processor_impl::process in mode 0 (CPU) / 1 (GPU) of one TB (nof_layers layers on nof_ports ports, precoding
/// `weights` [port][layer] complex float, one PRG) into grid_inout (nof_ports, 14, 12 grid_prb) bf16 pairs: the grid
/// keeps whatever it holds outside the PDSCH's REs.
static int chain_pdsch_process_impl(void* p, int mode, const chain_params* c, const float* weights, const uint8_t* tb,
                        unsigned tb_bytes, uint16_t* grid_inout)
{
  auto*          h   = static_cast<chain_harness*>(p);
  const unsigned P   = c->nof_ports;
  const unsigned L   = c->nof_layers;
  const unsigned nsc = 12 * c->grid_prb;
  resource_grid_impl grid(P, 14, nsc);
  load_grid(grid, grid_inout, P, nsc);

  const pdsch_processor::pdu_t pdu = make_pdsch_pdu(*c, weights);
  static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data;
  data.emplace_back(span<const uint8_t>(tb, tb_bytes));
  pdsch_done done;
  h->pdsch[mode]->process(grid.get_writer(), done, std::move(data), pdu);
  store_grid(grid, grid_inout, P, nsc);
  return done.done ? 0 : -1;
}

/// ofdm_slot_modulator of one port: mode 0 the reference (generic DFT), 1 the GPU binding. Returns the slot size.
static int chain_ofdm_modulate_impl(void* p, int mode, unsigned numerology, unsigned bw_rb, unsigned dft_size, float scale,
                        double center_freq_hz, unsigned slot, const uint16_t* grid_port, float* out, unsigned cap)
{
  auto*                        h = static_cast<chain_harness*>(p);
  ofdm_modulator_configuration cfg{numerology, bw_rb, dft_size, cyclic_prefix::NORMAL, scale, center_freq_hz};
  std::unique_ptr<ofdm_slot_modulator> m;
  if (mode == 0) {
    ofdm_modulator_common_configuration common;
    common.dft = std::make_unique<dft_processor_generic_impl>(
        dft_processor::configuration{dft_size, dft_processor::direction::INVERSE});
    m = std::make_unique<ofdm_slot_modulator_impl>(common, cfg);
  } else {
    m = h->ofdm_mod_gpu->create_ofdm_slot_modulator(cfg);
  }
  resource_grid_impl grid(1, 14, 12 * bw_rb);
  load_grid(grid, grid_port, 1, 12 * bw_rb);
  const unsigned n = m->get_slot_size(slot);
  if (n > cap) {
    return -1;
  }
  m->modulate(span<cf_t>(reinterpret_cast<cf_t*>(out), n), grid.get_reader(), 0, slot);
  return static_cast<int>(n);
}

/// ofdm_slot_demodulator of one port (mode 0 reference, 1 GPU) into grid_port (1, 14, 12 bw_rb) bf16 pairs.
static int chain_ofdm_demodulate_impl(void* p, int mode, unsigned numerology, unsigned bw_rb, unsigned dft_size, float scale,
                          double center_freq_hz, unsigned window_offset, unsigned slot, const float* in, unsigned n,
                          uint16_t* grid_port)
{
  auto*                          h = static_cast<chain_harness*>(p);
  ofdm_demodulator_configuration cfg{
      numerology, bw_rb, dft_size, cyclic_prefix::NORMAL, window_offset, scale, center_freq_hz};
  std::unique_ptr<ofdm_slot_demodulator> d;
  if (mode == 0) {
    ofdm_demodulator_common_configuration common;
    common.dft = std::make_unique<dft_processor_generic_impl>(
        dft_processor::configuration{dft_size, dft_processor::direction::DIRECT});
    d = std::make_unique<ofdm_slot_demodulator_impl>(common, cfg);
  } else {
    d = h->ofdm_demod_gpu->create_ofdm_slot_demodulator(cfg);
  }
  if (d->get_slot_size(slot) != n) {
    return -1;
  }
  resource_grid_impl grid(1, 14, 12 * bw_rb);
  grid.set_all_zero();
  d->demodulate(grid.get_writer(), span<const cf_t>(reinterpret_cast<const cf_t*>(in), n), 0, slot);
  store_grid(grid, grid_port, 1, 12 * bw_rb);
  return 0;
}

void* chain_create(int device, unsigned max_cb_ids)
{
  void* h = nullptr;
  guarded("chain_create", [&] {
    h = chain_create_impl(device, max_cb_ids);
    return 0;
  });
  return h;
}

int chain_ue_tx(void* p, const chain_params* c, const uint8_t* tb, unsigned tb_bytes, uint16_t* grid_out)
{
  return guarded("chain_ue_tx", [&] { return chain_ue_tx_impl(p, c, tb, tb_bytes, grid_out); });
}

int chain_pusch_process(void* p, int mode, const chain_params* c, const uint16_t* grid_in, uint8_t* tb,
                        unsigned tb_bytes, double* out)
{
  return guarded("chain_pusch_process", [&] { return chain_pusch_process_impl(p, mode, c, grid_in, tb, tb_bytes, out); });
}

int chain_pdsch_process(void* p, int mode, const chain_params* c, const float* weights, const uint8_t* tb,
                        unsigned tb_bytes, uint16_t* grid_inout)
{
  return guarded("chain_pdsch_process",
                 [&] { return chain_pdsch_process_impl(p, mode, c, weights, tb, tb_bytes, grid_inout); });
}

int chain_ofdm_modulate(void* p, int mode, unsigned numerology, unsigned bw_rb, unsigned dft_size, float scale,
                        double center_freq_hz, unsigned slot, const uint16_t* grid_port, float* out, unsigned cap)
{
  return guarded("chain_ofdm_modulate", [&] {
    return chain_ofdm_modulate_impl(p, mode, numerology, bw_rb, dft_size, scale, center_freq_hz, slot, grid_port, out,
                                    cap);
  });
}

int chain_ofdm_demodulate(void* p, int mode, unsigned numerology, unsigned bw_rb, unsigned dft_size, float scale,
                          double center_freq_hz, unsigned window_offset, unsigned slot, const float* in, unsigned n,
                          uint16_t* grid_port)
{
  return guarded("chain_ofdm_demodulate", [&] {
    return chain_ofdm_demodulate_impl(
        p, mode, numerology, bw_rb, dft_size, scale, center_freq_hz, window_offset, slot, in, n, grid_port);
  });
}

/// Throughput harness restating the reference's pusch_processor_benchmark.cpp "throughput_total" mode (the benchmark
/// itself cannot be built here: the reference's DFT factories need FFTW, absent from this image): nof_threads
/// persistent threads, each with its own pusch_processor_impl (mode 0 / 1 / 2 as chain_pusch_process; the benchmark's
/// estimator configuration: filter smoothing, interpolate time strategy, CFO compensation; ZF; EVM off; 2 LDPC
/// iterations with early stop, pusch_processor_benchmark.cpp:129-139, :630) and its own rx buffer, process the same PDU
/// `batch` times over one grid of random complex-normal REs (:700-720); seconds[r] = wall time of repetition r (all
/// threads). Returns the number of TBs whose CRC passed (0 on noise).
static int chain_pusch_bench_impl(int                 device,
                                  int                 mode,
                                  const chain_params* c,
                                  unsigned            tb_bytes,
                                  unsigned            nof_threads,
                                  unsigned            batch,
                                  unsigned            repetitions,
                                  double*             seconds)
{
  const unsigned     P   = c->nof_ports;
  const unsigned     nsc = 12 * c->grid_prb;
  resource_grid_impl grid(P, 14, nsc);
  {
    std::mt19937                    rgen(0);
    std::normal_distribution<float> n(0.0F, std::sqrt(0.5F));
    std::vector<cf_t>               row(nsc);
    for (unsigned p = 0; p != P; ++p) {
      for (unsigned l = 0; l != 14; ++l) {
        for (cf_t& v : row) {
          v = cf_t(n(rgen), n(rgen));
        }
        grid.get_writer().put(p, l, 0, row);
      }
    }
  }
  const pusch_processor::pdu_t pdu     = make_pusch_pdu(*c);
  const unsigned               nof_cbs = ldpc::compute_nof_codeblocks(
      units::bytes(tb_bytes).to_bits(), c->base_graph == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2);
  std::shared_ptr<pusch_decoder_hw_impl::hw_decoder_pool> hw_pool;
  if (mode == 2) {
    auto factory = hal::create_hw_accelerator_pusch_dec_factory_gpu(device, (nof_threads + 1) * CB_IDS_PER_HARQ);
    std::vector<std::unique_ptr<hal::hw_accelerator_pusch_dec>> accs;
    for (unsigned t = 0; t != nof_threads; ++t) {
      accs.push_back(factory->create());
    }
    hw_pool = std::make_shared<pusch_decoder_hw_impl::hw_decoder_pool>(std::move(accs));
  }
  std::vector<std::unique_ptr<pusch_processor>> procs;
  std::vector<std::unique_ptr<test_rx_buffer>>  rxb;
  std::vector<std::unique_ptr<bench_worker>>    workers;
  for (unsigned t = 0; t != nof_threads; ++t) {
    procs.push_back(new_pusch_processor(
        device, mode, port_channel_estimator_td_interpolation_strategy::interpolate, 2, false, hw_pool));
    rxb.push_back(std::make_unique<test_rx_buffer>(nof_cbs, t * CB_IDS_PER_HARQ));
    workers.push_back(std::make_unique<bench_worker>());
  }
  std::atomic<int> ok{0};
  auto run_batch = [&](unsigned t, unsigned n) {
    std::vector<uint8_t> data(tb_bytes);
    for (unsigned i = 0; i != n; ++i) {
      result_capture notifier;
      procs[t]->process(data, unique_rx_buffer(*rxb[t]), notifier, grid.get_reader(), pdu);
      ok += (notifier.have_sch && notifier.sch.data.tb_crc_ok) ? 1 : 0;
    }
  };
  // Warm-up: one PDU per thread (plans, pinned staging, first-call setup).
  for (unsigned t = 0; t != nof_threads; ++t) {
    workers[t]->post([&, t] { run_batch(t, 1); });
  }
  for (auto& w : workers) {
    w->wait();
  }
  ok = 0;
  for (unsigned r = 0; r != repetitions; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers[t]->post([&, t] { run_batch(t, batch); });
    }
    for (auto& w : workers) {
      w->wait();
    }
    seconds[r] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return ok.load();
}

/// The same harness for the reference's pdsch_processor_benchmark.cpp "throughput_total" mode: nof_threads persistent
/// threads, each with its own pdsch_processor_impl (mode 0 CPU, 1 GPU) and resource grid, process the same PDU with a
/// random TB `batch` times. seconds[r] = wall time of repetition r.
static int chain_pdsch_bench_impl(int                 device,
                                  int                 mode,
                                  const chain_params* c,
                                  const float*        weights,
                                  unsigned            tb_bytes,
                                  unsigned            nof_threads,
                                  unsigned            batch,
                                  unsigned            repetitions,
                                  double*             seconds)
{
  const pdsch_processor::pdu_t                     pdu = make_pdsch_pdu(*c, weights);
  std::vector<std::unique_ptr<pdsch_processor>>    procs;
  std::vector<std::unique_ptr<resource_grid_impl>> grids;
  std::vector<std::unique_ptr<bench_worker>>       workers;
  std::vector<uint8_t>                             tb(tb_bytes);
  std::mt19937                                     rgen(1);
  for (uint8_t& b : tb) {
    b = static_cast<uint8_t>(rgen());
  }
  for (unsigned t = 0; t != nof_threads; ++t) {
    procs.push_back(new_pdsch_processor(device, mode));
    grids.push_back(std::make_unique<resource_grid_impl>(c->nof_ports, 14, 12 * c->grid_prb));
    grids.back()->set_all_zero();
    workers.push_back(std::make_unique<bench_worker>());
  }
  std::atomic<int> done{0};
  auto run_batch = [&](unsigned t, unsigned n) {
    for (unsigned i = 0; i != n; ++i) {
      static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data;
      data.emplace_back(span<const uint8_t>(tb));
      pdsch_done notifier;
      procs[t]->process(grids[t]->get_writer(), notifier, std::move(data), pdu);
      done += notifier.done ? 1 : 0;
    }
  };
  for (unsigned t = 0; t != nof_threads; ++t) {
    workers[t]->post([&, t] { run_batch(t, 1); });
  }
  for (auto& w : workers) {
    w->wait();
  }
  done = 0;
  for (unsigned r = 0; r != repetitions; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers[t]->post([&, t] { run_batch(t, batch); });
    }
    for (auto& w : workers) {
      w->wait();
    }
    seconds[r] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return done.load();
}

int chain_pusch_bench(int device, int mode, const chain_params* c, unsigned tb_bytes, unsigned nof_threads,
                      unsigned batch, unsigned repetitions, double* seconds)
{
  return guarded("chain_pusch_bench", [&] {
    return chain_pusch_bench_impl(device, mode, c, tb_bytes, nof_threads, batch, repetitions, seconds);
  });
}

int chain_pdsch_bench(int device, int mode, const chain_params* c, const float* weights, unsigned tb_bytes,
                      unsigned nof_threads, unsigned batch, unsigned repetitions, double* seconds)
{
  return guarded("chain_pdsch_bench", [&] {
    return chain_pdsch_bench_impl(device, mode, c, weights, tb_bytes, nof_threads, batch, repetitions, seconds);
  });
}

} // extern "C"

// ---------------------------------------------------------------------------------------------------------------------
// Upper-PHY slot processors (row b6): the reference's own uplink_processor_impl and
// downlink_processor_single_executor_impl, once over the reference's CPU channel processors and once over the GPU slot
// batches of integration/upper_phy_gpu.cpp, fed the same slots (tests/test_upper_phy_gpu.py).
// ---------------------------------------------------------------------------------------------------------------------

namespace {

/// Runs every task on the caller (deterministic test order).
class inline_test_executor : public task_executor
{
public:
  bool execute(unique_task task) override
  {
    task();
    return true;
  }
  bool defer(unique_task task) override
  {
    task();
    return true;
  }
};

inline_test_executor& test_executor()
{
  static inline_test_executor e;
  return e;
}

// Channel processors the tests never drive (the reference's uplink / downlink processors require valid instances).
class stub_prach : public prach_detector
{
public:
  prach_detection_result detect(const prach_buffer&, const configuration&) override { return {}; }
};
class stub_pucch : public pucch_processor
{
public:
  pucch_processor_result process(const resource_grid_reader&, const format0_configuration&) override { return {}; }
  const pucch_format1_map<pucch_processor_result>& process(const resource_grid_reader&,
                                                           const format1_batch_configuration&) override
  {
    return f1;
  }
  pucch_processor_result process(const resource_grid_reader&, const format2_configuration&) override { return {}; }
  pucch_processor_result process(const resource_grid_reader&, const format3_configuration&) override { return {}; }
  pucch_processor_result process(const resource_grid_reader&, const format4_configuration&) override { return {}; }

private:
  pucch_format1_map<pucch_processor_result> f1;
};
class stub_srs : public srs_estimator
{
public:
  srs_estimator_result estimate(const resource_grid_reader&, const srs_estimator_configuration&) override
  {
    return {};
  }
};
class stub_pdcch : public pdcch_processor
{
public:
  void process(resource_grid_writer&, const pdu_t&) override {}
};
class stub_ssb : public ssb_processor
{
public:
  void process(resource_grid_writer&, const pdu_t&) override {}
};
class stub_csi_rs : public nzp_csi_rs_generator
{
public:
  void map(resource_grid_writer&, const config_t&) override {}
};
class stub_prs : public prs_generator
{
public:
  void generate(resource_grid_writer&, const prs_generator_configuration&) override {}
};

class demux_factory_ref : public ulsch_demultiplex_factory
{
public:
  std::unique_ptr<ulsch_demultiplex> create() override { return std::make_unique<ulsch_demultiplex_impl>(); }
};
class uci_factory_ref : public uci_decoder_factory
{
public:
  std::unique_ptr<uci_decoder> create() override { return cpu_uci_decoder(); }
};

// Factories of the stub channel processors (row b8: the GPU slot-processor factories take the channel factories of the
// channels they do not batch, as upper_phy_factories.cpp passes its PUCCH / PRACH / SRS / PDCCH / SSB / CSI-RS / PRS
// factories). Their validators accept every configuration.
template <typename V, typename... C>
class accept_all;
template <typename V, typename C>
class accept_all<V, C> : public V
{
public:
  error_type<std::string> is_valid(const C&) const override { return default_success_t(); }
};
class accept_all_pucch : public pucch_pdu_validator
{
public:
  error_type<std::string> is_valid(const pucch_processor::format0_configuration&) const override
  {
    return default_success_t();
  }
  error_type<std::string> is_valid(const pucch_processor::format1_configuration&) const override
  {
    return default_success_t();
  }
  error_type<std::string> is_valid(const pucch_processor::format2_configuration&) const override
  {
    return default_success_t();
  }
  error_type<std::string> is_valid(const pucch_processor::format3_configuration&) const override
  {
    return default_success_t();
  }
  error_type<std::string> is_valid(const pucch_processor::format4_configuration&) const override
  {
    return default_success_t();
  }
};
class stub_prach_factory : public prach_detector_factory
{
public:
  std::unique_ptr<prach_detector> create() override { return std::make_unique<stub_prach>(); }
  std::unique_ptr<prach_detector_validator> create_validator() override
  {
    return std::make_unique<accept_all<prach_detector_validator, prach_detector::configuration>>();
  }
};
class stub_pucch_factory : public pucch_processor_factory
{
public:
  std::unique_ptr<pucch_processor>     create() override { return std::make_unique<stub_pucch>(); }
  std::unique_ptr<pucch_pdu_validator> create_validator() override { return std::make_unique<accept_all_pucch>(); }
};
class stub_srs_factory : public srs_estimator_factory
{
public:
  std::unique_ptr<srs_estimator> create() override { return std::make_unique<stub_srs>(); }
  std::unique_ptr<srs_estimator_configuration_validator> create_validator() override
  {
    return std::make_unique<accept_all<srs_estimator_configuration_validator, srs_estimator_configuration>>();
  }
};
class stub_pdcch_factory : public pdcch_processor_factory
{
public:
  std::unique_ptr<pdcch_processor>     create() override { return std::make_unique<stub_pdcch>(); }
  std::unique_ptr<pdcch_pdu_validator> create_validator() override
  {
    return std::make_unique<accept_all<pdcch_pdu_validator, pdcch_processor::pdu_t>>();
  }
};
class stub_ssb_factory : public ssb_processor_factory
{
public:
  std::unique_ptr<ssb_processor>     create() override { return std::make_unique<stub_ssb>(); }
  std::unique_ptr<ssb_pdu_validator> create_validator() override
  {
    return std::make_unique<accept_all<ssb_pdu_validator, ssb_processor::pdu_t>>();
  }
};
class stub_csi_rs_factory : public nzp_csi_rs_generator_factory
{
public:
  std::unique_ptr<nzp_csi_rs_generator> create() override { return std::make_unique<stub_csi_rs>(); }
  std::unique_ptr<nzp_csi_rs_configuration_validator> create_validator() override
  {
    return std::make_unique<accept_all<nzp_csi_rs_configuration_validator, nzp_csi_rs_generator::config_t>>();
  }
};
class stub_prs_factory : public prs_generator_factory
{
public:
  std::unique_ptr<prs_generator>           create() override { return std::make_unique<stub_prs>(); }
  std::unique_ptr<prs_generator_validator> create_validator() override
  {
    return std::make_unique<accept_all<prs_generator_validator, prs_generator_configuration>>();
  }
};
class grid_factory_ref : public resource_grid_factory
{
public:
  std::unique_ptr<resource_grid> create(unsigned nof_ports, unsigned nof_symbols, unsigned nof_subc) override
  {
    return std::make_unique<resource_grid_impl>(nof_ports, nof_symbols, nof_subc);
  }
};
/// The reference's CPU PUSCH decoder (pusch_decoder_impl over the AVX2 dematcher and the host's fastest LDPC decoder).
class cpu_pusch_decoder_factory : public pusch_decoder_factory
{
public:
  std::unique_ptr<pusch_decoder> create() override { return cpu_pusch_decoder(); }
};
/// The reference's pdsch_encoder_hw_impl over the GPU PDSCH-encoder accelerator (row b2).
class gpu_pdsch_encoder_factory : public pdsch_encoder_factory
{
public:
  explicit gpu_pdsch_encoder_factory(int device_) : device(device_) {}
  std::unique_ptr<pdsch_encoder> create() override
  {
    auto seg_crc = sch_crc<ldpc_segmenter_tx_impl::sch_crc>();
    auto crcs    = sch_crc<pdsch_encoder_hw_impl::sch_crc>();
    return std::make_unique<pdsch_encoder_hw_impl>(crcs,
                                                   std::make_unique<ldpc_segmenter_tx_impl>(seg_crc),
                                                   hal::create_hw_accelerator_pdsch_enc_factory_gpu(device)->create());
  }

private:
  int device;
};
class ptrs_factory_ref : public ptrs_pdsch_generator_factory
{
public:
  std::unique_ptr<ptrs_pdsch_generator> create() override
  {
    return std::make_unique<ptrs_pdsch_generator_generic_impl>(std::make_unique<pseudo_random_generator_impl>(),
                                                               cpu_mapper());
  }
};

/// The GPU PUSCH processor factory of the fallback path (row b8): the reference's pusch_processor_impl over the GPU
/// estimator and demodulator (filter smoothing, CFO compensation, time strategy td; ZF with EVM and post-equalisation
/// SINR) and the reference's CPU decoder - what new_pusch_processor(device, 1, ...) assembles by hand.
std::shared_ptr<pusch_processor_factory>
gpu_pusch_factory(int device, port_channel_estimator_td_interpolation_strategy td, unsigned max_iter)
{
  pusch_processor_factory_gpu_configuration pc;
  pc.device      = device;
  pc.estimator   = gpu::make_pusch_estimator_options(port_channel_estimator_fd_smoothing_strategy::filter, td, true);
  pc.demux_factory          = std::make_shared<demux_factory_ref>();
  pc.decoder_factory        = std::make_shared<cpu_pusch_decoder_factory>();
  pc.uci_dec_factory        = std::make_shared<uci_factory_ref>();
  pc.ch_estimate_dimensions = channel_estimate::channel_estimate_dimensions{MAX_RB, MAX_NSYMB_PER_SLOT, 4, 4};
  pc.dec_nof_iterations     = max_iter;
  pc.dec_enable_early_stop  = true;
  pc.csi_sinr_calc_method   = channel_state_information::sinr_type::post_equalization;
  return create_pusch_processor_factory_gpu(pc);
}

/// PUSCH results as the upper PHY's notifier receives them, in arrival order.
struct ul_record {
  int                  rnti, harq_id, crc_ok, nof_cbs, ldpc_obs, ldpc_min, ldpc_max;
  float                ldpc_mean, sinr, evm, ta, cfo, epre, rsrp;
  std::vector<uint8_t> payload;
};

class ul_results_recorder : public upper_phy_rx_results_notifier
{
public:
  void on_new_prach_results(const ul_prach_results&) override {}
  void on_new_pusch_results_control(const ul_pusch_results_control& r) override
  {
    std::lock_guard<std::mutex> lock(mtx);
    ++nof_control;
    if (r.harq_ack.has_value()) {
      // HARQ-ACK on PUSCH: status and payload bits (LSB first) per RNTI.
      int bits = 0;
      for (unsigned b = 0; b != r.harq_ack->payload.size() && b < 30; ++b) {
        bits |= r.harq_ack->payload.test(b) ? (1 << b) : 0;
      }
      harq_ack[static_cast<int>(r.rnti)] = {static_cast<int>(r.harq_ack->status), bits};
    }
    // CSI Part 1 / Part 2: status (-1: not reported) and payload bits (size, first 30 bits LSB first).
    auto field = [](const std::optional<pusch_uci_field>& f) {
      std::array<int, 3> v = {-1, 0, 0};
      if (f.has_value()) {
        v[0] = static_cast<int>(f->status);
        v[1] = static_cast<int>(f->payload.size());
        for (unsigned b = 0; b != f->payload.size() && b < 30; ++b) {
          v[2] |= f->payload.test(b) ? (1 << b) : 0;
        }
      }
      return v;
    };
    csi[static_cast<int>(r.rnti)] = {field(r.csi1), field(r.csi2)};
  }
  void on_new_pusch_results_data(const ul_pusch_results_data& r) override
  {
    if (count_only) {
      // Benchmarks: results arrive on the GPU service's completion thread; only the count (and, when tracked, the
      // latency from the slot's reference instant) matters.
      if (track_latency) {
        const int64_t now = std::chrono::steady_clock::now().time_since_epoch().count();
        const int64_t ref = slot_ref[r.slot.slot_index() % slot_ref.size()].load(std::memory_order_acquire);
        std::lock_guard<std::mutex> lock(mtx);
        latency_ns.push_back(now - ref);
      }
      crc_ok += r.decoder_result.tb_crc_ok ? 1 : 0;
      ++nof_data;
      return;
    }
    std::lock_guard<std::mutex> lock(mtx);
    ++nof_data;
    ul_record x;
    x.rnti    = static_cast<int>(r.rnti);
    x.harq_id = static_cast<int>(r.harq_id);
    x.crc_ok  = r.decoder_result.tb_crc_ok ? 1 : 0;
    x.nof_cbs = static_cast<int>(r.decoder_result.nof_codeblocks_total);
    const auto& st = r.decoder_result.ldpc_decoder_stats;
    x.ldpc_obs     = static_cast<int>(st.get_nof_observations());
    x.ldpc_min     = st.get_nof_observations() ? static_cast<int>(st.get_min()) : -1;
    x.ldpc_max     = st.get_nof_observations() ? static_cast<int>(st.get_max()) : -1;
    x.ldpc_mean    = st.get_nof_observations() ? st.get_mean() : NAN;
    auto opt       = [](std::optional<float> v) { return v.has_value() ? *v : NAN; };
    x.sinr         = opt(r.csi.get_sinr_dB());
    x.evm          = opt(r.csi.get_total_evm());
    x.ta   = r.csi.get_time_alignment().has_value() ? static_cast<float>(r.csi.get_time_alignment()->to_seconds()) : NAN;
    x.cfo  = opt(r.csi.get_cfo_Hz());
    x.epre = opt(r.csi.get_epre_dB());
    x.rsrp = opt(r.csi.get_rsrp_dB());
    x.payload.assign(r.payload.begin(), r.payload.end());
    records.push_back(std::move(x));
  }
  void on_new_pucch_results(const ul_pucch_results&) override {}
  void on_new_srs_results(const ul_srs_results&) override {}

  /// Waits (asynchronous batches) until n data results have arrived since the last reset.
  void wait_for(unsigned n)
  {
    while (nof_data.load() < n) {
      std::this_thread::yield();
    }
  }
  void reset()
  {
    std::lock_guard<std::mutex> lock(mtx);
    records.clear();
    harq_ack.clear();
    csi.clear();
    latency_ns.clear();
    nof_data = 0;
    crc_ok   = 0;
  }

  /// Latency tracking (benchmarks): the reference instant (steady clock) of each slot - its last symbol - set by the
  /// slot's producer before the slot is processed; each data notification records now - reference. Keyed by the slot
  /// index within the frame: the harnesses' PDUs carry that index only (frame 0), and a sector has far fewer than a
  /// frame's slots in flight.
  void track(bool on)
  {
    track_latency = on;
    if (on && slot_ref.empty()) {
      slot_ref = std::vector<std::atomic<int64_t>>(20);
    }
  }
  void set_slot_reference(slot_point sp, std::chrono::steady_clock::time_point t)
  {
    slot_ref[sp.slot_index() % slot_ref.size()].store(t.time_since_epoch().count(), std::memory_order_release);
  }

  std::mutex                         mtx;
  std::vector<ul_record>             records;
  std::map<int, std::pair<int, int>> harq_ack;  ///< RNTI -> (uci_status, payload bits)
  std::map<int, std::pair<std::array<int, 3>, std::array<int, 3>>> csi;  ///< RNTI -> CSI Part 1, Part 2 fields
  unsigned                           nof_control = 0;
  bool                               count_only  = false;
  bool                               track_latency = false;
  std::vector<std::atomic<int64_t>>  slot_ref;
  std::vector<int64_t>               latency_ns;
  std::atomic<unsigned>              nof_data{0};
  std::atomic<unsigned>              crc_ok{0};
};

/// The reference's uplink_processor_impl over CPU processors (variant 0) or the GPU slot batch (variant 1).
struct ul_harness {
  unsigned                                   P, nsc, grid_prb;
  std::unique_ptr<rx_buffer_pool_controller> own_pool;
  rx_buffer_pool_controller*                 pool = nullptr;
  ul_results_recorder                        own_notifier;
  ul_results_recorder*                       notifier = &own_notifier;
  std::shared_ptr<uplink_processor_factory>  factory;  ///< GPU variants: the factory that made `proc` (row b8)
  std::unique_ptr<uplink_processor>          proc;
};

constexpr unsigned UL_POOL_CODEBLOCKS = 2048;

std::unique_ptr<rx_buffer_pool_controller> ul_pool()
{
  rx_buffer_pool_config pc;
  pc.max_codeblock_size   = ldpc::MAX_CODEBLOCK_SIZE;
  pc.nof_buffers          = 256;
  pc.nof_codeblocks       = UL_POOL_CODEBLOCKS;
  pc.expire_timeout_slots = 100;
  pc.external_soft_bits   = false;  // the fallback processor (CPU decoder) keeps its soft bits in the buffers
  return create_rx_buffer_pool(pc);
}

/// What the uplink processors of one sector share: the rx buffer pool, the HBM HARQ arena and the results notifier
/// (du_low builds several uplink processors per sector over one pool). The GPU service is shared by every sector.
struct ul_sector {
  std::unique_ptr<rx_buffer_pool_controller> pool;
  ul_results_recorder                        notifier;
};

/// The GPU uplink processor factory of the tests (row b8): stub PUCCH / PRACH / SRS, the reference's resource grid,
/// the GPU per-PDU PUSCH processor factory as the fallback, the reference's UCI decoder, inline executors.
/// service: nullptr for the device's shared service (gpu::get_pusch_gpu_service); multi: 1 three UE shards on the
/// device with the peer-copy transport, 2 one shard through RCCL at world size 1 (row b7).
std::shared_ptr<uplink_processor_factory> ul_factory(int                                              device,
                                                     port_channel_estimator_td_interpolation_strategy td,
                                                     unsigned                                         max_iter,
                                                     std::shared_ptr<gpu::pusch_gpu_service>          service,
                                                     bool                                             asynchronous,
                                                     int                                              multi)
{
  uplink_processor_factory_gpu_configuration fc;
  fc.pucch_factory   = std::make_shared<stub_pucch_factory>();
  fc.prach_factory   = std::make_shared<stub_prach_factory>();
  fc.srs_factory     = std::make_shared<stub_srs_factory>();
  fc.grid_factory    = std::make_shared<grid_factory_ref>();
  fc.pusch_factory   = gpu_pusch_factory(device, td, max_iter);
  fc.uci_dec_factory = std::make_shared<uci_factory_ref>();
  fc.pucch_executor  = &test_executor();
  fc.pusch_executor  = &test_executor();
  fc.srs_executor    = &test_executor();
  fc.prach_executor  = &test_executor();
  gpu::pusch_batch_configuration& bc = fc.batch;
  bc.device              = device;
  bc.estimator = gpu::make_pusch_estimator_options(port_channel_estimator_fd_smoothing_strategy::filter, td, true);
  bc.max_cb_ids          = UL_POOL_CODEBLOCKS;
  bc.nof_ldpc_iterations = max_iter;
  bc.asynchronous        = asynchronous;
  if (multi == 1) {
    bc.devices = {device, device, device};
  } else if (multi == 2) {
    bc.devices   = {device};
    bc.transport = gpu::create_pusch_rccl_transport({device});
  }
  fc.service                = std::move(service);
  fc.service_config.device  = device;
  return create_uplink_processor_factory_gpu(fc);
}

/// variant: 0 the reference's CPU PUSCH processor, 1 the GPU slot batch; + 2 with the "interpolate" time strategy of
/// the estimator (the batch then keeps per-symbol estimates) instead of du_low's "average". sector / service /
/// asynchronous: the uplink processor as one of several of a sector on a shared GPU service (else it owns its pool,
/// arena, notifier and a private service, and runs each slot synchronously).
ul_harness* ul_create(int                                     device,
                      int                                     variant,
                      unsigned                                P,
                      unsigned                                grid_prb,
                      unsigned                                max_iter,
                      ul_sector*                              sector       = nullptr,
                      std::shared_ptr<gpu::pusch_gpu_service> service      = nullptr,
                      bool                                    asynchronous = false,
                      int                                     multi        = 0)
{
  const auto td = variant >= 2 ? port_channel_estimator_td_interpolation_strategy::interpolate
                               : port_channel_estimator_td_interpolation_strategy::average;
  variant %= 2;
  auto* h     = new ul_harness();
  h->P        = P;
  h->grid_prb = grid_prb;
  h->nsc      = 12 * grid_prb;
  if (sector != nullptr) {
    h->pool     = sector->pool.get();
    h->notifier = &sector->notifier;
  } else {
    h->own_pool = ul_pool();
    h->pool     = h->own_pool.get();
  }

  if (variant == 0) {
    uplink_processor_impl::task_executor_collection execs{
        test_executor(), test_executor(), test_executor(), test_executor()};
    h->proc = std::make_unique<uplink_processor_impl>(std::make_unique<stub_prach>(),
                                                      new_pusch_processor(device, 0, td, max_iter, true, {}),
                                                      std::make_unique<stub_pucch>(),
                                                      std::make_unique<stub_srs>(),
                                                      std::make_unique<resource_grid_impl>(P, 14, h->nsc),
                                                      execs,
                                                      h->pool->get_pool(),
                                                      *h->notifier,
                                                      grid_prb,
                                                      4);
    return h;
  }
  // Row b8: the GPU uplink processor only through the uplink_processor_factory interface, as upper_phy_factories.cpp
  // would obtain it (create_ul_processor_pool -> factory.create(config)).
  h->factory = ul_factory(device, td, max_iter, service, asynchronous, multi);
  uplink_processor_config uc{*h->notifier, h->pool->get_pool(), P, grid_prb, 4};
  h->proc = h->factory->create(uc);
  return h;
}

/// PDSCH through the reference's downlink processor: the grid it sends.
class grid_capture : public upper_phy_rg_gateway
{
public:
  void send(const resource_grid_context& context, shared_resource_grid grid) override
  {
    if (forward) {
      forward(context, std::move(grid));  // du_low: on to the sector's lower-PHY PDxCH processor
      sent = true;
      return;
    }
    if (out != nullptr) {
      store_grid(grid.get(), out, P, nsc);
    }
    sent = true;
  }
  std::function<void(const resource_grid_context&, shared_resource_grid)> forward;
  uint16_t* out  = nullptr;
  unsigned  P    = 0;
  unsigned  nsc  = 0;
  bool      sent = false;
};

class one_grid_pool : public shared_resource_grid::pool_interface
{
public:
  one_grid_pool(unsigned P, unsigned nsc) : grid(P, 14, nsc) {}
  resource_grid& get(unsigned) override { return grid; }
  void           notify_release_scope(unsigned) override {}
  shared_resource_grid grab()
  {
    count = 1;
    return shared_resource_grid(*this, count, 0);
  }
  resource_grid_impl    grid;
  std::atomic<unsigned> count{0};
};

struct dl_harness {
  unsigned                                  P, nsc;
  grid_capture                              gateway;
  std::unique_ptr<one_grid_pool>            pool;
  std::shared_ptr<downlink_processor_factory> factory;  ///< GPU variant: the factory that made `proc` (row b8)
  std::unique_ptr<downlink_processor_base>  proc;
};

/// The GPU downlink processor factory of the tests (row b8).
std::shared_ptr<downlink_processor_factory> dl_factory(int device, bool multi = false)
{
  downlink_processor_factory_gpu_configuration fc;
  fc.device             = device;
  if (multi) {
    fc.devices = {device, device, device};  // three PDSCH shards on one GPU (the gather through peer reads)
  }
  fc.pdcch_factory      = std::make_shared<stub_pdcch_factory>();
  fc.pdsch_factory      = create_pdsch_processor_factory_gpu(device, std::make_shared<gpu_pdsch_encoder_factory>(device),
                                                        std::make_shared<ptrs_factory_ref>());
  fc.ssb_factory        = std::make_shared<stub_ssb_factory>();
  fc.nzp_csi_rs_factory = std::make_shared<stub_csi_rs_factory>();
  fc.prs_factory        = std::make_shared<stub_prs_factory>();
  fc.ptrs_factory       = std::make_shared<ptrs_factory_ref>();
  return create_downlink_processor_factory_gpu(fc);
}

dl_harness* dl_create(int device, int variant, unsigned P, unsigned grid_prb)
{
  auto* h = new dl_harness();
  h->P    = P;
  h->nsc  = 12 * grid_prb;
  h->pool = std::make_unique<one_grid_pool>(P, h->nsc);
  if (variant == 0) {
    h->proc = std::make_unique<downlink_processor_single_executor_impl>(h->gateway,
                                                                        std::make_unique<stub_pdcch>(),
                                                                        new_pdsch_processor(device, 0),
                                                                        std::make_unique<stub_ssb>(),
                                                                        std::make_unique<stub_csi_rs>(),
                                                                        std::make_unique<stub_prs>(),
                                                                        test_executor(),
                                                                        srslog::fetch_basic_logger("PHY", true));
    return h;
  }
  // Row b8: the GPU downlink processor only through the downlink_processor_factory interface; the PDSCHs the slot
  // batch does not cover go to the GPU per-PDU PDSCH processor factory (HAL encoder, GPU modulator and DM-RS).
  h->factory = dl_factory(device, (variant & 8) != 0);
  downlink_processor_config dc;
  dc.id       = 0;
  dc.gateway  = &h->gateway;
  dc.executor = &test_executor();
  h->proc     = h->factory->create(dc);
  return h;
}

} // namespace

extern "C" {

void* chain_ul_create(int device, int variant, unsigned nof_ports, unsigned grid_prb, unsigned max_iter)
{
  void* h = nullptr;
  guarded("chain_ul_create", [&] {
    // variant bit 2: the batch completes asynchronously (results from the service's completion thread).
    // variant bits 3 / 4: multi-GPU batch over {device} x 3 with peer copies / over {device} with RCCL.
    h = ul_create(device, variant & 3, nof_ports, grid_prb, max_iter, nullptr, nullptr, (variant & 4) != 0,
                  (variant & 8) != 0 ? 1 : ((variant & 16) != 0 ? 2 : 0));
    return 0;
  });
  return h;
}

void chain_ul_destroy(void* p)
{
  delete static_cast<ul_harness*>(p);
}

/// Process-wide grid transfer counts of the UL batches (gpu::get_pusch_multi_transfer_counters): out[0] host-to-device
/// grid uploads of multi-device batches, out[1] root-to-shard copy launches, out[2] bytes those copies moved, out[3]
/// single-device slots whose grid the lower PHY had written into its HBM twin.
void chain_multi_transfer_counters(uint64_t* out)
{
  const gpu::pusch_multi_transfer_counters c = gpu::get_pusch_multi_transfer_counters();
  out[0]                                     = c.host_uploads;
  out[1]                                     = c.shard_copies;
  out[2]                                     = c.shard_bytes;
  out[3]                                     = c.twin_grids;
}

/// Process-wide grid transfer counts of the PDSCH slot batches (gpu::get_pdsch_multi_transfer_counters): out[0]
/// device-to-host grid downloads, out[1] shard-to-root merges, out[2] bytes those merges moved, out[3] slots whose
/// PDSCH REs stayed in the grid's HBM twin for the GPU PDxCH.
void chain_pdsch_transfer_counters(uint64_t* out)
{
  const gpu::pdsch_multi_transfer_counters c = gpu::get_pdsch_multi_transfer_counters();
  out[0]                                     = c.grid_downloads;
  out[1]                                     = c.shard_merges;
  out[2]                                     = c.merge_bytes;
  out[3]                                     = c.twin_grids;
}

/// One UL slot: the PUSCH PDUs (tb_bytes[i] each) registered in the reference's PDU repository, the received grid
/// (nof_ports, 14, 12 grid_prb) bf16 pairs written into the processor's grid, then handle_rx_symbol(13). Results in
/// notification order: ints [rnti, harq, crc_ok, nof_cbs, ldpc_obs, ldpc_min, ldpc_max, harq_ack_status (-1: none),
/// harq_ack_bits, csi1 status / size / bits, csi2 status / size / bits], floats [ldpc_mean, sinr, evm, ta, cfo, epre, rsrp], payload bytes at tb_out + i * tb_stride.
/// Returns the number of results (< 0 on error).
int chain_ul_slot(void*               p,
                  unsigned            slot,
                  int                 nof_pdus,
                  const chain_params* pdus,
                  const int*          tb_bytes,
                  const uint16_t*     grid_in,
                  int*                out_i,
                  float*              out_f,
                  uint8_t*            tb_out,
                  int                 tb_stride)
{
  return guarded("chain_ul_slot", [&] {
    auto*            h  = static_cast<ul_harness*>(p);
    const slot_point sp(subcarrier_spacing::kHz30, slot);
    h->notifier->reset();
    unique_uplink_pdu_slot_repository repo = h->proc->get_pdu_slot_repository(sp);
    // An asynchronous batch releases the previous slot's grid right after its last notification.
    for (int tries = 0; !repo.is_valid() && tries != 100000; ++tries) {
      std::this_thread::sleep_for(std::chrono::microseconds(10));
      repo = h->proc->get_pdu_slot_repository(sp);
    }
    if (!repo.is_valid()) {
      return -2;
    }
    for (int i = 0; i != nof_pdus; ++i) {
      chain_params c = pdus[i];
      c.slot         = static_cast<int>(slot);
      uplink_pdu_slot_repository::pusch_pdu pdu{static_cast<unsigned>(c.harq_id),
                                                units::bytes(static_cast<unsigned>(tb_bytes[i])),
                                                make_pusch_pdu(c)};
      repo->add_pusch_pdu(pdu);
    }
    shared_resource_grid grid = repo.release();
    load_grid(grid.get(), grid_in, h->P, h->nsc);
    grid.release();
    h->proc->get_slot_processor(sp).handle_rx_symbol(13);
    h->notifier->wait_for(static_cast<unsigned>(nof_pdus));  // asynchronous batches notify from the service
    std::lock_guard<std::mutex> lock(h->notifier->mtx);
    const auto&                 recs = h->notifier->records;
    for (size_t i = 0; i != recs.size(); ++i) {
      const ul_record& r = recs[i];
      int*             oi = out_i + 15 * i;
      float*           of = out_f + 7 * i;
      oi[0] = r.rnti, oi[1] = r.harq_id, oi[2] = r.crc_ok, oi[3] = r.nof_cbs, oi[4] = r.ldpc_obs, oi[5] = r.ldpc_min;
      oi[6] = r.ldpc_max;
      auto ack = h->notifier->harq_ack.find(r.rnti);
      oi[7]    = ack != h->notifier->harq_ack.end() ? ack->second.first : -1;
      oi[8]    = ack != h->notifier->harq_ack.end() ? ack->second.second : 0;
      auto csi = h->notifier->csi.find(r.rnti);
      for (int k = 0; k != 6; ++k) {
        oi[9 + k] = csi == h->notifier->csi.end() ? (k % 3 == 0 ? -1 : 0)
                                                   : (k < 3 ? csi->second.first[k] : csi->second.second[k - 3]);
      }
      of[0] = r.ldpc_mean, of[1] = r.sinr, of[2] = r.evm, of[3] = r.ta, of[4] = r.cfo, of[5] = r.epre, of[6] = r.rsrp;
      std::memcpy(tb_out + i * tb_stride, r.payload.data(), std::min<size_t>(r.payload.size(), tb_stride));
    }
    return static_cast<int>(recs.size());
  });
}

/// Row b8: the PDU validators the GPU factories return (create_pdu_validator), against the reference's own PUSCH / PDSCH
/// validators (pusch_processor_validator_impl with the upper PHY's channel-estimate dimensions,
/// pdsch_processor_validator_impl). direction 0: PUSCH PDUs through the uplink factory's validator, 1: PDSCH PDUs (with
/// `weights`, nof_ports x nof_layers complex per PDU) through the downlink factory's. out[i]: bit 0 the factory's
/// validator accepts PDU i, bit 1 the reference's does, bit 2 their messages differ. Returns 0.
int chain_factory_validate(int device, int direction, int nof_pdus, const chain_params* pdus, const float* weights,
                           int* out)
{
  return guarded("chain_factory_validate", [&] {
    if (direction == 0) {
      std::unique_ptr<uplink_pdu_validator> v =
          ul_factory(device, port_channel_estimator_td_interpolation_strategy::average, 6, nullptr, false, 0)
              ->create_pdu_validator();
      pusch_processor_validator_impl ref(channel_estimate::channel_estimate_dimensions{MAX_RB, MAX_NSYMB_PER_SLOT, 4, 4});
      for (int i = 0; i != nof_pdus; ++i) {
        const pusch_processor::pdu_t pdu = make_pusch_pdu(pdus[i]);
        const auto                   a   = v->is_valid(pdu);
        const auto                   b   = ref.is_valid(pdu);
        out[i] = (a.has_value() ? 1 : 0) | (b.has_value() ? 2 : 0) |
                 (!a.has_value() && !b.has_value() && a.error() != b.error() ? 4 : 0);
      }
    } else {
      std::unique_ptr<downlink_pdu_validator> v = dl_factory(device)->create_pdu_validator();
      pdsch_processor_validator_impl          ref;
      const float*                            w = weights;
      for (int i = 0; i != nof_pdus; ++i) {
        const pdsch_processor::pdu_t pdu = make_pdsch_pdu(pdus[i], w);
        w += 2 * pdus[i].nof_ports * pdus[i].nof_layers;
        const auto a = v->is_valid(pdu);
        const auto b = ref.is_valid(pdu);
        out[i] = (a.has_value() ? 1 : 0) | (b.has_value() ? 2 : 0) |
                 (!a.has_value() && !b.has_value() && a.error() != b.error() ? 4 : 0);
      }
    }
    return 0;
  });
}

void* chain_dl_create(int device, int variant, unsigned nof_ports, unsigned grid_prb)
{
  void* h = nullptr;
  guarded("chain_dl_create", [&] {
    h = dl_create(device, variant, nof_ports, grid_prb);
    return 0;
  });
  return h;
}

void chain_dl_destroy(void* p)
{
  delete static_cast<dl_harness*>(p);
}

/// One DL slot: the grid is loaded with grid_inout (the content of other channels, kept where no PDSCH maps), the
/// reference's downlink processor configured with it, every PDSCH PDU processed (weights: nof_ports x nof_layers complex
/// per PDU, consecutive; TBs consecutive, tb_bytes[i] each), finish_processing_pdus; grid_inout receives the grid the
/// processor sent. Returns 0 when the grid was sent.
int chain_dl_slot(void*               p,
                  unsigned            slot,
                  int                 nof_pdus,
                  const chain_params* pdus,
                  const float*        weights,
                  const uint8_t*      tbs,
                  const int*          tb_bytes,
                  uint16_t*           grid_inout)
{
  return guarded("chain_dl_slot", [&] {
    auto* h = static_cast<dl_harness*>(p);
    load_grid(h->pool->grid, grid_inout, h->P, h->nsc);
    h->gateway.out  = grid_inout;
    h->gateway.P    = h->P;
    h->gateway.nsc  = h->nsc;
    h->gateway.sent = false;
    const slot_point          sp(subcarrier_spacing::kHz30, slot);
    unique_downlink_processor dl = h->proc->get_controller().configure_resource_grid({sp, 0}, h->pool->grab());
    if (!dl.is_valid()) {
      return -2;
    }
    const uint8_t* tb = tbs;
    const float*   w  = weights;
    for (int i = 0; i != nof_pdus; ++i) {
      chain_params c = pdus[i];
      c.slot         = static_cast<int>(slot);
      static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data;
      data.emplace_back(span<const uint8_t>(tb, static_cast<size_t>(tb_bytes[i])));
      dl->process_pdsch(std::move(data), make_pdsch_pdu(c, w));
      tb += tb_bytes[i];
      w += 2 * c.nof_ports * c.nof_layers;
    }
    dl.release();
    return h->gateway.sent ? 0 : -3;
  });
}


/// p50 / p90 / p99 / max / mean (us) of latencies (ns) and the fraction above budget_us; out[6] = samples.
void latency_summary(std::vector<int64_t> v, double budget_us, double* out)
{
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  auto         q = [&](double f) { return n ? static_cast<double>(v[std::min(n - 1, static_cast<size_t>(f * n))]) * 1e-3 : 0.0; };
  double       sum = 0, over = 0;
  for (int64_t x : v) {
    sum += static_cast<double>(x) * 1e-3;
    over += static_cast<double>(x) * 1e-3 > budget_us ? 1 : 0;
  }
  out[0] = q(0.5);
  out[1] = q(0.9);
  out[2] = q(0.99);
  out[3] = n ? static_cast<double>(v.back()) * 1e-3 : 0.0;
  out[4] = n ? sum / static_cast<double>(n) : 0.0;
  out[5] = n ? over / static_cast<double>(n) : 0.0;
  out[6] = static_cast<double>(n);
}

/// Slot-processor throughput (the reference's pusch_processor_benchmark / pdsch_processor_benchmark "throughput total"
/// scheme, at the granularity du_low drives: one uplink / downlink processor per thread, each running slots of
/// `nof_pdus` PDUs through the reference's uplink_processor_impl / downlink_processor_single_executor_impl, variant 0 =
/// reference CPU processors, 1 = GPU slot batches). seconds[r] = wall time of repetition r, in which every thread runs
/// `slots` slots. Returns the number of TB CRC passes of the last repetition (UL) or 0 (DL).
int chain_ul_bench(int                 device,
                   int                 variant,
                   unsigned            nof_threads,
                   unsigned            slots,
                   unsigned            repetitions,
                   int                 nof_pdus,
                   const chain_params* pdus,
                   const int*          tb_bytes,
                   const uint16_t*     grid_in,
                   unsigned            nof_ports,
                   unsigned            grid_prb,
                   double*             seconds,
                   double              pace_us,
                   double*             latency)
{
  return guarded("chain_ul_bench", [&] {
    // pace_us > 0: every thread (sector) submits its slot i at t0 + i pace_us - a radio's slot clock, the sectors
    // aligned - and each PUSCH data notification's latency from its slot's submission (handle_rx_symbol of the last
    // symbol) is recorded; latency[0..6] = latency_summary over all sectors (budget: du_low's max_processing_delay_slots
    // = 5 slots of pace_us, du_low_config.h:39), latency[7] = the largest lag of a submission behind its instant (us).
    // variant 0: reference CPU processors; 1: GPU slot batches, one synchronous uplink processor per thread (sector)
    // with a private GPU service; 2: du_low's structure on one shared GPU service - each sector (thread) a ring of
    // UL_RING uplink processors over one rx buffer pool and HARQ arena, slots completing asynchronously, the service
    // gathering the sectors' slots of one slot number into one launch.
    constexpr unsigned UL_RING = 4;
    const bool         shared  = variant == 2;
    std::vector<std::unique_ptr<bench_worker>> workers;
    std::vector<std::unique_ptr<ul_sector>>    sectors(nof_threads);
    std::vector<std::vector<ul_harness*>>      hs(nof_threads);
    std::shared_ptr<gpu::pusch_gpu_service>    service;
    if (shared) {
      gpu::pusch_service_configuration sc;
      sc.device                    = device;
      sc.nof_launch_sets           = 3;
      sc.max_slots_per_launch      = nof_threads;
      sc.expected_slots_per_launch = nof_threads;
      sc.gather_window_us          = 1000;
      sc.max_grids                 = nof_threads * UL_RING;
      service                      = gpu::create_pusch_gpu_service(sc);
    }
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers.push_back(std::make_unique<bench_worker>());
    }
    // Each worker builds its processors on its own thread (thread-local dependency pools bind there).
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers[t]->post([&, t] {
        if (shared) {
          sectors[t]                      = std::make_unique<ul_sector>();
          sectors[t]->pool                = ul_pool();
          sectors[t]->notifier.count_only = true;
          for (unsigned r = 0; r != UL_RING; ++r) {
            hs[t].push_back(ul_create(device, 1, nof_ports, grid_prb, 2, sectors[t].get(), service, true));
          }
        } else {
          // One synchronous uplink processor per thread on a private service (the per-thread batch of round 4).
          std::shared_ptr<gpu::pusch_gpu_service> own;
          if (variant == 1) {
            gpu::pusch_service_configuration sc;
            sc.device          = device;
            sc.nof_launch_sets = 2;
            sc.max_grids       = 4;
            own                = gpu::create_pusch_gpu_service(sc);
          }
          hs[t].push_back(ul_create(device, variant, nof_ports, grid_prb, 2, nullptr, own));
          hs[t].back()->notifier->count_only = true;
        }
      });
      workers[t]->wait();  // one at a time: the factories' first-use initialisation is not ours to race
    }
    const unsigned         nsc = 12 * grid_prb;
    std::vector<unsigned>  slot_no(nof_threads, 0);
    std::vector<unsigned>  submitted(nof_threads, 0);
    auto                   notifier_of = [&](unsigned t) -> ul_results_recorder& {
      return shared ? sectors[t]->notifier : *hs[t].front()->notifier;
    };
    using bclock = std::chrono::steady_clock;
    bclock::time_point  pace_t0;
    const bool          paced = pace_us > 0;
    std::vector<double> max_lag(nof_threads, 0.0);
    auto run_slots = [&](unsigned t, unsigned n, bool timed) {
      if (timed && paced) {
        (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
      }
      for (unsigned i = 0; i != n; ++i) {
        const unsigned   s  = slot_no[t]++;
        const slot_point sp(subcarrier_spacing::kHz30, s % 20480);
        ul_harness*      h  = hs[t][s % hs[t].size()];
        if (timed && paced) {
          const auto due = pace_t0 + std::chrono::nanoseconds(static_cast<int64_t>(pace_us * 1e3 * i));
          const auto now = bclock::now();
          if (now < due) {
            std::this_thread::sleep_until(due);
          } else {
            max_lag[t] = std::max(max_lag[t], std::chrono::duration<double, std::micro>(now - due).count());
          }
        }
        unique_uplink_pdu_slot_repository repo = h->proc->get_pdu_slot_repository(sp);
        while (!repo.is_valid()) {
          // The ring's processor still holds an earlier slot (its PUSCH results are not all notified yet).
          std::this_thread::yield();
          repo = h->proc->get_pdu_slot_repository(sp);
        }
        for (int k = 0; k != nof_pdus; ++k) {
          chain_params c = pdus[k];
          c.slot         = static_cast<int>(sp.slot_index());
          // A UE's HARQ process per slot in flight (du_low's UEs cycle their 16 processes).
          c.harq_id = (c.harq_id + static_cast<int>(s)) % 16;
          repo->add_pusch_pdu({static_cast<unsigned>(c.harq_id), units::bytes(static_cast<unsigned>(tb_bytes[k])),
                               make_pusch_pdu(c)});
        }
        shared_resource_grid g = repo.release();
        for (unsigned p = 0; p != nof_ports; ++p) {
          for (unsigned l = 0; l != 14; ++l) {
            std::memcpy(g.get().get_writer().get_view(p, l).data(),
                        grid_in + 2 * (static_cast<size_t>(p) * 14 + l) * nsc, nsc * sizeof(cbf16_t));
          }
        }
        g.release();
        if (notifier_of(t).track_latency) {
          notifier_of(t).set_slot_reference(sp, bclock::now());
        }
        h->proc->get_slot_processor(sp).handle_rx_symbol(13);
        submitted[t] += static_cast<unsigned>(nof_pdus);
      }
      notifier_of(t).wait_for(submitted[t]);  // every result of this thread's slots notified
    };
    // Warm-up over one frame (20 slots at 30 kHz): every slot number's DM-RS plans, pools, first touch - a DU runs
    // continuously, and the GPU batches cache their slot-dependent plans per slot number.
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers[t]->post([&, t] { run_slots(t, 20, false); });
    }
    for (auto& w : workers) {
      w->wait();
    }
    for (unsigned t = 0; t != nof_threads; ++t) {
      notifier_of(t).track(latency != nullptr);
    }
    int                  ok = 0;
    std::vector<int64_t> lat;
    for (unsigned r = 0; r != repetitions; ++r) {
      for (unsigned t = 0; t != nof_threads; ++t) {
        notifier_of(t).reset();
        submitted[t] = 0;
      }
      const auto t0 = std::chrono::steady_clock::now();
      pace_t0       = t0 + std::chrono::milliseconds(2);
      for (unsigned t = 0; t != nof_threads; ++t) {
        workers[t]->post([&, t] { run_slots(t, slots, true); });
      }
      for (auto& w : workers) {
        w->wait();
      }
      seconds[r] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      ok         = 0;
      for (unsigned t = 0; t != nof_threads; ++t) {
        ok += static_cast<int>(notifier_of(t).crc_ok.load());
        std::lock_guard<std::mutex> lock(notifier_of(t).mtx);
        lat.insert(lat.end(), notifier_of(t).latency_ns.begin(), notifier_of(t).latency_ns.end());
      }
    }
    if (latency != nullptr) {
      latency_summary(lat, 5.0 * (paced ? pace_us : 500.0), latency);
      latency[7] = *std::max_element(max_lag.begin(), max_lag.end());
    }
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers[t]->post([&, t] {
        for (ul_harness* h : hs[t]) {
          delete h;
        }
        sectors[t].reset();
      });
      workers[t]->wait();
    }
    service.reset();
    return ok;
  });
}

int chain_dl_bench(int                 device,
                   int                 variant,
                   unsigned            nof_threads,
                   unsigned            slots,
                   unsigned            repetitions,
                   int                 nof_pdus,
                   const chain_params* pdus,
                   const float*        weights,
                   const uint8_t*      tbs,
                   const int*          tb_bytes,
                   unsigned            nof_ports,
                   unsigned            grid_prb,
                   double*             seconds)
{
  return guarded("chain_dl_bench", [&] {
    std::vector<std::unique_ptr<bench_worker>> workers;
    std::vector<dl_harness*>                   hs(nof_threads, nullptr);
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers.push_back(std::make_unique<bench_worker>());
    }
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers[t]->post([&, t] { hs[t] = dl_create(device, variant, nof_ports, grid_prb); });
      workers[t]->wait();  // one at a time: the factories' first-use initialisation is not ours to race
    }
    for (auto& w : workers) {
      w->wait();
    }
    std::vector<unsigned> slot_no(nof_threads, 0);
    auto                  run_slots = [&](unsigned t, unsigned n) {
      dl_harness* h = hs[t];
      h->gateway.out = nullptr;
      for (unsigned i = 0; i != n; ++i) {
        const slot_point          sp(subcarrier_spacing::kHz30, slot_no[t]++ % 20480);
        unique_downlink_processor dl = h->proc->get_controller().configure_resource_grid({sp, 0}, h->pool->grab());
        const uint8_t*            tb = tbs;
        const float*              w  = weights;
        for (int k = 0; k != nof_pdus; ++k) {
          chain_params c = pdus[k];
          c.slot         = static_cast<int>(sp.slot_index());
          static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data;
          data.emplace_back(span<const uint8_t>(tb, static_cast<size_t>(tb_bytes[k])));
          dl->process_pdsch(std::move(data), make_pdsch_pdu(c, w));
          tb += tb_bytes[k];
          w += 2 * c.nof_ports * c.nof_layers;
        }
        dl.release();
      }
    };
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers[t]->post([&, t] { run_slots(t, 20); });  // one frame, as the UL bench
    }
    for (auto& w : workers) {
      w->wait();
    }
    for (unsigned r = 0; r != repetitions; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned t = 0; t != nof_threads; ++t) {
        workers[t]->post([&, t] { run_slots(t, slots); });
      }
      for (auto& w : workers) {
        w->wait();
      }
      seconds[r] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    for (unsigned t = 0; t != nof_threads; ++t) {
      workers[t]->post([&, t] { delete hs[t]; });
      workers[t]->wait();
    }
    return 0;
  });
}


/// du_low's UL on one GPU, paced at the radio's symbol rate (TEST INFRASTRUCTURE, tools/du_low_bench.py): every sector
/// a thread that, per slot, takes the grid of one of its ring of 4 uplink processors (the GPU slot batches on one shared
/// PUSCH service, as chain_ul_bench variant 2) with that slot's PUSCH PDUs, hands it to the sector's lower-PHY PUxCH
/// processor (handle_request) and delivers the slot's 14 symbols of samples (process_symbol) one symbol duration apart;
/// the PUxCH notifier's last symbol of the slot starts the uplink processor (handle_rx_symbol(13)), as the radio unit's
/// rx-symbol handler does in du_low. grouped: the sectors' PUxCH processors come from one lower_phy_sector_group (else
/// one GPU PUxCH processor each). samples: complex float, the two slots of a subframe, per symbol all ports (P x
/// (CP + N)) consecutively. Outputs per sector k: lag[4k..4k+3] = largest lag behind the pace (s), lag at the last
/// symbol (s), fraction of symbols more than a slot late, late PUxCH requests; results[2k], [2k+1] = PUSCH data results
/// and TB CRC passes. seconds: wall time. Returns 0 (< 0 on error).
int chain_du_low_ul(int                 device,
                    unsigned            nof_sectors,
                    unsigned            slots,
                    int                 nof_pdus,
                    const chain_params* pdus,
                    const int*          tb_bytes,
                    const float*        samples,
                    unsigned            nof_ports,
                    unsigned            grid_prb,
                    unsigned            dft_size,
                    int                 grouped,
                    unsigned            in_flight,
                    double*             lag,
                    int*                results,
                    double*             seconds,
                    double*             latency)
{
  return guarded("chain_du_low_ul", [&] {
    // latency (8 values, may be null): the PUSCH results' latency from the end of their slot on the radio's clock (the
    // instant its last symbol has been received) to the data notification, over every sector: latency_summary with
    // du_low's budget of max_processing_delay_slots = 5 slots (du_low_config.h:39), then the number of samples.
    using clock         = std::chrono::steady_clock;
    constexpr unsigned UL_RING = 4;
    const unsigned     nsc     = 12 * grid_prb;
    const double       srate   = static_cast<double>(dft_size) * 30e3;
    // Symbol sizes (CP + N) of the subframe's 28 symbols and where each symbol's samples start.
    std::vector<unsigned> size(28), start(28);
    size_t                pos = 0;
    for (unsigned s = 0; s != 28; ++s) {
      size[s]  = cyclic_prefix(cyclic_prefix::NORMAL).get_length(s, subcarrier_spacing::kHz30).to_samples(srate) +
                 dft_size;
      start[s] = static_cast<unsigned>(pos);
      pos += static_cast<size_t>(size[s]) * nof_ports;
    }
    gpu::pusch_service_configuration sc;
    sc.device                    = device;
    sc.nof_launch_sets           = 3;
    sc.max_slots_per_launch      = nof_sectors;
    sc.expected_slots_per_launch = nof_sectors;
    sc.gather_window_us          = 300;
    sc.max_grids                 = nof_sectors * UL_RING;
    auto service                 = gpu::create_pusch_gpu_service(sc);
    std::shared_ptr<lower_phy_sector_group> group;
    if (grouped != 0) {
      lower_phy_group_configuration gc;
      gc.device      = device;
      gc.nof_sectors = nof_sectors;
      group          = create_lower_phy_sector_group(gc);
    }

    struct du_ul_notifier : public puxch_processor_notifier {
      std::vector<ul_harness*>* ring = nullptr;
      std::atomic<unsigned>     late{0};
      void on_puxch_request_late(const resource_grid_context& /*c*/) override { ++late; }
      void on_rx_symbol(const shared_resource_grid& /*grid*/, const lower_phy_rx_symbol_context& c) override
      {
        if (c.nof_symbols == 13) {
          (*ring)[c.slot.system_slot() % ring->size()]->proc->get_slot_processor(c.slot).handle_rx_symbol(13);
        }
      }
    };
    struct reader : public baseband_gateway_buffer_reader {
      std::vector<span<const cf_t>> ch;
      unsigned                      get_nof_channels() const override { return ch.size(); }
      unsigned                      get_nof_samples() const override { return ch.empty() ? 0 : ch[0].size(); }
      span<const cf_t>              get_channel_buffer(unsigned i) const override { return ch[i]; }
    };
    struct sector_state {
      std::unique_ptr<ul_sector>       sec;
      std::vector<ul_harness*>         ring;
      du_ul_notifier                   notifier;
      std::unique_ptr<puxch_processor> puxch;
    };
    std::vector<std::unique_ptr<bench_worker>> workers;
    std::vector<std::unique_ptr<sector_state>> st(nof_sectors);
    for (unsigned k = 0; k != nof_sectors; ++k) {
      workers.push_back(std::make_unique<bench_worker>());
    }
    for (unsigned k = 0; k != nof_sectors; ++k) {
      workers[k]->post([&, k] {
        st[k]                           = std::make_unique<sector_state>();
        st[k]->sec                      = std::make_unique<ul_sector>();
        st[k]->sec->pool                = ul_pool();
        st[k]->sec->notifier.count_only = true;
        for (unsigned r = 0; r != UL_RING; ++r) {
          st[k]->ring.push_back(ul_create(device, 1, nof_ports, grid_prb, 2, st[k]->sec.get(), service, true));
        }
        st[k]->notifier.ring = &st[k]->ring;
        puxch_processor_configuration c;
        c.cp                = cyclic_prefix::NORMAL;
        c.scs               = subcarrier_spacing::kHz30;
        c.srate             = sampling_rate::from_Hz(srate);
        c.bandwidth_rb      = grid_prb;
        c.dft_window_offset = 0.5F;
        c.center_freq_Hz    = 3.5e9 + 2e7 * k;
        c.nof_rx_ports      = nof_ports;
        st[k]->puxch        = (group ? create_puxch_processor_factory_gpu(group, in_flight)
                                     : create_puxch_processor_factory_gpu(device, in_flight))
                           ->create(c);
        st[k]->puxch->connect(st[k]->notifier);
      });
      workers[k]->wait();  // one at a time: the factories' first-use initialisation is not ours to race
    }
    const clock::duration period = std::chrono::duration_cast<clock::duration>(std::chrono::nanoseconds(1000000 / 28));
    std::vector<unsigned> slot_no(nof_sectors, 0), submitted(nof_sectors, 0);
    // One sector's slots: paced (period > 0, from `t0`) or free-running; returns (largest lag, last lag, late count).
    auto run = [&](unsigned k, unsigned n, clock::time_point t0, bool paced, double* out) {
      if (paced) {
        (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
      }
      sector_state& s       = *st[k];
      reader        buf;
      double        max_lag = 0, last_lag = 0;
      long          late = 0, i_sym = 0;
      for (unsigned i = 0; i != n; ++i) {
        const unsigned   sl = slot_no[k]++;
        const slot_point sp(subcarrier_spacing::kHz30, sl % 20480);
        ul_harness*      h  = s.ring[sl % UL_RING];
        unique_uplink_pdu_slot_repository repo = h->proc->get_pdu_slot_repository(sp);
        while (!repo.is_valid()) {
          std::this_thread::yield();  // the ring's processor still holds an earlier slot
          repo = h->proc->get_pdu_slot_repository(sp);
        }
        for (int q = 0; q != nof_pdus; ++q) {
          chain_params c = pdus[q];
          c.slot         = static_cast<int>(sp.slot_index());
          c.harq_id      = (c.harq_id + static_cast<int>(sl)) % 16;
          repo->add_pusch_pdu({static_cast<unsigned>(c.harq_id), units::bytes(static_cast<unsigned>(tb_bytes[q])),
                               make_pusch_pdu(c)});
        }
        shared_resource_grid g = repo.release();
        s.puxch->get_request_handler().handle_request(g, {sp, k});
        g.release();
        submitted[k] += static_cast<unsigned>(nof_pdus);
        const unsigned q0 = sp.subframe_slot_index() * 14;
        if (paced && s.sec->notifier.track_latency) {
          s.sec->notifier.set_slot_reference(sp, t0 + period * (i_sym + 14));
        }
        for (unsigned l = 0; l != 14; ++l) {
          if (paced) {
            const clock::time_point due = t0 + period * i_sym++;
            const clock::time_point now = clock::now();
            if (now < due) {
              std::this_thread::sleep_until(due);
              last_lag = 0;
            } else {
              last_lag = std::chrono::duration<double>(now - due).count();
              max_lag  = std::max(max_lag, last_lag);
              late += (now - due) > period * 14 ? 1 : 0;
            }
          }
          buf.ch.clear();
          const unsigned ssz = size[q0 + l];
          for (unsigned p = 0; p != nof_ports; ++p) {
            buf.ch.emplace_back(reinterpret_cast<const cf_t*>(samples) + start[q0 + l] + static_cast<size_t>(p) * ssz,
                                ssz);
          }
          s.puxch->get_baseband().process_symbol(buf, lower_phy_rx_symbol_context{sp, k, l});
        }
      }
      s.sec->notifier.wait_for(submitted[k]);  // every result of the sector's slots notified
      out[0] = max_lag;
      out[1] = last_lag;
      out[2] = static_cast<double>(late) / std::max(1L, i_sym);
    };
    // Warm-up over one frame, free-running (plans per slot number, pools, first touch).
    std::vector<double> tmp(3 * nof_sectors);
    for (unsigned k = 0; k != nof_sectors; ++k) {
      workers[k]->post([&, k] { run(k, 20, clock::now(), false, &tmp[3 * k]); });
    }
    for (auto& w : workers) {
      w->wait();
    }
    for (unsigned k = 0; k != nof_sectors; ++k) {
      st[k]->sec->notifier.reset();
      st[k]->sec->notifier.track(latency != nullptr);
      st[k]->notifier.late = 0;
      submitted[k]         = 0;
    }
    const clock::time_point t0 = clock::now() + std::chrono::milliseconds(2);
    for (unsigned k = 0; k != nof_sectors; ++k) {
      workers[k]->post([&, k] { run(k, slots, t0, true, &tmp[3 * k]); });
    }
    for (auto& w : workers) {
      w->wait();
    }
    *seconds = std::chrono::duration<double>(clock::now() - t0).count();
    for (unsigned k = 0; k != nof_sectors; ++k) {
      lag[4 * k]         = tmp[3 * k];
      lag[4 * k + 1]     = tmp[3 * k + 1];
      lag[4 * k + 2]     = tmp[3 * k + 2];
      lag[4 * k + 3]     = st[k]->notifier.late.load();
      results[2 * k]     = static_cast<int>(st[k]->sec->notifier.nof_data.load());
      results[2 * k + 1] = static_cast<int>(st[k]->sec->notifier.crc_ok.load());
    }
    if (latency != nullptr) {
      std::vector<int64_t> all;
      for (unsigned k = 0; k != nof_sectors; ++k) {
        std::lock_guard<std::mutex> lock(st[k]->sec->notifier.mtx);
        all.insert(all.end(), st[k]->sec->notifier.latency_ns.begin(), st[k]->sec->notifier.latency_ns.end());
      }
      latency_summary(all, 5 * 500.0, latency);
      latency[7] = 0;
    }
    for (unsigned k = 0; k != nof_sectors; ++k) {
      workers[k]->post([&, k] {
        st[k]->puxch.reset();
        for (ul_harness* h : st[k]->ring) {
          delete h;
        }
        st[k].reset();
      });
      workers[k]->wait();
    }
    group.reset();
    service.reset();
    return 0;
  });
}

/// du_low's downlink on one GPU at the radio's pace (TEST INFRASTRUCTURE, tools/du_low_bench.py --direction dl):
/// every sector has an upper-PHY thread running its downlink processor (the GPU PDSCH slot batch) and a radio thread
/// that, at the start of slot s, asks the upper thread for slot s + 2 and then takes the 14 symbols of slot s from the
/// sector's lower-PHY PDxCH processor (process_symbol), one symbol duration apart; the downlink processor's grid goes
/// to the PDxCH processor (handle_request) through the upper-PHY gateway, as in du_low. grouped: the PDxCH processors
/// come from one lower_phy_sector_group. PDUs / weights / TBs as chain_dl_bench. Outputs per sector k: lag[4k..4k+3]
/// as chain_du_low_ul (the last entry: late PDxCH requests); results[2k], [2k+1] = symbols that carried a slot's
/// samples, DL slots the upper thread finished. Returns 0 (< 0 on error).
int chain_du_low_dl(int                 device,
                    unsigned            nof_sectors,
                    unsigned            slots,
                    int                 nof_pdus,
                    const chain_params* pdus,
                    const float*        weights,
                    const uint8_t*      tbs,
                    const int*          tb_bytes,
                    unsigned            nof_ports,
                    unsigned            grid_prb,
                    unsigned            dft_size,
                    int                 grouped,
                    double*             lag,
                    int*                results,
                    double*             seconds)
{
  return guarded("chain_du_low_dl", [&] {
    using clock     = std::chrono::steady_clock;
    const double srate = static_cast<double>(dft_size) * 30e3;
    std::vector<unsigned> size(28);
    for (unsigned s = 0; s != 28; ++s) {
      size[s] = cyclic_prefix(cyclic_prefix::NORMAL).get_length(s, subcarrier_spacing::kHz30).to_samples(srate) +
                dft_size;
    }
    std::shared_ptr<lower_phy_sector_group> group;
    if (grouped != 0) {
      lower_phy_group_configuration gc;
      gc.device      = device;
      gc.nof_sectors = nof_sectors;
      group          = create_lower_phy_sector_group(gc);
    }
    struct du_dl_notifier : public pdxch_processor_notifier {
      std::atomic<unsigned> late{0};
      void                  on_pdxch_request_late(const resource_grid_context& /*c*/) override { ++late; }
    };
    struct writer : public baseband_gateway_buffer_writer {
      std::vector<span<cf_t>> ch;
      unsigned                get_nof_channels() const override { return ch.size(); }
      unsigned                get_nof_samples() const override { return ch.empty() ? 0 : ch[0].size(); }
      span<cf_t>              get_channel_buffer(unsigned i) override { return ch[i]; }
    };
    struct sector_state {
      dl_harness*                      dl = nullptr;
      du_dl_notifier                   notifier;
      std::unique_ptr<pdxch_processor> pdxch;
      std::vector<cf_t>                out;  ///< one symbol of every port (a radio's baseband buffer)
      std::atomic<int>                 dl_slots{0};
    };
    std::vector<std::unique_ptr<bench_worker>> radio, upper;
    std::vector<std::unique_ptr<sector_state>> st(nof_sectors);
    for (unsigned k = 0; k != nof_sectors; ++k) {
      radio.push_back(std::make_unique<bench_worker>());
      upper.push_back(std::make_unique<bench_worker>());
    }
    for (unsigned k = 0; k != nof_sectors; ++k) {
      st[k] = std::make_unique<sector_state>();
      upper[k]->post([&, k] { st[k]->dl = dl_create(device, 1, nof_ports, grid_prb); });
      upper[k]->wait();
      radio[k]->post([&, k] {
        pdxch_processor_configuration c;
        c.cp             = cyclic_prefix::NORMAL;
        c.scs            = subcarrier_spacing::kHz30;
        c.srate          = sampling_rate::from_Hz(srate);
        c.bandwidth_rb   = grid_prb;
        c.center_freq_Hz = 3.5e9 + 2e7 * k;
        c.nof_tx_ports   = nof_ports;
        st[k]->pdxch     = (group ? create_pdxch_processor_factory_gpu(group) : create_pdxch_processor_factory_gpu(device))
                           ->create(c);
        st[k]->pdxch->connect(st[k]->notifier);
        st[k]->out.resize(static_cast<size_t>(nof_ports) * (dft_size + dft_size / 8));
      });
      radio[k]->wait();
      pdxch_processor* px = st[k]->pdxch.get();
      st[k]->dl->gateway.forward = [px](const resource_grid_context& c, shared_resource_grid g) {
        px->get_request_handler().handle_request(g, c);
      };
    }
    // The downlink processor of one slot (upper thread).
    auto dl_slot = [&](unsigned k, unsigned sl) {
      dl_harness*               h  = st[k]->dl;
      const slot_point          sp(subcarrier_spacing::kHz30, sl % 20480);
      unique_downlink_processor dl = h->proc->get_controller().configure_resource_grid({sp, k}, h->pool->grab());
      if (!dl.is_valid()) {
        return;
      }
      const uint8_t* tb = tbs;
      const float*   w  = weights;
      for (int q = 0; q != nof_pdus; ++q) {
        chain_params c = pdus[q];
        c.slot         = static_cast<int>(sp.slot_index());
        static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data;
        data.emplace_back(span<const uint8_t>(tb, static_cast<size_t>(tb_bytes[q])));
        dl->process_pdsch(std::move(data), make_pdsch_pdu(c, w));
        tb += tb_bytes[q];
        w += 2 * c.nof_ports * c.nof_layers;
      }
      dl.release();
      ++st[k]->dl_slots;
    };
    const clock::duration period = std::chrono::duration_cast<clock::duration>(std::chrono::nanoseconds(1000000 / 28));
    std::vector<unsigned> slot_no(nof_sectors, 0);
    std::vector<double>   tmp(4 * nof_sectors, 0.0);
    auto run = [&](unsigned k, unsigned n, clock::time_point t0, bool paced) {
      if (paced) {
        (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
      }
      sector_state& s = *st[k];
      writer        buf;
      double        max_lag = 0, last_lag = 0;
      long          late = 0, i_sym = 0, with_data = 0;
      for (unsigned i = 0; i != n; ++i) {
        const unsigned   sl = slot_no[k]++;
        const slot_point sp(subcarrier_spacing::kHz30, sl % 20480);
        upper[k]->wait();  // the slot before's DL job has finished (it had a whole slot)
        upper[k]->post([&, k, sl] { dl_slot(k, sl + 2); });
        const unsigned q0 = sp.subframe_slot_index() * 14;
        for (unsigned l = 0; l != 14; ++l) {
          if (paced) {
            const clock::time_point due = t0 + period * i_sym++;
            const clock::time_point now = clock::now();
            if (now < due) {
              std::this_thread::sleep_until(due);
              last_lag = 0;
            } else {
              last_lag = std::chrono::duration<double>(now - due).count();
              max_lag  = std::max(max_lag, last_lag);
              late += (now - due) > period * 14 ? 1 : 0;
            }
          }
          const unsigned ssz = size[q0 + l];
          buf.ch.clear();
          for (unsigned p = 0; p != nof_ports; ++p) {
            buf.ch.emplace_back(s.out.data() + static_cast<size_t>(p) * (dft_size + dft_size / 8), ssz);
          }
          with_data += s.pdxch->get_baseband().process_symbol(buf, {sp, k, l}) ? 1 : 0;
        }
      }
      upper[k]->wait();
      tmp[4 * k]     = max_lag;
      tmp[4 * k + 1] = last_lag;
      tmp[4 * k + 2] = static_cast<double>(late) / std::max(1L, i_sym);
      tmp[4 * k + 3] = static_cast<double>(with_data);
    };
    for (unsigned k = 0; k != nof_sectors; ++k) {
      radio[k]->post([&, k] { run(k, 20, clock::now(), false); });
    }
    for (auto& w : radio) {
      w->wait();
    }
    for (unsigned k = 0; k != nof_sectors; ++k) {
      st[k]->notifier.late = 0;
      st[k]->dl_slots      = 0;
    }
    const clock::time_point t0 = clock::now() + std::chrono::milliseconds(2);
    for (unsigned k = 0; k != nof_sectors; ++k) {
      radio[k]->post([&, k] { run(k, slots, t0, true); });
    }
    for (auto& w : radio) {
      w->wait();
    }
    *seconds = std::chrono::duration<double>(clock::now() - t0).count();
    for (unsigned k = 0; k != nof_sectors; ++k) {
      lag[4 * k]         = tmp[4 * k];
      lag[4 * k + 1]     = tmp[4 * k + 1];
      lag[4 * k + 2]     = tmp[4 * k + 2];
      lag[4 * k + 3]     = st[k]->notifier.late.load();
      results[2 * k]     = static_cast<int>(tmp[4 * k + 3]);
      results[2 * k + 1] = st[k]->dl_slots.load();
    }
    for (unsigned k = 0; k != nof_sectors; ++k) {
      st[k]->dl->gateway.forward = nullptr;
      radio[k]->post([&, k] { st[k]->pdxch.reset(); });
      radio[k]->wait();
      upper[k]->post([&, k] { delete st[k]->dl; });
      upper[k]->wait();
    }
    group.reset();
    return 0;
  });
}

/// One sector's downlink on the calling thread: the GPU downlink processor (PDSCH slot batch, row b8) hands each
/// slot's grid to the GPU PDxCH processor (gateway -> handle_request, as du_low's upper-PHY gateway does), which
/// modulates it; `slots` slots, with the downlink HBM grid twin enabled or not (gpu::dl_grid_twins::set_enabled).
/// Before its PDSCHs every slot's grid gets host-written REs (random, in symbols 0-1 and above PRB 270 as PDCCH /
/// CSI-RS would put them), so the twin's merge of device and host REs is exercised. out: every slot's 14 symbols x
/// nof_ports complex samples in order [slot][symbol][port][sample] (as float pairs); counters: [PDSCH grid downloads,
/// slots through the twin, late PDxCH requests] over the run.
int chain_dl_twin_samples(int                 device,
                          int                 twin,
                          unsigned            slots,
                          int                 nof_pdus,
                          const chain_params* pdus,
                          const float*        weights,
                          const uint8_t*      tbs,
                          const int*          tb_bytes,
                          unsigned            nof_ports,
                          unsigned            grid_prb,
                          unsigned            dft_size,
                          float*              out,
                          uint64_t*           counters)
{
  return guarded("chain_dl_twin_samples", [&] {
    gpu::dl_grid_twins::set_enabled(twin != 0);
    const double                srate = static_cast<double>(dft_size) * 30e3;
    std::unique_ptr<dl_harness> h(dl_create(device, 1, nof_ports, grid_prb));
    struct late_notifier : public pdxch_processor_notifier {
      std::atomic<unsigned> late{0};
      void                  on_pdxch_request_late(const resource_grid_context& /*c*/) override { ++late; }
    } notifier;
    struct writer : public baseband_gateway_buffer_writer {
      std::vector<span<cf_t>> ch;
      unsigned                get_nof_channels() const override { return ch.size(); }
      unsigned                get_nof_samples() const override { return ch.empty() ? 0 : ch[0].size(); }
      span<cf_t>              get_channel_buffer(unsigned i) override { return ch[i]; }
    };
    pdxch_processor_configuration c;
    c.cp                                 = cyclic_prefix::NORMAL;
    c.scs                                = subcarrier_spacing::kHz30;
    c.srate                              = sampling_rate::from_Hz(srate);
    c.bandwidth_rb                       = grid_prb;
    c.center_freq_Hz                     = 3.5e9;
    c.nof_tx_ports                       = nof_ports;
    std::unique_ptr<pdxch_processor> px  = create_pdxch_processor_factory_gpu(device)->create(c);
    px->connect(notifier);
    std::atomic<unsigned> forwarded{0};
    pdxch_processor*      pxp = px.get();
    h->gateway.forward        = [pxp, &forwarded](const resource_grid_context& ctx, shared_resource_grid g) {
      pxp->get_request_handler().handle_request(g, ctx);
      ++forwarded;
    };
    const gpu::pdsch_multi_transfer_counters before = gpu::get_pdsch_multi_transfer_counters();
    std::mt19937                             rng(7);
    std::normal_distribution<float>          nd(0.F, 0.5F);
    const unsigned                           nsc = 12 * grid_prb;
    std::vector<cf_t>                        row(nsc);
    std::vector<cf_t>                        buf(static_cast<size_t>(nof_ports) * (dft_size + dft_size / 8));
    size_t                                   o = 0;
    for (unsigned i = 0; i != slots; ++i) {
      const slot_point          sp(subcarrier_spacing::kHz30, i);
      unique_downlink_processor dl = h->proc->get_controller().configure_resource_grid({sp, 0}, h->pool->grab());
      if (!dl.is_valid()) {
        throw std::runtime_error("downlink processor not available");
      }
      resource_grid& g = h->pool->grid;
      g.set_all_zero();
      for (unsigned p = 0; p != nof_ports; ++p) {
        for (unsigned l = 0; l != 14; ++l) {
          const unsigned k0 = l < 2 ? 0 : std::min(nsc, 270U * 12);
          for (unsigned k = k0; k < nsc; ++k) {
            row[k] = cf_t(nd(rng), nd(rng));
          }
          if (k0 < nsc) {
            g.get_writer().put(p, l, k0, span<const cf_t>(row.data() + k0, nsc - k0));
          }
        }
      }
      const uint8_t* tb = tbs;
      const float*   w  = weights;
      for (int q = 0; q != nof_pdus; ++q) {
        chain_params cq = pdus[q];
        cq.slot         = static_cast<int>(sp.slot_index());
        static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data;
        data.emplace_back(span<const uint8_t>(tb, static_cast<size_t>(tb_bytes[q])));
        dl->process_pdsch(std::move(data), make_pdsch_pdu(cq, w));
        tb += tb_bytes[q];
        w += 2 * cq.nof_ports * cq.nof_layers;
      }
      dl.release();
      for (int t = 0; forwarded.load() != i + 1; ++t) {  // the grid reaches the PDxCH (inline executor: at once)
        if (t == 5000) {
          throw std::runtime_error("the grid of a slot never reached the PDxCH processor");
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      for (unsigned l = 0; l != 14; ++l) {
        const unsigned n = cyclic_prefix(cyclic_prefix::NORMAL)
                               .get_length(sp.subframe_slot_index() * 14 + l, subcarrier_spacing::kHz30)
                               .to_samples(srate) +
                           dft_size;
        writer wb;
        for (unsigned p = 0; p != nof_ports; ++p) {
          wb.ch.emplace_back(buf.data() + static_cast<size_t>(p) * (dft_size + dft_size / 8), n);
        }
        const bool any = pxp->get_baseband().process_symbol(wb, {sp, 0, l});
        for (unsigned p = 0; p != nof_ports; ++p) {
          for (unsigned k = 0; k != n; ++k) {
            const cf_t v = any ? wb.ch[p][k] : cf_t();
            out[o++]     = v.real();
            out[o++]     = v.imag();
          }
        }
      }
    }
    const gpu::pdsch_multi_transfer_counters after = gpu::get_pdsch_multi_transfer_counters();
    counters[0]                                    = after.grid_downloads - before.grid_downloads;
    counters[1]                                    = after.twin_grids - before.twin_grids;
    counters[2]                                    = notifier.late.load();
    h->gateway.forward                             = nullptr;
    px.reset();
    h.reset();
    gpu::dl_grid_twins::set_enabled(true);
    return 0;
  });
}

} // extern "C"
