// TEST INFRASTRUCTURE ONLY: C entry points over the reference's own PUSCH demodulator (pusch_demodulator_impl with
// the generic channel equalizer, the demodulation mapper and the pseudo-random descrambler) and demodulation mapper,
// compiled from the reference sources by oracle/build_ref.sh into oracle/_ref/libsrsref.so. Used to pin the numpy
// restatement (oracle/pusch_demod_oracle.py) and to generate golden vectors; never shipped.
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran/phy/upper/channel_estimation.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_codeword_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_demodulator_notifier.h"

#include "lib/phy/support/resource_grid_impl.h"
#include "lib/phy/generic_functions/transform_precoding/transform_precoder_dft_impl.h"
#include "lib/phy/upper/channel_modulation/demodulation_mapper_impl.h"
#include "lib/phy/upper/channel_modulation/evm_calculator_generic_impl.h"
#include "lib/phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_demodulator_impl.h"
#include "lib/phy/upper/equalization/channel_equalizer_generic_impl.h"
#include "lib/phy/upper/sequence_generators/pseudo_random_generator_impl.h"

#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

using namespace srsran;

namespace {

modulation_scheme mod_from_qm(int qm)
{
  switch (qm) {
    case 1: return modulation_scheme::BPSK;
    case 2: return modulation_scheme::QPSK;
    case 4: return modulation_scheme::QAM16;
    case 6: return modulation_scheme::QAM64;
    default: return modulation_scheme::QAM256;
  }
}

/// Codeword buffer collecting every block the demodulator produces, in order.
class collecting_codeword_buffer : public pusch_codeword_buffer
{
public:
  explicit collecting_codeword_buffer(unsigned capacity) : data(capacity) {}
  span<log_likelihood_ratio> get_next_block_view(unsigned block_size) override
  {
    unsigned n = std::min(block_size, static_cast<unsigned>(data.size()) - pos);
    return span<log_likelihood_ratio>(data).subspan(pos, n);
  }
  void on_new_block(span<const log_likelihood_ratio> block, const bit_buffer& /**/) override { pos += block.size(); }
  void on_end_codeword() override {}

  std::vector<log_likelihood_ratio> data;
  unsigned                          pos = 0;
};

class null_notifier : public pusch_demodulator_notifier
{
public:
  void on_provisional_stats(unsigned /**/, const demodulation_stats& /**/) override {}
  void on_end_stats(const demodulation_stats& /**/) override {}
};

/// Exact DFT (float64 accumulation) behind the reference's dft_processor interface. The upper PHY builds the
/// transform precoder's DFTs with FFTW (upper_phy_factories.cpp:364, dft_processor_fftw_impl.cpp), which this image
/// lacks, and the generic DFT only has the OFDM sizes; this test implementation of the interface lets the reference's
/// own transform_precoder_dft_impl (scaling, noise handling) and pusch_demodulator_impl run on every 12 x 2^a 3^b 5^c
/// size. Test infrastructure only.
class exact_dft_processor : public dft_processor
{
public:
  exact_dft_processor(unsigned size, direction dir_) : dir(dir_), input(size), output(size) {}
  direction        get_direction() const override { return dir; }
  unsigned         get_size() const override { return static_cast<unsigned>(input.size()); }
  span<cf_t>       get_input() override { return input; }
  span<const cf_t> run() override
  {
    const size_t n    = input.size();
    const double sign = (dir == direction::DIRECT) ? -1.0 : 1.0;
    for (size_t k = 0; k != n; ++k) {
      double re = 0, im = 0;
      for (size_t i = 0; i != n; ++i) {
        const double a = sign * 2.0 * M_PI * static_cast<double>((i * k) % n) / static_cast<double>(n);
        const double c = std::cos(a), s = std::sin(a);
        re += input[i].real() * c - input[i].imag() * s;
        im += input[i].real() * s + input[i].imag() * c;
      }
      output[k] = cf_t(static_cast<float>(re), static_cast<float>(im));
    }
    return output;
  }

private:
  direction         dir;
  std::vector<cf_t> input, output;
};

/// Notifier recording the per-symbol (provisional) and end statistics: rows 0..13 per OFDM symbol, row 14 the end
/// stats, (SINR dB, EVM) each, NaN when absent.
class stats_notifier : public pusch_demodulator_notifier
{
public:
  explicit stats_notifier(float* out_) : out(out_)
  {
    for (unsigned i = 0; i != 30; ++i) {
      out[i] = std::nanf("");
    }
  }
  void on_provisional_stats(unsigned i_symbol, const demodulation_stats& s) override { put(i_symbol, s); }
  void on_end_stats(const demodulation_stats& s) override { put(14, s); }

private:
  void put(unsigned row, const demodulation_stats& s)
  {
    if (s.sinr_dB.has_value()) {
      out[2 * row] = *s.sinr_dB;
    }
    if (s.evm.has_value()) {
      out[2 * row + 1] = *s.evm;
    }
  }
  float* out;
};

} // namespace

extern "C" {

/// PUSCH demodulation of one transmission: contiguous CRB allocation [rb_start, rb_start + nof_rb), rx grid
/// (nof_rx_ports x 14 x 12 * grid_nof_prb bf16 pairs), channel estimates [layer][port][14][12 * grid_nof_prb] bf16
/// pairs, per-port noise variances. equalizer: 0 ZF, 1 MMSE. Writes the descrambled codeword LLRs; returns their count.
int ref_pusch_demodulate(int             rnti,
                         int             n_id,
                         int             qm,
                         int             nof_layers,
                         int             nof_rx_ports,
                         int             start_symbol,
                         int             nof_symbols,
                         unsigned        dmrs_symbol_mask,
                         int             dmrs_type2,
                         int             nof_cdm_groups_without_data,
                         int             rb_start,
                         int             nof_rb,
                         int             grid_nof_prb,
                         int             equalizer_mmse,
                         const uint16_t* grid_in,
                         const uint16_t* ch_est_in,
                         const float*    noise_var,
                         int8_t*         llr_out,
                         int             max_llrs)
{
  const unsigned     nsc = 12 * grid_nof_prb;
  resource_grid_impl grid(nof_rx_ports, 14, nsc);
  grid.set_all_zero();
  std::vector<cbf16_t> row(nsc);
  for (int p = 0; p < nof_rx_ports; ++p) {
    for (unsigned l = 0; l != 14; ++l) {
      const uint16_t* src = grid_in + 2 * (static_cast<size_t>(p) * 14 + l) * nsc;
      for (unsigned k = 0; k != nsc; ++k) {
        row[k].real = bf16_t(src[2 * k]);
        row[k].imag = bf16_t(src[2 * k + 1]);
      }
      grid.get_writer().put(p, l, 0, 1, row);
    }
  }
  channel_estimate est({static_cast<unsigned>(grid_nof_prb), 14, static_cast<unsigned>(nof_rx_ports),
                        static_cast<unsigned>(nof_layers)});
  for (int ly = 0; ly < nof_layers; ++ly) {
    for (int p = 0; p < nof_rx_ports; ++p) {
      span<cbf16_t>   path = est.get_path_ch_estimate(p, ly);
      const uint16_t* src  = ch_est_in + 2 * (static_cast<size_t>(ly) * nof_rx_ports + p) * 14 * nsc;
      for (size_t i = 0; i != path.size(); ++i) {
        path[i].real = bf16_t(src[2 * i]);
        path[i].imag = bf16_t(src[2 * i + 1]);
      }
    }
  }
  for (int p = 0; p < nof_rx_ports; ++p) {
    est.set_noise_variance(noise_var[p], p);
  }

  pusch_demodulator_impl demod(
      std::make_unique<channel_equalizer_generic_impl>(equalizer_mmse ? channel_equalizer_algorithm_type::mmse
                                                                      : channel_equalizer_algorithm_type::zf),
      nullptr,
      std::make_unique<demodulation_mapper_impl>(),
      nullptr,
      std::make_unique<pseudo_random_generator_impl>(),
      grid_nof_prb,
      true);

  pusch_demodulator::configuration cfg;
  cfg.rnti    = static_cast<uint16_t>(rnti);
  cfg.rb_mask = crb_bitmap(grid_nof_prb);
  cfg.rb_mask.fill(rb_start, rb_start + nof_rb);
  cfg.modulation         = mod_from_qm(qm);
  cfg.start_symbol_index = start_symbol;
  cfg.nof_symbols        = nof_symbols;
  cfg.dmrs_symb_pos      = symbol_slot_mask(14);
  for (unsigned l = 0; l != 14; ++l) {
    cfg.dmrs_symb_pos.set(l, ((dmrs_symbol_mask >> l) & 1U) != 0);
  }
  cfg.dmrs_config_type            = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.nof_cdm_groups_without_data = nof_cdm_groups_without_data;
  cfg.n_id                        = n_id;
  cfg.nof_tx_layers               = nof_layers;
  cfg.enable_transform_precoding  = false;
  for (int p = 0; p < nof_rx_ports; ++p) {
    cfg.rx_ports.push_back(static_cast<uint8_t>(p));
  }
  collecting_codeword_buffer buf(static_cast<unsigned>(max_llrs));
  null_notifier              notifier;
  demod.demodulate(buf, notifier, grid.get_reader(), est, cfg);
  std::memcpy(llr_out, buf.data.data(), buf.pos);
  return static_cast<int>(buf.pos);
}

/// Soft demapping of n symbols (interleaved (re, im) floats) with per-symbol noise variances into n * qm LLRs.
void ref_demodulate_soft(int qm, const float* symbols, const float* noise_vars, int n, int8_t* llrs)
{
  demodulation_mapper_impl demapper;
  std::vector<log_likelihood_ratio> out(static_cast<size_t>(n) * qm);
  demapper.demodulate_soft(out,
                           span<const cf_t>(reinterpret_cast<const cf_t*>(symbols), n),
                           span<const float>(noise_vars, n),
                           mod_from_qm(qm));
  std::memcpy(llrs, out.data(), out.size());
}

/// As ref_pusch_demodulate with the general configuration: crb_mask (one byte per grid CRB, NULL = the contiguous
/// allocation), transform precoding (transform_precoder_dft_impl over exact DFTs for every valid PRB count), the
/// EVM calculator (evm_calculator_generic_impl with the LUT modulation mapper) and the post-equalization SINR, as the
/// upper PHY factory builds the demodulator (upper_phy_factories.cpp:423). stats_out: 15 x (SINR dB, EVM).
int ref_pusch_demodulate_ex(int             rnti,
                            int             n_id,
                            int             qm,
                            int             nof_layers,
                            int             nof_rx_ports,
                            int             start_symbol,
                            int             nof_symbols,
                            unsigned        dmrs_symbol_mask,
                            int             dmrs_type2,
                            int             nof_cdm_groups_without_data,
                            int             rb_start,
                            int             nof_rb,
                            const uint8_t*  crb_mask,
                            int             transform_precoding,
                            int             grid_nof_prb,
                            int             equalizer_mmse,
                            const uint16_t* grid_in,
                            const uint16_t* ch_est_in,
                            const float*    noise_var,
                            int8_t*         llr_out,
                            int             max_llrs,
                            float*          stats_out)
{
  const unsigned     nsc = 12 * grid_nof_prb;
  resource_grid_impl grid(nof_rx_ports, 14, nsc);
  grid.set_all_zero();
  std::vector<cbf16_t> row(nsc);
  for (int p = 0; p < nof_rx_ports; ++p) {
    for (unsigned l = 0; l != 14; ++l) {
      const uint16_t* src = grid_in + 2 * (static_cast<size_t>(p) * 14 + l) * nsc;
      for (unsigned k = 0; k != nsc; ++k) {
        row[k].real = bf16_t(src[2 * k]);
        row[k].imag = bf16_t(src[2 * k + 1]);
      }
      grid.get_writer().put(p, l, 0, 1, row);
    }
  }
  channel_estimate est({static_cast<unsigned>(grid_nof_prb), 14, static_cast<unsigned>(nof_rx_ports),
                        static_cast<unsigned>(nof_layers)});
  for (int ly = 0; ly < nof_layers; ++ly) {
    for (int p = 0; p < nof_rx_ports; ++p) {
      span<cbf16_t>   path = est.get_path_ch_estimate(p, ly);
      const uint16_t* src  = ch_est_in + 2 * (static_cast<size_t>(ly) * nof_rx_ports + p) * 14 * nsc;
      for (size_t i = 0; i != path.size(); ++i) {
        path[i].real = bf16_t(src[2 * i]);
        path[i].imag = bf16_t(src[2 * i + 1]);
      }
    }
  }
  for (int p = 0; p < nof_rx_ports; ++p) {
    est.set_noise_variance(noise_var[p], p);
  }

  std::unique_ptr<transform_precoder> precoder;
  if (transform_precoding) {
    transform_precoder_dft_impl::collection_dft_processors dfts;
    for (unsigned nof_prb = 1; nof_prb <= static_cast<unsigned>(grid_nof_prb); ++nof_prb) {
      if (transform_precoding::is_nof_prbs_valid(nof_prb)) {
        dfts.emplace(nof_prb, std::make_unique<exact_dft_processor>(NRE * nof_prb, dft_processor::direction::INVERSE));
      }
    }
    precoder = std::make_unique<transform_precoder_dft_impl>(std::move(dfts));
  }
  pusch_demodulator_impl demod(
      std::make_unique<channel_equalizer_generic_impl>(equalizer_mmse ? channel_equalizer_algorithm_type::mmse
                                                                      : channel_equalizer_algorithm_type::zf),
      std::move(precoder),
      std::make_unique<demodulation_mapper_impl>(),
      std::make_unique<evm_calculator_generic_impl>(std::make_unique<modulation_mapper_lut_impl>()),
      std::make_unique<pseudo_random_generator_impl>(),
      grid_nof_prb,
      true);

  pusch_demodulator::configuration cfg;
  cfg.rnti    = static_cast<uint16_t>(rnti);
  cfg.rb_mask = crb_bitmap(grid_nof_prb);
  if (crb_mask != nullptr) {
    for (int rb = 0; rb < grid_nof_prb; ++rb) {
      cfg.rb_mask.set(rb, crb_mask[rb] != 0);
    }
  } else {
    cfg.rb_mask.fill(rb_start, rb_start + nof_rb);
  }
  cfg.modulation         = mod_from_qm(qm);
  cfg.start_symbol_index = start_symbol;
  cfg.nof_symbols        = nof_symbols;
  cfg.dmrs_symb_pos      = symbol_slot_mask(14);
  for (unsigned l = 0; l != 14; ++l) {
    cfg.dmrs_symb_pos.set(l, ((dmrs_symbol_mask >> l) & 1U) != 0);
  }
  cfg.dmrs_config_type            = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.nof_cdm_groups_without_data = nof_cdm_groups_without_data;
  cfg.n_id                        = n_id;
  cfg.nof_tx_layers               = nof_layers;
  cfg.enable_transform_precoding  = transform_precoding != 0;
  for (int p = 0; p < nof_rx_ports; ++p) {
    cfg.rx_ports.push_back(static_cast<uint8_t>(p));
  }
  collecting_codeword_buffer buf(static_cast<unsigned>(max_llrs));
  stats_notifier             notifier(stats_out);
  demod.demodulate(buf, notifier, grid.get_reader(), est, cfg);
  std::memcpy(llr_out, buf.data.data(), buf.pos);
  return static_cast<int>(buf.pos);
}

} // extern "C"
