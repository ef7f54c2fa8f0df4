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
#include "lib/phy/upper/channel_modulation/demodulation_mapper_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_demodulator_impl.h"
#include "lib/phy/upper/equalization/channel_equalizer_generic_impl.h"
#include "lib/phy/upper/sequence_generators/pseudo_random_generator_impl.h"

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

} // extern "C"
