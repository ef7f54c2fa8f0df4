// TEST INFRASTRUCTURE ONLY: C entry point over the reference's own PUSCH DM-RS channel estimator
// (dmrs_pusch_estimator_impl with port_channel_estimator_average_impl, the linear interpolator and the DFT time
// alignment estimator), compiled from the reference sources by oracle/build_ref.sh into oracle/_ref/libsrsref.so. Used
// to pin the numpy restatement (oracle/pusch_chest_oracle.py) and to generate golden vectors; never shipped.
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran/phy/upper/channel_estimation.h"

#include "lib/phy/generic_functions/dft_processor_generic_impl.h"
#include "lib/phy/support/interpolator/interpolator_linear_impl.h"
#include "lib/phy/support/resource_grid_impl.h"
#include "lib/phy/support/time_alignment_estimator/time_alignment_estimator_dft_impl.h"
#include "lib/phy/upper/sequence_generators/low_papr_sequence_generator_impl.h"
#include "lib/phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "lib/phy/upper/signal_processors/dmrs_pusch_estimator_impl.h"
#include "lib/phy/upper/signal_processors/port_channel_estimator_average_impl.h"

#include <cstring>
#include <memory>
#include <vector>

using namespace srsran;

extern "C" {

/// DM-RS based channel estimation of one single-layer PUSCH transmission (pseudo-random DM-RS sequence, CRB allocation
/// crb_mask (one byte per grid CRB) or, when NULL, the contiguous [rb_start, rb_start + nof_rb)) on every rx port of a (nof_rx_ports x 14 x 12 * grid_nof_prb) bf16 grid.
/// fd_strategy: 0 none, 1 mean, 2 filter; td_strategy: 0 average, 1 interpolate. Outputs: ch_est
/// [port][14][12 * grid_nof_prb] bf16 pairs, and per port noise variance, RSRP, EPRE, time alignment (s), CFO (Hz or
/// NaN).
int ref_pusch_chest_mask(int             numerology,
                    int             low_papr_id,
                    int             slot_index,
                    int             scrambling_id,
                    int             n_scid,
                    int             dmrs_type2,
                    int             nof_layers,
                    float           scaling,
                    unsigned        dmrs_symbol_mask,
                    int             first_symbol,
                    int             nof_symbols,
                    int             rb_start,
                    int             nof_rb,
                    const uint8_t*  crb_mask,
                    int             grid_nof_prb,
                    int             nof_rx_ports,
                    int             fd_strategy,
                    int             td_strategy,
                    int             compensate_cfo,
                    const uint16_t* grid_in,
                    uint16_t*       ch_est_out,
                    float*          noise_var,
                    float*          rsrp,
                    float*          epre,
                    float*          ta_s,
                    float*          cfo_hz)
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
  const port_channel_estimator_fd_smoothing_strategy fd =
      fd_strategy == 0 ? port_channel_estimator_fd_smoothing_strategy::none
                       : (fd_strategy == 1 ? port_channel_estimator_fd_smoothing_strategy::mean
                                           : port_channel_estimator_fd_smoothing_strategy::filter);
  const port_channel_estimator_td_interpolation_strategy td =
      td_strategy == 0 ? port_channel_estimator_td_interpolation_strategy::average
                       : port_channel_estimator_td_interpolation_strategy::interpolate;
  time_alignment_estimator_dft_impl::collection_dft_processors dfts;
  for (unsigned n = time_alignment_estimator_dft_impl::min_dft_size; n <= time_alignment_estimator_dft_impl::max_dft_size;
       n *= 2) {
    dfts.emplace(n, std::make_unique<dft_processor_generic_impl>(
                        dft_processor::configuration{n, time_alignment_estimator_dft_impl::dft_direction}));
  }
  auto ta = std::make_unique<time_alignment_estimator_dft_impl>(std::move(dfts));
  auto port_est = std::make_unique<port_channel_estimator_average_impl>(
      std::make_unique<interpolator_linear_impl>(), std::move(ta), fd, td, compensate_cfo != 0);
  dmrs_pusch_estimator_impl est(std::make_unique<pseudo_random_generator_impl>(),
                                std::make_unique<low_papr_sequence_generator_impl>(),
                                std::move(port_est));

  dmrs_pusch_estimator::configuration cfg;
  cfg.slot = slot_point(to_subcarrier_spacing(numerology), slot_index);
  if (low_papr_id >= 0) {
    // Transform precoding: low-PAPR DM-RS sequence (dmrs_pusch_estimator_impl.cpp:77), type 1, one layer.
    dmrs_pusch_estimator::low_papr_sequence_configuration lp;
    lp.n_rs_id          = static_cast<unsigned>(low_papr_id);
    cfg.sequence_config = lp;
  } else {
    dmrs_pusch_estimator::pseudo_random_sequence_configuration seq;
    seq.type            = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
    seq.nof_tx_layers   = nof_layers;
    seq.scrambling_id   = scrambling_id;
    seq.n_scid          = n_scid != 0;
    cfg.sequence_config = seq;
  }
  cfg.scaling         = scaling;
  cfg.c_prefix        = cyclic_prefix::NORMAL;
  cfg.symbols_mask    = bounded_bitset<MAX_NSYMB_PER_SLOT>(14);
  for (unsigned l = 0; l != 14; ++l) {
    cfg.symbols_mask.set(l, ((dmrs_symbol_mask >> l) & 1U) != 0);
  }
  cfg.rb_mask = crb_bitmap(grid_nof_prb);
  if (crb_mask != nullptr) {
    for (int rb = 0; rb < grid_nof_prb; ++rb) {
      cfg.rb_mask.set(rb, crb_mask[rb] != 0);
    }
  } else {
    cfg.rb_mask.fill(rb_start, rb_start + nof_rb);
  }
  cfg.first_symbol = first_symbol;
  cfg.nof_symbols  = nof_symbols;
  for (int p = 0; p < nof_rx_ports; ++p) {
    cfg.rx_ports.push_back(static_cast<uint8_t>(p));
  }
  channel_estimate ce({static_cast<unsigned>(grid_nof_prb), 14, static_cast<unsigned>(nof_rx_ports),
                       static_cast<unsigned>(nof_layers)});
  for (int p = 0; p < nof_rx_ports; ++p) {
    span<cbf16_t> path = ce.get_path_ch_estimate(p, 0);
    std::fill(path.begin(), path.end(), cbf16_t());
  }
  est.estimate(ce, grid.get_reader(), cfg);
  for (int p = 0; p < nof_rx_ports; ++p) {
    span<const cbf16_t> path = ce.get_path_ch_estimate(p, 0);
    const unsigned      n    = std::min<unsigned>(path.size(), 14 * nsc);
    for (unsigned i = 0; i != n; ++i) {
      ch_est_out[2 * (static_cast<size_t>(p) * 14 * nsc + i)]     = path[i].real.value();
      ch_est_out[2 * (static_cast<size_t>(p) * 14 * nsc + i) + 1] = path[i].imag.value();
    }
    noise_var[p]                = ce.get_noise_variance(p);
    rsrp[p]                     = ce.get_rsrp(p, 0);
    epre[p]                     = ce.get_epre(p);
    ta_s[p]                     = static_cast<float>(ce.get_time_alignment(p, 0).to_seconds());
    std::optional<float> cfo    = ce.get_cfo_Hz(p, 0);
    cfo_hz[p]                   = cfo.has_value() ? *cfo : std::numeric_limits<float>::quiet_NaN();
  }
  return 0;
}

int ref_pusch_chest(int             numerology,
                    int             slot_index,
                    int             scrambling_id,
                    int             n_scid,
                    int             dmrs_type2,
                    int             nof_layers,
                    float           scaling,
                    unsigned        dmrs_symbol_mask,
                    int             first_symbol,
                    int             nof_symbols,
                    int             rb_start,
                    int             nof_rb,
                    int             grid_nof_prb,
                    int             nof_rx_ports,
                    int             fd_strategy,
                    int             td_strategy,
                    int             compensate_cfo,
                    const uint16_t* grid_in,
                    uint16_t*       ch_est_out,
                    float*          noise_var,
                    float*          rsrp,
                    float*          epre,
                    float*          ta_s,
                    float*          cfo_hz)
{
  return ref_pusch_chest_mask(numerology, -1, slot_index, scrambling_id, n_scid, dmrs_type2, nof_layers, scaling,
                              dmrs_symbol_mask, first_symbol, nof_symbols, rb_start, nof_rb, nullptr, grid_nof_prb,
                              nof_rx_ports, fd_strategy, td_strategy, compensate_cfo, grid_in, ch_est_out, noise_var,
                              rsrp, epre, ta_s, cfo_hz);
}

/// The reference's low-PAPR sequence r^(alpha, delta)_(u,v)(n) of length m (low_papr_sequence_generator_impl::generate
/// with alpha = 0, the estimator's call): m complex floats.
void ref_low_papr_generate(unsigned u, unsigned v, unsigned m, float* out)
{
  static low_papr_sequence_generator_impl gen;
  std::vector<cf_t>                       seq(m);
  gen.generate(seq, u, v, 0, 1);
  std::memcpy(out, seq.data(), m * sizeof(cf_t));
}

} // extern "C"
