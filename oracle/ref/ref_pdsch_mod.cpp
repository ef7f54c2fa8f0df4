// TEST INFRASTRUCTURE ONLY: C entry point over the reference's own PDSCH modulator (pdsch_modulator_impl with the
// LUT modulation mapper, the pseudo-random generator, the resource-grid mapper and the generic channel precoder),
// compiled from the reference sources by oracle/build_ref.sh into oracle/_ref/libsrsref.so. Used to pin the CPU
// restatement (oracle/oracle.cpp: orc_pdsch_modulate) and to generate golden vectors; never shipped.
#include "srsran/phy/support/precoding_configuration.h"
#include "srsran/phy/support/re_pattern.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/upper/channel_processors/pdsch/pdsch_modulator.h"
#include "srsran/phy/upper/dmrs_mapping.h"
#include "srsran/phy/upper/rb_allocation.h"
#include "srsran/srsvec/bit.h"
#include "srsran/support/units.h"

// Concrete classes (their headers live next to the sources).
#include "lib/phy/generic_functions/precoding/channel_precoder_generic.h"
#include "lib/phy/support/resource_grid_impl.h"
#include "lib/phy/support/resource_grid_mapper_impl.h"
#include "lib/phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_modulator_impl.h"
#include "lib/phy/upper/sequence_generators/pseudo_random_generator_impl.h"

#include <cstring>
#include <memory>

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
} // namespace

extern "C" {

/// Modulates one codeword into a zeroed resource grid of nof_ports x 14 x (12 * grid_nof_prb) and writes the grid
/// as interleaved (re, im) bf16 bit patterns, port-major then symbol then subcarrier. Contiguous VRB allocation
/// [rb_start, rb_start + nof_rb) of the BWP, no reserved REs other than the DM-RS, wideband precoding with the given
/// nof_ports x nof_layers complex weights (row-major by port). Returns 0 on success.
int ref_pdsch_modulate(int             rnti,
                       int             n_id,
                       int             qm,
                       int             nof_layers,
                       int             nof_ports,
                       int             bwp_start_rb,
                       int             bwp_size_rb,
                       int             rb_start,
                       int             nof_rb,
                       int             start_symbol,
                       int             nof_symbols,
                       unsigned        dmrs_symbol_mask,
                       int             dmrs_type2,
                       int             nof_cdm_groups_without_data,
                       float           scaling,
                       const float*    weights,
                       const uint8_t*  codeword_packed,
                       int             nof_bits,
                       int             grid_nof_prb,
                       uint16_t*       grid_out)
{
  auto precoder = std::make_unique<channel_precoder_generic>();
  auto mapper   = std::make_unique<resource_grid_mapper_impl>(std::move(precoder));
  pdsch_modulator_impl modulator(std::make_unique<modulation_mapper_lut_impl>(),
                                 std::make_unique<pseudo_random_generator_impl>(), std::move(mapper));
  resource_grid_impl grid(nof_ports, 14, 12 * grid_nof_prb);
  grid.set_all_zero();

  pdsch_modulator::config_t cfg;
  cfg.rnti                        = static_cast<uint16_t>(rnti);
  cfg.bwp_size_rb                 = bwp_size_rb;
  cfg.bwp_start_rb                = bwp_start_rb;
  cfg.modulation1                 = mod_from_qm(qm);
  cfg.modulation2                 = mod_from_qm(qm);
  cfg.freq_allocation             = rb_allocation::make_type1(rb_start, nof_rb);
  cfg.start_symbol_index          = start_symbol;
  cfg.nof_symbols                 = nof_symbols;
  cfg.dmrs_symb_pos               = symbol_slot_mask(14);
  for (unsigned l = 0; l != 14; ++l) {
    cfg.dmrs_symb_pos.set(l, ((dmrs_symbol_mask >> l) & 1U) != 0);
  }
  cfg.dmrs_config_type            = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.nof_cdm_groups_without_data = nof_cdm_groups_without_data;
  cfg.n_id                        = n_id;
  cfg.scaling                     = scaling;
  cfg.precoding                   = precoding_configuration(nof_layers, nof_ports, 1, MAX_NOF_PRBS);
  for (int p = 0; p < nof_ports; ++p) {
    for (int l = 0; l < nof_layers; ++l) {
      cfg.precoding.set_coefficient(cf_t(weights[2 * (p * nof_layers + l)], weights[2 * (p * nof_layers + l) + 1]),
                                    l, p, 0);
    }
  }

  dynamic_bit_buffer cw(nof_bits);
  srsvec::copy_offset(cw, span<const uint8_t>(codeword_packed, (nof_bits + 7) / 8), 0);
  const bit_buffer cws[1] = {cw};
  modulator.modulate(grid.get_writer(), span<const bit_buffer>(cws, 1), cfg);

  const resource_grid_reader& reader = grid.get_reader();
  const unsigned              nsc    = 12 * grid_nof_prb;
  for (int p = 0; p < nof_ports; ++p) {
    for (unsigned l = 0; l != 14; ++l) {
      span<const cbf16_t> v = reader.get_view(p, l);
      for (unsigned k = 0; k != nsc; ++k) {
        grid_out[2 * ((p * 14 + l) * nsc + k)]     = v[k].real.value();
        grid_out[2 * ((p * 14 + l) * nsc + k) + 1] = v[k].imag.value();
      }
    }
  }
  return 0;
}

} // extern "C"
