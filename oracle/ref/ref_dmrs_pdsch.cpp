// TEST INFRASTRUCTURE ONLY: C entry point over the reference's own PDSCH DM-RS processor (dmrs_pdsch_processor_impl
// with the pseudo-random generator and the resource-grid mapper / generic precoder), compiled from the reference
// sources by oracle/build_ref.sh into oracle/_ref/libsrsref.so. Pins oracle/pdsch_dmrs_oracle.py; never shipped.
#include "srsran/phy/support/precoding_configuration.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/upper/signal_processors/dmrs_pdsch_processor.h"

#include "lib/phy/generic_functions/precoding/channel_precoder_generic.h"
#include "lib/phy/support/resource_grid_impl.h"
#include "lib/phy/support/resource_grid_mapper_impl.h"
#include "lib/phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "lib/phy/upper/signal_processors/dmrs_pdsch_processor_impl.h"

#include <memory>

using namespace srsran;

extern "C" {

/// Maps the DM-RS of one PDSCH transmission (CRB allocation rb_mask: crb_mask, one byte per grid CRB, or the
/// contiguous [rb_start, rb_start + nof_rb) when crb_mask is NULL; wideband precoding nof_ports x nof_layers weights,
/// row-major by port) into a zeroed (nof_ports x 14 x 12 * grid_nof_prb) grid; writes it as bf16 pairs.
int ref_dmrs_pdsch_map_mask(int             numerology,
                       int             slot_index,
                       int             scrambling_id,
                       int             n_scid,
                       int             dmrs_type2,
                       int             nof_layers,
                       int             nof_ports,
                       unsigned        dmrs_symbol_mask,
                       int             reference_point_k_rb,
                       int             rb_start,
                       int             nof_rb,
                       float           amplitude,
                       const float*    weights,
                       const uint8_t*  crb_mask,
                       int             grid_nof_prb,
                       uint16_t*       grid_out)
{
  dmrs_pdsch_processor_impl proc(
      std::make_unique<pseudo_random_generator_impl>(),
      std::make_unique<resource_grid_mapper_impl>(std::make_unique<channel_precoder_generic>()));
  const unsigned     nsc = 12 * grid_nof_prb;
  resource_grid_impl grid(nof_ports, 14, nsc);
  grid.set_all_zero();
  dmrs_pdsch_processor::config_t cfg;
  cfg.slot                 = slot_point(to_subcarrier_spacing(numerology), slot_index);
  cfg.reference_point_k_rb = reference_point_k_rb;
  cfg.type                 = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.scrambling_id        = scrambling_id;
  cfg.n_scid               = n_scid != 0;
  cfg.amplitude            = amplitude;
  cfg.symbols_mask         = symbol_slot_mask(14);
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
  cfg.precoding = precoding_configuration(nof_layers, nof_ports, 1, MAX_NOF_PRBS);
  for (int p = 0; p < nof_ports; ++p) {
    for (int l = 0; l < nof_layers; ++l) {
      cfg.precoding.set_coefficient(cf_t(weights[2 * (p * nof_layers + l)], weights[2 * (p * nof_layers + l) + 1]),
                                    l, p, 0);
    }
  }
  proc.map(grid.get_writer(), cfg);
  for (int p = 0; p < nof_ports; ++p) {
    for (unsigned l = 0; l != 14; ++l) {
      span<const cbf16_t> v = grid.get_reader().get_view(p, l);
      for (unsigned k = 0; k != nsc; ++k) {
        grid_out[2 * ((static_cast<size_t>(p) * 14 + l) * nsc + k)]     = v[k].real.value();
        grid_out[2 * ((static_cast<size_t>(p) * 14 + l) * nsc + k) + 1] = v[k].imag.value();
      }
    }
  }
  return 0;
}

int ref_dmrs_pdsch_map(int          numerology,
                       int          slot_index,
                       int          scrambling_id,
                       int          n_scid,
                       int          dmrs_type2,
                       int          nof_layers,
                       int          nof_ports,
                       unsigned     dmrs_symbol_mask,
                       int          reference_point_k_rb,
                       int          rb_start,
                       int          nof_rb,
                       float        amplitude,
                       const float* weights,
                       int          grid_nof_prb,
                       uint16_t*    grid_out)
{
  return ref_dmrs_pdsch_map_mask(numerology,
                                 slot_index,
                                 scrambling_id,
                                 n_scid,
                                 dmrs_type2,
                                 nof_layers,
                                 nof_ports,
                                 dmrs_symbol_mask,
                                 reference_point_k_rb,
                                 rb_start,
                                 nof_rb,
                                 amplitude,
                                 weights,
                                 nullptr,
                                 grid_nof_prb,
                                 grid_out);
}

} // extern "C"
