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
#include "srsran/ran/resource_allocation/vrb_to_prb.h"
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

/// General allocation: VRB bitmap vrb_mask (one byte per VRB, nof_vrb entries) of a type-0 allocation, mapped
/// non-interleaved (interleave_l = 0) or interleaved with bundle size 2 / 4 (vrb_to_prb::create_interleaved_other);
/// nof_reserved reserved patterns besides the DM-RS, pattern i covering the CRBs whose byte in
/// res_crb[i * grid_nof_prb ..] is set, the PRB subcarriers of res_re[i] and the symbols of res_sym[i]; nof_prg PRGs of
/// prg_size PRBs with weights [prg][port][layer] (re, im) (prg_size 0: wideband `weights`). Writes the grid as
/// ref_pdsch_modulate does and the reference's CRB mask (rb_allocation::get_crb_mask, one byte per grid CRB) to
/// crb_out. Returns 0, or -1 when the codeword does not fill the allocation.
int ref_pdsch_modulate_ex(int             rnti,
                          int             n_id,
                          int             qm,
                          int             nof_layers,
                          int             nof_ports,
                          int             bwp_start_rb,
                          int             bwp_size_rb,
                          const uint8_t*  vrb_mask,
                          int             nof_vrb,
                          int             interleave_l,
                          int             start_symbol,
                          int             nof_symbols,
                          unsigned        dmrs_symbol_mask,
                          int             dmrs_type2,
                          int             nof_cdm_groups_without_data,
                          float           scaling,
                          const float*    weights,
                          int             nof_reserved,
                          const uint8_t*  res_crb,
                          const uint16_t* res_re,
                          const uint16_t* res_sym,
                          int             prg_size,
                          int             nof_prg,
                          const float*    prg_weights,
                          const uint8_t*  codeword_packed,
                          int             nof_bits,
                          int             grid_nof_prb,
                          uint16_t*       grid_out,
                          uint8_t*        crb_out)
{
  auto precoder = std::make_unique<channel_precoder_generic>();
  auto mapper   = std::make_unique<resource_grid_mapper_impl>(std::move(precoder));
  pdsch_modulator_impl modulator(std::make_unique<modulation_mapper_lut_impl>(),
                                 std::make_unique<pseudo_random_generator_impl>(), std::move(mapper));
  resource_grid_impl grid(nof_ports, 14, 12 * grid_nof_prb);
  grid.set_all_zero();

  vrb_bitmap vrbs(nof_vrb);
  for (int v = 0; v != nof_vrb; ++v) {
    vrbs.set(v, vrb_mask[v] != 0);
  }
  std::optional<vrb_to_prb::configuration> vtp;
  if (interleave_l != 0) {
    vtp = vrb_to_prb::create_interleaved_other(
        bwp_start_rb, bwp_size_rb,
        interleave_l == 2 ? vrb_to_prb::mapping_type::interleaved_n2 : vrb_to_prb::mapping_type::interleaved_n4);
  }

  pdsch_modulator::config_t cfg;
  cfg.rnti                        = static_cast<uint16_t>(rnti);
  cfg.bwp_size_rb                 = bwp_size_rb;
  cfg.bwp_start_rb                = bwp_start_rb;
  cfg.modulation1                 = mod_from_qm(qm);
  cfg.modulation2                 = mod_from_qm(qm);
  cfg.freq_allocation             = rb_allocation::make_type0(vrbs, vtp);
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
  for (int i = 0; i != nof_reserved; ++i) {
    re_pattern pat;
    pat.crb_mask = crb_bitmap(grid_nof_prb);
    for (int rb = 0; rb != grid_nof_prb; ++rb) {
      pat.crb_mask.set(rb, res_crb[i * grid_nof_prb + rb] != 0);
    }
    for (unsigned k = 0; k != 12; ++k) {
      pat.re_mask.set(k, ((res_re[i] >> k) & 1U) != 0);
    }
    pat.symbols = symbol_slot_mask(14);
    for (unsigned l = 0; l != 14; ++l) {
      pat.symbols.set(l, ((res_sym[i] >> l) & 1U) != 0);
    }
    cfg.reserved.merge(pat);
  }
  if (prg_size > 0) {
    cfg.precoding = precoding_configuration(nof_layers, nof_ports, nof_prg, prg_size);
    for (int g = 0; g < nof_prg; ++g) {
      for (int p = 0; p < nof_ports; ++p) {
        for (int l = 0; l < nof_layers; ++l) {
          const float* w = prg_weights + 2 * ((g * nof_ports + p) * nof_layers + l);
          cfg.precoding.set_coefficient(cf_t(w[0], w[1]), l, p, g);
        }
      }
    }
  } else {
    cfg.precoding = precoding_configuration(nof_layers, nof_ports, 1, MAX_NOF_PRBS);
    for (int p = 0; p < nof_ports; ++p) {
      for (int l = 0; l < nof_layers; ++l) {
        cfg.precoding.set_coefficient(cf_t(weights[2 * (p * nof_layers + l)], weights[2 * (p * nof_layers + l) + 1]),
                                      l, p, 0);
      }
    }
  }

  const crb_bitmap crbs = cfg.freq_allocation.get_crb_mask(bwp_start_rb, bwp_size_rb);
  for (int rb = 0; rb != grid_nof_prb; ++rb) {
    crb_out[rb] = (rb < static_cast<int>(crbs.size()) && crbs.test(rb)) ? 1 : 0;
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
