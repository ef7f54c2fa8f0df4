// TEST INFRASTRUCTURE ONLY: C entry points over the reference's own OFDM slot modulator / demodulator
// (lib/phy/lower/modulation/ofdm_modulator_impl.cpp, ofdm_demodulator_impl.cpp) with the generic DFT
// (lib/phy/generic_functions/dft_processor_generic_impl.cpp), compiled from the reference sources by
// oracle/build_ref.sh into oracle/_ref/libsrsref.so. Used to pin the numpy restatement (oracle/ofdm_oracle.py) and
// to generate golden vectors; never shipped.
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"

#include "lib/phy/generic_functions/dft_processor_generic_impl.h"
#include "lib/phy/lower/modulation/ofdm_demodulator_impl.h"
#include "lib/phy/lower/modulation/ofdm_modulator_impl.h"
#include "lib/phy/support/resource_grid_impl.h"

#include <cstring>
#include <memory>

using namespace srsran;

extern "C" {

/// Samples of one slot of one port.
int ref_ofdm_slot_size(int numerology, int bw_rb, int dft_size, int cp_extended, int slot_index)
{
  ofdm_modulator_common_configuration common;
  common.dft = std::make_unique<dft_processor_generic_impl>(
      dft_processor::configuration{static_cast<unsigned>(dft_size), dft_processor::direction::INVERSE});
  ofdm_modulator_configuration cfg{static_cast<unsigned>(numerology), static_cast<unsigned>(bw_rb),
                                   static_cast<unsigned>(dft_size),
                                   cp_extended ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL, 1.0F, 0.0};
  ofdm_slot_modulator_impl mod(common, cfg);
  return static_cast<int>(mod.get_slot_size(static_cast<unsigned>(slot_index)));
}

/// Modulates every port of a (nof_ports x nsymb x 12 * bw_rb) bf16 grid ((re, im) uint16 pairs) for `slot_index`
/// within the subframe; out holds nof_ports consecutive slots of (re, im) floats.
int ref_ofdm_modulate(int             numerology,
                      int             bw_rb,
                      int             dft_size,
                      int             cp_extended,
                      float           scale,
                      double          center_freq_hz,
                      int             slot_index,
                      int             nof_ports,
                      const uint16_t* grid_in,
                      float*          out)
{
  ofdm_modulator_common_configuration common;
  common.dft = std::make_unique<dft_processor_generic_impl>(
      dft_processor::configuration{static_cast<unsigned>(dft_size), dft_processor::direction::INVERSE});
  const cyclic_prefix          cp = cp_extended ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL;
  ofdm_modulator_configuration cfg{static_cast<unsigned>(numerology), static_cast<unsigned>(bw_rb),
                                   static_cast<unsigned>(dft_size), cp, scale, center_freq_hz};
  ofdm_slot_modulator_impl     mod(common, cfg);
  const unsigned               nsymb = get_nsymb_per_slot(cp);
  const unsigned               nsc   = 12 * bw_rb;
  resource_grid_impl           grid(nof_ports, nsymb, nsc);
  grid.set_all_zero();
  std::vector<cbf16_t> row(nsc);
  for (int p = 0; p < nof_ports; ++p) {
    for (unsigned l = 0; l != nsymb; ++l) {
      const uint16_t* src = grid_in + 2 * (static_cast<size_t>(p) * nsymb + l) * nsc;
      for (unsigned k = 0; k != nsc; ++k) {
        row[k].real = bf16_t(src[2 * k]);
        row[k].imag = bf16_t(src[2 * k + 1]);
      }
      grid.get_writer().put(p, l, 0, 1, row);
    }
  }
  const unsigned    slot_sz = mod.get_slot_size(static_cast<unsigned>(slot_index));
  std::vector<cf_t> buf(slot_sz);
  for (int p = 0; p < nof_ports; ++p) {
    mod.modulate(buf, grid.get_reader(), p, static_cast<unsigned>(slot_index));
    std::memcpy(out + 2 * static_cast<size_t>(p) * slot_sz, buf.data(), slot_sz * sizeof(cf_t));
  }
  return 0;
}

/// Demodulates nof_ports consecutive slots of (re, im) float samples into a (nof_ports x nsymb x 12 * bw_rb) bf16 grid.
int ref_ofdm_demodulate(int          numerology,
                        int          bw_rb,
                        int          dft_size,
                        int          cp_extended,
                        float        scale,
                        double       center_freq_hz,
                        int          window_offset,
                        int          slot_index,
                        int          nof_ports,
                        const float* in,
                        uint16_t*    grid_out)
{
  ofdm_demodulator_common_configuration common;
  common.dft = std::make_unique<dft_processor_generic_impl>(
      dft_processor::configuration{static_cast<unsigned>(dft_size), dft_processor::direction::DIRECT});
  const cyclic_prefix            cp = cp_extended ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL;
  ofdm_demodulator_configuration cfg{static_cast<unsigned>(numerology),   static_cast<unsigned>(bw_rb),
                                     static_cast<unsigned>(dft_size),     cp,
                                     static_cast<unsigned>(window_offset), scale,
                                     center_freq_hz};
  ofdm_slot_demodulator_impl     demod(common, cfg);
  const unsigned                 nsymb   = get_nsymb_per_slot(cp);
  const unsigned                 nsc     = 12 * bw_rb;
  const unsigned                 slot_sz = demod.get_slot_size(static_cast<unsigned>(slot_index));
  resource_grid_impl             grid(nof_ports, nsymb, nsc);
  grid.set_all_zero();
  std::vector<cf_t> buf(slot_sz);
  for (int p = 0; p < nof_ports; ++p) {
    std::memcpy(buf.data(), in + 2 * static_cast<size_t>(p) * slot_sz, slot_sz * sizeof(cf_t));
    demod.demodulate(grid.get_writer(), buf, p, static_cast<unsigned>(slot_index));
  }
  for (int p = 0; p < nof_ports; ++p) {
    for (unsigned l = 0; l != nsymb; ++l) {
      span<const cbf16_t> v = grid.get_reader().get_view(p, l);
      for (unsigned k = 0; k != nsc; ++k) {
        grid_out[2 * ((static_cast<size_t>(p) * nsymb + l) * nsc + k)]     = v[k].real.value();
        grid_out[2 * ((static_cast<size_t>(p) * nsymb + l) * nsc + k) + 1] = v[k].imag.value();
      }
    }
  }
  return 0;
}

} // extern "C"
