// TEST INFRASTRUCTURE ONLY: drives lower-PHY baseband processors through a scripted sequence of upper-PHY requests and
// baseband symbols, for tests/test_lower_phy_gpu.py:
//   * the reference's own pdxch_processor_impl / puxch_processor_impl (lib/phy/lower/processors/downlink/pdxch/
//     pdxch_processor_impl.cpp, uplink/puxch/puxch_processor_impl.cpp, compiled from their sources by
//     oracle/build_chain.sh) on the reference's OFDM symbol (de)modulator with the generic DFT (variant 0) or on the GPU
//     symbol objects of integration/ofdm_gpu.cpp (variant 1);
//   * the GPU processors of integration/lower_phy_gpu.cpp (variant 2).
// Every variant sees the same requests, grids and samples; the test compares samples, grids, return values and the
// notifications (late requests, received symbols). Never shipped.
#include "signal_chain_gpu.h"

#include "lib/phy/generic_functions/dft_processor_generic_impl.h"
#include "lib/phy/lower/modulation/ofdm_demodulator_impl.h"
#include "lib/phy/lower/modulation/ofdm_modulator_impl.h"
#include "lib/phy/lower/processors/downlink/pdxch/pdxch_processor_impl.h"
#include "lib/phy/lower/processors/uplink/puxch/puxch_processor_impl.h"
#include "lib/phy/support/resource_grid_impl.h"
#include "srsran/gateways/baseband/buffer/baseband_gateway_buffer_reader.h"
#include "srsran/gateways/baseband/buffer/baseband_gateway_buffer_writer.h"
#include "srsran/phy/lower/lower_phy_rx_symbol_context.h"
#include "srsran/phy/lower/processors/downlink/pdxch/pdxch_processor_baseband.h"
#include "srsran/phy/lower/processors/downlink/pdxch/pdxch_processor_notifier.h"
#include "srsran/phy/lower/processors/downlink/pdxch/pdxch_processor_request_handler.h"
#include "srsran/phy/lower/processors/uplink/puxch/puxch_processor_baseband.h"
#include "srsran/phy/lower/processors/uplink/puxch/puxch_processor_notifier.h"
#include "srsran/phy/lower/processors/uplink/puxch/puxch_processor_request_handler.h"
#include "srsran/phy/support/resource_grid_context.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"

#include <cstring>
#include <memory>
#include <vector>

using namespace srsran;

namespace {

/// A fixed set of grids handed out as shared_resource_grid (one reference per request, released by the processors).
class harness_pool : public shared_resource_grid::pool_interface
{
public:
  harness_pool(unsigned n, unsigned ports, unsigned nsymb, unsigned nsc) : counts(n)
  {
    for (unsigned i = 0; i != n; ++i) {
      grids.emplace_back(std::make_unique<resource_grid_impl>(ports, nsymb, nsc));
      grids.back()->set_all_zero();
    }
  }
  resource_grid& get(unsigned id) override { return *grids[id]; }
  void           notify_release_scope(unsigned /*id*/) override {}
  shared_resource_grid grab(unsigned id)
  {
    counts[id] = 1;
    return shared_resource_grid(*this, counts[id], id);
  }

private:
  std::vector<std::unique_ptr<resource_grid_impl>> grids;
  std::vector<std::atomic<unsigned>>               counts;
};

class span_writer : public baseband_gateway_buffer_writer
{
public:
  std::vector<span<cf_t>> ch;
  unsigned                get_nof_channels() const override { return ch.size(); }
  unsigned                get_nof_samples() const override { return ch.empty() ? 0 : ch[0].size(); }
  span<cf_t>              get_channel_buffer(unsigned i) override { return ch[i]; }
};

class span_reader : public baseband_gateway_buffer_reader
{
public:
  std::vector<span<const cf_t>> ch;
  unsigned                      get_nof_channels() const override { return ch.size(); }
  unsigned                      get_nof_samples() const override { return ch.empty() ? 0 : ch[0].size(); }
  span<const cf_t>              get_channel_buffer(unsigned i) const override { return ch[i]; }
};

struct pdxch_recorder : public pdxch_processor_notifier {
  std::vector<int> late;
  void             on_pdxch_request_late(const resource_grid_context& c) override { late.push_back(c.slot.system_slot()); }
};

struct puxch_recorder : public puxch_processor_notifier {
  std::vector<int> late;
  std::vector<int> rx;  ///< (system slot, symbol) pairs in notification order.
  void on_puxch_request_late(const resource_grid_context& c) override { late.push_back(c.slot.system_slot()); }
  void on_rx_symbol(const shared_resource_grid& /*grid*/, const lower_phy_rx_symbol_context& c) override
  {
    rx.push_back(c.slot.system_slot());
    rx.push_back(c.nof_symbols);
  }
};

subcarrier_spacing scs_of(int numerology)
{
  return to_subcarrier_spacing(static_cast<unsigned>(numerology));
}

unsigned symbol_size(int numerology, int dft_size, cyclic_prefix cp, unsigned symbol_subframe)
{
  const subcarrier_spacing scs = scs_of(numerology);
  return cp.get_length(symbol_subframe, scs).to_samples(static_cast<double>(dft_size) * scs_to_khz(scs) * 1000.0) +
         dft_size;
}

} // namespace

extern "C" {

/// PDxCH scenario. grids: nof_grids x ports x nsymb x nsc bf16 pairs; port_mask[g]: bit p set = port p of grid g is
/// written (the others stay empty). events: nof_events x {kind, system slot, a, b}: kind 0 = handle_request(grid a),
/// kind 1 = process_symbol for symbols [a, b) of the slot. Outputs, in event order: the samples of every processed
/// symbol and port (sentinel 1e30 where the processor leaves the buffer untouched), one return flag per symbol, the
/// late-request slots. Returns the number of samples written (< 0 on error).
long ref_lower_pdxch_run(int             variant,
                         int             numerology,
                         int             bw_rb,
                         int             dft_size,
                         int             cp_extended,
                         double          center_freq_hz,
                         int             nof_ports,
                         int             nof_grids,
                         const uint16_t* grids,
                         const uint32_t* port_mask,
                         int             nof_events,
                         const int*      events,
                         float*          samples_out,
                         long            samples_cap,
                         uint8_t*        processed_out,
                         int*            late_out,
                         int*            nof_late)
{
  const cyclic_prefix      cp    = cp_extended ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL;
  const subcarrier_spacing scs   = scs_of(numerology);
  const unsigned           nsymb = get_nsymb_per_slot(cp);
  const unsigned           nsc   = 12 * bw_rb;
  harness_pool             pool(nof_grids, nof_ports, nsymb, nsc);
  for (int g = 0; g < nof_grids; ++g) {
    resource_grid_writer& w = pool.get(g).get_writer();
    for (int p = 0; p < nof_ports; ++p) {
      if (((port_mask[g] >> p) & 1U) == 0) {
        continue;
      }
      for (unsigned l = 0; l != nsymb; ++l) {
        const auto* row = reinterpret_cast<const cbf16_t*>(grids + 2 * ((static_cast<size_t>(g) * nof_ports + p) * nsymb + l) * nsc);
        w.put(p, l, 0, 1, span<const cbf16_t>(row, nsc));
      }
    }
  }

  std::unique_ptr<pdxch_processor> proc;
  if (variant == 2) {
    pdxch_processor_configuration c;
    c.cp             = cp;
    c.scs            = scs;
    c.srate          = sampling_rate::from_Hz(static_cast<double>(dft_size) * scs_to_khz(scs) * 1000.0);
    c.bandwidth_rb   = bw_rb;
    c.center_freq_Hz = center_freq_hz;
    c.nof_tx_ports   = nof_ports;
    proc             = create_pdxch_processor_factory_gpu(0)->create(c);
  } else {
    ofdm_modulator_configuration mc{static_cast<unsigned>(numerology), static_cast<unsigned>(bw_rb),
                                    static_cast<unsigned>(dft_size), cp, 1.0F, center_freq_hz};
    std::unique_ptr<ofdm_symbol_modulator> mod;
    if (variant == 0) {
      ofdm_modulator_common_configuration common;
      common.dft = std::make_unique<dft_processor_generic_impl>(
          dft_processor::configuration{static_cast<unsigned>(dft_size), dft_processor::direction::INVERSE});
      mod = std::make_unique<ofdm_symbol_modulator_impl>(common, mc);
    } else {
      mod = create_ofdm_modulator_factory_gpu(0)->create_ofdm_symbol_modulator(mc);
    }
    pdxch_processor_impl::configuration pc{cp, static_cast<unsigned>(nof_ports), 16};
    proc = std::make_unique<pdxch_processor_impl>(std::move(mod), pc);
  }
  pdxch_recorder rec;
  proc->connect(rec);

  long              pos = 0;
  size_t            nflag = 0;
  span_writer       buf;
  std::vector<cf_t> store;
  for (int e = 0; e < nof_events; ++e) {
    const int*       ev = events + 4 * e;
    const slot_point slot(static_cast<uint32_t>(numerology), static_cast<uint32_t>(ev[1]));
    if (ev[0] == 0) {
      proc->get_request_handler().handle_request(pool.grab(static_cast<unsigned>(ev[2])), {slot, 0});
      continue;
    }
    for (int l = ev[2]; l < ev[3]; ++l) {
      const unsigned n = symbol_size(numerology, dft_size, cp, slot.subframe_slot_index() * nsymb + l);
      if (pos + static_cast<long>(n) * nof_ports > samples_cap) {
        return -1;
      }
      buf.ch.clear();
      for (int p = 0; p < nof_ports; ++p) {
        auto* dst = reinterpret_cast<cf_t*>(samples_out) + pos + static_cast<long>(p) * n;
        std::fill(dst, dst + n, cf_t(1e30F, 1e30F));
        buf.ch.emplace_back(dst, n);
      }
      pdxch_processor_baseband::symbol_context ctx{slot, 0, static_cast<unsigned>(l)};
      processed_out[nflag++] = proc->get_baseband().process_symbol(buf, ctx) ? 1 : 0;
      pos += static_cast<long>(n) * nof_ports;
    }
  }
  *nof_late = static_cast<int>(rec.late.size());
  std::copy(rec.late.begin(), rec.late.end(), late_out);
  return pos;
}

/// PUxCH scenario. events as for PDxCH (kind 0 = handle_request(grid a), kind 1 = process_symbol for symbols [a, b)),
/// samples_in: the samples of every processed symbol and port in event order. max_in_flight: variant 2's
/// max_symbols_in_flight. Outputs: the final contents of every grid (nof_grids x ports x nsymb x nsc bf16 pairs), one
/// return flag per symbol, the received-symbol notifications ((system slot, symbol) pairs) and late-request slots.
int ref_lower_puxch_run(int          variant,
                        int          max_in_flight,
                        int          numerology,
                        int          bw_rb,
                        int          dft_size,
                        int          cp_extended,
                        float        dft_window_offset,
                        double       center_freq_hz,
                        int          nof_ports,
                        int          nof_grids,
                        int          nof_events,
                        const int*   events,
                        const float* samples_in,
                        uint16_t*    grids_out,
                        uint8_t*     processed_out,
                        int*         rx_out,
                        int*         nof_rx,
                        int*         late_out,
                        int*         nof_late)
{
  const cyclic_prefix      cp    = cp_extended ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL;
  const subcarrier_spacing scs   = scs_of(numerology);
  const unsigned           nsymb = get_nsymb_per_slot(cp);
  const unsigned           nsc   = 12 * bw_rb;
  const double             srate = static_cast<double>(dft_size) * scs_to_khz(scs) * 1000.0;
  harness_pool             pool(nof_grids, nof_ports, nsymb, nsc);

  std::unique_ptr<puxch_processor> proc;
  if (variant == 2) {
    puxch_processor_configuration c;
    c.cp                = cp;
    c.scs               = scs;
    c.srate             = sampling_rate::from_Hz(srate);
    c.bandwidth_rb      = bw_rb;
    c.dft_window_offset = dft_window_offset;
    c.center_freq_Hz    = center_freq_hz;
    c.nof_rx_ports      = nof_ports;
    proc                = create_puxch_processor_factory_gpu(0, static_cast<unsigned>(max_in_flight))->create(c);
  } else {
    // puxch_processor_factory_sw::create (puxch_processor_factories.cpp:41-57).
    const unsigned woff = static_cast<unsigned>(static_cast<float>(cp.get_length(1, scs).to_samples(srate)) *
                                                dft_window_offset);
    ofdm_demodulator_configuration dc{static_cast<unsigned>(numerology), static_cast<unsigned>(bw_rb),
                                      static_cast<unsigned>(dft_size), cp, woff,
                                      1.0F / std::sqrt(static_cast<float>(bw_rb * 12)), center_freq_hz};
    std::unique_ptr<ofdm_symbol_demodulator> demod;
    if (variant == 0) {
      ofdm_demodulator_common_configuration common;
      common.dft = std::make_unique<dft_processor_generic_impl>(
          dft_processor::configuration{static_cast<unsigned>(dft_size), dft_processor::direction::DIRECT});
      demod = std::make_unique<ofdm_symbol_demodulator_impl>(common, dc);
    } else {
      demod = create_ofdm_demodulator_factory_gpu(0)->create_ofdm_symbol_demodulator(dc);
    }
    puxch_processor_impl::configuration pc{cp, static_cast<unsigned>(nof_ports), 16};
    proc = std::make_unique<puxch_processor_impl>(std::move(demod), pc);
  }
  puxch_recorder rec;
  proc->connect(rec);

  long        pos   = 0;
  size_t      nflag = 0;
  span_reader buf;
  for (int e = 0; e < nof_events; ++e) {
    const int*       ev = events + 4 * e;
    const slot_point slot(static_cast<uint32_t>(numerology), static_cast<uint32_t>(ev[1]));
    if (ev[0] == 0) {
      proc->get_request_handler().handle_request(pool.grab(static_cast<unsigned>(ev[2])), {slot, 0});
      continue;
    }
    for (int l = ev[2]; l < ev[3]; ++l) {
      const unsigned n = symbol_size(numerology, dft_size, cp, slot.subframe_slot_index() * nsymb + l);
      buf.ch.clear();
      for (int p = 0; p < nof_ports; ++p) {
        buf.ch.emplace_back(reinterpret_cast<const cf_t*>(samples_in) + pos + static_cast<long>(p) * n, n);
      }
      lower_phy_rx_symbol_context ctx{slot, 0, static_cast<unsigned>(l)};
      processed_out[nflag++] = proc->get_baseband().process_symbol(buf, ctx) ? 1 : 0;
      pos += static_cast<long>(n) * nof_ports;
    }
  }
  proc.reset();
  for (int g = 0; g < nof_grids; ++g) {
    const resource_grid_reader& r = pool.get(g).get_reader();
    for (int p = 0; p < nof_ports; ++p) {
      for (unsigned l = 0; l != nsymb; ++l) {
        std::memcpy(grids_out + 2 * ((static_cast<size_t>(g) * nof_ports + p) * nsymb + l) * nsc,
                    r.get_view(p, l).data(), nsc * sizeof(cbf16_t));
      }
    }
  }
  *nof_rx   = static_cast<int>(rec.rx.size() / 2);
  *nof_late = static_cast<int>(rec.late.size());
  std::copy(rec.rx.begin(), rec.rx.end(), rx_out);
  std::copy(rec.late.begin(), rec.late.end(), late_out);
  return 0;
}

} // extern "C"
