// TEST INFRASTRUCTURE ONLY: drives lower-PHY baseband processors through a scripted sequence of upper-PHY requests and
// baseband symbols, for tests/test_lower_phy_gpu.py:
//   * the reference's own pdxch_processor_impl / puxch_processor_impl (lib/phy/lower/processors/downlink/pdxch/
//     pdxch_processor_impl.cpp, uplink/puxch/puxch_processor_impl.cpp, compiled from their sources by
//     oracle/build_chain.sh) on the reference's OFDM symbol (de)modulator with the generic DFT (variant 0) or on the GPU
//     symbol objects of integration/ofdm_gpu.cpp (variant 1);
//   * the GPU processors of integration/lower_phy_gpu.cpp (variant 2), and those of a sector group (variant 3, several
//     sectors driven from their own threads: ref_lower_sectors_run).
// Every variant sees the same requests, grids and samples; the test compares samples, grids, return values and the
// notifications (late requests, received symbols). Never shipped.
#include "gpu_staging.h"
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

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <sys/prctl.h>
#include <thread>
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
  /// Maps (or unmaps) every grid's storage for the devices (gpu::host_blocks), as a GPU uplink processor's PUSCH slot
  /// batch does with its grid: the GPU lower PHY then demodulates into the rows directly.
  void map_grids(bool on)
  {
    for (auto& g : grids) {
      const resource_grid_reader& r    = g->get_reader();
      const void*                 base = r.get_view(0, 0).data();
      if (on) {
        (void)gpu::host_blocks::add(base, static_cast<size_t>(r.get_nof_ports()) * r.get_nof_symbols() *
                                              r.get_nof_subc() * sizeof(cbf16_t));
      } else {
        gpu::host_blocks::remove(base);
      }
    }
  }
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

/// The lower-PHY configuration every sector of a scenario shares (the carrier frequency is per sector).
struct scenario {
  int           numerology;
  int           bw_rb;
  int           dft_size;
  cyclic_prefix cp;
  float         dft_window_offset;
  int           nof_ports;

  subcarrier_spacing scs() const { return scs_of(numerology); }
  unsigned           nsymb() const { return get_nsymb_per_slot(cp); }
  unsigned           nsc() const { return 12 * bw_rb; }
  double             srate() const { return static_cast<double>(dft_size) * scs_to_khz(scs()) * 1000.0; }
};

/// Variants 0 (reference processor, generic DFT), 1 (reference processor, GPU symbol objects), 2 (GPU processor) and
/// 3 (GPU processor of a sector group).
std::unique_ptr<pdxch_processor>
make_pdxch(int variant, const scenario& sc, double center_freq_hz, const std::shared_ptr<lower_phy_sector_group>& group)
{
  if (variant >= 2) {
    pdxch_processor_configuration c;
    c.cp             = sc.cp;
    c.scs            = sc.scs();
    c.srate          = sampling_rate::from_Hz(sc.srate());
    c.bandwidth_rb   = sc.bw_rb;
    c.center_freq_Hz = center_freq_hz;
    c.nof_tx_ports   = sc.nof_ports;
    return (variant == 3 ? create_pdxch_processor_factory_gpu(group) : create_pdxch_processor_factory_gpu(0))->create(c);
  }
  ofdm_modulator_configuration mc{static_cast<unsigned>(sc.numerology), static_cast<unsigned>(sc.bw_rb),
                                  static_cast<unsigned>(sc.dft_size), sc.cp, 1.0F, center_freq_hz};
  std::unique_ptr<ofdm_symbol_modulator> mod;
  if (variant == 0) {
    ofdm_modulator_common_configuration common;
    common.dft = std::make_unique<dft_processor_generic_impl>(
        dft_processor::configuration{static_cast<unsigned>(sc.dft_size), dft_processor::direction::INVERSE});
    mod = std::make_unique<ofdm_symbol_modulator_impl>(common, mc);
  } else {
    mod = create_ofdm_modulator_factory_gpu(0)->create_ofdm_symbol_modulator(mc);
  }
  pdxch_processor_impl::configuration pc{sc.cp, static_cast<unsigned>(sc.nof_ports), 16};
  return std::make_unique<pdxch_processor_impl>(std::move(mod), pc);
}

std::unique_ptr<puxch_processor> make_puxch(int                                            variant,
                                            int                                            max_in_flight,
                                            const scenario&                                sc,
                                            double                                         center_freq_hz,
                                            const std::shared_ptr<lower_phy_sector_group>& group)
{
  if (variant >= 2) {
    puxch_processor_configuration c;
    c.cp                = sc.cp;
    c.scs               = sc.scs();
    c.srate             = sampling_rate::from_Hz(sc.srate());
    c.bandwidth_rb      = sc.bw_rb;
    c.dft_window_offset = sc.dft_window_offset;
    c.center_freq_Hz    = center_freq_hz;
    c.nof_rx_ports      = sc.nof_ports;
    const unsigned f    = static_cast<unsigned>(max_in_flight);
    return (variant == 3 ? create_puxch_processor_factory_gpu(group, f) : create_puxch_processor_factory_gpu(0, f))
        ->create(c);
  }
  // puxch_processor_factory_sw::create (puxch_processor_factories.cpp:41-57).
  const unsigned woff = static_cast<unsigned>(static_cast<float>(sc.cp.get_length(1, sc.scs()).to_samples(sc.srate())) *
                                              sc.dft_window_offset);
  ofdm_demodulator_configuration dc{static_cast<unsigned>(sc.numerology), static_cast<unsigned>(sc.bw_rb),
                                    static_cast<unsigned>(sc.dft_size), sc.cp, woff,
                                    1.0F / std::sqrt(static_cast<float>(sc.bw_rb * 12)), center_freq_hz};
  std::unique_ptr<ofdm_symbol_demodulator> demod;
  if (variant == 0) {
    ofdm_demodulator_common_configuration common;
    common.dft = std::make_unique<dft_processor_generic_impl>(
        dft_processor::configuration{static_cast<unsigned>(sc.dft_size), dft_processor::direction::DIRECT});
    demod = std::make_unique<ofdm_symbol_demodulator_impl>(common, dc);
  } else {
    demod = create_ofdm_demodulator_factory_gpu(0)->create_ofdm_symbol_demodulator(dc);
  }
  puxch_processor_impl::configuration pc{sc.cp, static_cast<unsigned>(sc.nof_ports), 16};
  return std::make_unique<puxch_processor_impl>(std::move(demod), pc);
}

/// A grid pool holding the scenario's DL grids (port_mask bit p clear: port p stays empty).
/// Variants 4 and 5: the GPU processor of a two-sector group in which another sector registered first (the group takes
/// its launch parameters and buffer sizes from the first sector's plans). 4: that sector was removed again (its processor
/// and plans destroyed) before the tested one runs; 5: it stays, with the other cyclic prefix (at 60 kHz: the same
/// slot length, 12 instead of 14 symbols: a normal-CP sector has more jobs per slot than the group's job table holds per
/// entry and must run alone). The first sector is returned (nullptr for variant 4).
template <typename Proc, typename Make>
std::unique_ptr<Proc> group_prelude(int variant, const scenario& sc, double center_freq_hz,
                                    std::shared_ptr<lower_phy_sector_group>& group, Make make)
{
  lower_phy_group_configuration gc;
  gc.device      = 0;
  gc.nof_sectors = 2;
  group          = create_lower_phy_sector_group(gc);
  scenario other = sc;
  if (variant == 5) {
    other.cp = sc.cp == cyclic_prefix::NORMAL ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL;
  }
  std::unique_ptr<Proc> first = make(other, center_freq_hz + 1e7);
  if (variant == 4) {
    first.reset();
  }
  return first;
}

void fill_pool(harness_pool& pool, const scenario& sc, int nof_grids, const uint16_t* grids, const uint32_t* port_mask)
{
  const unsigned nsymb = sc.nsymb();
  const unsigned nsc   = sc.nsc();
  for (int g = 0; g < nof_grids; ++g) {
    resource_grid_writer& w = pool.get(g).get_writer();
    for (int p = 0; p < sc.nof_ports; ++p) {
      if (((port_mask[g] >> p) & 1U) == 0) {
        continue;
      }
      for (unsigned l = 0; l != nsymb; ++l) {
        const auto* row =
            reinterpret_cast<const cbf16_t*>(grids + 2 * ((static_cast<size_t>(g) * sc.nof_ports + p) * nsymb + l) * nsc);
        w.put(p, l, 0, 1, span<const cbf16_t>(row, nsc));
      }
    }
  }
}

/// Real-time pacing of a script: symbol i of the script may start at start + i x period (the radio delivers / wants a
/// symbol every period). Lag statistics: the latest a symbol started behind its time, the lag of the last symbol (a
/// sector that cannot keep up falls further behind symbol after symbol; one that can recovers from a hiccup) and the
/// symbols that started more than one slot behind. period 0: free-running.
struct pacer {
  using clock = std::chrono::steady_clock;
  clock::time_point start;
  clock::duration   period{0};
  clock::duration   slot{0};
  double            max_lag   = 0;
  double            final_lag = 0;
  long              late      = 0;
  long              i         = 0;
  clock::time_point call;            ///< start of the current process_symbol call
  double            max_call   = 0;  ///< longest process_symbol call (s)
  long              calls_over = 0;  ///< calls longer than one symbol duration

  void done()
  {
    if (period.count() == 0) {
      return;
    }
    const auto d = clock::now() - call;
    max_call     = std::max(max_call, std::chrono::duration<double>(d).count());
    calls_over += d > period ? 1 : 0;
  }

  void next()
  {
    if (period.count() == 0) {
      return;
    }
    const clock::time_point due = start + period * i++;
    clock::time_point       now = clock::now();
    if (now < due) {
      // Sleep (the thread of a radio unit blocks on its baseband device): spinning sectors would take the CPUs the
      // processors need. The thread's timer slack is 1 us (set_timer_slack), so the wake-up lands within microseconds.
      std::this_thread::sleep_until(due);
      final_lag = 0;
    } else {
      final_lag = std::chrono::duration<double>(now - due).count();
      max_lag   = std::max(max_lag, final_lag);
      late += (now - due) > slot ? 1 : 0;
    }
    call = clock::now();
  }
};

/// The DL script (see ref_lower_pdxch_run). Returns the number of samples produced, -1 when they overflow samples_cap.
long run_pdxch_script(pdxch_processor&  proc,
                      harness_pool&     pool,
                      const scenario&   sc,
                      int               nof_events,
                      const int*        events,
                      float*            samples_out,
                      long              samples_cap,
                      uint8_t*          processed_out,
                      pacer*            pace = nullptr)
{
  long        pos   = 0;
  size_t      nflag = 0;
  span_writer buf;
  for (int e = 0; e < nof_events; ++e) {
    const int*       ev = events + 4 * e;
    const slot_point slot(static_cast<uint32_t>(sc.numerology), static_cast<uint32_t>(ev[1]));
    if (ev[0] == 0) {
      proc.get_request_handler().handle_request(pool.grab(static_cast<unsigned>(ev[2])), {slot, 0});
      continue;
    }
    for (int l = ev[2]; l < ev[3]; ++l) {
      const unsigned n    = symbol_size(sc.numerology, sc.dft_size, sc.cp, slot.subframe_slot_index() * sc.nsymb() + l);
      const long     need = static_cast<long>(n) * sc.nof_ports;
      long           at   = pos;
      if (samples_cap < 0) {
        if (need > -samples_cap) {
          return -1;
        }
        at = (pos % -samples_cap) + need > -samples_cap ? 0 : pos % -samples_cap;
      } else if (pos + need > samples_cap) {
        return -1;
      }
      buf.ch.clear();
      for (int p = 0; p < sc.nof_ports; ++p) {
        auto* dst = reinterpret_cast<cf_t*>(samples_out) + at + static_cast<long>(p) * n;
        if (samples_cap >= 0) {
          std::fill(dst, dst + n, cf_t(1e30F, 1e30F));
        }
        buf.ch.emplace_back(dst, n);
      }
      pdxch_processor_baseband::symbol_context ctx{slot, 0, static_cast<unsigned>(l)};
      if (pace != nullptr) {
        pace->next();
      }
      processed_out[nflag++] = proc.get_baseband().process_symbol(buf, ctx) ? 1 : 0;
      if (pace != nullptr) {
        pace->done();
      }
      pos += need;
    }
  }
  return pos;
}

/// The UL script (see ref_lower_puxch_run).
void run_puxch_script(puxch_processor& proc,
                      harness_pool&    pool,
                      const scenario&  sc,
                      int              nof_events,
                      const int*       events,
                      const float*     samples_in,
                      uint8_t*         processed_out,
                      pacer*           pace = nullptr)
{
  long        pos   = 0;
  size_t      nflag = 0;
  span_reader buf;
  for (int e = 0; e < nof_events; ++e) {
    const int*       ev = events + 4 * e;
    const slot_point slot(static_cast<uint32_t>(sc.numerology), static_cast<uint32_t>(ev[1]));
    if (ev[0] == 0) {
      proc.get_request_handler().handle_request(pool.grab(static_cast<unsigned>(ev[2])), {slot, 0});
      continue;
    }
    for (int l = ev[2]; l < ev[3]; ++l) {
      const unsigned n = symbol_size(sc.numerology, sc.dft_size, sc.cp, slot.subframe_slot_index() * sc.nsymb() + l);
      buf.ch.clear();
      for (int p = 0; p < sc.nof_ports; ++p) {
        buf.ch.emplace_back(reinterpret_cast<const cf_t*>(samples_in) + pos + static_cast<long>(p) * n, n);
      }
      lower_phy_rx_symbol_context ctx{slot, 0, static_cast<unsigned>(l)};
      if (pace != nullptr) {
        pace->next();
      }
      processed_out[nflag++] = proc.get_baseband().process_symbol(buf, ctx) ? 1 : 0;
      if (pace != nullptr) {
        pace->done();
      }
      pos += static_cast<long>(n) * sc.nof_ports;
    }
  }
}

/// Final grid contents (nof_grids x ports x nsymb x nsc bf16 pairs).
void dump_pool(harness_pool& pool, const scenario& sc, int nof_grids, uint16_t* grids_out)
{
  const unsigned nsymb = sc.nsymb();
  const unsigned nsc   = sc.nsc();
  for (int g = 0; g < nof_grids; ++g) {
    const resource_grid_reader& r = pool.get(g).get_reader();
    for (int p = 0; p < sc.nof_ports; ++p) {
      for (unsigned l = 0; l != nsymb; ++l) {
        std::memcpy(grids_out + 2 * ((static_cast<size_t>(g) * sc.nof_ports + p) * nsymb + l) * nsc,
                    r.get_view(p, l).data(), nsc * sizeof(cbf16_t));
      }
    }
  }
}

/// All sector threads meet here between the DL and UL scripts.
class barrier
{
public:
  explicit barrier(unsigned n_) : n(n_) {}
  void wait()
  {
    std::unique_lock<std::mutex> lock(mtx);
    const unsigned               gen = generation;
    if (++count == n) {
      count = 0;
      ++generation;
      cv.notify_all();
      return;
    }
    cv.wait(lock, [&]() { return generation != gen; });
  }

private:
  std::mutex              mtx;
  std::condition_variable cv;
  unsigned                n;
  unsigned                count      = 0;
  unsigned                generation = 0;
};

} // namespace

extern "C" {

/// PDxCH scenario (variants 0-2 as make_pdxch, 4-5 as group_prelude). grids: nof_grids x ports x nsymb x nsc bf16 pairs; port_mask[g]: bit p set = port p of grid g is
/// written (the others stay empty). events: nof_events x {kind, system slot, a, b}: kind 0 = handle_request(grid a),
/// kind 1 = process_symbol for symbols [a, b) of the slot. Outputs, in event order: the samples of every processed
/// symbol and port (sentinel 1e30 where the processor leaves the buffer untouched), one return flag per symbol, the
/// late-request slots. Returns the number of samples written (< 0 on error). Benchmark mode, samples_cap < 0: the
/// samples go round a ring of -samples_cap samples (a radio's reused baseband buffer: no page faults on fresh memory, no
/// sentinel fill), the return value still counts every sample.
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
  const scenario sc{numerology, bw_rb, dft_size, cp_extended ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL, 0.0F,
                    nof_ports};
  harness_pool   pool(nof_grids, nof_ports, sc.nsymb(), sc.nsc());
  fill_pool(pool, sc, nof_grids, grids, port_mask);
  std::shared_ptr<lower_phy_sector_group> group;
  std::unique_ptr<pdxch_processor>        first;
  if (variant >= 4) {
    first = group_prelude<pdxch_processor>(variant, sc, center_freq_hz, group, [&](const scenario& o, double f) {
      return make_pdxch(3, o, f, group);
    });
  }
  std::unique_ptr<pdxch_processor> proc = make_pdxch(variant >= 4 ? 3 : variant, sc, center_freq_hz, group);
  pdxch_recorder                   rec;
  proc->connect(rec);
  const long pos = run_pdxch_script(*proc, pool, sc, nof_events, events, samples_out, samples_cap, processed_out);
  *nof_late      = static_cast<int>(rec.late.size());
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
  const scenario sc{numerology,        bw_rb,    dft_size, cp_extended ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL,
                    dft_window_offset, nof_ports};
  harness_pool   pool(nof_grids, nof_ports, sc.nsymb(), sc.nsc());
  std::shared_ptr<lower_phy_sector_group> group;
  std::unique_ptr<puxch_processor>        first;
  if (variant >= 4) {
    first = group_prelude<puxch_processor>(variant, sc, center_freq_hz, group, [&](const scenario& o, double f) {
      return make_puxch(3, max_in_flight, o, f, group);
    });
  }
  std::unique_ptr<puxch_processor> proc =
      make_puxch(variant >= 4 ? 3 : variant, max_in_flight, sc, center_freq_hz, group);
  puxch_recorder                   rec;
  proc->connect(rec);
  run_puxch_script(*proc, pool, sc, nof_events, events, samples_in, processed_out);
  proc.reset();
  dump_pool(pool, sc, nof_grids, grids_out);
  *nof_rx   = static_cast<int>(rec.rx.size() / 2);
  *nof_late = static_cast<int>(rec.late.size());
  std::copy(rec.rx.begin(), rec.rx.end(), rx_out);
  std::copy(rec.late.begin(), rec.late.end(), late_out);
  return 0;
}

/// Several sectors at once, as the reference's radio unit runs them (one lower-PHY sector per cell, each driven by its
/// own thread: lib/ru/generic/ru_factory_generic_impl.cpp:75-90): nof_sectors threads, sector k with carrier
/// center_freq_hz[k], its own grids (dl_grids + k * grid block, dl_port_mask + k * nof_grids) and UL samples
/// (ul_samples + k * ul_stride complex samples), first all run the DL script together, then (after a barrier) the UL
/// script. Variant 3: the sectors' GPU processors come from one lower_phy_sector_group (window_us: its gather windows,
/// 0 = defaults). Outputs per sector k at k x the stride of one sector: DL samples (dl_cap < 0: a ring per sector, as
/// ref_lower_pdxch_run), DL and UL return flags, UL grids, UL notifications (nof_rx[k] pairs) and late slots
/// (nof_late[k], DL then UL); seconds[2k], seconds[2k+1]: the sector's DL and UL script wall time. group_counts (8
/// values, variant 3): lower_phy_group_counters in declaration order. paced != 0: every sector runs at the radio's pace, one symbol per
/// symbol duration (1 ms / symbols per subframe) from a common start; lag[10k .. 10k+9]: sector k's DL and UL largest
/// lag behind that pace (s), DL and UL lag at the last symbol (s), DL and UL fraction of symbols started more than one
/// slot behind, DL and UL longest process_symbol call (s), DL and UL fraction of calls longer than a symbol. Returns 0, -1 on a sample overflow.
int ref_lower_sectors_run(int             variant,
                          int             max_in_flight,
                          int             nof_sectors,
                          int             numerology,
                          int             bw_rb,
                          int             dft_size,
                          int             cp_extended,
                          float           dft_window_offset,
                          const double*   center_freq_hz,
                          int             nof_ports,
                          int             nof_grids,
                          int             window_us,
                          const uint16_t* dl_grids,
                          const uint32_t* dl_port_mask,
                          int             nof_dl_events,
                          const int*      dl_events,
                          float*          dl_samples_out,
                          long            dl_cap,
                          uint8_t*        dl_processed,
                          int             nof_ul_events,
                          const int*      ul_events,
                          const float*    ul_samples,
                          long            ul_stride,
                          uint16_t*       ul_grids_out,
                          uint8_t*        ul_processed,
                          int*            rx_out,
                          int*            nof_rx,
                          int*            late_out,
                          int*            nof_late,
                          double*         seconds,
                          uint64_t*       group_counts,
                          int             paced,
                          double*         lag)
{
  const scenario sc{numerology,        bw_rb,    dft_size, cp_extended ? cyclic_prefix::EXTENDED : cyclic_prefix::NORMAL,
                    dft_window_offset, nof_ports};
  const size_t   grid_block = static_cast<size_t>(nof_grids) * nof_ports * sc.nsymb() * sc.nsc() * 2;
  int            n_dl_proc = 0, n_ul_proc = 0;
  for (int e = 0; e < nof_dl_events; ++e) {
    n_dl_proc += dl_events[4 * e] == 1 ? dl_events[4 * e + 3] - dl_events[4 * e + 2] : 0;
  }
  for (int e = 0; e < nof_ul_events; ++e) {
    n_ul_proc += ul_events[4 * e] == 1 ? ul_events[4 * e + 3] - ul_events[4 * e + 2] : 0;
  }
  const long dl_stride   = 2 * std::labs(dl_cap);
  const int  late_stride = nof_dl_events + nof_ul_events + 1;

  // Variant 6: the sector group (variant 3) with the UL grids mapped for the devices, so that the group demodulates
  // into them directly (srsgpu_ofdm_jobs_execute_direct) instead of staging and copying the rows.
  const bool mapped_ul = variant == 6;
  if (mapped_ul) {
    variant = 3;
  }
  std::shared_ptr<lower_phy_sector_group> group;
  if (variant == 3) {
    lower_phy_group_configuration gc;
    gc.device      = 0;
    gc.nof_sectors = static_cast<unsigned>(nof_sectors);
    if (window_us > 0) {
      gc.ul_window_us = static_cast<unsigned>(window_us);
      gc.dl_window_us = static_cast<unsigned>(window_us);
    }
    group = create_lower_phy_sector_group(gc);
  }
  std::vector<std::unique_ptr<harness_pool>>    dl_pools, ul_pools;
  std::vector<std::unique_ptr<pdxch_processor>> dl;
  std::vector<std::unique_ptr<puxch_processor>> ul;
  std::vector<pdxch_recorder>                   dl_rec(nof_sectors);
  std::vector<puxch_recorder>                   ul_rec(nof_sectors);
  for (int k = 0; k < nof_sectors; ++k) {
    dl_pools.emplace_back(std::make_unique<harness_pool>(nof_grids, nof_ports, sc.nsymb(), sc.nsc()));
    fill_pool(*dl_pools.back(), sc, nof_grids, dl_grids + k * grid_block, dl_port_mask + k * nof_grids);
    ul_pools.emplace_back(std::make_unique<harness_pool>(nof_grids, nof_ports, sc.nsymb(), sc.nsc()));
    if (mapped_ul) {
      ul_pools.back()->map_grids(true);
    }
    dl.push_back(make_pdxch(variant, sc, center_freq_hz[k], group));
    dl.back()->connect(dl_rec[k]);
    ul.push_back(make_puxch(variant, max_in_flight, sc, center_freq_hz[k], group));
    ul.back()->connect(ul_rec[k]);
  }
  barrier                  meet(static_cast<unsigned>(nof_sectors));
  std::vector<long>        produced(nof_sectors, 0);
  std::vector<std::thread> threads;
  using clock = std::chrono::steady_clock;
  const clock::duration period =
      paced != 0 ? std::chrono::duration_cast<clock::duration>(std::chrono::nanoseconds(
                       1000000 / (sc.nsymb() * get_nof_slots_per_subframe(sc.scs()))))
                 : clock::duration(0);
  std::array<clock::time_point, 2> start;
  for (int k = 0; k < nof_sectors; ++k) {
    threads.emplace_back([&, k]() {
      if (period.count() != 0) {
        (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);  // 1 us timer slack: paced sleeps wake on time
      }
      pacer pdl, pul;
      pdl.period = pul.period = period;
      pdl.slot = pul.slot = period * static_cast<long>(sc.nsymb());
      if (k == 0) {
        start[0] = clock::now() + std::chrono::milliseconds(1);
      }
      meet.wait();
      pdl.start   = start[0];
      auto t0     = clock::now();
      produced[k] = run_pdxch_script(*dl[k], *dl_pools[k], sc, nof_dl_events, dl_events, dl_samples_out + k * dl_stride,
                                     dl_cap, dl_processed + static_cast<size_t>(k) * n_dl_proc, &pdl);
      seconds[2 * k] = std::chrono::duration<double>(clock::now() - t0).count();
      meet.wait();
      if (k == 0) {
        start[1] = clock::now() + std::chrono::milliseconds(1);
      }
      meet.wait();
      pul.start = start[1];
      t0        = clock::now();
      run_puxch_script(*ul[k], *ul_pools[k], sc, nof_ul_events, ul_events, ul_samples + 2 * k * ul_stride,
                       ul_processed + static_cast<size_t>(k) * n_ul_proc, &pul);
      seconds[2 * k + 1] = std::chrono::duration<double>(clock::now() - t0).count();
      const double nd = static_cast<double>(std::max(1L, pdl.i)), nu = static_cast<double>(std::max(1L, pul.i));
      const double v[10] = {pdl.max_lag,  pul.max_lag,  pdl.final_lag,       pul.final_lag,       pdl.late / nd,
                            pul.late / nu, pdl.max_call, pul.max_call, pdl.calls_over / nd, pul.calls_over / nu};
      std::copy(v, v + 10, lag + 10 * k);
    });
  }
  for (std::thread& t : threads) {
    t.join();
  }
  dl.clear();
  ul.clear();
  for (int k = 0; k < nof_sectors; ++k) {
    if (mapped_ul) {
      ul_pools[k]->map_grids(false);
    }
    dump_pool(*ul_pools[k], sc, nof_grids, ul_grids_out + k * grid_block);
    nof_rx[k] = static_cast<int>(ul_rec[k].rx.size() / 2);
    std::copy(ul_rec[k].rx.begin(), ul_rec[k].rx.end(), rx_out + static_cast<size_t>(k) * 2 * n_ul_proc);
    int* late = late_out + static_cast<size_t>(k) * late_stride;
    late      = std::copy(dl_rec[k].late.begin(), dl_rec[k].late.end(), late);
    std::copy(ul_rec[k].late.begin(), ul_rec[k].late.end(), late);
    nof_late[k] = static_cast<int>(dl_rec[k].late.size() + ul_rec[k].late.size());
  }
  if (group) {
    const lower_phy_group_counters c = get_lower_phy_group_counters(*group);
    const uint64_t v[8] = {c.ul_launches, c.ul_batched, c.ul_alone, c.ul_windowed,
                           c.dl_launches, c.dl_batched, c.dl_alone, c.dl_windowed};
    std::copy(v, v + 8, group_counts);
  }
  for (long p : produced) {
    if (p < 0) {
      return -1;
    }
  }
  return 0;
}

} // extern "C"
