// Reference-side bindings of the lower PHY's baseband processors (the file a srsRAN maintainer adds next to
// lib/phy/lower/processors/): srsran::pdxch_processor and srsran::puxch_processor
// (include/srsran/phy/lower/processors/downlink/pdxch/pdxch_processor.h, uplink/puxch/puxch_processor.h) created by
// pdxch_processor_factory / puxch_processor_factory implementations over the srsgpu C ABI, plus GPU symbol-granularity
// OFDM objects for the generic factories (integration/ofdm_gpu.cpp).
//
// These are the objects du_low's radio unit drives (lib/ru/generic/lower_phy/lower_phy_factory.cpp:70/:84 builds them
// with create_pdxch_processor_factory_sw / create_puxch_processor_factory_sw). The reference processors
// (pdxch_processor_impl.cpp:45-115, puxch_processor_impl.cpp:30-103) call an OFDM symbol (de)modulator once per port
// and symbol from the real-time baseband thread. On the GPU a symbol of one port is far too small a launch, so:
//
//  * PDxCH (downlink): the whole slot is modulated when the upper PHY hands the grid over (handle_request): every
//    non-empty port's 14 grid rows go up, one launch modulates all ports and symbols, the samples come back into a
//    pinned buffer of the request, all asynchronously on the processor's stream. process_symbol() only waits for that
//    slot's event at its first symbol (long finished: requests arrive max_processing_delay slots ahead) and copies
//    the symbol's CP + N samples of every port. The request bookkeeping (one entry per slot modulo 16, the late-request
//    notifications, empty grids discarded) is the reference's.
//
//  * PUxCH (uplink): the symbols arrive one by one. process_symbol() stages the symbol's samples of every port into
//    pinned memory and launches its demodulation (one plan per symbol of the subframe, all ports) without waiting.
//    Symbols whose demodulation has finished are written into the request's grid and notified (on_rx_symbol) in
//    order; at most `max_symbols_in_flight` are outstanding (0: every symbol is demodulated and notified before
//    process_symbol returns, the reference's timing), and the slot's last symbol drains everything, so every symbol of
//    a slot is notified, in order, before the slot's last process_symbol() returns.
#include "signal_chain_gpu.h"

#include "gpu_staging.h"
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
#include "srsran/phy/support/shared_resource_grid.h"

#include <array>
#include <atomic>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace srsran {

namespace {

/// Requests indexed by slot modulo 16 (resource_grid_request_pool.h:40-83): exchange() swaps an entry under its lock.
template <typename Payload>
class request_ring
{
public:
  struct request {
    slot_point slot;
    Payload    payload;
  };

  request exchange(request r)
  {
    entry&                      e = entries[r.slot.system_slot() % SIZE];
    std::lock_guard<std::mutex> lock(e.mtx);
    request                     old = std::move(e.req);
    e.req                           = std::move(r);
    return old;
  }

private:
  static constexpr unsigned SIZE = 16;
  struct entry {
    request    req = {slot_point(), Payload()};
    std::mutex mtx;
  };
  std::array<entry, SIZE> entries;
};

/// Cyclic prefix + DFT samples of every symbol of a subframe and where each starts within its slot.
struct symbol_geometry {
  symbol_geometry(subcarrier_spacing scs, cyclic_prefix cp, unsigned dft_size) :
    nsymb(get_nsymb_per_slot(cp)), nslot(get_nof_slots_per_subframe(scs))
  {
    const double srate = static_cast<double>(dft_size) * scs_to_khz(scs) * 1000.0;
    size.resize(nsymb * nslot);
    start.resize(nsymb * nslot);
    for (unsigned s = 0; s != nsymb * nslot; ++s) {
      size[s]  = cp.get_length(s, scs).to_samples(srate) + dft_size;
      start[s] = (s % nsymb == 0) ? 0 : start[s - 1] + size[s - 1];
    }
  }
  unsigned slot_size(unsigned slot) const { return start[slot * nsymb + nsymb - 1] + size[slot * nsymb + nsymb - 1]; }

  unsigned              nsymb;
  unsigned              nslot;
  std::vector<unsigned> size;   ///< CP + N of symbol s of the subframe.
  std::vector<unsigned> start;  ///< First sample of symbol s within its slot.
};

srsgpu_ofdm_config ofdm_config(subcarrier_spacing scs, cyclic_prefix cp, unsigned bw_rb, unsigned dft_size,
                               unsigned window_offset, float scale, double center_freq_hz)
{
  srsgpu_ofdm_config c;
  std::memset(&c, 0, sizeof(c));
  c.numerology                = to_numerology_value(scs);
  c.bw_rb                     = bw_rb;
  c.dft_size                  = dft_size;
  c.cp_extended               = (cp == cyclic_prefix::EXTENDED) ? 1 : 0;
  c.nof_samples_window_offset = window_offset;
  c.scale                     = scale;
  c.center_freq_hz            = center_freq_hz;
  return c;
}

// ---------------------------------------------------------------------------------------------------------------------
// PDxCH
// ---------------------------------------------------------------------------------------------------------------------

class pdxch_processor_gpu : public pdxch_processor,
                            private pdxch_processor_baseband,
                            private pdxch_processor_request_handler
{
  static constexpr const char* WHO = "pdxch_processor_gpu";

  /// One slot's modulation: staging, result and completion event. Recycled through the free list.
  struct job {
    explicit job(const char* who) : grid(who), samples(who) {}
    ~job()
    {
      drop_graphs();
      if (done != nullptr) {
        (void)hipEventDestroy(done);
      }
    }
    void drop_graphs()
    {
      for (hipGraphExec_t& g : graphs) {
        if (g != nullptr) {
          (void)hipGraphExecDestroy(g);
          g = nullptr;
        }
      }
    }
    gpu::staged_buffer grid;
    gpu::staged_buffer samples;
    hipEvent_t         done = nullptr;
    /// Per slot of the subframe: upload + modulation + download captured over this job's buffers (graph_buffers).
    std::vector<hipGraphExec_t> graphs;
    const void*                 graph_buffers[2] = {nullptr, nullptr};
    std::vector<bool>  port_empty;
    unsigned           subframe_slot = 0;
    bool               launched      = false;  ///< false: the request's grid was empty (nothing to transmit).
  };
  using job_ptr = std::unique_ptr<job>;

public:
  pdxch_processor_gpu(std::shared_ptr<srsgpu_context> owner_, const pdxch_processor_configuration& config) :
    owner(std::move(owner_)),
    ctx(owner.get()),
    stream(ctx, WHO),
    geo(config.scs, config.cp, config.srate.get_dft_size(config.scs)),
    nof_ports(config.nof_tx_ports),
    nsc(config.bandwidth_rb * NRE)
  {
    gpu::device_scope dev(ctx, WHO);
    // pdxch_processor_factory_sw: modulator scaling 1 (pdxch_processor_factories.cpp:59).
    const srsgpu_ofdm_config c = ofdm_config(config.scs, config.cp, config.bandwidth_rb,
                                             config.srate.get_dft_size(config.scs), 0, 1.0F, config.center_freq_Hz);
    for (unsigned s = 0; s != geo.nslot; ++s) {
      srsgpu_ofdm_plan* p = nullptr;
      gpu::srsgpu_check(srsgpu_ofdm_modulator_plan_create(ctx, &c, 1, nof_ports, &s, &p), WHO);
      plans.push_back(p);
    }
  }

  ~pdxch_processor_gpu() override
  {
    (void)hipStreamSynchronize(stream.get());
    for (srsgpu_ofdm_plan* p : plans) {
      srsgpu_ofdm_plan_destroy(p);
    }
  }

  void                             connect(pdxch_processor_notifier& n) override { notifier = &n; }
  void                             stop() override { stopped = true; }
  pdxch_processor_request_handler& get_request_handler() override { return *this; }
  pdxch_processor_baseband&        get_baseband() override { return *this; }

private:
  bool process_symbol(baseband_gateway_buffer_writer& samples, const symbol_context& context) override
  {
    srsran_assert(notifier != nullptr, "Notifier has not been connected.");
    if (context.slot != current_slot) {
      current_slot = context.slot;
      recycle(std::move(current));
      auto r = requests.exchange({context.slot, job_ptr()});
      if (!r.payload) {
        return false;  // no request for this slot
      }
      if (current_slot != r.slot) {
        resource_grid_context late;
        late.slot   = r.slot;
        late.sector = context.sector;
        notifier->on_pdxch_request_late(late);
        recycle(std::move(r.payload));
        return false;
      }
      if (!r.payload->launched) {
        recycle(std::move(r.payload));  // nothing to transmit (empty grid)
        return false;
      }
      current = std::move(r.payload);
      gpu::device_scope dev(ctx, WHO);
      gpu::hip_check(hipEventSynchronize(current->done), WHO, "modulation");
    }
    if (!current) {
      return false;
    }
    const unsigned s     = context.slot.subframe_slot_index() * geo.nsymb + context.symbol;
    const unsigned n     = geo.size[s];
    const size_t   slotn = geo.slot_size(current->subframe_slot);
    for (unsigned p = 0; p != nof_ports; ++p) {
      span<cf_t> out = samples.get_channel_buffer(p);
      srsran_assert(out.size() == n, "The output buffer size ({}) does not match the symbol size ({}).", out.size(), n);
      if (current->port_empty[p]) {
        std::fill(out.begin(), out.end(), cf_t());  // ofdm_modulator_impl.cpp:77: an empty port transmits zeros
      } else {
        std::memcpy(out.data(), current->samples.host<cf_t>((p * slotn + geo.start[s]) * sizeof(cf_t)), n * sizeof(cf_t));
      }
    }
    return true;
  }

  void handle_request(const shared_resource_grid& grid, const resource_grid_context& context) override
  {
    if (stopped) {
      return;
    }
    srsran_assert(notifier != nullptr, "Notifier has not been connected.");
    job_ptr j = acquire();
    j->launched = false;
    const resource_grid_reader& reader = grid.get_reader();
    if (!reader.is_empty()) {
      launch(*j, reader, context.slot.subframe_slot_index());
    }
    auto old = requests.exchange({context.slot, std::move(j)});
    if (old.payload) {
      resource_grid_context late;
      late.slot   = old.slot;
      late.sector = context.sector;
      notifier->on_pdxch_request_late(late);
      recycle(std::move(old.payload));
    }
  }

  /// Stages the grid's non-empty ports and modulates the whole slot on the processor's stream (no waiting).
  void launch(job& j, const resource_grid_reader& reader, unsigned subframe_slot)
  {
    gpu::device_scope           dev(ctx, WHO);
    std::lock_guard<std::mutex> lock(launch_mtx);
    const size_t                row   = static_cast<size_t>(nsc) * sizeof(uint32_t);
    const size_t                slotn = geo.slot_size(subframe_slot);
    hipStream_t                 s     = stream.get();
    j.grid.reserve(nof_ports * geo.nsymb * row);
    j.samples.reserve(nof_ports * slotn * sizeof(cf_t));
    if (j.done == nullptr) {
      gpu::hip_check(hipEventCreateWithFlags(&j.done, hipEventDisableTiming), WHO, "event");
    }
    j.port_empty.assign(nof_ports, false);
    for (unsigned p = 0; p != nof_ports; ++p) {
      j.port_empty[p] = reader.is_empty(p);
      if (j.port_empty[p]) {
        continue;  // its rows stay stale on the device; the port's output is zeros
      }
      for (unsigned l = 0; l != geo.nsymb; ++l) {
        std::memcpy(j.grid.host((p * geo.nsymb + l) * row), reader.get_view(p, l).data(), row);
      }
    }
    // Upload, modulation and download as one captured graph per (job, slot of the subframe), built on first use.
    if (j.graph_buffers[0] != j.grid.dev() || j.graph_buffers[1] != j.samples.dev()) {
      j.drop_graphs();  // the job's buffers grew: the graphs captured their old addresses
      j.graph_buffers[0] = j.grid.dev();
      j.graph_buffers[1] = j.samples.dev();
    }
    j.graphs.resize(plans.size(), nullptr);
    hipGraphExec_t& exec = j.graphs[subframe_slot];
    if (exec == nullptr) {
      std::lock_guard<std::recursive_mutex> setup(gpu::hip_setup_mutex());
      gpu::hip_check(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed), WHO, "begin capture");
      hipGraph_t graph = nullptr;
      try {
        j.grid.upload(0, nof_ports * geo.nsymb * row, s);
        gpu::srsgpu_check(srsgpu_ofdm_modulator_plan_execute(plans[subframe_slot], j.grid.dev<uint32_t>(),
                                                             j.samples.dev<float>(), s),
                          WHO);
        j.samples.download(0, nof_ports * slotn * sizeof(cf_t), s);
      } catch (...) {
        (void)hipStreamEndCapture(s, &graph);
        (void)hipGraphDestroy(graph);
        throw;
      }
      gpu::hip_check(hipStreamEndCapture(s, &graph), WHO, "end capture");
      const hipError_t r = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      gpu::hip_check(r, WHO, "graph instantiate");
    }
    gpu::hip_check(hipGraphLaunch(exec, s), WHO, "graph launch");
    gpu::hip_check(hipEventRecord(j.done, s), WHO, "event");
    j.subframe_slot = subframe_slot;
    j.launched      = true;
  }

  /// A job from the free list (its previous transfers finished before its buffers are rewritten) or a new one.
  job_ptr acquire()
  {
    job_ptr j;
    {
      std::lock_guard<std::mutex> lock(free_mtx);
      if (!free_jobs.empty()) {
        j = std::move(free_jobs.back());
        free_jobs.pop_back();
      }
    }
    if (!j) {
      return std::make_unique<job>(WHO);
    }
    if (j->launched) {
      gpu::device_scope dev(ctx, WHO);
      gpu::hip_check(hipEventSynchronize(j->done), WHO, "job reuse");
    }
    return j;
  }

  void recycle(job_ptr j)
  {
    if (j) {
      std::lock_guard<std::mutex> lock(free_mtx);
      free_jobs.push_back(std::move(j));
    }
  }

  std::shared_ptr<srsgpu_context> owner;
  srsgpu_context*                 ctx;
  gpu::owned_stream               stream;
  symbol_geometry                 geo;
  unsigned                        nof_ports;
  unsigned                        nsc;
  std::vector<srsgpu_ofdm_plan*>  plans;  ///< One whole-slot plan (all ports) per slot of the subframe.
  std::atomic<bool>               stopped  = false;
  pdxch_processor_notifier*       notifier = nullptr;
  slot_point                      current_slot;
  job_ptr                         current;
  request_ring<job_ptr>           requests;
  std::mutex                      launch_mtx;
  std::mutex                      free_mtx;
  std::vector<job_ptr>            free_jobs;
};

// ---------------------------------------------------------------------------------------------------------------------
// PUxCH
// ---------------------------------------------------------------------------------------------------------------------

class puxch_processor_gpu : public puxch_processor,
                            private puxch_processor_baseband,
                            private puxch_processor_request_handler
{
  static constexpr const char* WHO = "puxch_processor_gpu";

  /// Staging of one symbol of the slot (indexed by the symbol within the slot; reused slot after slot).
  struct symbol_stage {
    explicit symbol_stage(const char* who) : in(who), out(who) {}
    ~symbol_stage()
    {
      if (done != nullptr) {
        (void)hipEventDestroy(done);
      }
    }
    gpu::staged_buffer in;
    gpu::staged_buffer out;
    hipEvent_t         done = nullptr;
  };

public:
  puxch_processor_gpu(std::shared_ptr<srsgpu_context> owner_,
                      const puxch_processor_configuration& config,
                      unsigned                             max_symbols_in_flight_) :
    owner(std::move(owner_)),
    ctx(owner.get()),
    stream(ctx, WHO),
    geo(config.scs, config.cp, config.srate.get_dft_size(config.scs)),
    nof_ports(config.nof_rx_ports),
    nsc(config.bandwidth_rb * NRE),
    max_symbols_in_flight(max_symbols_in_flight_)
  {
    gpu::device_scope dev(ctx, WHO);
    const unsigned    N = config.srate.get_dft_size(config.scs);
    // puxch_processor_factory_sw (puxch_processor_factories.cpp:41-57): DFT window offset as a fraction of the CP of
    // symbol 1, scaling 1 / sqrt(subcarriers).
    const unsigned window_offset = static_cast<unsigned>(
        static_cast<float>(config.cp.get_length(1, config.scs).to_samples(config.srate.to_Hz())) *
        config.dft_window_offset);
    const srsgpu_ofdm_config c =
        ofdm_config(config.scs, config.cp, config.bandwidth_rb, N, window_offset,
                    1.0F / std::sqrt(static_cast<float>(config.bandwidth_rb * NRE)), config.center_freq_Hz);
    for (unsigned s = 0; s != geo.nslot; ++s) {
      for (unsigned l = 0; l != geo.nsymb; ++l) {
        srsgpu_ofdm_plan* p = nullptr;
        gpu::srsgpu_check(srsgpu_ofdm_demodulator_symbols_plan_create(ctx, &c, nof_ports, s, l, 1, &p), WHO);
        plans.push_back(p);
      }
    }
    graphs.assign(plans.size(), nullptr);
    unsigned max_size = 0;
    for (unsigned n : geo.size) {
      max_size = std::max(max_size, n);
    }
    for (unsigned l = 0; l != geo.nsymb; ++l) {
      stages.emplace_back(std::make_unique<symbol_stage>(WHO));
      stages.back()->in.reserve(static_cast<size_t>(nof_ports) * max_size * sizeof(cf_t));
      stages.back()->out.reserve(static_cast<size_t>(nof_ports) * nsc * sizeof(uint32_t));
      gpu::hip_check(hipEventCreateWithFlags(&stages.back()->done, hipEventDisableTiming), WHO, "event");
    }
  }

  ~puxch_processor_gpu() override
  {
    (void)hipStreamSynchronize(stream.get());
    for (hipGraphExec_t g : graphs) {
      if (g != nullptr) {
        (void)hipGraphExecDestroy(g);
      }
    }
    for (srsgpu_ofdm_plan* p : plans) {
      srsgpu_ofdm_plan_destroy(p);
    }
  }

  void                             connect(puxch_processor_notifier& n) override { notifier = &n; }
  void                             stop() override { stopped = true; }
  puxch_processor_request_handler& get_request_handler() override { return *this; }
  puxch_processor_baseband&        get_baseband() override { return *this; }

private:
  bool process_symbol(const baseband_gateway_buffer_reader& samples, const lower_phy_rx_symbol_context& context) override
  {
    srsran_assert(notifier != nullptr, "Notifier has not been connected.");
    gpu::device_scope dev(ctx, WHO);
    if (context.slot != current_slot) {
      drain(0);  // a slot left before its last symbol: what was demodulated is still delivered
      current_grid.release();
      current_slot = context.slot;
      auto r       = requests.exchange({context.slot, shared_resource_grid()});
      if (!r.payload) {
        // no request for this slot
      } else if (current_slot != r.slot) {
        resource_grid_context late;
        late.slot   = r.slot;
        late.sector = context.sector;
        notifier->on_puxch_request_late(late);
      } else {
        current_grid = std::move(r.payload);
      }
    }
    if (!current_grid) {
      return false;
    }
    const unsigned l = context.nof_symbols;
    const unsigned s = context.slot.subframe_slot_index() * geo.nsymb + l;
    const unsigned n = geo.size[s];
    symbol_stage&  st = *stages[l];
    hipStream_t    hs = stream.get();
    for (unsigned p = 0; p != nof_ports; ++p) {
      span<const cf_t> in = samples.get_channel_buffer(p);
      srsran_assert(in.size() == n, "The input buffer size ({}) does not match the symbol size ({}).", in.size(), n);
      std::memcpy(st.in.host<cf_t>(static_cast<size_t>(p) * n * sizeof(cf_t)), in.data(), n * sizeof(cf_t));
    }
    // Upload, demodulation and download of this symbol position as one captured graph (built on first use): a
    // symbol costs one launch instead of three dependent queue operations (~9 us apart each).
    hipGraphExec_t& exec = graphs[s];
    if (exec == nullptr) {
      std::lock_guard<std::recursive_mutex> lock(gpu::hip_setup_mutex());
      gpu::hip_check(hipStreamBeginCapture(hs, hipStreamCaptureModeRelaxed), WHO, "begin capture");
      hipGraph_t graph = nullptr;
      try {
        st.in.upload(0, static_cast<size_t>(nof_ports) * n * sizeof(cf_t), hs);
        gpu::srsgpu_check(
            srsgpu_ofdm_demodulator_plan_execute(plans[s], st.in.dev<float>(), st.out.dev<uint32_t>(), hs), WHO);
        st.out.download(0, static_cast<size_t>(nof_ports) * nsc * sizeof(uint32_t), hs);
      } catch (...) {
        (void)hipStreamEndCapture(hs, &graph);
        (void)hipGraphDestroy(graph);
        throw;
      }
      gpu::hip_check(hipStreamEndCapture(hs, &graph), WHO, "end capture");
      const hipError_t r = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      gpu::hip_check(r, WHO, "graph instantiate");
    }
    gpu::hip_check(hipGraphLaunch(exec, hs), WHO, "graph launch");
    gpu::hip_check(hipEventRecord(st.done, hs), WHO, "event");
    pending.push_back({l, context});
    // Deliver what has finished; bound the symbols in flight; the slot's last symbol drains the slot.
    if (l == geo.nsymb - 1) {
      drain(0);
      current_grid.release();
    } else {
      drain(max_symbols_in_flight);
    }
    return true;
  }

  void handle_request(const shared_resource_grid& grid, const resource_grid_context& context) override
  {
    if (stopped) {
      return;
    }
    srsran_assert(notifier != nullptr, "Notifier has not been connected.");
    auto old = requests.exchange({context.slot, grid.copy()});
    if (old.payload) {
      resource_grid_context late;
      late.slot   = old.slot;
      late.sector = context.sector;
      notifier->on_puxch_request_late(late);
    }
  }

  /// Writes the demodulated symbols into the grid and notifies them, oldest first: every finished one, and enough
  /// unfinished ones (waiting) that at most `keep` stay in flight.
  void drain(unsigned keep)
  {
    while (!pending.empty()) {
      const pending_symbol& ps = pending.front();
      symbol_stage&         st = *stages[ps.symbol];
      if (pending.size() > keep) {
        gpu::hip_check(hipEventSynchronize(st.done), WHO, "demodulation");
      } else if (hipEventQuery(st.done) != hipSuccess) {
        break;
      }
      resource_grid_writer& writer = current_grid.get().get_writer();
      for (unsigned p = 0; p != nof_ports; ++p) {
        writer.put(p, ps.symbol, 0, 1,
                   span<const cbf16_t>(st.out.host<cbf16_t>(static_cast<size_t>(p) * nsc * sizeof(uint32_t)), nsc));
      }
      notifier->on_rx_symbol(current_grid, ps.context);
      pending.pop_front();
    }
  }

  struct pending_symbol {
    unsigned                    symbol;
    lower_phy_rx_symbol_context context;
  };

  std::shared_ptr<srsgpu_context>            owner;
  srsgpu_context*                            ctx;
  gpu::owned_stream                          stream;
  symbol_geometry                            geo;
  unsigned                                   nof_ports;
  unsigned                                   nsc;
  unsigned                                   max_symbols_in_flight;
  std::vector<srsgpu_ofdm_plan*>             plans;  ///< One plan (all ports) per symbol of the subframe.
  std::vector<hipGraphExec_t>                graphs;  ///< per plan: upload + demodulation + download
  std::vector<std::unique_ptr<symbol_stage>> stages;
  std::deque<pending_symbol>                 pending;
  std::atomic<bool>                          stopped  = false;
  puxch_processor_notifier*                  notifier = nullptr;
  slot_point                                 current_slot;
  shared_resource_grid                       current_grid;
  request_ring<shared_resource_grid>         requests;
};

class pdxch_processor_factory_gpu : public pdxch_processor_factory
{
public:
  explicit pdxch_processor_factory_gpu(int device) : ctx(gpu::shared_context(device)) {}
  std::unique_ptr<pdxch_processor> create(const pdxch_processor_configuration& config) override
  {
    return std::make_unique<pdxch_processor_gpu>(ctx, config);
  }

private:
  std::shared_ptr<srsgpu_context> ctx;
};

class puxch_processor_factory_gpu : public puxch_processor_factory
{
public:
  puxch_processor_factory_gpu(int device, unsigned max_symbols_in_flight_) :
    ctx(gpu::shared_context(device)), max_symbols_in_flight(max_symbols_in_flight_)
  {
  }
  std::unique_ptr<puxch_processor> create(const puxch_processor_configuration& config) override
  {
    return std::make_unique<puxch_processor_gpu>(ctx, config, max_symbols_in_flight);
  }

private:
  std::shared_ptr<srsgpu_context> ctx;
  unsigned                        max_symbols_in_flight;
};

} // namespace

std::shared_ptr<pdxch_processor_factory> create_pdxch_processor_factory_gpu(int device)
{
  return std::make_shared<pdxch_processor_factory_gpu>(device);
}

std::shared_ptr<puxch_processor_factory> create_puxch_processor_factory_gpu(int device, unsigned max_symbols_in_flight)
{
  return std::make_shared<puxch_processor_factory_gpu>(device, max_symbols_in_flight);
}

} // namespace srsran
