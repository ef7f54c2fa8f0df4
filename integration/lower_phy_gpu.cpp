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
//    non-empty port's 14 grid rows are staged in mapped host memory, one launch modulates all ports and symbols
//    reading them in place and writes the samples in place into mapped memory of the request, asynchronously on the
//    processor's stream (zero-copy: below a few MB a DMA copy costs several times the PCIe transfer). process_symbol()
//    only waits for that slot's event at its first symbol (long finished: requests arrive max_processing_delay slots
//    ahead) and copies the symbol's CP + N samples of every port. The request bookkeeping (one entry per slot modulo
//    16, the late-request notifications, empty grids discarded) is the reference's.
//
//  * PUxCH (uplink): the symbols arrive one by one. process_symbol() stages the symbol's samples of every port into
//    mapped memory and launches its demodulation (one plan per symbol of the subframe, all ports) without waiting.
//    Symbols whose demodulation has finished are written into the request's grid and notified (on_rx_symbol) in
//    order; at most `max_symbols_in_flight` are outstanding (0: every symbol is demodulated and notified before
//    process_symbol returns, the reference's timing), and the slot's last symbol drains everything, so every symbol of
//    a slot is notified, in order, before the slot's last process_symbol() returns.
//
//  * Sector group (lower_phy_sector_group, optional): the processors of several sectors on one GPU share launches:
//    the same UL symbol / DL slot of every sector runs as one OFDM launch over the sectors' plans concatenated.
#include "signal_chain_gpu.h"

#include "batch_graph.h"
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

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
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

  template <typename F>
  void for_each(F&& f)
  {
    for (entry& e : entries) {
      std::lock_guard<std::mutex> lock(e.mtx);
      f(e.req.payload);
    }
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
// Sector group
// ---------------------------------------------------------------------------------------------------------------------

/// One direction of a sector group. A round is the work of every sector at one position (UL: a symbol, key = system
/// slot x symbols per slot + symbol; DL: a slot, key = system slot), run as one OFDM launch of the sectors' plans
/// concatenated (srsgpu_ofdm_plan_concat) that reads the round's input region (all sectors) from mapped host memory
/// and writes its output region there (zero-copy: no DMA copy on the path). Rounds sit in a ring of a whole number of
/// periods (a subframe's symbols or slots), so a ring entry always serves the same position and owns one captured
/// launch over its own buffers; consecutive rounds go to different streams.
class sector_rounds
{
public:
  using clock = std::chrono::steady_clock;

  sector_rounds(srsgpu_context* ctx_, const char* who_, bool inverse_, unsigned nof_sectors_, unsigned period_,
                unsigned nof_rounds, std::chrono::microseconds window_) :
    ctx(ctx_),
    who(who_),
    inverse(inverse_),
    nof_sectors(nof_sectors_),
    all((nof_sectors_ >= 32) ? ~0u : ((1u << nof_sectors_) - 1)),
    period(period_),
    window(window_),
    members(nof_sectors_)
  {
    for (auto& st : streams) {
      st = std::make_unique<gpu::owned_stream>(ctx_, who_);
    }
    for (unsigned r = 0; r != nof_rounds; ++r) {
      rounds.emplace_back(std::make_unique<round>(who, r));
    }
    dispatcher = std::thread([this]() { dispatch_loop(); });
  }

  ~sector_rounds()
  {
    {
      std::lock_guard<std::mutex> lock(mtx);
      stopping = true;
    }
    dispatch_cv.notify_all();
    dispatcher.join();
    for (auto& st : streams) {
      (void)hipStreamSynchronize(st->get());
    }
    std::lock_guard<std::recursive_mutex> setup(gpu::hip_setup_mutex());
    for (auto& rd : rounds) {
      if (rd->graph != nullptr) {
        (void)hipGraphExecDestroy(rd->graph);
      }
      if (rd->done != nullptr) {
        (void)hipEventDestroy(rd->done);
      }
    }
    rounds.clear();
    for (srsgpu_ofdm_plan* p : plans) {
      srsgpu_ofdm_plan_destroy(p);
    }
  }

  /// A sector's plans, one per position of the period (kept by the caller while it is registered); returns the
  /// sector's index, or -1 when every index is taken. The last sector builds the concatenated plans, the rounds'
  /// buffers and graphs (the caller holds gpu::hip_setup_mutex). Sectors whose plans do not concatenate leave the
  /// group disabled: every sector then runs alone.
  int add_sector(const std::vector<srsgpu_ofdm_plan*>& sector_plans)
  {
    std::lock_guard<std::mutex> lock(mtx);
    if (registered == nof_sectors || sector_plans.size() != period) {
      return -1;
    }
    const int index     = static_cast<int>(registered++);
    members[index]      = sector_plans;
    if (registered == nof_sectors) {
      build();
    }
    return index;
  }

  /// Deregistration (the sector's plans are going away): rounds no longer wait for it; before the group is built, the
  /// group stays disabled.
  void remove_sector(int sector)
  {
    std::vector<round*> go;
    {
      std::lock_guard<std::mutex> lock(mtx);
      gone |= 1u << sector;
      members[sector].clear();
      const auto now = clock::now();
      for (auto& rd : rounds) {
        if (rd->key != UINT64_MAX && !rd->closed) {
          rd->arrived |= 1u << sector;
          if (try_close(*rd, now)) {
            go.push_back(rd.get());
          }
        }
      }
    }
    for (round* rd : go) {
      launch(*rd);
    }
  }

  bool enabled() const { return built; }

  /// Sector `sector` reaches the round of `key`: present (it has work: returns the ring entry it writes its input into
  /// before calling written()) or absent (no request: returns -1, the round stops waiting for it). -1 also when the
  /// round launched already or its ring entry is still busy with an older key: the sector runs alone.
  int join(int sector, uint64_t key, bool present)
  {
    if (!built || sector < 0) {
      return -1;
    }
    std::unique_lock<std::mutex> lock(mtx);
    const unsigned               r  = static_cast<unsigned>(key % rounds.size());
    round&                       rd = *rounds[r];
    if (rd.key != key) {
      if (rd.consumers != 0 || (rd.arrived != 0 && !rd.closed)) {
        ++alone;
        return -1;
      }
      rd.key      = key;
      rd.arrived  = gone;
      rd.present  = 0;
      rd.written  = 0;
      rd.closed   = false;
      rd.launched = false;
      rd.first    = clock::now();
      if (dispatcher_idle) {
        dispatch_cv.notify_one();  // a busy dispatcher already waits for an earlier deadline
      }
    }
    const uint32_t bit = 1u << sector;
    if (rd.closed || (rd.arrived & bit) != 0) {
      if (present) {
        ++alone;
      }
      return -1;
    }
    rd.arrived |= bit;
    if (!present) {
      if (try_close(rd, clock::now())) {
        lock.unlock();
        launch(rd);
      }
      return -1;
    }
    rd.present |= bit;
    ++rd.consumers;
    ++grouped;
    return static_cast<int>(r);
  }

  uint8_t* input(int r, int sector) { return rounds[r]->in.host(in_off[r % period][sector]); }
  const uint8_t* output(int r, int sector) { return rounds[r]->out.host(out_off[r % period][sector]); }

  /// The sector's input of round r is in place.
  void written(int r, int sector)
  {
    round& rd = *rounds[r];
    bool   go;
    {
      std::lock_guard<std::mutex> lock(mtx);
      rd.written |= 1u << sector;
      go = try_close(rd, clock::now());
    }
    if (go) {
      launch(rd);
    }
  }

  /// Whether round r's outputs are ready; wait: block until they are.
  bool ready(int r, bool wait)
  {
    round& rd = *rounds[r];
    {
      std::unique_lock<std::mutex> lock(mtx);
      if (!rd.launched) {
        if (!wait) {
          return false;
        }
        launched_cv.wait(lock, [&rd]() { return rd.launched; });
      }
    }
    if (wait) {
      gpu::hip_check(hipEventSynchronize(rd.done), who, "sector group round");
      return true;
    }
    return hipEventQuery(rd.done) == hipSuccess;
  }

  /// A present sector is done with round r's outputs.
  void release(int r)
  {
    std::lock_guard<std::mutex> lock(mtx);
    --rounds[r]->consumers;
  }

  uint64_t nof_rounds() const { return launches.load(); }
  uint64_t nof_grouped() const { return grouped.load(); }
  uint64_t nof_alone() const { return alone.load(); }

private:
  struct round {
    round(const char* w, unsigned i) : index(i), in(w), out(w) {}
    unsigned            index;
    uint64_t            key       = UINT64_MAX;
    uint32_t            arrived   = 0;  ///< sectors that reached the round (present or absent; gone ones count)
    uint32_t            present   = 0;  ///< sectors with input in the round
    uint32_t            written   = 0;  ///< present sectors whose input is in place
    unsigned            consumers = 0;  ///< present sectors that have not released the outputs
    bool                closed    = false;  ///< no more sectors join (launched, or nothing to launch)
    bool                launched  = false;
    clock::time_point   first;
    gpu::mapped_buffer  in;   ///< every sector's input, read in place by the OFDM kernel
    gpu::mapped_buffer  out;  ///< every sector's output, written in place
    hipEvent_t          done  = nullptr;
    hipGraphExec_t      graph = nullptr;
  };

  /// Closes a round once every sector arrived or its window ran out, and every present sector's input is in place;
  /// true: the caller launches it (after releasing mtx). A round nobody is present in retires without a launch. Holds
  /// mtx.
  bool try_close(round& rd, clock::time_point now)
  {
    if (rd.closed || rd.written != rd.present || (rd.arrived != all && now - rd.first < window)) {
      return false;
    }
    rd.closed = true;
    return rd.present != 0;
  }

  /// The round's captured launch, outside mtx (the sectors of the next round keep joining meanwhile). Consecutive
  /// rounds go to different streams: a round still reading / writing host memory does not hold the next.
  void launch(round& rd)
  {
    gpu::device_scope dev(ctx, who);
    hipStream_t       hs = streams[rd.index % streams.size()]->get();
    gpu::hip_check(hipGraphLaunch(rd.graph, hs), who, "graph launch");
    gpu::hip_check(hipEventRecord(rd.done, hs), who, "event");
    {
      std::lock_guard<std::mutex> lock(mtx);
      rd.launched = true;
    }
    ++launches;
    launched_cv.notify_all();
  }

  void dispatch_loop()
  {
    std::unique_lock<std::mutex> lock(mtx);
    std::vector<round*>          go;
    while (!stopping) {
      clock::time_point next = clock::time_point::max();
      const auto        now  = clock::now();
      for (auto& rd : rounds) {
        if (rd->arrived == 0 || rd->closed || rd->key == UINT64_MAX) {
          continue;
        }
        if (try_close(*rd, now)) {
          go.push_back(rd.get());
        } else if (!rd->closed) {
          // waiting for its window, or (window over) for a sector still copying its input
          next = std::min(next, rd->first + window > now ? rd->first + window : now + std::chrono::microseconds(20));
        }
      }
      if (!go.empty()) {
        lock.unlock();
        for (round* rd : go) {
          launch(*rd);
        }
        go.clear();
        lock.lock();
        continue;
      }
      dispatcher_idle = next == clock::time_point::max();
      if (dispatcher_idle) {
        dispatch_cv.wait(lock);
      } else {
        dispatch_cv.wait_until(lock, next);
      }
      dispatcher_idle = false;
    }
  }

  /// Concatenated plans, per-sector offsets, round buffers and graphs. Holds mtx (and gpu::hip_setup_mutex).
  void build()
  {
    gpu::device_scope dev(ctx, who);
    for (unsigned k = 0; k != nof_sectors; ++k) {
      if (members[k].size() != period) {
        return;  // a sector left before the group was complete
      }
    }
    std::vector<srsgpu_ofdm_plan*> cat(period, nullptr);
    for (unsigned pos = 0; pos != period; ++pos) {
      std::vector<const srsgpu_ofdm_plan*> m;
      for (unsigned k = 0; k != nof_sectors; ++k) {
        m.push_back(members[k][pos]);
      }
      if (srsgpu_ofdm_plan_concat(ctx, m.data(), nof_sectors, &cat[pos]) != SRSGPU_OK) {
        for (srsgpu_ofdm_plan* p : cat) {
          srsgpu_ofdm_plan_destroy(p);
        }
        return;  // sectors differ in what one launch shares: no group
      }
    }
    plans = cat;
    in_off.assign(period, std::vector<size_t>(nof_sectors));
    out_off.assign(period, std::vector<size_t>(nof_sectors));
    std::vector<size_t> in_bytes(period), out_bytes(period);  // per position
    for (unsigned pos = 0; pos != period; ++pos) {
      const size_t words = srsgpu_ofdm_plan_nof_grid_words(plans[pos]) / nof_sectors;  // equal per sector
      for (unsigned k = 0; k != nof_sectors; ++k) {
        const size_t samples = srsgpu_ofdm_plan_sample_offset(plans[pos], k, 0) * sizeof(cf_t);
        in_off[pos][k]       = inverse ? k * words * sizeof(uint32_t) : samples;
        out_off[pos][k]      = inverse ? samples : k * words * sizeof(uint32_t);
      }
      const size_t grid_bytes   = srsgpu_ofdm_plan_nof_grid_words(plans[pos]) * sizeof(uint32_t);
      const size_t sample_bytes = srsgpu_ofdm_plan_nof_samples(plans[pos]) * sizeof(cf_t);
      in_bytes[pos]             = inverse ? grid_bytes : sample_bytes;
      out_bytes[pos]            = inverse ? sample_bytes : grid_bytes;
    }
    hipStream_t hs = streams[0]->get();
    for (unsigned r = 0; r != rounds.size(); ++r) {
      round&         rd  = *rounds[r];
      const unsigned pos = r % period;
      rd.in.reserve(in_bytes[pos]);
      rd.out.reserve(out_bytes[pos]);
      gpu::hip_check(hipEventCreateWithFlags(&rd.done, hipEventDisableTiming), who, "event");
      rd.graph = gpu::capture_graph(hs, who, [&]() {
        if (inverse) {
          gpu::srsgpu_check(srsgpu_ofdm_modulator_plan_execute(plans[pos], rd.in.dev<uint32_t>(), rd.out.dev<float>(),
                                                               hs),
                            who);
        } else {
          gpu::srsgpu_check(srsgpu_ofdm_demodulator_plan_execute(plans[pos], rd.in.dev<float>(),
                                                                 rd.out.dev<uint32_t>(), hs),
                            who);
        }
      });
    }
    built = true;
  }

  srsgpu_context*                              ctx;
  const char*                                  who;
  bool                                         inverse;
  unsigned                                     nof_sectors;
  uint32_t                                     all;
  unsigned                                     period;
  std::chrono::microseconds                    window;
  std::array<std::unique_ptr<gpu::owned_stream>, 3> streams;
  std::vector<std::vector<srsgpu_ofdm_plan*>>  members;
  std::vector<srsgpu_ofdm_plan*>               plans;    ///< per position: every sector's plan concatenated
  std::vector<std::vector<size_t>>             in_off;   ///< per position and sector: byte offset of its input
  std::vector<std::vector<size_t>>             out_off;  ///< ... and of its output
  std::vector<std::unique_ptr<round>>          rounds;
  unsigned                                     registered = 0;
  uint32_t                                     gone       = 0;
  std::atomic<bool>                            built      = false;
  bool                                         stopping   = false;
  bool                                         dispatcher_idle = true;
  std::atomic<uint64_t>                        launches   = 0;
  std::atomic<uint64_t>                        grouped    = 0;
  std::atomic<uint64_t>                        alone      = 0;
  std::mutex                                   mtx;
  std::condition_variable                      launched_cv;
  std::condition_variable                      dispatch_cv;
  std::thread                                  dispatcher;
};

} // namespace

/// The group: one sector_rounds per direction, made by the first processor of that direction (its geometry sets the
/// period: the subframe's symbols for UL, its slots for DL).
class lower_phy_sector_group
{
public:
  explicit lower_phy_sector_group(const lower_phy_group_configuration& cfg_) :
    cfg(cfg_), owner(gpu::shared_context(cfg_.device))
  {
    if (cfg.nof_sectors == 0 || cfg.nof_sectors > 32) {
      throw std::invalid_argument("lower_phy_sector_group: 1 to 32 sectors");
    }
  }

  sector_rounds& rounds(bool downlink, unsigned period)
  {
    std::lock_guard<std::mutex> lock(mtx);
    std::unique_ptr<sector_rounds>& r = downlink ? dl : ul;
    if (!r) {
      // A whole number of periods (one graph per ring entry): at least 8 slots of DL (requests run a few slots ahead
      // of the slot being transmitted) and 4 slots of UL symbols (a sector holds at most a slot's symbols).
      const unsigned n = downlink ? period * std::max(1u, 8u / period) : period * std::max(2u, 56u / period);
      r = std::make_unique<sector_rounds>(owner.get(), downlink ? "pdxch_sector_group" : "puxch_sector_group",
                                          downlink, cfg.nof_sectors, period, n,
                                          std::chrono::microseconds(downlink ? cfg.dl_window_us : cfg.ul_window_us));
    }
    return *r;
  }

  lower_phy_group_counters counters() const
  {
    lower_phy_group_counters c;
    std::lock_guard<std::mutex> lock(mtx);
    if (ul) {
      c.ul_rounds  = ul->nof_rounds();
      c.ul_grouped = ul->nof_grouped();
      c.ul_alone   = ul->nof_alone();
    }
    if (dl) {
      c.dl_rounds  = dl->nof_rounds();
      c.dl_grouped = dl->nof_grouped();
      c.dl_alone   = dl->nof_alone();
    }
    return c;
  }

  const lower_phy_group_configuration cfg;
  std::shared_ptr<srsgpu_context>      owner;

private:
  mutable std::mutex             mtx;
  std::unique_ptr<sector_rounds> ul;
  std::unique_ptr<sector_rounds> dl;
};

namespace {

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
    gpu::mapped_buffer grid;     ///< the slot's grid rows, read in place by the modulation
    gpu::mapped_buffer samples;  ///< the slot's samples, written in place
    hipEvent_t         done = nullptr;
    /// Per slot of the subframe: the modulation captured over this job's buffers (graph_buffers).
    std::vector<hipGraphExec_t> graphs;
    const void*                 graph_buffers[2] = {nullptr, nullptr};
    std::vector<bool>  port_empty;
    unsigned           subframe_slot = 0;
    bool               launched      = false;  ///< false: the request's grid was empty (nothing to transmit).
    bool               own           = false;  ///< launched on this job's own buffers (done is recorded)
    int                round         = -1;     ///< launched in the sector group's round (its outputs hold the slot)
  };
  using job_ptr = std::unique_ptr<job>;

public:
  pdxch_processor_gpu(std::shared_ptr<srsgpu_context>         owner_,
                      const pdxch_processor_configuration&    config,
                      std::shared_ptr<lower_phy_sector_group> group_) :
    group_owner(std::move(group_)),
    owner(std::move(owner_)),
    ctx(owner.get()),
    stream(ctx, WHO),
    geo(config.scs, config.cp, config.srate.get_dft_size(config.scs)),
    nof_ports(config.nof_tx_ports),
    nsc(config.bandwidth_rb * NRE)
  {
    gpu::device_scope                     dev(ctx, WHO);
    std::lock_guard<std::recursive_mutex> setup(gpu::hip_setup_mutex());  // plan allocations vs other sectors' captures
    // pdxch_processor_factory_sw: modulator scaling 1 (pdxch_processor_factories.cpp:59).
    const srsgpu_ofdm_config c = ofdm_config(config.scs, config.cp, config.bandwidth_rb,
                                             config.srate.get_dft_size(config.scs), 0, 1.0F, config.center_freq_Hz);
    for (unsigned s = 0; s != geo.nslot; ++s) {
      srsgpu_ofdm_plan* p = nullptr;
      gpu::srsgpu_check(srsgpu_ofdm_modulator_plan_create(ctx, &c, 1, nof_ports, &s, &p), WHO);
      plans.push_back(p);
    }
    if (group_owner) {
      group  = &group_owner->rounds(true, geo.nslot);
      sector = group->add_sector(plans);
    }
  }

  ~pdxch_processor_gpu() override
  {
    recycle(std::move(current));
    requests.for_each([this](job_ptr& j) { recycle(std::move(j)); });
    if (sector >= 0) {
      group->remove_sector(sector);
    }
    (void)hipStreamSynchronize(stream.get());
    std::lock_guard<std::recursive_mutex> setup(gpu::hip_setup_mutex());
    free_jobs.clear();
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
      if (current->round >= 0) {
        group->ready(current->round, true);
      } else {
        gpu::hip_check(hipEventSynchronize(current->done), WHO, "modulation");
      }
    }
    if (!current) {
      return false;
    }
    const unsigned s     = context.slot.subframe_slot_index() * geo.nsymb + context.symbol;
    const unsigned n     = geo.size[s];
    const size_t   slotn = geo.slot_size(current->subframe_slot);
    const auto*    slot_samples =
        reinterpret_cast<const cf_t*>(current->round >= 0 ? group->output(current->round, sector) : current->samples.host());
    for (unsigned p = 0; p != nof_ports; ++p) {
      span<cf_t> out = samples.get_channel_buffer(p);
      srsran_assert(out.size() == n, "The output buffer size ({}) does not match the symbol size ({}).", out.size(), n);
      if (current->port_empty[p]) {
        std::fill(out.begin(), out.end(), cf_t());  // ofdm_modulator_impl.cpp:77: an empty port transmits zeros
      } else {
        std::memcpy(out.data(), slot_samples + p * slotn + geo.start[s], n * sizeof(cf_t));
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
    const bool                  empty  = reader.is_empty();
    const int r = sector >= 0 ? group->join(sector, context.slot.system_slot(), !empty) : -1;
    if (r >= 0) {
      stage_grid(*j, reader, group->input(r, sector));
      group->written(r, sector);
      j->round         = r;
      j->subframe_slot = context.slot.subframe_slot_index();
      j->launched      = true;
    } else if (!empty) {
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
      std::lock_guard<std::recursive_mutex> setup(gpu::hip_setup_mutex());
      gpu::hip_check(hipEventCreateWithFlags(&j.done, hipEventDisableTiming), WHO, "event");
    }
    stage_grid(j, reader, j.grid.host());
    // The modulation reads the rows and writes the samples in mapped host memory (no DMA copies), one captured launch
    // per (job, slot of the subframe), built on first use.
    if (j.graph_buffers[0] != j.grid.dev() || j.graph_buffers[1] != j.samples.dev()) {
      j.drop_graphs();  // the job's buffers grew: the graphs captured their old addresses
      j.graph_buffers[0] = j.grid.dev();
      j.graph_buffers[1] = j.samples.dev();
    }
    j.graphs.resize(plans.size(), nullptr);
    hipGraphExec_t& exec = j.graphs[subframe_slot];
    if (exec == nullptr) {
      std::lock_guard<std::recursive_mutex> setup(gpu::hip_setup_mutex());
      exec = gpu::capture_graph(s, WHO, [&]() {
        gpu::srsgpu_check(srsgpu_ofdm_modulator_plan_execute(plans[subframe_slot], j.grid.dev<uint32_t>(),
                                                             j.samples.dev<float>(), s),
                          WHO);
      });
    }
    gpu::hip_check(hipGraphLaunch(exec, s), WHO, "graph launch");
    gpu::hip_check(hipEventRecord(j.done, s), WHO, "event");
    j.subframe_slot = subframe_slot;
    j.launched      = true;
    j.own           = true;
  }

  /// The grid rows of every non-empty port into `dst` ([port][symbol][subcarrier] uint32), the empty ports noted.
  void stage_grid(job& j, const resource_grid_reader& reader, uint8_t* dst)
  {
    const size_t row = static_cast<size_t>(nsc) * sizeof(uint32_t);
    j.port_empty.assign(nof_ports, false);
    for (unsigned p = 0; p != nof_ports; ++p) {
      j.port_empty[p] = reader.is_empty(p);
      if (j.port_empty[p]) {
        continue;  // its rows stay stale on the device; the port's output is zeros
      }
      for (unsigned l = 0; l != geo.nsymb; ++l) {
        std::memcpy(dst + (p * geo.nsymb + l) * row, reader.get_view(p, l).data(), row);
      }
    }
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
    if (j->own) {
      gpu::device_scope dev(ctx, WHO);
      gpu::hip_check(hipEventSynchronize(j->done), WHO, "job reuse");
      j->own = false;
    }
    return j;
  }

  void recycle(job_ptr j)
  {
    if (j) {
      if (j->round >= 0) {
        group->release(j->round);
        j->round = -1;
      }
      std::lock_guard<std::mutex> lock(free_mtx);
      free_jobs.push_back(std::move(j));
    }
  }

  std::shared_ptr<lower_phy_sector_group> group_owner;
  sector_rounds*                  group  = nullptr;
  int                             sector = -1;  ///< index in the group, -1: not grouped
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
    gpu::mapped_buffer in;   ///< the symbol's samples (all ports), read in place by the demodulation
    gpu::mapped_buffer out;  ///< the demodulated rows, written in place
    hipEvent_t         done = nullptr;
  };

public:
  puxch_processor_gpu(std::shared_ptr<srsgpu_context>         owner_,
                      const puxch_processor_configuration&    config,
                      unsigned                                max_symbols_in_flight_,
                      std::shared_ptr<lower_phy_sector_group> group_) :
    group_owner(std::move(group_)),
    owner(std::move(owner_)),
    ctx(owner.get()),
    stream(ctx, WHO),
    geo(config.scs, config.cp, config.srate.get_dft_size(config.scs)),
    nof_ports(config.nof_rx_ports),
    nsc(config.bandwidth_rb * NRE),
    max_symbols_in_flight(max_symbols_in_flight_)
  {
    gpu::device_scope                     dev(ctx, WHO);
    std::lock_guard<std::recursive_mutex> setup(gpu::hip_setup_mutex());  // plan allocations vs other sectors' captures
    const unsigned                        N = config.srate.get_dft_size(config.scs);
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
    if (group_owner) {
      group  = &group_owner->rounds(false, geo.nslot * geo.nsymb);
      sector = group->add_sector(plans);
    }
  }

  ~puxch_processor_gpu() override
  {
    for (const pending_symbol& ps : pending) {
      if (ps.round >= 0) {
        group->release(ps.round);
      }
    }
    if (sector >= 0) {
      group->remove_sector(sector);
    }
    (void)hipStreamSynchronize(stream.get());
    std::lock_guard<std::recursive_mutex> setup(gpu::hip_setup_mutex());
    stages.clear();
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
    const unsigned l   = context.nof_symbols;
    const uint64_t key = static_cast<uint64_t>(context.slot.system_slot()) * geo.nsymb + l;
    if (!current_grid) {
      if (sector >= 0) {
        group->join(sector, key, false);  // the group's round for this symbol stops waiting for this sector
      }
      return false;
    }
    const unsigned s = context.slot.subframe_slot_index() * geo.nsymb + l;
    const unsigned n = geo.size[s];
    // Grouped: the samples go into the group's round for this symbol, launched with the other sectors' samples.
    const int r = sector >= 0 ? group->join(sector, key, true) : -1;
    if (r >= 0) {
      uint8_t* dst = group->input(r, sector);
      for (unsigned p = 0; p != nof_ports; ++p) {
        span<const cf_t> in = samples.get_channel_buffer(p);
        srsran_assert(in.size() == n, "The input buffer size ({}) does not match the symbol size ({}).", in.size(), n);
        std::memcpy(dst + static_cast<size_t>(p) * n * sizeof(cf_t), in.data(), n * sizeof(cf_t));
      }
      group->written(r, sector);
      pending.push_back({l, context, r});
      if (l == geo.nsymb - 1) {
        drain(0);
        current_grid.release();
      } else {
        drain(max_symbols_in_flight);
      }
      return true;
    }
    symbol_stage& st = *stages[l];
    hipStream_t   hs = stream.get();
    for (unsigned p = 0; p != nof_ports; ++p) {
      span<const cf_t> in = samples.get_channel_buffer(p);
      srsran_assert(in.size() == n, "The input buffer size ({}) does not match the symbol size ({}).", in.size(), n);
      std::memcpy(st.in.host<cf_t>(static_cast<size_t>(p) * n * sizeof(cf_t)), in.data(), n * sizeof(cf_t));
    }
    // The demodulation of this symbol position reads the samples and writes the rows in mapped host memory (no DMA
    // copies), captured once per position.
    hipGraphExec_t& exec = graphs[s];
    if (exec == nullptr) {
      std::lock_guard<std::recursive_mutex> lock(gpu::hip_setup_mutex());
      exec = gpu::capture_graph(hs, WHO, [&]() {
        gpu::srsgpu_check(
            srsgpu_ofdm_demodulator_plan_execute(plans[s], st.in.dev<float>(), st.out.dev<uint32_t>(), hs), WHO);
      });
    }
    gpu::hip_check(hipGraphLaunch(exec, hs), WHO, "graph launch");
    gpu::hip_check(hipEventRecord(st.done, hs), WHO, "event");
    pending.push_back({l, context, -1});
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
      const uint8_t*        rows;
      if (ps.round >= 0) {
        if (!group->ready(ps.round, pending.size() > keep)) {
          break;
        }
        rows = group->output(ps.round, sector);
      } else {
        symbol_stage& st = *stages[ps.symbol];
        if (pending.size() > keep) {
          gpu::hip_check(hipEventSynchronize(st.done), WHO, "demodulation");
        } else if (hipEventQuery(st.done) != hipSuccess) {
          break;
        }
        rows = st.out.host();
      }
      resource_grid_writer& writer = current_grid.get().get_writer();
      for (unsigned p = 0; p != nof_ports; ++p) {
        writer.put(p, ps.symbol, 0, 1,
                   span<const cbf16_t>(reinterpret_cast<const cbf16_t*>(rows + static_cast<size_t>(p) * nsc *
                                                                                    sizeof(uint32_t)),
                                       nsc));
      }
      if (ps.round >= 0) {
        group->release(ps.round);
      }
      notifier->on_rx_symbol(current_grid, ps.context);
      pending.pop_front();
    }
  }

  struct pending_symbol {
    unsigned                    symbol;
    lower_phy_rx_symbol_context context;
    int                         round;  ///< the group's round holding the result, -1: this processor's own stage
  };

  std::shared_ptr<lower_phy_sector_group>    group_owner;
  sector_rounds*                             group  = nullptr;
  int                                        sector = -1;  ///< index in the group, -1: not grouped
  std::shared_ptr<srsgpu_context>            owner;
  srsgpu_context*                            ctx;
  gpu::owned_stream                          stream;
  symbol_geometry                            geo;
  unsigned                                   nof_ports;
  unsigned                                   nsc;
  unsigned                                   max_symbols_in_flight;
  std::vector<srsgpu_ofdm_plan*>             plans;  ///< One plan (all ports) per symbol of the subframe.
  std::vector<hipGraphExec_t>                graphs;  ///< per plan: the demodulation over the stage's buffers
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
  pdxch_processor_factory_gpu(int device, std::shared_ptr<lower_phy_sector_group> g) :
    ctx(gpu::shared_context(device)), group(std::move(g))
  {
  }
  std::unique_ptr<pdxch_processor> create(const pdxch_processor_configuration& config) override
  {
    return std::make_unique<pdxch_processor_gpu>(ctx, config, group);
  }

private:
  std::shared_ptr<srsgpu_context>         ctx;
  std::shared_ptr<lower_phy_sector_group> group;
};

class puxch_processor_factory_gpu : public puxch_processor_factory
{
public:
  puxch_processor_factory_gpu(int device, unsigned max_symbols_in_flight_, std::shared_ptr<lower_phy_sector_group> g) :
    ctx(gpu::shared_context(device)), max_symbols_in_flight(max_symbols_in_flight_), group(std::move(g))
  {
  }
  std::unique_ptr<puxch_processor> create(const puxch_processor_configuration& config) override
  {
    return std::make_unique<puxch_processor_gpu>(ctx, config, max_symbols_in_flight, group);
  }

private:
  std::shared_ptr<srsgpu_context>         ctx;
  unsigned                                max_symbols_in_flight;
  std::shared_ptr<lower_phy_sector_group> group;
};

} // namespace

std::shared_ptr<pdxch_processor_factory> create_pdxch_processor_factory_gpu(int device)
{
  return std::make_shared<pdxch_processor_factory_gpu>(device, nullptr);
}

std::shared_ptr<puxch_processor_factory> create_puxch_processor_factory_gpu(int device, unsigned max_symbols_in_flight)
{
  return std::make_shared<puxch_processor_factory_gpu>(device, max_symbols_in_flight, nullptr);
}

std::shared_ptr<lower_phy_sector_group> create_lower_phy_sector_group(const lower_phy_group_configuration& config)
{
  return std::make_shared<lower_phy_sector_group>(config);
}

std::shared_ptr<pdxch_processor_factory> create_pdxch_processor_factory_gpu(std::shared_ptr<lower_phy_sector_group> group)
{
  const int device = group->cfg.device;
  return std::make_shared<pdxch_processor_factory_gpu>(device, std::move(group));
}

std::shared_ptr<puxch_processor_factory> create_puxch_processor_factory_gpu(std::shared_ptr<lower_phy_sector_group> group,
                                                                            unsigned max_symbols_in_flight)
{
  const int device = group->cfg.device;
  return std::make_shared<puxch_processor_factory_gpu>(device, max_symbols_in_flight, std::move(group));
}

lower_phy_group_counters get_lower_phy_group_counters(const lower_phy_sector_group& group)
{
  return group.counters();
}

} // namespace srsran
