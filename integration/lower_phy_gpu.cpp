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

/// Waits for a lower-PHY launch by polling its event: the launches take tens of microseconds, and a blocking
/// hipEventSynchronize sleeps until an interrupt that can come that much later again (a real-time sector thread would
/// lose the time of its next symbol).
inline void wait_event(hipEvent_t e, const char* who)
{
  for (;;) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) {
      return;
    }
    if (r != hipErrorNotReady) {
      gpu::hip_check(r, who, "event");
    }
    std::this_thread::yield();
  }
}

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

/// One direction of a sector group: the sectors' OFDM work (UL: one symbol of one sector; DL: one slot) in shared
/// launches. A sector stages its input in an entry of its own ring in mapped host memory and submits it; a launch
/// takes every submitted entry — whatever sector, slot or symbol — and runs them as one job list
/// (srsgpu_ofdm_jobs_execute: each entry's jobs are its plan's, moved to the entry's place in the shared buffers),
/// reading the inputs and writing the outputs in place (zero-copy). A launch goes out as soon as every active sector
/// (one that submitted within the last `activity`) has an entry waiting, or `window` after the oldest waiting entry;
/// the last sector to submit launches it, a dispatcher thread handles the windows. Nothing waits for a particular
/// sector: a sector that falls behind has its entries taken by whichever launch comes next. Completion: the stream
/// writes each launch's sequence number into its completion word in mapped memory, which the sectors poll (no HIP
/// call on their per-symbol path).
class ofdm_batcher
{
public:
  using clock = std::chrono::steady_clock;

  ofdm_batcher(srsgpu_context*           ctx_,
               const char*               who_,
               bool                      inverse_,
               unsigned                  nof_sectors_,
               unsigned                  depth_,
               std::chrono::microseconds window_,
               clock::duration           activity_) :
    ctx(ctx_),
    who(who_),
    inverse(inverse_),
    nof_sectors(nof_sectors_),
    depth(depth_),
    window(window_),
    activity(activity_),
    sectors(nof_sectors_),
    jobs_buf(who_),
    in_all(who_),
    out_all(who_),
    flags(who_)
  {
    for (auto& st : streams) {
      st = std::make_unique<gpu::owned_stream>(ctx_, who_);
    }
    dispatcher = std::thread([this]() { dispatch_loop(); });
  }

  ~ofdm_batcher()
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
    if (launcher != nullptr) {
      srsgpu_ofdm_plan_destroy(launcher);
    }
  }

  /// Registers a sector's plans, one per position of its period (kept by the caller while registered): its index, or
  /// -1 (no free index, or plans that cannot share a launch with the first sector's: that sector runs alone). The
  /// first sector sizes the shared buffers (the caller holds gpu::hip_setup_mutex).
  int add_sector(const std::vector<srsgpu_ofdm_plan*>& plans)
  {
    std::lock_guard<std::mutex> lock(mtx);
    int k = -1;
    for (unsigned i = 0; i != nof_sectors; ++i) {
      if (!sectors[i].used) {
        k = static_cast<int>(i);
        break;
      }
    }
    if (k < 0 || plans.empty()) {
      return -1;
    }
    if (launcher == nullptr) {
      if (!size_buffers(plans)) {
        return -1;
      }
    } else if (!compatible(plans)) {
      return -1;
    }
    sector_state& sc = sectors[k];
    sc.used          = true;
    sc.templates.assign(plans.size(), {});
    for (size_t pos = 0; pos != plans.size(); ++pos) {
      uint32_t n = 0;
      gpu::srsgpu_check(srsgpu_ofdm_plan_get_jobs(plans[pos], nullptr, 0, &n), who);
      sc.templates[pos].resize(n);
      gpu::srsgpu_check(srsgpu_ofdm_plan_get_jobs(plans[pos], sc.templates[pos].data(), n, &n), who);
    }
    sc.entries   = std::vector<entry>(depth);
    sc.head      = 0;
    sc.row_words = static_cast<uint32_t>(srsgpu_ofdm_plan_nof_grid_words(plans[0]) /
                                         std::max<size_t>(sc.templates[0].size(), 1));  // one job per grid row
    return k;
  }

  void remove_sector(int sector)
  {
    std::lock_guard<std::mutex> lock(mtx);
    sectors[sector].used        = false;
    sectors[sector].last_submit = clock::time_point();
  }

  /// The sector's next staging entry, or -1 while it is still in use (the sector then runs that work alone).
  int acquire(int sector)
  {
    sector_state& sc = sectors[sector];
    const int     e  = static_cast<int>(sc.head % depth);
    entry&        en = sc.entries[e];
    if (en.busy.load(std::memory_order_acquire)) {
      ++alone;
      return -1;
    }
    en.busy.store(true, std::memory_order_relaxed);
    en.launched.store(false, std::memory_order_relaxed);
    ++sc.head;
    return e;
  }

  uint8_t*       input(int sector, int e) { return in_all.host(entry_index(sector, e) * in_max); }
  const uint8_t* output(int sector, int e) { return out_all.host(entry_index(sector, e) * out_max); }
  /// Whether the entry's rows went to the direct destination given at submit (not to its staging output).
  bool           direct(int sector, int e) const { return sectors[sector].entries[e].direct; }

  /// Where a demodulation entry's grid rows go instead of its staging output: the device address of port 0's row and
  /// the distance between ports' rows (a mapped uplink resource grid, gpu::host_blocks).
  struct direct_rows {
    uint8_t* row0        = nullptr;
    size_t   port_stride = 0;
    uint8_t* twin0       = nullptr;  ///< the same rows of the grid's HBM twin (gpu::host_blocks::twin), or nullptr
  };

  /// The entry's input for position `pos` is in place; rows: its demodulated rows' destination (default: the entry's
  /// staging output).
  void submit(int sector, int e, unsigned pos) { submit(sector, e, pos, direct_rows()); }
  void submit(int sector, int e, unsigned pos, direct_rows rows)
  {
    std::vector<pending_entry> batch;
    {
      std::lock_guard<std::mutex> lock(mtx);
      const auto now = clock::now();
      sectors[sector].last_submit = now;
      sectors[sector].entries[e].direct = rows.row0 != nullptr && !inverse;
      queue.push_back({sector, e, pos, now, rows});
      if (queue.size() == 1) {
        dispatch_cv.notify_one();  // a window to watch
      }
      if (queue.size() >= active_sectors(now)) {
        batch.swap(queue);
      }
    }
    if (!batch.empty()) {
      launch(batch);
    }
  }

  /// Whether the entry's output is ready; wait: until it is.
  bool ready(int sector, int e, bool wait)
  {
    entry& en = sectors[sector].entries[e];
    if (!en.launched.load(std::memory_order_acquire)) {
      if (!wait) {
        return false;
      }
      std::unique_lock<std::mutex> lock(mtx);
      launched_cv.wait(lock, [&en]() { return en.launched.load(std::memory_order_acquire); });
    }
    const uint32_t* word = flags.host<uint32_t>(en.batch * 64);
    for (;;) {
      // the words count up (wrapping): reached once the difference is no longer negative
      if (static_cast<int32_t>(__atomic_load_n(word, __ATOMIC_ACQUIRE) - en.seq) >= 0) {
        return true;
      }
      if (!wait) {
        return false;
      }
      std::this_thread::yield();
    }
  }

  void release(int sector, int e) { sectors[sector].entries[e].busy.store(false, std::memory_order_release); }

  uint64_t nof_launches() const { return launches.load(); }
  uint64_t nof_grouped() const { return grouped.load(); }
  uint64_t nof_alone() const { return alone.load(); }
  uint64_t nof_windowed() const { return windowed.load(); }
  double   mean_batch() const { return launches ? static_cast<double>(grouped.load()) / launches.load() : 0; }

private:
  struct entry {
    std::atomic<bool> busy     = false;  ///< acquired and not yet released
    std::atomic<bool> launched = false;
    unsigned          batch    = 0;      ///< batch ring index of its launch
    uint32_t          seq      = 0;      ///< that launch's sequence number
    bool              direct   = false;  ///< rows written to the submit's direct destination
  };
  struct sector_state {
    bool                                      used = false;
    std::vector<std::vector<srsgpu_ofdm_job>> templates;  ///< per position: the plan's jobs
    std::vector<entry>                        entries;
    uint64_t                                  head      = 0;
    uint32_t                                  row_words = 1;  ///< uint32 words of a grid row (12 * bw_rb)
    clock::time_point                         last_submit;
  };
  struct pending_entry {
    int               sector;
    int               e;
    unsigned          pos;
    clock::time_point at;
    direct_rows       rows;
  };
  static constexpr unsigned NOF_BATCHES = 16;

  size_t entry_index(int sector, int e) const { return static_cast<size_t>(sector) * depth + e; }

  /// Sectors that submitted within `activity` (at least one). Holds mtx.
  size_t active_sectors(clock::time_point now) const
  {
    size_t n = 0;
    for (const sector_state& sc : sectors) {
      n += (sc.used && now - sc.last_submit < activity) ? 1 : 0;
    }
    return std::max<size_t>(n, 1);
  }

  /// Shared buffers sized from the first sector's plans. Holds mtx and gpu::hip_setup_mutex.
  bool size_buffers(const std::vector<srsgpu_ofdm_plan*>& plans)
  {
    // The launch parameters come from a plan of the batcher's own (a copy of the first plan): the sector that
    // registered first may be removed, and its plans destroyed, while the others keep submitting.
    srsgpu_ofdm_plan* own = nullptr;
    if (srsgpu_ofdm_plan_concat(ctx, const_cast<const srsgpu_ofdm_plan* const*>(plans.data()), 1, &own) !=
        SRSGPU_OK) {
      return false;
    }
    for (srsgpu_ofdm_plan* p : plans) {
      if (!joins(own, p) || !runs_job_lists(p)) {
        srsgpu_ofdm_plan_destroy(own);
        return false;
      }
    }
    for (srsgpu_ofdm_plan* p : plans) {
      const size_t grid  = srsgpu_ofdm_plan_nof_grid_words(p) * sizeof(uint32_t);
      const size_t samp  = srsgpu_ofdm_plan_nof_samples(p) * sizeof(cf_t);
      uint32_t     njobs = 0;
      gpu::srsgpu_check(srsgpu_ofdm_plan_get_jobs(p, nullptr, 0, &njobs), who);
      // entries 256-byte aligned; offsets in samples (8 bytes) and grid words (4 bytes) stay exact
      in_max        = std::max(in_max, (inverse ? grid : samp) + 255) / 256 * 256;
      out_max       = std::max(out_max, (inverse ? samp : grid) + 255) / 256 * 256;
      jobs_per_entry = std::max<size_t>(jobs_per_entry, njobs);
    }
    const size_t entries = static_cast<size_t>(nof_sectors) * depth;
    if ((entries * in_max) / sizeof(uint32_t) >= (1ull << 32) || (entries * out_max) / sizeof(uint32_t) >= (1ull << 32)) {
      in_max = out_max = jobs_per_entry = 0;
      srsgpu_ofdm_plan_destroy(own);
      return false;  // beyond the jobs' 32-bit offsets
    }
    in_all.reserve(entries * in_max);
    out_all.reserve(entries * out_max);
    jobs_buf.reserve(NOF_BATCHES * entries * jobs_per_entry * sizeof(srsgpu_ofdm_direct_job));
    flags.reserve(NOF_BATCHES * 64);
    for (unsigned b = 0; b != NOF_BATCHES; ++b) {
      *flags.host<uint32_t>(b * 64) = 0;
    }
    launcher = own;
    return true;
  }

  /// Whether two plans can run in one launch (srsgpu_ofdm_plan_concat accepts them: same direction, DFT size,
  /// bandwidth, DFT window offset and ports).
  bool joins(const srsgpu_ofdm_plan* a, const srsgpu_ofdm_plan* b) const
  {
    const srsgpu_ofdm_plan* pair[2] = {a, b};
    srsgpu_ofdm_plan*       joined  = nullptr;
    if (srsgpu_ofdm_plan_concat(ctx, pair, 2, &joined) != SRSGPU_OK) {
      return false;
    }
    srsgpu_ofdm_plan_destroy(joined);
    return true;
  }

  /// Whether the plan's DFT size runs from job lists (not the split sizes 9216...98304): a zero-job trial, which
  /// launches nothing.
  static bool runs_job_lists(const srsgpu_ofdm_plan* p)
  {
    uint64_t dummy = 0;
    return srsgpu_ofdm_jobs_execute(p, nullptr, 0, &dummy, &dummy, nullptr) == SRSGPU_OK;
  }

  /// Whether every position's plan can share a launch with the first sector's and fits the shared buffers: its
  /// input and output in an entry, its jobs in an entry's slice of the job table (sized from the first sector; a
  /// normal-CP sector joining an extended-CP group has more jobs per slot with the same sample count).
  bool compatible(const std::vector<srsgpu_ofdm_plan*>& plans) const
  {
    for (srsgpu_ofdm_plan* p : plans) {
      if (!joins(launcher, p) || !runs_job_lists(p)) {
        return false;
      }
      const size_t grid  = srsgpu_ofdm_plan_nof_grid_words(p) * sizeof(uint32_t);
      const size_t samp  = srsgpu_ofdm_plan_nof_samples(p) * sizeof(cf_t);
      uint32_t     njobs = 0;
      if (srsgpu_ofdm_plan_get_jobs(p, nullptr, 0, &njobs) != SRSGPU_OK || njobs > jobs_per_entry) {
        return false;
      }
      if ((inverse ? grid : samp) > in_max || (inverse ? samp : grid) > out_max) {
        return false;
      }
    }
    return true;
  }

  /// One launch of the entries: their jobs moved to the entries' places, the OFDM kernel over them, the completion
  /// word. Without mtx.
  void launch(const std::vector<pending_entry>& batch)
  {
    std::lock_guard<std::mutex> serial(launch_mtx);  // batch ring order = sequence order
    const unsigned              b     = static_cast<unsigned>(next_seq % NOF_BATCHES);
    const uint32_t              seq   = static_cast<uint32_t>(++next_seq);
    const uint32_t*             word  = flags.host<uint32_t>(b * 64);
    // The batch record's previous launch (NOF_BATCHES launches ago) must have finished reading its job table.
    while (static_cast<int32_t>(__atomic_load_n(word, __ATOMIC_ACQUIRE) - (seq - NOF_BATCHES)) < 0 &&
           seq > NOF_BATCHES) {
      std::this_thread::yield();
    }
    // Direct-address jobs: every entry's buffers are its staging slices, except the grid rows of a demodulation entry
    // submitted with a direct destination (the uplink grid itself).
    const size_t            stride = static_cast<size_t>(nof_sectors) * depth * jobs_per_entry;
    srsgpu_ofdm_direct_job* jobs   = jobs_buf.host<srsgpu_ofdm_direct_job>(b * stride * sizeof(srsgpu_ofdm_direct_job));
    size_t                  n      = 0;
    for (const pending_entry& pe : batch) {
      uint8_t* in_dev   = in_all.dev<uint8_t>(entry_index(pe.sector, pe.e) * in_max);
      uint8_t* out_dev  = out_all.dev<uint8_t>(entry_index(pe.sector, pe.e) * out_max);
      uint8_t* grid_dev = inverse ? in_dev : out_dev;
      uint8_t* samp_dev = inverse ? out_dev : in_dev;
      for (const srsgpu_ofdm_job& jb : sectors[pe.sector].templates[pe.pos]) {
        srsgpu_ofdm_direct_job& d = jobs[n++];
        d.grid                    = reinterpret_cast<uint64_t>(grid_dev + static_cast<size_t>(jb.grid_offset) * 4);
        d.grid_copy = 0;
        if (!inverse && pe.rows.row0 != nullptr) {
          // the templates' rows are [port][symbol - first] of one symbol: row = port
          const size_t port = jb.grid_offset / sectors[pe.sector].row_words;
          d.grid            = reinterpret_cast<uint64_t>(pe.rows.row0 + port * pe.rows.port_stride);
          if (pe.rows.twin0 != nullptr) {
            d.grid_copy = reinterpret_cast<uint64_t>(pe.rows.twin0 + port * pe.rows.port_stride);
          }
        }
        d.samples  = reinterpret_cast<uint64_t>(samp_dev + static_cast<size_t>(jb.sample_offset) * sizeof(cf_t));
        d.cp_len   = jb.cp_len;
        d.coef_re  = jb.coef_re;
        d.coef_im  = jb.coef_im;
        d.reserved = 0;
      }
    }
    gpu::device_scope dev(ctx, who);
    hipStream_t       hs = streams[b % streams.size()]->get();
    gpu::srsgpu_check(
        srsgpu_ofdm_jobs_execute_direct(
            launcher, jobs_buf.dev<srsgpu_ofdm_direct_job>(b * stride * sizeof(srsgpu_ofdm_direct_job)),
            static_cast<uint32_t>(n), hs),
        who);
    gpu::hip_check(hipStreamWriteValue32(hs, flags.dev<uint32_t>(b * 64), seq, 0), who, "completion word");
    for (const pending_entry& pe : batch) {
      entry& en = sectors[pe.sector].entries[pe.e];
      en.batch  = b;
      en.seq    = seq;
      en.launched.store(true, std::memory_order_release);
    }
    ++launches;
    grouped += batch.size();
    {
      std::lock_guard<std::mutex> lock(mtx);  // pairs with the waiters' predicate check
    }
    launched_cv.notify_all();
  }

  void dispatch_loop()
  {
    std::unique_lock<std::mutex> lock(mtx);
    while (!stopping) {
      if (queue.empty()) {
        dispatch_cv.wait(lock);
        continue;
      }
      const auto deadline = queue.front().at + window;
      if (clock::now() < deadline) {
        dispatch_cv.wait_until(lock, deadline);
        continue;
      }
      std::vector<pending_entry> batch;
      batch.swap(queue);
      lock.unlock();
      ++windowed;
      launch(batch);
      lock.lock();
    }
  }

  srsgpu_context*                                   ctx;
  const char*                                       who;
  bool                                              inverse;
  unsigned                                          nof_sectors;
  unsigned                                          depth;  ///< staging entries per sector
  std::chrono::microseconds                         window;
  clock::duration                                   activity;
  std::vector<sector_state>                         sectors;
  srsgpu_ofdm_plan*                                 launcher = nullptr;  ///< owned copy of the first plan: launch params
  size_t                                            in_max = 0, out_max = 0, jobs_per_entry = 0;
  gpu::mapped_buffer                                jobs_buf;  ///< NOF_BATCHES job tables
  gpu::mapped_buffer                                in_all;    ///< every sector's entries' inputs
  gpu::mapped_buffer                                out_all;   ///< ... and outputs
  gpu::mapped_buffer                                flags;     ///< completion word per batch record
  std::array<std::unique_ptr<gpu::owned_stream>, 3> streams;
  std::vector<pending_entry>                        queue;
  uint64_t                                          next_seq = 0;
  bool                                              stopping = false;
  std::atomic<uint64_t>                             launches = 0, grouped = 0, alone = 0, windowed = 0;
  std::mutex                                        mtx;
  std::mutex                                        launch_mtx;
  std::condition_variable                           launched_cv;
  std::condition_variable                           dispatch_cv;
  std::thread                                       dispatcher;
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

  /// The direction's batcher, made by its first processor: `positions` = slots (DL) or symbols (UL) per subframe.
  ofdm_batcher& batcher(bool downlink, unsigned positions)
  {
    std::lock_guard<std::mutex> lock(mtx);
    std::unique_ptr<ofdm_batcher>& r = downlink ? dl : ul;
    if (!r) {
      // Staging entries per sector: a UL sector holds at most a slot's symbols, a DL sector the requests of a few
      // slots ahead. A sector is active while it submitted within 3 symbols (UL) / 1.5 slots (DL).
      const auto position = std::chrono::nanoseconds(1000000 / positions);
      r = std::make_unique<ofdm_batcher>(owner.get(), downlink ? "pdxch_sector_group" : "puxch_sector_group", downlink,
                                         cfg.nof_sectors, downlink ? 8 : 16,
                                         std::chrono::microseconds(downlink ? cfg.dl_window_us : cfg.ul_window_us),
                                         downlink ? position * 3 / 2 : position * 3);
    }
    return *r;
  }

  lower_phy_group_counters counters() const
  {
    lower_phy_group_counters c;
    std::lock_guard<std::mutex> lock(mtx);
    if (ul) {
      c.ul_launches = ul->nof_launches();
      c.ul_batched  = ul->nof_grouped();
      c.ul_alone    = ul->nof_alone();
      c.ul_windowed = ul->nof_windowed();
    }
    if (dl) {
      c.dl_launches = dl->nof_launches();
      c.dl_batched  = dl->nof_grouped();
      c.dl_alone    = dl->nof_alone();
      c.dl_windowed = dl->nof_windowed();
    }
    return c;
  }

  const lower_phy_group_configuration cfg;
  std::shared_ptr<srsgpu_context>      owner;

private:
  mutable std::mutex            mtx;
  std::unique_ptr<ofdm_batcher> ul;
  std::unique_ptr<ofdm_batcher> dl;
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
    int                entry         = -1;     ///< staged in the sector group's entry (its output holds the slot)
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
    gpu::hip_check(hipGetDevice(&device_id), WHO, "device");
    if (group_owner) {
      group  = &group_owner->batcher(true, geo.nslot);
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
    for (const void* key : twin_keys) {
      gpu::dl_grid_twins::unsubscribe(key);
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
      if (current->entry >= 0) {
        group->ready(sector, current->entry, true);
      } else {
        wait_event(current->done, WHO);
      }
    }
    if (!current) {
      return false;
    }
    const unsigned s     = context.slot.subframe_slot_index() * geo.nsymb + context.symbol;
    const unsigned n     = geo.size[s];
    const size_t   slotn = geo.slot_size(current->subframe_slot);
    const auto*    slot_samples =
        reinterpret_cast<const cf_t*>(current->entry >= 0 ? group->output(sector, current->entry) : current->samples.host());
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
    // An ungrouped sector modulates the grid itself: it takes the PDSCH REs from the grid's HBM twin when the PDSCH
    // slot batch of its device left them there (gpu::dl_grid_twins).
    const void* twin_key = nullptr;
    if (sector < 0 && geo.nsymb == 14) {
      twin_key = &grid.get_writer();
      if (std::find(twin_keys.begin(), twin_keys.end(), twin_key) == twin_keys.end()) {
        gpu::dl_grid_twins::subscribe(twin_key, device_id, static_cast<size_t>(nof_ports) * 14 * nsc * sizeof(uint32_t));
        twin_keys.push_back(twin_key);
      }
    }
    const int e = (sector >= 0 && !empty) ? group->acquire(sector) : -1;
    if (e >= 0) {
      // Grouped: the rows go into this sector's staging entry, modulated in the group's next launch.
      stage_grid(*j, reader, group->input(sector, e));
      group->submit(sector, e, context.slot.subframe_slot_index());
      j->entry         = e;
      j->subframe_slot = context.slot.subframe_slot_index();
      j->launched      = true;
    } else if (twin_key != nullptr || !empty) {
      launch(*j, reader, context.slot.subframe_slot_index(), twin_key, context.slot.to_uint());
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

  /// Stages the grid's non-empty ports and modulates the whole slot on the processor's stream (no waiting). With
  /// `twin_key`, the PDSCH REs come from the grid's HBM twin when one was published for `slot` (then every port is
  /// staged and modulated); without a twin an empty grid launches nothing.
  void launch(job& j, const resource_grid_reader& reader, unsigned subframe_slot, const void* twin_key = nullptr,
              uint32_t slot = 0)
  {
    gpu::device_scope           dev(ctx, WHO);
    std::lock_guard<std::mutex> lock(launch_mtx);
    const size_t                row   = static_cast<size_t>(nsc) * sizeof(uint32_t);
    const size_t                slotn = geo.slot_size(subframe_slot);
    hipStream_t                 s     = stream.get();
    const size_t                gsize = nof_ports * geo.nsymb * row;
    const uint8_t*              twin  = twin_key != nullptr ? gpu::dl_grid_twins::take(twin_key, slot, gsize, s) : nullptr;
    if (twin == nullptr && reader.is_empty()) {
      return;  // nothing to transmit
    }
    j.grid.reserve(nof_ports * geo.nsymb * row);
    j.samples.reserve(nof_ports * slotn * sizeof(cf_t));
    if (j.done == nullptr) {
      std::lock_guard<std::recursive_mutex> setup(gpu::hip_setup_mutex());
      gpu::hip_check(hipEventCreateWithFlags(&j.done, hipEventDisableTiming), WHO, "event");
    }
    stage_grid(j, reader, j.grid.host(), twin != nullptr);
    if (twin != nullptr) {
      gpu::srsgpu_check(srsgpu_ofdm_modulator_plan_execute_twin(plans[subframe_slot], j.grid.dev<uint32_t>(),
                                                                reinterpret_cast<const uint32_t*>(twin),
                                                                j.samples.dev<float>(), s),
                        WHO);
      gpu::dl_grid_twins::release(twin_key, s);
      gpu::hip_check(hipEventRecord(j.done, s), WHO, "event");
      j.subframe_slot = subframe_slot;
      j.launched      = true;
      j.own           = true;
      return;
    }
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
  /// `all_ports` (an HBM twin holds the PDSCH REs): no port is empty, an empty one's rows are zeros.
  void stage_grid(job& j, const resource_grid_reader& reader, uint8_t* dst, bool all_ports = false)
  {
    const size_t row = static_cast<size_t>(nsc) * sizeof(uint32_t);
    j.port_empty.assign(nof_ports, false);
    for (unsigned p = 0; p != nof_ports; ++p) {
      j.port_empty[p] = reader.is_empty(p);
      if (j.port_empty[p] && all_ports) {
        j.port_empty[p] = false;
        std::memset(dst + p * geo.nsymb * row, 0, geo.nsymb * row);
        continue;
      }
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
      if (j->entry >= 0) {
        group->ready(sector, j->entry, true);  // a late or dropped request's launch may still write the entry
        group->release(sector, j->entry);
        j->entry = -1;
      }
      std::lock_guard<std::mutex> lock(free_mtx);
      free_jobs.push_back(std::move(j));
    }
  }

  std::shared_ptr<lower_phy_sector_group> group_owner;
  ofdm_batcher*                   group  = nullptr;
  int                             sector = -1;  ///< index in the group, -1: not grouped
  std::shared_ptr<srsgpu_context> owner;
  srsgpu_context*                 ctx;
  gpu::owned_stream               stream;
  symbol_geometry                 geo;
  unsigned                        nof_ports;
  unsigned                        nsc;
  std::vector<srsgpu_ofdm_plan*>  plans;  ///< One whole-slot plan (all ports) per slot of the subframe.
  int                             device_id = 0;
  std::vector<const void*>        twin_keys;  ///< grids subscribed to (gpu::dl_grid_twins)
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
      group  = &group_owner->batcher(false, geo.nslot * geo.nsymb);
      sector = group->add_sector(plans);
    }
  }

  ~puxch_processor_gpu() override
  {
    for (const pending_symbol& ps : pending) {
      if (ps.entry >= 0) {
        group->ready(sector, ps.entry, true);  // the launch still writes the entry
        group->release(sector, ps.entry);
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
      grid_dev = nullptr;
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
        find_grid_rows();
      }
    }
    const unsigned l = context.nof_symbols;
    if (!current_grid) {
      return false;
    }
    const unsigned s = context.slot.subframe_slot_index() * geo.nsymb + l;
    const unsigned n = geo.size[s];
    // Grouped: the samples go into this sector's staging entry, demodulated in the group's next launch.
    const int e = sector >= 0 ? group->acquire(sector) : -1;
    if (e >= 0) {
      uint8_t* dst = group->input(sector, e);
      for (unsigned p = 0; p != nof_ports; ++p) {
        span<const cf_t> in = samples.get_channel_buffer(p);
        srsran_assert(in.size() == n, "The input buffer size ({}) does not match the symbol size ({}).", in.size(), n);
        std::memcpy(dst + static_cast<size_t>(p) * n * sizeof(cf_t), in.data(), n * sizeof(cf_t));
      }
      ofdm_batcher::direct_rows rows;
      if (grid_dev != nullptr) {
        const size_t off = static_cast<size_t>(l) * nsc * sizeof(uint32_t);
        rows             = {grid_dev + off, grid_port_stride, twin.dev != nullptr ? twin.dev + off : nullptr};
      }
      group->submit(sector, e, s, rows);
      if (grid_dev != nullptr && twin.dev != nullptr) {
        // The symbol goes to the twin too; the PUSCH batch copies nothing for a slot whose 14 symbols all did (the
        // launch is queued before this symbol's notification, which precedes the uplink processor's PUSCH job).
        twin.symbols->fetch_or(1u << l, std::memory_order_acq_rel);
      }
      pending.push_back({l, context, e});
      if (l == geo.nsymb - 1) {
        drain(0);
        current_grid.release();
        grid_dev = nullptr;
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
      grid_dev = nullptr;
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
      if (ps.entry >= 0) {
        if (!group->ready(sector, ps.entry, pending.size() > keep)) {
          break;
        }
        rows = group->output(sector, ps.entry);
      } else {
        symbol_stage& st = *stages[ps.symbol];
        if (pending.size() > keep) {
          wait_event(st.done, WHO);
        } else if (hipEventQuery(st.done) != hipSuccess) {
          break;
        }
        rows = st.out.host();
      }
      resource_grid_writer& writer = current_grid.get().get_writer();
      if (ps.entry >= 0 && group->direct(sector, ps.entry)) {
        // Demodulated straight into the grid's rows: only the ports' non-empty marks remain (a put of each row's first
        // element onto itself, resource_grid_writer_impl.cpp clear_empty).
        const resource_grid_reader& reader = current_grid.get().get_reader();
        for (unsigned p = 0; p != nof_ports; ++p) {
          const cbf16_t v = reader.get_view(p, ps.symbol)[0];
          writer.put(p, ps.symbol, 0, 1, span<const cbf16_t>(&v, 1));
        }
      } else {
        for (unsigned p = 0; p != nof_ports; ++p) {
          writer.put(p, ps.symbol, 0, 1,
                     span<const cbf16_t>(reinterpret_cast<const cbf16_t*>(rows + static_cast<size_t>(p) * nsc *
                                                                                      sizeof(uint32_t)),
                                         nsc));
        }
      }
      if (ps.entry >= 0) {
        group->release(sector, ps.entry);
      }
      notifier->on_rx_symbol(current_grid, ps.context);
      pending.pop_front();
    }
  }

  struct pending_symbol {
    unsigned                    symbol;
    lower_phy_rx_symbol_context context;
    int                         entry;  ///< the group staging entry holding the result, -1: this processor's own stage
  };

  /// The current grid's rows in device-mapped host memory (gpu::host_blocks: mapped by the grid's owner, the GPU
  /// uplink processor's PUSCH slot batch), for the sector group to demodulate into directly; nullptr: the rows are
  /// staged and copied into the grid (drain). Needs the reference grid's layout: one [port][symbol][subcarrier] block.
  void find_grid_rows()
  {
    grid_dev = nullptr;
    if (sector < 0 || !current_grid) {
      return;
    }
    const resource_grid_reader& r = current_grid.get().get_reader();
    if (r.get_nof_ports() < nof_ports || r.get_nof_subc() != nsc || r.get_nof_symbols() < geo.nsymb) {
      return;
    }
    const size_t row   = static_cast<size_t>(nsc) * sizeof(uint32_t);
    const size_t nsymb = r.get_nof_symbols();
    const auto*  base  = reinterpret_cast<const uint8_t*>(r.get_view(0, 0).data());
    for (unsigned p = 0; p != nof_ports; ++p) {
      for (unsigned l = 0; l != geo.nsymb; ++l) {
        if (reinterpret_cast<const uint8_t*>(r.get_view(p, l).data()) != base + (p * nsymb + l) * row) {
          return;
        }
      }
    }
    grid_dev         = static_cast<uint8_t*>(gpu::host_blocks::find(base, nof_ports * nsymb * row));
    grid_port_stride = nsymb * row;
    // The HBM twin only when it has the grid's exact shape (the PUSCH batch's grid slot: [port][14][subcarrier]).
    twin = gpu::host_blocks::find_twin(base);
    if (grid_dev == nullptr || nsymb != 14 || geo.nsymb != 14 || twin.bytes != nof_ports * nsymb * row) {
      twin = {};
    }
  }

  std::shared_ptr<lower_phy_sector_group>    group_owner;
  ofdm_batcher*                              group  = nullptr;
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
  uint8_t*                                   grid_dev         = nullptr;  ///< find_grid_rows
  size_t                                     grid_port_stride = 0;
  gpu::host_blocks::twin                     twin;  ///< find_grid_rows: the grid's HBM twin (dev nullptr: none)
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
