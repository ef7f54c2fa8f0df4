// Slot-batched GPU processing behind the reference's downlink slot processor (the uplink side is pusch_batch_gpu.cpp):
// see upper_phy_gpu.h for the design.
#include "upper_phy_gpu.h"
#include <cstdlib>
#include <chrono>
#include <unordered_map>
#include "srsran/support/error_handling.h"

#include "batch_graph.h"
#include "chain_convert.h"
#include "gpu_staging.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_processor_helpers.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_processor_impl.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"
#include "srsran/phy/upper/channel_coding/ldpc/ldpc.h"
#include "srsran/phy/upper/channel_processors/pdsch/pdsch_encoder.h"
#include "srsran/phy/upper/channel_processors/pusch/factories.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_notifier.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_result.h"
#include "srsran/phy/upper/channel_processors/uci/factories.h"
#include "srsran/phy/upper/rx_buffer.h"
#include "srsran/phy/upper/unique_rx_buffer.h"
#include "srsran/phy/upper/uplink_slot_processor.h"
#include "srsran/ran/pusch/ulsch_info.h"
#include "srsran/ran/sch/sch_dmrs_power.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <map>
#include <mutex>
#include <thread>

namespace srsran {
namespace gpu {

// ---------------------------------------------------------------------------------------------------------------------
// PDSCH slot batch
// ---------------------------------------------------------------------------------------------------------------------

namespace {

/// One recorded PDSCH transmission.
struct pdsch_entry {
  resource_grid_writer*          grid     = nullptr;
  pdsch_processor_notifier*      notifier = nullptr;
  srsgpu_pdsch_tb_config         tb;  ///< tb_offset / cw_offset are set per launch
  std::vector<uint8_t>           data;
  unsigned                       cw_bytes = 0;
  crb_bitmap                     crbs;  ///< the allocation's CRBs (the multi-device gather moves these bands)
  uint32_t                       slot = 0;  ///< pdu.slot (the HBM twin's publication tag)
  pdsch_modulator::config_t      mod;
  dmrs_pdsch_processor::config_t dmrs;
};

/// Captures the DM-RS configuration pdsch_process_dmrs builds (pdsch_processor_helpers.h:43-70).
class recording_dmrs : public dmrs_pdsch_processor
{
public:
  dmrs_pdsch_processor::config_t* out = nullptr;
  void map(resource_grid_writer& /*grid*/, const config_t& config) override { *out = config; }
};

thread_local bool pdsch_inline_scope = false;

/// Grid transfers of the multi-device PDSCH batches, process-wide.
struct {
  std::atomic<uint64_t> grid_downloads{0};
  std::atomic<uint64_t> shard_merges{0};
  std::atomic<uint64_t> merge_bytes{0};
  std::atomic<uint64_t> twin_grids{0};
} pdsch_transfers;


/// One device's part of a PDSCH slot batch: its launch plans and captured graphs, TB staging, codewords and a
/// sentinel-filled scratch grid into which the encoder, DM-RS and modulator map its PDSCHs.
class pdsch_shard
{
  static constexpr const char* WHO = "pdsch_slot_batch";

public:
  explicit pdsch_shard(int device_) :
    device(device_),
    owner(shared_context(device_)),
    ctx(owner.get()),
    stream(ctx, WHO),
    enc_plans(srsgpu_pdsch_encoder_plan_destroy, 16),
    mod_plans(srsgpu_pdsch_modulator_plan_destroy, 16),
    dmrs_plans(srsgpu_pdsch_dmrs_plan_destroy, SLOT_PLANS),
    graphs(destroy_graph_exec, SLOT_PLANS),
    tb_buf(WHO),
    grid_buf(WHO)
  {
    device_scope dev(ctx, WHO);
    hip_check(hipEventCreateWithFlags(&done, hipEventDisableTiming), WHO, "event");
  }

  ~pdsch_shard()
  {
    device_scope dev(ctx, WHO);
    (void)hipStreamSynchronize(stream.get());
    (void)hipFree(d_cw);
    (void)hipEventDestroy(done);
  }

  /// The scratch grid (P x 14 rows of `row` bytes) on the device, grown when needed.
  void reserve_grid(size_t bytes)
  {
    device_scope                          dev(ctx, WHO);
    std::lock_guard<std::recursive_mutex> setup_lock(gpu::hip_setup_mutex());
    grid_buf.reserve(bytes);
  }

  /// Queues the PDSCHs `es` on the stream as one captured graph (cached per layout): TB upload, sentinel scratch grid,
  /// encoder, DM-RS, modulator, and, with `download`, the grid back into the host image. Without PDSCHs only the
  /// sentinel fill.
  void launch(const std::vector<const pdsch_entry*>& es, unsigned grid_prb, unsigned P, bool download)
  {
    device_scope   dev(ctx, WHO);
    const unsigned nsc   = grid_prb * NRE;
    const size_t   row   = static_cast<size_t>(nsc) * sizeof(uint32_t);
    const size_t   gsize = static_cast<size_t>(P) * 14 * row;
    hipStream_t    s     = stream.get();
    reserve_grid(gsize);
    if (es.empty()) {
      hip_check(hipMemsetAsync(grid_buf.dev(), 0xff, gsize, s), WHO, "scratch");
      return;
    }
    const unsigned                      n = static_cast<unsigned>(es.size());
    std::vector<srsgpu_pdsch_tb_config> tcs;
    std::vector<pdsch_mod_desc>         mods;
    std::vector<pdsch_dmrs_desc>        dmrss;
    std::vector<uint8_t>                enc_key, mod_key, dmrs_key, tbs;
    unsigned                            cw_bytes = 0;
    gpu::key_append(mod_key, grid_prb);
    gpu::key_append(dmrs_key, grid_prb);
    for (const pdsch_entry* e : es) {
      srsgpu_pdsch_tb_config tc = e->tb;
      tc.tb_offset              = static_cast<uint32_t>(tbs.size());
      tc.cw_offset              = cw_bytes;
      tbs.insert(tbs.end(), e->data.begin(), e->data.end());
      tbs.resize((tbs.size() + 15) / 16 * 16, 0);
      cw_bytes += e->cw_bytes;
      tcs.push_back(tc);
      gpu::key_append(enc_key, tc);
      const unsigned nof_bits = tc.nof_ch_symbols * tc.modulation_order;
      mods.push_back(make_pdsch_mod_desc(e->mod, nof_bits, grid_prb, P, WHO));
      mods.back().c.cw_offset = tc.cw_offset;
      mods.back().append_key(mod_key);
      dmrss.push_back(make_pdsch_dmrs_desc(e->dmrs, grid_prb, P, WHO));
      dmrss.back().append_key(dmrs_key);
    }
    srsgpu_pdsch_encoder_plan* enc = enc_plans.get(enc_key, [&] {
      srsgpu_pdsch_encoder_plan* p = nullptr;
      srsgpu_check(srsgpu_pdsch_encoder_plan_create(ctx, tcs.data(), n, &p), WHO);
      return p;
    });
    srsgpu_pdsch_modulator_plan* mod = mod_plans.get(mod_key, [&] {
      std::vector<srsgpu_pdsch_mod_config> c;
      std::vector<srsgpu_alloc_ext>        x;
      for (pdsch_mod_desc& d : mods) {
        c.push_back(d.c);
        x.push_back(d.ext());
      }
      srsgpu_pdsch_modulator_plan* p = nullptr;
      srsgpu_check(srsgpu_pdsch_modulator_plan_create_ex(ctx, c.data(), x.data(), n, grid_prb, P, &p), WHO);
      return p;
    });
    srsgpu_pdsch_dmrs_plan* dmrs = dmrs_plans.get(dmrs_key, [&] {
      std::vector<srsgpu_pdsch_dmrs_config> c;
      std::vector<srsgpu_alloc_ext>         x;
      for (const pdsch_dmrs_desc& d : dmrss) {
        c.push_back(d.c);
        x.push_back(d.ext());
      }
      srsgpu_pdsch_dmrs_plan* p = nullptr;
      srsgpu_check(srsgpu_pdsch_dmrs_plan_create_ex(ctx, c.data(), x.data(), n, grid_prb, P, &p), WHO);
      return p;
    });
    {
      // Buffer growth and the graph capture call synchronous HIP APIs, which fail while any thread captures a
      // stream: both run under gpu::hip_setup_mutex, as the UL slot batch's do.
      std::lock_guard<std::recursive_mutex> setup_lock(gpu::hip_setup_mutex());
      tb_buf.reserve(std::max<size_t>(tbs.size(), 16));
      if (cw_bytes > d_cw_cap) {
        (void)hipFree(d_cw);
        d_cw     = nullptr;
        d_cw_cap = 0;
        hip_check(hipMalloc(&d_cw, cw_bytes), WHO, "codewords");
        d_cw_cap = cw_bytes;
      }
    }
    std::memcpy(tb_buf.host(), tbs.data(), tbs.size());

    // The shard's device work as one captured graph per layout (cached like the plans it runs), so a slot costs one
    // graph launch instead of six queue operations.
    std::vector<uint8_t> graph_key;
    for (const std::vector<uint8_t>* k : {&enc_key, &mod_key, &dmrs_key}) {
      gpu::key_append(graph_key, k->size());
      graph_key.insert(graph_key.end(), k->begin(), k->end());
    }
    for (const void* ptr : {static_cast<const void*>(tb_buf.host()), static_cast<const void*>(tb_buf.dev()),
                            static_cast<const void*>(grid_buf.host()), static_cast<const void*>(grid_buf.dev()),
                            static_cast<const void*>(d_cw)}) {
      gpu::key_append(graph_key, ptr);
    }
    gpu::key_append(graph_key, tbs.size());
    gpu::key_append(graph_key, P);
    gpu::key_append(graph_key, download);
    std::unique_lock<std::recursive_mutex> setup_lock(gpu::hip_setup_mutex());
    // A plan evicted since the last slot invalidates the graphs that run it.
    const uint64_t generation = enc_plans.evictions() + mod_plans.evictions() + dmrs_plans.evictions();
    if (generation != plan_generation) {
      graphs.clear();
      plan_generation = generation;
    }
    hipGraphExec_t exec = graphs.get(graph_key, [&] { return capture_graph(s, WHO, [&] {
      tb_buf.upload(0, tbs.size(), s);
      // Sentinel scratch grid: exactly the REs the PDSCH and its DM-RS map come back.
      hip_check(hipMemsetAsync(grid_buf.dev(), 0xff, gsize, s), WHO, "scratch");
      srsgpu_check(srsgpu_pdsch_encoder_plan_execute(enc, tb_buf.dev<uint8_t>(), d_cw, s), WHO);
      srsgpu_check(srsgpu_pdsch_dmrs_plan_execute(dmrs, grid_buf.dev<uint32_t>(), s), WHO);
      srsgpu_check(srsgpu_pdsch_modulator_plan_execute(mod, d_cw, grid_buf.dev<uint32_t>(), s), WHO);
      if (download) {
        grid_buf.download(0, gsize, s);
      }
    }); });
    setup_lock.unlock();
    hip_check(hipGraphLaunch(exec, s), WHO, "graph launch");
  }

  int                                               device;
  std::shared_ptr<srsgpu_context>                   owner;
  srsgpu_context*                                   ctx;
  owned_stream                                      stream;
  plan_cache<srsgpu_pdsch_encoder_plan>             enc_plans;
  plan_cache<srsgpu_pdsch_modulator_plan>           mod_plans;
  plan_cache<srsgpu_pdsch_dmrs_plan>                dmrs_plans;
  plan_cache<std::remove_pointer_t<hipGraphExec_t>> graphs;
  uint64_t                                          plan_generation = 0;
  staged_buffer                                     tb_buf;
  staged_buffer                                     grid_buf;
  uint8_t*                                          d_cw     = nullptr;
  size_t                                            d_cw_cap = 0;
  hipEvent_t                                        done     = nullptr;
};

} // namespace

pdsch_multi_transfer_counters get_pdsch_multi_transfer_counters()
{
  return {pdsch_transfers.grid_downloads.load(), pdsch_transfers.shard_merges.load(),
          pdsch_transfers.merge_bytes.load(), pdsch_transfers.twin_grids.load()};
}

class pdsch_slot_batch
{
  static constexpr const char* WHO = "pdsch_slot_batch";

public:
  pdsch_slot_batch(const pdsch_batch_configuration&      config,
                   std::unique_ptr<ptrs_pdsch_generator> ptrs_,
                   std::unique_ptr<pdsch_processor>      fallback_) :
    ptrs(std::move(ptrs_)), fallback(std::move(fallback_)), spans(WHO)
  {
    if (!ptrs || !fallback) {
      throw std::invalid_argument(std::string(WHO) + ": invalid dependencies");
    }
    const std::vector<int> devs = config.devices.empty() ? std::vector<int>{config.device} : config.devices;
    for (int d : devs) {
      shards.push_back(std::make_unique<pdsch_shard>(d));
    }
  }

  /// pdsch_processor_impl::process (pdsch_processor_impl.cpp:42-90) up to the point where the encoder, modulator and
  /// DM-RS would run: their configurations are recorded for the batch; PT-RS is generated into the grid right away.
  void add(resource_grid_writer&                                                           grid,
           pdsch_processor_notifier&                                                       notifier,
           static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data,
           const pdsch_processor::pdu_t&                                                   pdu)
  {
    const unsigned nof_layers = pdu.precoding.get_nof_layers();
    if (nof_layers == 0 || nof_layers > 4 || pdu.precoding.get_nof_ports() > 4 || data.size() != 1) {
      fallback->process(grid, notifier, std::move(data), pdu);  // two codewords (more than four layers)
      return;
    }
    std::lock_guard<std::mutex> lock(mtx);
    pdsch_entry                 e;
    e.grid                     = &grid;
    e.notifier                 = &notifier;
    e.slot                     = pdu.slot.to_uint();
    span<const uint8_t> tb     = data[0].get_buffer();
    const unsigned      nre    = pdsch_compute_nof_data_re(pdu);
    const unsigned      qm     = get_bits_per_symbol(pdu.codewords[0].modulation);
    const units::bits   tbs    = units::bytes(tb.size()).to_bits();
    std::memset(&e.tb, 0, sizeof(e.tb));
    e.tb.base_graph       = bg_number(pdu.ldpc_base_graph);
    e.tb.rv               = static_cast<uint8_t>(pdu.codewords[0].rv);
    e.tb.modulation_order = static_cast<uint8_t>(qm);
    e.tb.nof_layers       = static_cast<uint8_t>(nof_layers);
    e.tb.tbs_bytes        = static_cast<uint32_t>(tb.size());
    e.tb.nof_ch_symbols   = nre * nof_layers;
    e.tb.Nref = ldpc::compute_N_ref(pdu.tbs_lbrm, ldpc::compute_nof_codeblocks(tbs, pdu.ldpc_base_graph)).value();
    e.data.assign(tb.begin(), tb.end());
    e.cw_bytes = (nre * nof_layers * qm + 31) / 32 * 4;
    e.crbs     = pdu.freq_alloc.get_crb_mask(pdu.bwp_start_rb, pdu.bwp_size_rb);

    // The modulator configuration pdsch_processor_impl::modulate builds (pdsch_processor_impl.cpp:143-161; one
    // codeword; dmrs_config_type is not set there, so it keeps its default, type 1).
    pdsch_modulator::config_t& m     = e.mod;
    m.rnti                        = pdu.rnti;
    m.bwp_size_rb                 = pdu.bwp_size_rb;
    m.bwp_start_rb                = pdu.bwp_start_rb;
    m.modulation1                 = pdu.codewords[0].modulation;
    m.modulation2                 = modulation_scheme::BPSK;
    m.freq_allocation             = pdu.freq_alloc;
    m.start_symbol_index          = pdu.start_symbol_index;
    m.nof_symbols                 = pdu.nof_symbols;
    m.dmrs_symb_pos               = pdu.dmrs_symbol_mask;
    m.nof_cdm_groups_without_data = pdu.nof_cdm_groups_without_data;
    m.n_id                        = pdu.n_id;
    m.scaling                     = convert_dB_to_amplitude(-pdu.ratio_pdsch_data_to_sss_dB);
    m.reserved                    = pdu.reserved;
    m.precoding                   = pdu.precoding;
    if (pdu.ptrs) {
      pdsch_process_ptrs(grid, *ptrs, pdu);
    }
    recording_dmrs rec;
    rec.out = &e.dmrs;
    pdsch_process_dmrs(grid, rec, pdu);
    entries.push_back(std::move(e));
  }

  /// Encodes, modulates and maps every recorded PDSCH, stores the REs into the slot's grid and reports each PDSCH
  /// finished (after which the reference's downlink processor sends the grid). One device: one launch sequence and one
  /// download. Several devices (row b7's DL counterpart): a UE's PDSCH runs on the device of its RNTI modulo the number
  /// of devices, every shard maps into its own sentinel-filled grid, the other shards' subcarrier bands are merged into
  /// the root's grid on the root (peer reads over xGMI, sentinel words skipped) and the root's grid comes back once.
  void flush()
  {
    std::vector<pdsch_entry> es;
    {
      std::lock_guard<std::mutex> lock(mtx);
      es = std::exchange(entries, {});
    }
    if (es.empty()) {
      return;
    }
    std::lock_guard<std::mutex> lock(run_mtx);
    resource_grid_writer&       grid     = *es.front().grid;
    const unsigned              nsc      = grid.get_nof_subc();
    const unsigned              grid_prb = nsc / NRE;
    const unsigned              P        = grid.get_nof_ports();
    const unsigned              D        = static_cast<unsigned>(shards.size());
    const size_t                row      = static_cast<size_t>(nsc) * sizeof(uint32_t);
    const size_t                gsize    = static_cast<size_t>(P) * 14 * row;
    std::vector<std::vector<const pdsch_entry*>> part(D);
    for (const pdsch_entry& e : es) {
      if (e.grid != &grid) {
        throw std::logic_error(std::string(WHO) + ": PDSCH of one batch in different resource grids");
      }
      part[D == 1 ? 0 : e.mod.rnti % D].push_back(&e);
    }
    pdsch_shard& root = *shards[0];
    if (D == 1) {
      // A GPU PDxCH on this device modulates the grid (gpu::dl_grid_twins): the REs stay in the grid's HBM twin.
      uint8_t* twin = nullptr;
      {
        device_scope rdev(root.ctx, WHO);
        twin = gpu::dl_grid_twins::begin(&grid, root.device, gsize, root.stream.get());
        if (twin != nullptr) {
          // Without the download's synchronisation below, the previous slot's launch is waited for here, before this
          // one rewrites its TB staging.
          hip_check(hipStreamSynchronize(root.stream.get()), WHO, "synchronise");
        }
      }
      if (twin != nullptr) {
        root.launch(part[0], grid_prb, P, false);
        device_scope rdev(root.ctx, WHO);
        hip_check(hipMemcpyAsync(twin, root.grid_buf.dev(), gsize, hipMemcpyDeviceToDevice, root.stream.get()), WHO,
                  "twin copy");
        gpu::dl_grid_twins::publish(&grid, es.front().slot, root.stream.get());
        pdsch_transfers.twin_grids.fetch_add(1, std::memory_order_relaxed);
        for (pdsch_entry& e : es) {
          e.notifier->on_finish_processing();
        }
        return;
      }
      root.launch(part[0], grid_prb, P, true);
    } else {
      // The shards' launches first, so that they run while the root maps its own UEs.
      for (unsigned s = 1; s != D; ++s) {
        if (!part[s].empty()) {
          shards[s]->launch(part[s], grid_prb, P, false);
          device_scope sdev(shards[s]->ctx, WHO);
          hip_check(hipEventRecord(shards[s]->done, shards[s]->stream.get()), WHO, "event");
        }
      }
      root.launch(part[0], grid_prb, P, false);
      // Each shard's bands: its UEs' allocations, merged.
      size_t nspans = 0;
      std::vector<std::vector<std::pair<unsigned, unsigned>>> bands(D);
      for (unsigned s = 1; s != D; ++s) {
        for (const pdsch_entry* e : part[s]) {
          if (e->crbs.any()) {
            bands[s].emplace_back(static_cast<unsigned>(e->crbs.find_lowest()) * NRE,
                                  (static_cast<unsigned>(e->crbs.find_highest()) + 1) * NRE);
          }
        }
        std::sort(bands[s].begin(), bands[s].end());
        std::vector<std::pair<unsigned, unsigned>> merged;
        for (const auto& r : bands[s]) {
          if (!merged.empty() && r.first <= merged.back().second) {
            merged.back().second = std::max(merged.back().second, r.second);
          } else {
            merged.push_back(r);
          }
        }
        bands[s] = std::move(merged);
        nspans += bands[s].size() * P * 14;
      }
      device_scope rdev(root.ctx, WHO);
      hipStream_t  rs = root.stream.get();
      spans.reserve(std::max<size_t>(nspans, 1) * sizeof(srsgpu_copy_span));
      auto*    sp   = spans.host<srsgpu_copy_span>();
      size_t   next = 0;
      uint64_t most = 0;
      for (unsigned s = 1; s != D; ++s) {
        if (part[s].empty()) {
          continue;
        }
        for (const auto& b : bands[s]) {
          const size_t off = static_cast<size_t>(b.first) * sizeof(uint32_t);
          const size_t len = static_cast<size_t>(b.second - b.first) * sizeof(uint32_t);
          for (unsigned r = 0; r != P * 14; ++r) {
            sp[next++] = {shards[s]->grid_buf.dev(r * row + off), root.grid_buf.dev(r * row + off), len};
            pdsch_transfers.merge_bytes.fetch_add(len, std::memory_order_relaxed);
          }
          most = std::max<uint64_t>(most, len);
        }
        hip_check(hipStreamWaitEvent(rs, shards[s]->done, 0), WHO, "wait for a shard");
        pdsch_transfers.shard_merges.fetch_add(1, std::memory_order_relaxed);
      }
      if (next != 0) {
        srsgpu_check(srsgpu_merge_spans(spans.dev<srsgpu_copy_span>(), static_cast<uint32_t>(next), most,
                                        GRID_SENTINEL, rs),
                     WHO);
      }
      root.grid_buf.download(0, gsize, rs);
    }
    pdsch_transfers.grid_downloads.fetch_add(1, std::memory_order_relaxed);
    {
      device_scope rdev(root.ctx, WHO);
      hip_check(hipStreamSynchronize(root.stream.get()), WHO, "synchronise");
    }
    store_written_res(grid, root.grid_buf.host<uint32_t>(), P, nsc, 0, 14);
    for (pdsch_entry& e : es) {
      e.notifier->on_finish_processing();
    }
  }

private:
  std::unique_ptr<ptrs_pdsch_generator>     ptrs;
  std::unique_ptr<pdsch_processor>          fallback;
  std::vector<std::unique_ptr<pdsch_shard>> shards;
  mapped_buffer                             spans;  ///< the multi-device gather's merge list
  std::mutex                                mtx;
  std::vector<pdsch_entry>                  entries;
  std::mutex                                run_mtx;
};

std::shared_ptr<pdsch_slot_batch> create_pdsch_slot_batch(const pdsch_batch_configuration&      config,
                                                          std::unique_ptr<ptrs_pdsch_generator> ptrs,
                                                          std::unique_ptr<pdsch_processor>      fallback)
{
  return std::make_shared<pdsch_slot_batch>(config, std::move(ptrs), std::move(fallback));
}

std::shared_ptr<pdsch_slot_batch> create_pdsch_slot_batch(int                                   device,
                                                          std::unique_ptr<ptrs_pdsch_generator> ptrs,
                                                          std::unique_ptr<pdsch_processor>      fallback)
{
  pdsch_batch_configuration c;
  c.device = device;
  return create_pdsch_slot_batch(c, std::move(ptrs), std::move(fallback));
}

namespace {

class pdsch_processor_batch_gpu : public pdsch_processor
{
public:
  explicit pdsch_processor_batch_gpu(std::shared_ptr<pdsch_slot_batch> batch_) : batch(std::move(batch_)) {}

  void process(resource_grid_writer&                                           grid,
               pdsch_processor_notifier&                                       notifier,
               static_vector<shared_transport_block, MAX_NOF_TRANSPORT_BLOCKS> data,
               const pdu_t&                                                    pdu) override
  {
    batch->add(grid, notifier, std::move(data), pdu);
  }

private:
  std::shared_ptr<pdsch_slot_batch> batch;
};

/// The reference's downlink processor with the slot's PDSCHs recorded inline and run as one batch at the end.
class downlink_processor_batch_gpu : public downlink_processor_base,
                                     private downlink_processor_controller,
                                     private unique_downlink_processor::downlink_processor_callback
{
public:
  downlink_processor_batch_gpu(std::unique_ptr<downlink_processor_base> inner_,
                               std::shared_ptr<pdsch_slot_batch>        batch_,
                               task_executor&                           executor_) :
    inner(std::move(inner_)), batch(std::move(batch_)), executor(executor_)
  {
  }

  downlink_processor_controller& get_controller() override { return *this; }
  void                           stop() override { inner->stop(); }

private:
  unique_downlink_processor configure_resource_grid(const resource_grid_context& context,
                                                    shared_resource_grid         grid) override
  {
    current = inner->get_controller().configure_resource_grid(context, std::move(grid));
    if (!current.is_valid()) {
      return {};
    }
    return unique_downlink_processor(*this);
  }

  void process_pdcch(const pdcch_processor::pdu_t& pdu) override { current->process_pdcch(pdu); }
  void process_ssb(const ssb_processor::pdu_t& pdu) override { current->process_ssb(pdu); }
  void process_nzp_csi_rs(const nzp_csi_rs_generator::config_t& config) override
  {
    current->process_nzp_csi_rs(config);
  }
  void process_prs(const prs_generator_configuration& config) override { current->process_prs(config); }

  void process_pdsch(static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data,
                     const pdsch_processor::pdu_t&                                                    pdu) override
  {
    // The reference enqueues the PDSCH task on its executor (pdsch_batch_executor): within this scope it runs here,
    // and the batch pdsch_processor records the transmission.
    pdsch_inline_scope = true;
    current->process_pdsch(std::move(data), pdu);
    pdsch_inline_scope = false;
  }

  void finish_processing_pdus() override
  {
    // The reference's state machine sends the grid once every task, including the batched PDSCHs, has completed.
    unique_downlink_processor         proc = std::move(current);
    std::shared_ptr<pdsch_slot_batch> b    = batch;
    auto job = [b]() {
      try {
        b->flush();
      } catch (const std::exception& e) {
        report_fatal_error("pdsch_slot_batch: {}", e.what());  // as the UL batch
      }
    };
    if (!executor.execute(job)) {
      job();
    }
    proc.release();
  }

  std::unique_ptr<downlink_processor_base> inner;
  std::shared_ptr<pdsch_slot_batch>        batch;
  task_executor&                           executor;
  unique_downlink_processor                current;
};

} // namespace

bool pdsch_batch_executor::execute(unique_task task)
{
  if (pdsch_inline_scope) {
    task();
    return true;
  }
  return real.execute(std::move(task));
}

bool pdsch_batch_executor::defer(unique_task task)
{
  if (pdsch_inline_scope) {
    task();
    return true;
  }
  return real.defer(std::move(task));
}

std::unique_ptr<pdsch_processor> create_pdsch_processor_batch_gpu(std::shared_ptr<pdsch_slot_batch> batch)
{
  return std::make_unique<pdsch_processor_batch_gpu>(std::move(batch));
}

std::unique_ptr<downlink_processor_base> create_downlink_processor_batch_gpu(std::unique_ptr<downlink_processor_base> inner,
                                                                             std::shared_ptr<pdsch_slot_batch> batch,
                                                                             task_executor&                    executor)
{
  return std::make_unique<downlink_processor_batch_gpu>(std::move(inner), std::move(batch), executor);
}

} // namespace gpu
} // namespace srsran
