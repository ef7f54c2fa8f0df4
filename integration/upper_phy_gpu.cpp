// Slot-batched GPU processing behind the reference's upper-PHY slot processors: see upper_phy_gpu.h for the design.
#include "upper_phy_gpu.h"
#include <cstdlib>
#include <chrono>
#include <unordered_map>
#include "srsran/support/error_handling.h"

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

#include <array>
#include <cstdio>
#include <map>
#include <mutex>
#include <thread>

namespace srsran {
namespace gpu {

namespace {

constexpr unsigned HARQ_SLOT_BYTES = 66 * 384;  ///< N of BG1 at Z = 384: one arena slot per codeblock.

uint8_t bg_number(ldpc_base_graph_type bg)
{
  return bg == ldpc_base_graph_type::BG1 ? 1 : 2;
}

/// Codeblock length N (soft bits kept for HARQ) and message bits K Z of a transport block's codeblocks.
void ldpc_lengths(units::bits tbs, ldpc_base_graph_type bg, unsigned& N, unsigned& KZ)
{
  const unsigned Z = ldpc::compute_lifting_size(tbs, bg, ldpc::compute_nof_codeblocks(tbs, bg));
  N                = (bg == ldpc_base_graph_type::BG1 ? 66 : 50) * Z;
  KZ               = (bg == ldpc_base_graph_type::BG1 ? 22 : 10) * Z;
}

} // namespace

// ---------------------------------------------------------------------------------------------------------------------
// HARQ arena
// ---------------------------------------------------------------------------------------------------------------------

class pusch_harq_arena
{
public:
  pusch_harq_arena(int device, unsigned max_cb_ids_) : ctx(shared_context(device)), max_cb_ids(max_cb_ids_)
  {
    device_scope dev(ctx.get(), "pusch_harq_arena");
    // Zero-initialised like the reference's codeblock pool storage; never cleared afterwards (the reference's
    // rx_buffer soft bits persist across reservations: a new transmission overwrites what the dematcher writes).
    hip_check(hipMalloc(&d_soft, static_cast<size_t>(max_cb_ids) * HARQ_SLOT_BYTES), "pusch_harq_arena", "arena");
    hip_check(hipMemset(d_soft, 0, static_cast<size_t>(max_cb_ids) * HARQ_SLOT_BYTES), "pusch_harq_arena", "arena");
  }
  ~pusch_harq_arena() { (void)hipFree(d_soft); }

  std::shared_ptr<srsgpu_context> ctx;
  unsigned                        max_cb_ids;
  int8_t*                         d_soft = nullptr;
};

std::shared_ptr<pusch_harq_arena> create_pusch_harq_arena(int device, unsigned max_cb_ids)
{
  return std::make_shared<pusch_harq_arena>(device, max_cb_ids);
}

// ---------------------------------------------------------------------------------------------------------------------
// PUSCH slot batch
// ---------------------------------------------------------------------------------------------------------------------

namespace {

/// One registered PUSCH transmission and what the batch derives for it.
struct pusch_entry {
  pusch_processor::pdu_t           pdu;
  span<uint8_t>                    data;
  unique_rx_buffer                 rm;
  pusch_processor_result_notifier* notifier = nullptr;
  const resource_grid_reader*      grid     = nullptr;
  // Layout within the batch.
  unsigned nof_rb     = 0;
  unsigned nof_cbs    = 0;
  unsigned cb0        = 0;  ///< First codeblock of the TB in the batch.
  unsigned llr_offset = 0;
  unsigned nof_llrs   = 0;
  unsigned tb_offset  = 0;
  unsigned harq0      = 0;  ///< First byte of the TB's HARQ soft bits in the batch HARQ buffer.
  unsigned cb_N       = 0;
  unsigned cb_KZ      = 0;
  bool     new_data   = true;
  int      demux_index  = -1;  ///< UCI on PUSCH: the transmission's entry in the demultiplexer plan.
  unsigned sch_offset   = 0;   ///< First UL-SCH LLR the decoder reads.
  unsigned nof_sch_llrs = 0;
};

/// Replay stages: the reference's pusch_processor_impl runs per PDU on the batch's results.
class replay_estimator : public dmrs_pusch_estimator
{
public:
  const float* nv = nullptr;
  const float* m  = nullptr;

  void estimate(channel_estimate& estimate, const resource_grid_reader& /*grid*/, const configuration& config) override
  {
    const unsigned P = config.rx_ports.size();
    const unsigned L = config.get_nof_tx_layers();
    estimate.resize({static_cast<unsigned>(config.rb_mask.size()), config.first_symbol + config.nof_symbols, P, L});
    write_chest_metrics(estimate, nv, m, P, L);
  }
};

class replay_demodulator : public pusch_demodulator
{
public:
  pusch_demodulator_options opts;
  const int8_t*             llrs     = nullptr;
  const uint32_t*           seq      = nullptr;
  const float*              stats    = nullptr;
  unsigned                  nof_llrs = 0;
  unsigned                  nof_rb   = 0;

  void demodulate(pusch_codeword_buffer&      codeword_buffer,
                  pusch_demodulator_notifier& notifier,
                  const resource_grid_reader& /*grid*/,
                  const channel_estimate& /*estimates*/,
                  const configuration& config) override
  {
    feed_codeword(codeword_buffer, notifier, config, nof_rb, llrs, seq, nof_llrs, stats, opts, seq_bytes, block_seq,
                  "pusch_slot_batch");
  }

private:
  std::vector<uint8_t> seq_bytes;
  dynamic_bit_buffer   block_seq;
};

/// The decoder stage of the replay: the TB was decoded on the GPU; on_end_softbits() settles the rx buffer like
/// pusch_decoder_impl::join_and_notify (pusch_decoder_impl.cpp:386-440) and notifies the result.
class replay_decoder : public pusch_decoder, private pusch_decoder_buffer
{
public:
  const uint8_t* cb_flags = nullptr;  ///< CB CRC flags after the decode (batch-wide array, first of the TB).
  const int32_t* cb_iters = nullptr;  ///< Iterations per CB (> 0 on success).
  const uint8_t* tb       = nullptr;  ///< Decoded TB bytes.
  const uint8_t* cb_msgs  = nullptr;  ///< Decoded messages, SRSGPU_CB_MSG_STRIDE bytes per CB.
  const uint8_t* decoded  = nullptr;  ///< 1: the CB went through the LDPC decoder in this transmission.
  bool           tb_ok    = false;
  unsigned       cb_KZ    = 0;
  unsigned       max_iter = 6;

  pusch_decoder_buffer& new_data(span<uint8_t>           transport_block_,
                                 unique_rx_buffer        rm_,
                                 pusch_decoder_notifier& notifier_,
                                 const configuration& /*cfg*/) override
  {
    transport_block = transport_block_;
    rm              = std::move(rm_);
    notifier        = &notifier_;
    return *this;
  }

  void set_nof_softbits(units::bits /*nof_softbits*/) override {}

private:
  span<log_likelihood_ratio> get_next_block_view(unsigned block_size) override
  {
    scratch.resize(std::max<size_t>(scratch.size(), block_size));
    return span<log_likelihood_ratio>(scratch).first(block_size);
  }
  void on_new_softbits(span<const log_likelihood_ratio> /*softbits*/) override {}

  void on_end_softbits() override
  {
    span<bool>           crcs    = rm->get_codeblocks_crc();
    const unsigned       nof_cbs = crcs.size();
    pusch_decoder_result result;
    result.tb_crc_ok            = tb_ok;
    result.nof_codeblocks_total = nof_cbs;
    result.ldpc_decoder_stats.reset();
    if (cb_stats.size() < nof_cbs) {
      cb_stats.resize(nof_cbs, 0);
    }
    for (unsigned c = 0; c != nof_cbs; ++c) {
      // pusch_decoder_impl.cpp:339-352: the iterations of a decoded CB (all of them on failure); a CB whose CRC had
      // already passed is not decoded again and keeps its previous statistic.
      if (decoded[c] != 0) {
        cb_stats[c] = cb_iters[c] > 0 ? static_cast<unsigned>(cb_iters[c]) : max_iter;
      }
      result.ldpc_decoder_stats.update(cb_stats[c]);
      crcs[c] = cb_flags[c] != 0;
    }
    if (tb_ok) {
      std::memcpy(transport_block.data(), tb, transport_block.size());
      rm.release();
    } else {
      // Codeblocks that passed keep their message for the retransmission (rx_buffer::get_codeblock_data_bits).
      const unsigned nbytes = (cb_KZ + 7) / 8;
      for (unsigned c = 0; c != nof_cbs; ++c) {
        if (crcs[c]) {
          bit_buffer bits = rm->get_codeblock_data_bits(c, cb_KZ);
          for (unsigned i = 0; i != nbytes; ++i) {
            bits.set_byte(cb_msgs[static_cast<size_t>(c) * SRSGPU_CB_MSG_STRIDE + i], i);
          }
        }
      }
      rm.unlock();
    }
    notifier->on_sch_data(result);
  }

  span<uint8_t>                     transport_block;
  unique_rx_buffer                  rm;
  pusch_decoder_notifier*           notifier = nullptr;
  std::vector<log_likelihood_ratio> scratch;
  std::vector<unsigned>             cb_stats;
};

/// Capacity of the caches whose plans depend on the slot number (DM-RS sequences, and the UL slot graphs that run
/// them): a grant pattern repeats every frame, i.e. every 10 x 2^mu slots (40 at 60 kHz), so a few patterns of a frame
/// stay resident instead of every slot missing.
constexpr size_t SLOT_PLANS = 160;

void destroy_graph_exec(hipGraphExec_t x)
{
  (void)hipGraphExecDestroy(x);
}

/// Captures the queue operations `body` issues on `s` (relaxed mode; the caller holds gpu::hip_setup_mutex) into an
/// instantiated graph. A capture an error interrupts is ended, so the stream stays usable.
template <typename F>
hipGraphExec_t capture_graph(hipStream_t s, const char* who, F&& body)
{
  hip_check(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed), who, "begin capture");
  struct capture_guard {
    hipStream_t s;
    bool        open = true;
    ~capture_guard()
    {
      if (open) {
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphDestroy(g);
      }
    }
  } guard{s};
  body();
  hipGraph_t g = nullptr;
  guard.open   = false;
  hip_check(hipStreamEndCapture(s, &g), who, "end capture");
  hipGraphExec_t   x = nullptr;
  const hipError_t r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  hip_check(r, who, "graph instantiate");
  return x;
}

/// A reference pusch_processor_impl over the replay stages (one per thread that runs batches: the processor's
/// dependency pool binds its instances to threads, concurrent_thread_local_object_pool.h:67-96).
struct replay_processor {
  replay_estimator*               est   = nullptr;
  replay_demodulator*             demod = nullptr;
  replay_decoder*                 dec   = nullptr;
  std::unique_ptr<pusch_processor> proc;
};

} // namespace

class pusch_slot_batch
{
  static constexpr const char* WHO = "pusch_slot_batch";

public:
  pusch_slot_batch(const pusch_batch_configuration&           cfg_,
                   std::shared_ptr<pusch_harq_arena>          arena_,
                   std::shared_ptr<ulsch_demultiplex_factory> demux_factory_,
                   std::shared_ptr<uci_decoder_factory>       uci_factory_,
                   std::unique_ptr<pusch_processor>           fallback_) :
    cfg(cfg_),
    arena(std::move(arena_)),
    ctx(arena->ctx.get()),
    demux_factory(std::move(demux_factory_)),
    uci_factory(std::move(uci_factory_)),
    fallback(std::move(fallback_)),
    stream(ctx, WHO),
    chest_plans(srsgpu_pusch_chest_plan_destroy, SLOT_PLANS),
    demod_plans(srsgpu_pusch_demodulator_plan_destroy, 16),
    dec_plans(srsgpu_pusch_decoder_plan_destroy, 16),
    demux_plans(srsgpu_ulsch_demux_plan_destroy, 16),
    io(WHO),
    graphs(destroy_graph_exec, SLOT_PLANS)
  {
    if (!fallback || !demux_factory || !uci_factory) {
      throw std::invalid_argument(std::string(WHO) + ": invalid dependencies");
    }
  }

  ~pusch_slot_batch()
  {
    if (timing && timed_slots > 0) {
      // SRSGPU_BATCH_TIMING=1: mean host-clock time per slot of each phase of run() (diagnostics).
      std::fprintf(stderr,
                   "pusch_slot_batch: %llu slots, us per slot: setup %.1f, host fill %.1f, graph lookup %.1f, "
                   "launch+GPU+sync %.1f, replay %.1f\n",
                   static_cast<unsigned long long>(timed_slots), phase_us[0] / timed_slots,
                   phase_us[1] / timed_slots, phase_us[2] / timed_slots, phase_us[3] / timed_slots,
                   phase_us[4] / timed_slots);
    }
    (void)hipStreamSynchronize(stream.get());
    (void)hipFree(d_ce);
    (void)hipFree(d_harq);
  }

  void add(pusch_entry&& e)
  {
    std::lock_guard<std::mutex> lock(pending_mtx);
    pending.push_back(std::move(e));
  }

  std::vector<pusch_entry> take()
  {
    std::lock_guard<std::mutex> lock(pending_mtx);
    return std::exchange(pending, {});
  }

  void run(std::vector<pusch_entry>& entries);

private:
  /// PDUs the batch covers: SCH data (with or without HARQ-ACK / CSI Part 1 on PUSCH), identity rx port list, up to
  /// four layers. CSI Part 2 needs the decoded CSI Part 1 before the UL-SCH bits are known
  /// (pusch_processor_impl.cpp:60-100), so those PDUs go to the fallback processor.
  static bool batchable(const pusch_entry& e)
  {
    const pusch_processor::pdu_t& pdu = e.pdu;
    if (!pdu.codeword.has_value() || !pdu.uci.csi_part2_size.entries.empty() || pdu.nof_tx_layers == 0 ||
        pdu.nof_tx_layers > 4 ||
        pdu.rx_ports.empty() || pdu.rx_ports.size() > 4 || pdu.cp != cyclic_prefix::NORMAL) {
      return false;
    }
    for (unsigned p = 0; p != pdu.rx_ports.size(); ++p) {
      if (pdu.rx_ports[p] != p) {
        return false;
      }
    }
    return true;
  }

  replay_processor& replay_for_this_thread();

  template <typename T>
  static void reserve_device(T*& ptr, size_t& cap, size_t bytes, const char* what)
  {
    if (bytes <= cap) {
      return;
    }
    (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    hip_check(hipMalloc(reinterpret_cast<void**>(&ptr), bytes), WHO, what);
    cap = bytes;
  }

  pusch_batch_configuration                     cfg;
  std::shared_ptr<pusch_harq_arena>             arena;
  srsgpu_context*                               ctx;
  std::shared_ptr<ulsch_demultiplex_factory>    demux_factory;
  std::shared_ptr<uci_decoder_factory>          uci_factory;
  std::unique_ptr<pusch_processor>              fallback;
  owned_stream                                  stream;
  plan_cache<srsgpu_pusch_chest_plan>           chest_plans;
  plan_cache<srsgpu_pusch_demodulator_plan>     demod_plans;
  plan_cache<srsgpu_pusch_decoder_plan>         dec_plans;
  plan_cache<srsgpu_ulsch_demux_plan>           demux_plans;
  staged_buffer                                 io;  ///< A slot's inputs and outputs (layout in run()).
  plan_cache<std::remove_pointer_t<hipGraphExec_t>> graphs;
  std::unordered_map<std::string, std::vector<std::vector<uint32_t>>> seq_cache;  ///< demodulator key -> sequences
  uint64_t                                      plan_generation = 0;
  const bool                                    timing          = std::getenv("SRSGPU_BATCH_TIMING") != nullptr;
  double                                        phase_us[5]     = {};
  uint64_t                                      timed_slots     = 0;
  uint32_t*                                     d_ce      = nullptr;
  size_t                                        d_ce_cap  = 0;
  int8_t*                                       d_harq    = nullptr;
  size_t                                        d_harq_cap = 0;
  std::mutex                                    pending_mtx;
  std::vector<pusch_entry>                      pending;
  std::mutex                                    run_mtx;
  std::map<std::thread::id, replay_processor>   replays;
  std::vector<uint8_t>                          decoded_flags;
};

replay_processor& pusch_slot_batch::replay_for_this_thread()
{
  auto it = replays.find(std::this_thread::get_id());
  if (it != replays.end()) {
    return it->second;
  }
  replay_processor r;
  auto             est   = std::make_unique<replay_estimator>();
  auto             demod = std::make_unique<replay_demodulator>();
  auto             dec   = std::make_unique<replay_decoder>();
  r.est                  = est.get();
  r.demod                = demod.get();
  r.dec                  = dec.get();
  demod->opts            = cfg.demodulator;
  std::vector<std::unique_ptr<pusch_processor_impl::concurrent_dependencies>> deps;
  deps.push_back(std::make_unique<pusch_processor_impl::concurrent_dependencies>(
      std::move(est),
      std::move(demod),
      demux_factory->create(),
      uci_factory->create(),
      channel_estimate::channel_estimate_dimensions{MAX_RB, MAX_NSYMB_PER_SLOT, 4, 4}));
  pusch_processor_impl::configuration pc;
  pc.thread_local_dependencies_pool =
      std::make_shared<pusch_processor_impl::concurrent_dependencies_pool_type>(std::move(deps));
  pc.decoder               = std::move(dec);
  pc.dec_nof_iterations    = cfg.nof_ldpc_iterations;
  pc.dec_enable_early_stop = cfg.ldpc_early_stop;
  pc.csi_sinr_calc_method  = cfg.csi_sinr_calc_method;
  r.proc                   = std::make_unique<pusch_processor_impl>(pc);
  return replays.emplace(std::this_thread::get_id(), std::move(r)).first->second;
}

void pusch_slot_batch::run(std::vector<pusch_entry>& all)
{
  std::lock_guard<std::mutex> lock(run_mtx);
  device_scope                dev(ctx, WHO);

  // PDUs outside the batch's scope go through the fallback processor, one by one, as the reference would.
  std::vector<pusch_entry*> batch;
  for (pusch_entry& e : all) {
    if (batchable(e)) {
      batch.push_back(&e);
    } else {
      fallback->process(e.data, std::move(e.rm), *e.notifier, *e.grid, e.pdu);
    }
  }
  if (batch.empty()) {
    return;
  }
  const resource_grid_reader& grid     = *batch.front()->grid;
  const unsigned              nsc      = grid.get_nof_subc();
  const unsigned              grid_prb = nsc / NRE;
  unsigned                    P        = 0;
  for (pusch_entry* e : batch) {
    P = std::max<unsigned>(P, e->pdu.rx_ports.size());
  }

  // Estimates in the compact layout with the "average" time strategy (one row per allocation and rx port, the CFO
  // rotation of each symbol applied by the demodulator; the LLRs equal the per-symbol layout's bit for bit,
  // tests/test_pusch_chest_gpu.py): the estimator writes 1 / 14 of the words. "interpolate" needs every symbol.
  const uint8_t layout = cfg.estimator.td_strategy == SRSGPU_CHEST_TD_AVERAGE ? SRSGPU_CE_COMPACT : SRSGPU_CE_PER_SYMBOL;

  // The estimator / demodulator / decoder configurations pusch_processor_impl derives from each PDU
  // (pusch_processor_impl.cpp:150-337), as srsgpu descriptors, and the batch layout.
  std::vector<pusch_chest_desc>       chests;
  std::vector<pusch_demod_desc>       demods;
  std::vector<srsgpu_pusch_tb_config> tbs;
  std::vector<srsgpu_harq_copy_job>   jobs;
  std::vector<srsgpu_ulsch_demux_config> demuxes;
  std::vector<uint8_t>                chest_key, demod_key, dec_key, demux_key;
  unsigned                            llr_total = 0, cb_total = 0, tb_total = 0, harq_total = 0;
  gpu::key_append(chest_key, grid_prb);
  gpu::key_append(demod_key, grid_prb);
  for (pusch_entry* ep : batch) {
    pusch_entry&                  e   = *ep;
    const pusch_processor::pdu_t& pdu = e.pdu;
    const crb_bitmap              rb_mask = pdu.freq_alloc.get_crb_mask(pdu.bwp_start_rb, pdu.bwp_size_rb);
    e.nof_rb                              = pdu.freq_alloc.get_nof_rb();

    unsigned  scrambling_id = 0, n_rs_id = 0, cdm_groups = 2;
    bool      n_scid = false, tp = false;
    dmrs_type dmrs   = dmrs_type::TYPE1;
    if (std::holds_alternative<pusch_processor::dmrs_configuration>(pdu.dmrs)) {
      const auto& d = std::get<pusch_processor::dmrs_configuration>(pdu.dmrs);
      scrambling_id = d.scrambling_id;
      n_scid        = d.n_scid;
      cdm_groups    = d.nof_cdm_groups_without_data;
      dmrs          = d.dmrs;
    } else {
      tp      = true;
      n_rs_id = std::get<pusch_processor::dmrs_transform_precoding_configuration>(pdu.dmrs).n_rs_id;
    }

    dmrs_pusch_estimator::configuration est;
    est.slot = pdu.slot;
    if (tp) {
      est.sequence_config = dmrs_pusch_estimator::low_papr_sequence_configuration{.n_rs_id = n_rs_id};
    } else {
      est.sequence_config = dmrs_pusch_estimator::pseudo_random_sequence_configuration{
          .type = dmrs, .nof_tx_layers = pdu.nof_tx_layers, .scrambling_id = scrambling_id, .n_scid = n_scid};
    }
    est.scaling      = convert_dB_to_amplitude(-get_sch_to_dmrs_ratio_dB(cdm_groups));
    est.c_prefix     = pdu.cp;
    est.symbols_mask = pdu.dmrs_symbol_mask;
    est.rb_mask      = rb_mask;
    est.first_symbol = pdu.start_symbol_index;
    est.nof_symbols  = pdu.nof_symbols;
    est.rx_ports.assign(pdu.rx_ports.begin(), pdu.rx_ports.end());
    chests.push_back(make_pusch_chest_desc(est, grid_prb, cfg.estimator, layout, WHO));
    chests.back().append_key(chest_key);

    pusch_demodulator::configuration dem;
    dem.rnti                        = pdu.rnti;
    dem.rb_mask                     = rb_mask;
    dem.modulation                  = pdu.mcs_descr.modulation;
    dem.start_symbol_index          = pdu.start_symbol_index;
    dem.nof_symbols                 = pdu.nof_symbols;
    dem.dmrs_symb_pos               = pdu.dmrs_symbol_mask;
    dem.dmrs_config_type            = dmrs;
    dem.nof_cdm_groups_without_data = cdm_groups;
    dem.n_id                        = pdu.n_id;
    dem.nof_tx_layers               = pdu.nof_tx_layers;
    dem.enable_transform_precoding  = tp;
    dem.rx_ports                    = pdu.rx_ports;
    demods.push_back(make_pusch_demod_desc(dem, grid_prb, cfg.demodulator, layout, WHO));
    pusch_demod_desc& dd = demods.back();
    dd.c.cfo_compensated = (layout == SRSGPU_CE_COMPACT && cfg.estimator.compensate_cfo) ? 1 : 0;
    dd.c.numerology      = static_cast<uint8_t>(pdu.slot.numerology());  // the symbol epochs of the rotation

    // Codeword LLRs: nof_rb REs per data symbol (minus the DM-RS REs) x layers x Qm.
    const unsigned dmrs_re = cdm_groups * (dmrs == dmrs_type::TYPE1 ? 6 : 4);
    unsigned       nre     = 0;
    for (unsigned l = pdu.start_symbol_index; l != pdu.start_symbol_index + pdu.nof_symbols; ++l) {
      nre += e.nof_rb * (pdu.dmrs_symbol_mask.test(l) ? NRE - dmrs_re : NRE);
    }
    e.nof_llrs      = nre * pdu.nof_tx_layers * dd.qm;
    e.llr_offset    = llr_total;
    dd.c.llr_offset = llr_total;
    llr_total += (e.nof_llrs + 63) / 64 * 64;
    dd.append_key(demod_key);

    // UCI on PUSCH (pusch_processor_impl.cpp:180-202, 244-262): the UL-SCH LLRs are the demultiplexer's SCH stream,
    // written after the codewords (the reference's own demultiplexer splits the UCI LLRs again during the replay).
    unsigned nof_sch_llrs = e.nof_llrs;
    e.sch_offset          = e.llr_offset;
    if (pdu.uci.nof_harq_ack != 0 || pdu.uci.nof_csi_part1 != 0) {
      bool overlap_dc = false;
      if (pdu.dc_position.has_value()) {
        overlap_dc = rb_mask.test(*pdu.dc_position / NRE);
      }
      ulsch_configuration uc;
      uc.tbs                         = units::bytes(e.data.size()).to_bits();
      uc.mcs_descr                   = pdu.mcs_descr;
      uc.nof_harq_ack_bits           = units::bits(pdu.uci.nof_harq_ack);
      uc.nof_csi_part1_bits          = units::bits(pdu.uci.nof_csi_part1);
      uc.nof_csi_part2_bits          = units::bits(0);
      uc.alpha_scaling               = pdu.uci.alpha_scaling;
      uc.beta_offset_harq_ack        = pdu.uci.beta_offset_harq_ack;
      uc.beta_offset_csi_part1       = pdu.uci.beta_offset_csi_part1;
      uc.beta_offset_csi_part2       = pdu.uci.beta_offset_csi_part2;
      uc.nof_rb                      = e.nof_rb;
      uc.start_symbol_index          = pdu.start_symbol_index;
      uc.nof_symbols                 = pdu.nof_symbols;
      uc.dmrs_type                   = dmrs == dmrs_type::TYPE1 ? dmrs_config_type::type1 : dmrs_config_type::type2;
      uc.dmrs_symbol_mask            = pdu.dmrs_symbol_mask;
      uc.nof_cdm_groups_without_data = cdm_groups;
      uc.nof_layers                  = pdu.nof_tx_layers;
      uc.contains_dc                 = overlap_dc;
      const ulsch_information info   = get_ulsch_information(uc);
      srsgpu_ulsch_demux_config d;
      std::memset(&d, 0, sizeof(d));
      d.modulation_order            = static_cast<uint8_t>(dd.qm);
      d.nof_layers                  = static_cast<uint8_t>(pdu.nof_tx_layers);
      d.nof_prb                     = static_cast<uint16_t>(e.nof_rb);
      d.start_symbol                = static_cast<uint8_t>(pdu.start_symbol_index);
      d.nof_symbols                 = static_cast<uint8_t>(pdu.nof_symbols);
      d.dmrs_symbol_mask            = symbol_mask_bits(pdu.dmrs_symbol_mask);
      d.dmrs_type                   = dmrs == dmrs_type::TYPE1 ? 1 : 2;
      d.nof_cdm_groups_without_data = static_cast<uint8_t>(cdm_groups);
      d.rnti                        = pdu.rnti;
      d.n_id                        = static_cast<uint16_t>(pdu.n_id);
      d.nof_harq_ack_rvd            = info.nof_harq_ack_rvd.value();
      d.nof_harq_ack_bits           = pdu.uci.nof_harq_ack;
      d.nof_enc_harq_ack_bits       = info.nof_harq_ack_bits.value();
      d.nof_csi_part1_bits          = pdu.uci.nof_csi_part1;
      d.nof_enc_csi_part1_bits      = info.nof_csi_part1_bits.value();
      d.llr_offset                  = e.llr_offset;
      demuxes.push_back(d);  // sch_offset set once the codeword region's size is known
      e.demux_index = static_cast<int>(demuxes.size()) - 1;
      nof_sch_llrs  = info.nof_ul_sch_bits.value();
    }
    e.nof_sch_llrs = nof_sch_llrs;

    // TB decoding (pusch_processor_impl.cpp:278-296).
    const units::bits tb_bits = units::bytes(e.data.size()).to_bits();
    const auto        bg      = pdu.codeword->ldpc_base_graph;
    e.nof_cbs                 = ldpc::compute_nof_codeblocks(tb_bits, bg);
    ldpc_lengths(tb_bits, bg, e.cb_N, e.cb_KZ);
    e.cb0       = cb_total;
    e.tb_offset = tb_total;
    e.harq0     = harq_total;
    e.new_data  = pdu.codeword->new_data;
    srsgpu_pusch_tb_config t;
    std::memset(&t, 0, sizeof(t));
    t.base_graph       = bg_number(bg);
    t.rv               = static_cast<uint8_t>(pdu.codeword->rv);
    t.modulation_order = static_cast<uint8_t>(dd.qm);
    t.nof_layers       = static_cast<uint8_t>(pdu.nof_tx_layers);
    t.new_data         = e.new_data ? 1 : 0;
    t.use_early_stop   = cfg.ldpc_early_stop ? 1 : 0;
    t.max_iterations   = static_cast<uint8_t>(cfg.nof_ldpc_iterations);
    t.scaling_factor   = 0.8F;  // ldpc_decoder::configuration::algorithm_details default (ldpc_decoder.h:50)
    t.tbs_bytes        = static_cast<uint32_t>(e.data.size());
    t.nof_ch_symbols   = nof_sch_llrs / dd.qm;
    t.Nref             = ldpc::compute_N_ref(pdu.tbs_lbrm, e.nof_cbs).value();
    t.llr_offset       = e.llr_offset;
    t.harq_offset      = e.harq0;
    t.cb_offset        = e.cb0;
    t.tb_offset        = e.tb_offset;
    tbs.push_back(t);
    gpu::key_append(dec_key, t);
    for (unsigned c = 0; c != e.nof_cbs; ++c) {
      const unsigned id = e.rm->get_absolute_codeblock_id(c);
      if (id >= arena->max_cb_ids) {
        throw std::out_of_range(std::string(WHO) + ": absolute codeblock id " + std::to_string(id) +
                                " beyond the HARQ arena");
      }
      jobs.push_back({id, e.harq0 + c * e.cb_N, e.cb_N, 0});
    }
    cb_total += e.nof_cbs;
    tb_total += (static_cast<unsigned>(e.data.size()) + 15) / 16 * 16;
    harq_total += e.nof_cbs * e.cb_N;
  }
  const unsigned n = batch.size();
  // UL-SCH streams of the UCI transmissions after the codewords in the same LLR buffer, then their HARQ-ACK and
  // CSI Part 1 streams (the plan writes every stream it routes; the replay decodes the UCI from the codeword LLRs).
  for (pusch_entry* ep : batch) {
    if (ep->demux_index >= 0) {
      srsgpu_ulsch_demux_config& d = demuxes[static_cast<size_t>(ep->demux_index)];
      d.sch_offset                 = llr_total;
      ep->sch_offset               = llr_total;
      llr_total += (ep->nof_sch_llrs + 63) / 64 * 64;
      d.harq_offset = llr_total;
      llr_total += (d.nof_enc_harq_ack_bits + 63) / 64 * 64;
      d.csi1_offset = llr_total;
      llr_total += (d.nof_enc_csi_part1_bits + 63) / 64 * 64;
      gpu::key_append(demux_key, d);
      gpu::key_append(dec_key, d.sch_offset);
      for (srsgpu_pusch_tb_config& t : tbs) {
        if (t.cb_offset == ep->cb0) {
          t.llr_offset = ep->sch_offset;
        }
      }
    }
  }

  // Plans (cached: a cell's grants repeat). Plan creation and buffer growth call synchronous HIP APIs, which fail
  // while any thread captures a stream: they and the slot graph's capture run under gpu::hip_setup_mutex (a cache hit
  // holds it for microseconds).
  const auto                   t_start = std::chrono::steady_clock::now();
  std::unique_lock<std::recursive_mutex> setup_lock(gpu::hip_setup_mutex());
  srsgpu_pusch_chest_plan* chest = chest_plans.get(chest_key, [&] {
    std::vector<srsgpu_pusch_chest_config> c;
    std::vector<srsgpu_alloc_ext>          x;
    for (const pusch_chest_desc& d : chests) {
      c.push_back(d.c);
      x.push_back(d.ext());
    }
    srsgpu_pusch_chest_plan* p = nullptr;
    srsgpu_check(srsgpu_pusch_chest_plan_create_ex(ctx, c.data(), x.data(), n, grid_prb, P, &p), WHO);
    return p;
  });
  srsgpu_pusch_demodulator_plan* demod = demod_plans.get(demod_key, [&] {
    std::vector<srsgpu_pusch_demod_config> c;
    std::vector<srsgpu_alloc_ext>          x;
    for (const pusch_demod_desc& d : demods) {
      c.push_back(d.c);
      x.push_back(d.ext());
    }
    srsgpu_pusch_demodulator_plan* p = nullptr;
    srsgpu_check(srsgpu_pusch_demodulator_plan_create_ex(ctx, c.data(), x.data(), n, grid_prb, P, &p), WHO);
    return p;
  });
  // A plan evicted above invalidates the graphs that run it and its cached sequences.
  const uint64_t generation = chest_plans.evictions() + demod_plans.evictions() + demux_plans.evictions() +
                              dec_plans.evictions();
  if (generation != plan_generation) {
    graphs.clear();  // a captured graph references the plans' device descriptors
    seq_cache.clear();
    plan_generation = generation;
  }

  // The replay hands the reference's codeword buffer each transmission's scrambling sequence: a property of the
  // demodulator plan (RNTI, n_ID, length), fetched once per plan instead of copied out every slot.
  const std::string                   seq_key(demod_key.begin(), demod_key.end());
  const std::vector<std::vector<uint32_t>>& seq_words = [&]() -> const std::vector<std::vector<uint32_t>>& {
    auto it = seq_cache.find(seq_key);
    if (it != seq_cache.end()) {
      return it->second;
    }
    std::vector<std::vector<uint32_t>> words(n);
    size_t                              most = 0;
    for (unsigned i = 0; i != n; ++i) {
      most = std::max<size_t>(most, (batch[i]->nof_llrs + 31) / 32);
    }
    uint32_t* d_seq = nullptr;
    hip_check(hipMalloc(reinterpret_cast<void**>(&d_seq), std::max<size_t>(most, 1) * sizeof(uint32_t)), WHO, "seq");
    for (unsigned i = 0; i != n; ++i) {
      words[i].resize((batch[i]->nof_llrs + 31) / 32);
      srsgpu_check(srsgpu_pusch_demodulator_plan_scrambling(demod, i, d_seq, stream.get()), WHO);
      hip_check(hipMemcpyAsync(words[i].data(), d_seq, words[i].size() * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               stream.get()),
                WHO, "seq download");
      hip_check(hipStreamSynchronize(stream.get()), WHO, "seq download");
    }
    (void)hipFree(d_seq);
    return seq_cache.emplace(seq_key, std::move(words)).first->second;
  }();
  srsgpu_ulsch_demux_plan* demux = nullptr;
  if (!demuxes.empty()) {
    demux = demux_plans.get(demux_key, [&] {
      srsgpu_ulsch_demux_plan* p = nullptr;
      srsgpu_check(srsgpu_ulsch_demux_plan_create(ctx, demuxes.data(), demuxes.size(), &p), WHO);
      return p;
    });
  }
  srsgpu_pusch_decoder_plan* dec = dec_plans.get(dec_key, [&] {
    srsgpu_pusch_decoder_plan* p = nullptr;
    srsgpu_check(srsgpu_pusch_decoder_plan_create(ctx, SRSGPU_LDPC_IMPL_SIMD, tbs.data(), n, &p), WHO);
    return p;
  });

  hipStream_t  s   = stream.get();
  const size_t row = static_cast<size_t>(nsc) * sizeof(uint32_t);

  // One pinned staging image per slot, inputs first: [grid | copy jobs | CB messages | CB CRC flags] are uploaded,
  // [CB CRC flags | iterations | TB CRC flags | nv | metrics | statistics | LLRs | scrambling words | TBs] downloaded
  // (the CRC flags are the HARQ context in and the result out). Two copies per slot instead of one per array.
  auto         align  = [](size_t x) { return (x + 63) / 64 * 64; };
  const size_t grid_o = 0;
  const size_t jobs_o = align(grid_o + static_cast<size_t>(P) * 14 * row);
  const size_t msgs_o = align(jobs_o + jobs.size() * sizeof(srsgpu_harq_copy_job));
  const size_t flag_o = align(msgs_o + static_cast<size_t>(cb_total) * SRSGPU_CB_MSG_STRIDE);
  const size_t iter_o = align(flag_o + cb_total);
  const size_t tbok_o = align(iter_o + static_cast<size_t>(cb_total) * sizeof(int32_t));
  const size_t nv_o   = align(tbok_o + n);
  const size_t m_o    = align(nv_o + 4 * n * sizeof(float));
  const size_t st_o   = align(m_o + 4 * n * SRSGPU_CHEST_METRICS * sizeof(float));
  const size_t llr_o  = align(st_o + n * SRSGPU_DEMOD_STATS * sizeof(float));
  const size_t tb_o  = align(llr_o + llr_total);
  const size_t end_o = tb_o + std::max<size_t>(tb_total, 16);
  io.reserve(end_o);
  reserve_device(d_ce, d_ce_cap, static_cast<size_t>(4) * P * 14 * row, "channel estimates");
  reserve_device(d_harq, d_harq_cap, std::max<size_t>(harq_total, 16), "HARQ batch buffer");
  setup_lock.unlock();
  const auto t_setup = std::chrono::steady_clock::now();

  // Host inputs: the rx grid (every symbol of ports 0..P-1, [port][symbol][subcarrier]), the HARQ arena copy jobs,
  // and the HARQ context from the rx buffers: CB CRC flags and the messages of CBs that already passed (a new
  // transmission's flags are reset by the plan, pusch_decoder_impl.cpp:133-136).
  for (unsigned p = 0; p != P; ++p) {
    for (unsigned l = 0; l != 14; ++l) {
      std::memcpy(io.host(grid_o + (p * 14 + l) * row), grid.get_view(p, l).data(), row);
    }
  }
  std::memcpy(io.host(jobs_o), jobs.data(), jobs.size() * sizeof(srsgpu_harq_copy_job));
  decoded_flags.assign(cb_total, 0);
  for (unsigned i = 0; i != n; ++i) {
    pusch_entry&     e    = *batch[i];
    span<const bool> crcs = e.rm->get_codeblocks_crc();
    for (unsigned c = 0; c != e.nof_cbs; ++c) {
      const bool ok                    = !e.new_data && crcs[c];
      *io.host<uint8_t>(flag_o + e.cb0 + c) = ok ? 1 : 0;
      decoded_flags[e.cb0 + c]         = ok ? 0 : 1;
      if (ok) {
        const bit_buffer bits = e.rm->get_codeblock_data_bits(c, e.cb_KZ);
        uint8_t*         dst  = io.host<uint8_t>(msgs_o + static_cast<size_t>(e.cb0 + c) * SRSGPU_CB_MSG_STRIDE);
        for (unsigned b = 0; b != (e.cb_KZ + 7) / 8; ++b) {
          dst[b] = bits.get_byte(b);
        }
      }
    }
  }

  const auto t_fill = std::chrono::steady_clock::now();
  setup_lock.lock();
  // The slot's device work as one captured graph per layout (cached like the plans it runs: a cell's grants repeat),
  // so a slot costs one graph launch instead of some thirty queue operations.
  std::vector<uint8_t> graph_key;
  for (const std::vector<uint8_t>* k : {&chest_key, &demod_key, &demux_key, &dec_key}) {
    gpu::key_append(graph_key, k->size());
    graph_key.insert(graph_key.end(), k->begin(), k->end());
  }
  for (const void* ptr : {static_cast<const void*>(io.host()), static_cast<const void*>(io.dev()),
                          static_cast<const void*>(d_ce), static_cast<const void*>(d_harq)}) {
    gpu::key_append(graph_key, ptr);
  }
  gpu::key_append(graph_key, P);
  gpu::key_append(graph_key, end_o);
  for (unsigned i = 0; i != n; ++i) {
    const pusch_processor::pdu_t& pdu = batch[i]->pdu;
    gpu::key_append(graph_key, pdu.dc_position.has_value() ? static_cast<int>(*pdu.dc_position) : -1);
  }
  hipGraphExec_t exec = graphs.get(graph_key, [&] { return capture_graph(s, WHO, [&] {
    io.upload(0, iter_o, s);
    srsgpu_check(srsgpu_pusch_chest_plan_execute(chest, io.dev<uint32_t>(grid_o), d_ce, io.dev<float>(nv_o),
                                                 io.dev<float>(m_o), s),
                 WHO);
    // pusch_processor_impl.cpp:222-240: the DC subcarrier's estimate is zeroed for CP-OFDM transmissions over it.
    for (unsigned i = 0; i != n; ++i) {
      const pusch_processor::pdu_t& pdu = batch[i]->pdu;
      if (pdu.dc_position.has_value() && std::holds_alternative<pusch_processor::dmrs_configuration>(pdu.dmrs) &&
          *pdu.dc_position < nsc) {
        for (unsigned ly = 0; ly != pdu.nof_tx_layers; ++ly) {
          for (unsigned p = 0; p != pdu.rx_ports.size(); ++p) {
            uint8_t* base = reinterpret_cast<uint8_t*>(d_ce) +
                            ((static_cast<size_t>(ly) * P + p) * 14 + pdu.start_symbol_index) * row +
                            static_cast<size_t>(*pdu.dc_position) * sizeof(uint32_t);
            // Compact layout: the one row every symbol reads.
            const unsigned rows = layout == SRSGPU_CE_COMPACT ? 1u : pdu.nof_symbols;
            hip_check(hipMemset2DAsync(base, row, 0, sizeof(uint32_t), rows, s), WHO, "DC");
          }
        }
      }
    }
    srsgpu_check(srsgpu_pusch_demodulator_plan_execute_ex(demod, io.dev<uint32_t>(grid_o), d_ce, io.dev<float>(nv_o),
                                                          io.dev<int8_t>(llr_o), io.dev<float>(st_o), s),
                 WHO);
    if (demux != nullptr) {
      // Only the UL-SCH stream is used on the device: the UCI streams are split again by the reference's own
      // demultiplexer during the replay, from the codeword LLRs.
      int8_t* llr_base = io.dev<int8_t>(llr_o);
      srsgpu_check(srsgpu_ulsch_demux_plan_execute(demux, llr_base, llr_base, llr_base, llr_base, llr_base, s), WHO);
    }
    srsgpu_check(srsgpu_harq_copy(ctx, SRSGPU_HARQ_TO_BATCH, arena->d_soft, HARQ_SLOT_BYTES, d_harq,
                                  io.dev<srsgpu_harq_copy_job>(jobs_o), jobs.size(), s),
                 WHO);
    srsgpu_check(srsgpu_pusch_decoder_plan_execute(dec, io.dev<int8_t>(llr_o), d_harq, io.dev<uint8_t>(flag_o),
                                                   io.dev<uint8_t>(msgs_o), io.dev<int32_t>(iter_o),
                                                   io.dev<uint8_t>(tb_o), io.dev<uint8_t>(tbok_o), s),
                 WHO);
    srsgpu_check(srsgpu_harq_copy(ctx, SRSGPU_HARQ_TO_ARENA, arena->d_soft, HARQ_SLOT_BYTES, d_harq,
                                  io.dev<srsgpu_harq_copy_job>(jobs_o), jobs.size(), s),
                 WHO);
    io.download(flag_o, end_o - flag_o, s);
  }); });
  setup_lock.unlock();
  const auto t_graph = std::chrono::steady_clock::now();
  hip_check(hipGraphLaunch(exec, s), WHO, "graph launch");
  hip_check(hipStreamSynchronize(s), WHO, "synchronise");
  const auto t_gpu = std::chrono::steady_clock::now();

  // Messages of the passed CBs of failed TBs are kept in the rx buffer for the retransmission.
  bool need_msgs = false;
  for (unsigned i = 0; i != n && !need_msgs; ++i) {
    const pusch_entry& e = *batch[i];
    if (*io.host<uint8_t>(tbok_o + i) == 0) {
      for (unsigned c = 0; c != e.nof_cbs; ++c) {
        need_msgs = need_msgs || *io.host<uint8_t>(flag_o + e.cb0 + c) != 0;
      }
    }
  }
  if (need_msgs) {
    io.download(msgs_o, static_cast<size_t>(cb_total) * SRSGPU_CB_MSG_STRIDE, s);
    hip_check(hipStreamSynchronize(s), WHO, "synchronise");
  }

  // Result assembly and notification by the reference's own processor, PDU by PDU.
  replay_processor& r = replay_for_this_thread();
  for (unsigned i = 0; i != n; ++i) {
    pusch_entry& e      = *batch[i];
    r.est->nv           = io.host<float>(nv_o + 4 * i * sizeof(float));
    r.est->m            = io.host<float>(m_o + 4 * i * SRSGPU_CHEST_METRICS * sizeof(float));
    r.demod->llrs       = io.host<int8_t>(llr_o + e.llr_offset);
    r.demod->seq        = seq_words[i].data();
    r.demod->stats      = io.host<float>(st_o + i * SRSGPU_DEMOD_STATS * sizeof(float));
    r.demod->nof_llrs   = e.nof_llrs;
    r.demod->nof_rb     = e.nof_rb;
    r.dec->cb_flags     = io.host<uint8_t>(flag_o + e.cb0);
    r.dec->cb_iters     = io.host<int32_t>(iter_o + e.cb0 * sizeof(int32_t));
    r.dec->tb           = io.host<uint8_t>(tb_o + e.tb_offset);
    r.dec->cb_msgs      = io.host<uint8_t>(msgs_o + static_cast<size_t>(e.cb0) * SRSGPU_CB_MSG_STRIDE);
    r.dec->decoded      = decoded_flags.data() + e.cb0;
    r.dec->tb_ok        = *io.host<uint8_t>(tbok_o + i) != 0;
    r.dec->cb_KZ        = e.cb_KZ;
    r.dec->max_iter     = cfg.nof_ldpc_iterations;
    r.proc->process(e.data, std::move(e.rm), *e.notifier, *e.grid, e.pdu);
  }
  if (timing) {
    const auto t_end = std::chrono::steady_clock::now();
    auto       us    = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    phase_us[0] += us(t_start, t_setup);
    phase_us[1] += us(t_setup, t_fill);
    phase_us[2] += us(t_fill, t_graph);
    phase_us[3] += us(t_graph, t_gpu);
    phase_us[4] += us(t_gpu, t_end);
    ++timed_slots;
  }
}

std::shared_ptr<pusch_slot_batch> create_pusch_slot_batch(const pusch_batch_configuration&           config,
                                                          std::shared_ptr<pusch_harq_arena>          arena,
                                                          std::shared_ptr<ulsch_demultiplex_factory> demux,
                                                          std::shared_ptr<uci_decoder_factory>       uci,
                                                          std::unique_ptr<pusch_processor>           fallback)
{
  return std::make_shared<pusch_slot_batch>(config, std::move(arena), std::move(demux), std::move(uci),
                                            std::move(fallback));
}

namespace {

class pusch_processor_batch_gpu : public pusch_processor
{
public:
  explicit pusch_processor_batch_gpu(std::shared_ptr<pusch_slot_batch> batch_) : batch(std::move(batch_)) {}

  void process(span<uint8_t>                    data,
               unique_rx_buffer                 rm_buffer,
               pusch_processor_result_notifier& notifier,
               const resource_grid_reader&      grid,
               const pdu_t&                     pdu) override
  {
    pusch_entry e;
    e.pdu      = pdu;
    e.data     = data;
    e.rm       = std::move(rm_buffer);
    e.notifier = &notifier;
    e.grid     = &grid;
    batch->add(std::move(e));
  }

private:
  std::shared_ptr<pusch_slot_batch> batch;
};

class inline_executor : public task_executor
{
public:
  bool execute(unique_task task) override
  {
    task();
    return true;
  }
  bool defer(unique_task task) override
  {
    task();
    return true;
  }
};

/// The reference's uplink processor with the batch run after each handle_rx_symbol.
class uplink_processor_batch_gpu : public uplink_processor
{
  /// The slot processor handed out for one slot (a ring indexed by slot, like the reference's request pools).
  class slot_processor : public uplink_slot_processor
  {
  public:
    uplink_processor_batch_gpu* owner = nullptr;
    slot_point                  slot;

    void handle_rx_symbol(unsigned end_symbol_index) override
    {
      owner->inner->get_slot_processor(slot).handle_rx_symbol(end_symbol_index);
      owner->flush();
    }
    void process_prach(const prach_buffer& buffer, const prach_buffer_context& context) override
    {
      owner->inner->get_slot_processor(slot).process_prach(buffer, context);
    }
    void discard_slot() override
    {
      owner->inner->get_slot_processor(slot).discard_slot();
      owner->flush();
    }
  };

public:
  uplink_processor_batch_gpu(std::unique_ptr<uplink_processor> inner_,
                             std::shared_ptr<pusch_slot_batch> batch_,
                             task_executor&                    executor_) :
    inner(std::move(inner_)), batch(std::move(batch_)), executor(executor_)
  {
    for (slot_processor& s : slots) {
      s.owner = this;
    }
  }

  unique_uplink_pdu_slot_repository get_pdu_slot_repository(slot_point slot) override
  {
    return inner->get_pdu_slot_repository(slot);
  }

  uplink_slot_processor& get_slot_processor(slot_point slot) override
  {
    slot_processor& s = slots[slot.system_slot() % slots.size()];
    s.slot            = slot;
    return s;
  }

  void stop() override { inner->stop(); }

private:
  /// Hands the PDUs registered by the last reference call to the PUSCH executor as one job.
  void flush()
  {
    auto entries = std::make_shared<std::vector<pusch_entry>>(batch->take());
    if (entries->empty()) {
      return;
    }
    std::shared_ptr<pusch_slot_batch> b   = batch;
    auto                              job = [b, entries]() {
      // A GPU or configuration error leaves the slot's PUSCH results undeliverable: fatal, with its reason, as the
      // reference's own processors treat failures they cannot notify (error_handling.h report_fatal_error).
      try {
        b->run(*entries);
      } catch (const std::exception& e) {
        report_fatal_error("pusch_slot_batch: {}", e.what());
      }
    };
    if (!executor.execute(job)) {
      job();  // the executor refused the job: run it here rather than lose the PDUs' notifications
    }
  }

  std::unique_ptr<uplink_processor>  inner;
  std::shared_ptr<pusch_slot_batch>  batch;
  task_executor&                     executor;
  std::array<slot_processor, 16>     slots;
};

} // namespace

std::unique_ptr<pusch_processor> create_pusch_processor_batch_gpu(std::shared_ptr<pusch_slot_batch> batch)
{
  return std::make_unique<pusch_processor_batch_gpu>(std::move(batch));
}

task_executor& pusch_inline_executor()
{
  static inline_executor exec;
  return exec;
}

std::unique_ptr<uplink_processor> create_uplink_processor_batch_gpu(std::unique_ptr<uplink_processor>  inner,
                                                                    std::shared_ptr<pusch_slot_batch> batch,
                                                                    task_executor&                    executor)
{
  return std::make_unique<uplink_processor_batch_gpu>(std::move(inner), std::move(batch), executor);
}

// ---------------------------------------------------------------------------------------------------------------------
// PDSCH slot batch
// ---------------------------------------------------------------------------------------------------------------------

namespace {

/// One recorded PDSCH transmission.
struct pdsch_entry {
  resource_grid_writer*          grid     = nullptr;
  pdsch_processor_notifier*      notifier = nullptr;
  srsgpu_pdsch_tb_config         tb;
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

} // namespace

class pdsch_slot_batch
{
  static constexpr const char* WHO = "pdsch_slot_batch";

public:
  pdsch_slot_batch(int device, std::unique_ptr<ptrs_pdsch_generator> ptrs_, std::unique_ptr<pdsch_processor> fallback_) :
    owner(shared_context(device)),
    ctx(owner.get()),
    ptrs(std::move(ptrs_)),
    fallback(std::move(fallback_)),
    stream(ctx, WHO),
    enc_plans(srsgpu_pdsch_encoder_plan_destroy, 16),
    mod_plans(srsgpu_pdsch_modulator_plan_destroy, 16),
    dmrs_plans(srsgpu_pdsch_dmrs_plan_destroy, SLOT_PLANS),
    graphs(destroy_graph_exec, SLOT_PLANS),
    tb_buf(WHO),
    grid_buf(WHO)
  {
    if (!ptrs || !fallback) {
      throw std::invalid_argument(std::string(WHO) + ": invalid dependencies");
    }
  }

  ~pdsch_slot_batch()
  {
    (void)hipStreamSynchronize(stream.get());
    (void)hipFree(d_cw);
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
    e.tb.tb_offset = static_cast<uint32_t>(tb_bytes.size());
    tb_bytes.insert(tb_bytes.end(), tb.begin(), tb.end());
    tb_bytes.resize((tb_bytes.size() + 15) / 16 * 16, 0);
    e.tb.cw_offset = cw_total;
    cw_total += (nre * nof_layers * qm + 31) / 32 * 4;

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

  /// Encodes, modulates and maps every recorded PDSCH as one launch sequence, stores the REs into the slot's grid and
  /// reports each PDSCH finished (after which the reference's downlink processor sends the grid).
  void flush()
  {
    std::vector<pdsch_entry> es;
    std::vector<uint8_t>     tbs;
    unsigned                 cw_bytes = 0;
    {
      std::lock_guard<std::mutex> lock(mtx);
      es       = std::exchange(entries, {});
      tbs      = std::exchange(tb_bytes, {});
      cw_bytes = std::exchange(cw_total, 0u);
    }
    if (es.empty()) {
      return;
    }
    std::lock_guard<std::mutex> lock(run_mtx);
    device_scope                dev(ctx, WHO);
    resource_grid_writer&       grid     = *es.front().grid;
    const unsigned              nsc      = grid.get_nof_subc();
    const unsigned              grid_prb = nsc / NRE;
    const unsigned              P        = grid.get_nof_ports();
    const unsigned              n        = es.size();

    std::vector<srsgpu_pdsch_tb_config> tcs;
    std::vector<pdsch_mod_desc>         mods;
    std::vector<pdsch_dmrs_desc>        dmrss;
    std::vector<uint8_t>                enc_key, mod_key, dmrs_key;
    gpu::key_append(mod_key, grid_prb);
    gpu::key_append(dmrs_key, grid_prb);
    for (const pdsch_entry& e : es) {
      if (e.grid != &grid) {
        throw std::logic_error(std::string(WHO) + ": PDSCH of one batch in different resource grids");
      }
      tcs.push_back(e.tb);
      gpu::key_append(enc_key, e.tb);
      const unsigned nof_bits = e.tb.nof_ch_symbols * e.tb.modulation_order;
      mods.push_back(make_pdsch_mod_desc(e.mod, nof_bits, grid_prb, P, WHO));
      mods.back().c.cw_offset = e.tb.cw_offset;
      mods.back().append_key(mod_key);
      dmrss.push_back(make_pdsch_dmrs_desc(e.dmrs, grid_prb, P, WHO));
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

    hipStream_t  s   = stream.get();
    const size_t row = static_cast<size_t>(nsc) * sizeof(uint32_t);
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
      grid_buf.reserve(P * 14 * row);
    }
    std::memcpy(tb_buf.host(), tbs.data(), tbs.size());

    // The slot's device work as one captured graph per layout (cached like the plans it runs), so a slot costs one
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
      hip_check(hipMemsetAsync(grid_buf.dev(), 0xff, P * 14 * row, s), WHO, "scratch");
      srsgpu_check(srsgpu_pdsch_encoder_plan_execute(enc, tb_buf.dev<uint8_t>(), d_cw, s), WHO);
      srsgpu_check(srsgpu_pdsch_dmrs_plan_execute(dmrs, grid_buf.dev<uint32_t>(), s), WHO);
      srsgpu_check(srsgpu_pdsch_modulator_plan_execute(mod, d_cw, grid_buf.dev<uint32_t>(), s), WHO);
      grid_buf.download(0, P * 14 * row, s);
    }); });
    setup_lock.unlock();
    hip_check(hipGraphLaunch(exec, s), WHO, "graph launch");
    hip_check(hipStreamSynchronize(s), WHO, "synchronise");
    store_written_res(grid, grid_buf.host<uint32_t>(), P, nsc, 0, 14);
    for (pdsch_entry& e : es) {
      e.notifier->on_finish_processing();
    }
  }

private:
  std::shared_ptr<srsgpu_context>       owner;
  srsgpu_context*                       ctx;
  std::unique_ptr<ptrs_pdsch_generator> ptrs;
  std::unique_ptr<pdsch_processor>      fallback;
  owned_stream                          stream;
  plan_cache<srsgpu_pdsch_encoder_plan>   enc_plans;
  plan_cache<srsgpu_pdsch_modulator_plan> mod_plans;
  plan_cache<srsgpu_pdsch_dmrs_plan>      dmrs_plans;
  plan_cache<std::remove_pointer_t<hipGraphExec_t>> graphs;
  uint64_t                              plan_generation = 0;
  staged_buffer                         tb_buf;
  staged_buffer                         grid_buf;
  uint8_t*                              d_cw     = nullptr;
  size_t                                d_cw_cap = 0;
  std::mutex                            mtx;
  std::vector<pdsch_entry>              entries;
  std::vector<uint8_t>                  tb_bytes;
  unsigned                              cw_total = 0;
  std::mutex                            run_mtx;
};

std::shared_ptr<pdsch_slot_batch> create_pdsch_slot_batch(int                                   device,
                                                          std::unique_ptr<ptrs_pdsch_generator> ptrs,
                                                          std::unique_ptr<pdsch_processor>      fallback)
{
  return std::make_shared<pdsch_slot_batch>(device, std::move(ptrs), std::move(fallback));
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
