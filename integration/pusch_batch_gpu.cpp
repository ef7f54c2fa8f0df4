// Slot-batched PUSCH processing behind the reference's uplink processor (see upper_phy_gpu.h for the interface).
//
// Structure (one per GPU, shared by every sector on it):
//
//   PUSCH executor threads (one per cell)            pusch_gpu_service
//   ------------------------------------------      -------------------------------------------------------------------
//   uplink_processor_impl::handle_rx_symbol          dispatcher thread: gathers the submitted slots of one slot number
//     -> pusch_slot_batch::run(PDUs)                   (up to max_slots_per_launch, waiting up to gather_window_us for
//        copy the rx grid into pinned memory,          expected_slots_per_launch of them), builds the launch's plans
//        upload it to the batch's HBM grid slot        (cached by layout), orders its stream after the grids' uploads
//        (own stream), submit the slot                 and replays one captured graph: estimator, DC zeroing,
//                                                      demodulator, UL-SCH demultiplexer, HARQ arena gathers, decoder,
//                                                      TB assembly, arena scatters, one download of the results
//                                                    completion thread: waits for each launch in order and replays
//                                                      every PDU through the reference's pusch_processor_impl over
//                                                      replay stages (metrics, statistics, UCI streams, decoded TBs),
//                                                      which notifies the reference's uplink processor
//
// Nothing codeword-sized crosses PCIe: the LLRs stay in HBM; only the HARQ-ACK / CSI Part 1 streams of PDUs with UCI
// come back, fed to the reference's UCI decoders symbol by symbol (srsgpu_ulsch_demux_plan_symbol_llrs) so that UCI is
// decoded and notified when the reference's demultiplexer would do it.
#include "upper_phy_gpu.h"
#include "batch_graph.h"
#include "chain_convert.h"
#include "gpu_staging.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_processor_impl.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_notifier.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_result.h"
#include "srsran/phy/upper/channel_processors/pusch/ulsch_demultiplex.h"
#include "srsran/phy/upper/rx_buffer.h"
#include "srsran/phy/upper/unique_rx_buffer.h"
#include "srsran/phy/upper/uplink_slot_processor.h"
#include "srsran/ran/pusch/ulsch_info.h"
#include "srsran/ran/sch/sch_dmrs_power.h"
#include "srsran/support/error_handling.h"

#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <thread>

#include <rccl/rccl.h>

namespace srsran {
namespace gpu {

namespace {

constexpr unsigned HARQ_SLOT_BYTES = 66 * 384;  ///< N of BG1 at Z = 384: one arena slot per codeblock.

using clock_type = std::chrono::steady_clock;

double us_between(clock_type::time_point a, clock_type::time_point b)
{
  return std::chrono::duration<double, std::micro>(b - a).count();
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
    device_scope                          dev(ctx.get(), "pusch_harq_arena");
    std::lock_guard<std::recursive_mutex> lock(hip_setup_mutex());
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
// Replay stages: the reference's pusch_processor_impl runs per PDU on the launch's results.
// ---------------------------------------------------------------------------------------------------------------------

namespace {

/// Process-wide grid transfer counts of the multi-device UL batches (get_pusch_multi_transfer_counters).
struct {
  std::atomic<uint64_t> host_uploads{0}, shard_copies{0}, shard_bytes{0};
  std::atomic<uint64_t> twin_grids{0};  ///< single-device slots whose grid the lower PHY had written into HBM
} multi_transfers;

/// One registered PUSCH transmission and where its results are in its launch.
struct pusch_entry {
  pusch_processor::pdu_t           pdu;
  span<uint8_t>                    data;
  unique_rx_buffer                 rm;
  pusch_processor_result_notifier* notifier = nullptr;
  const resource_grid_reader*      grid     = nullptr;
  // Layout within the launch.
  unsigned tx         = 0;  ///< Transmission index in the launch's plans.
  unsigned nof_rb     = 0;
  unsigned nof_cbs    = 0;
  unsigned cb0        = 0;  ///< First codeblock of the TB in the launch.
  unsigned llr_offset = 0;
  unsigned nof_llrs   = 0;
  unsigned tb_offset  = 0;
  unsigned harq0      = 0;  ///< First byte of the TB's HARQ soft bits in the launch's HARQ buffer.
  unsigned cb_N       = 0;
  unsigned cb_KZ      = 0;
  bool     new_data   = true;
  int      demux_index  = -1;  ///< UCI on PUSCH: the transmission's entry in the demultiplexer plan.
  unsigned sch_offset   = 0;   ///< First UL-SCH LLR the decoder reads.
  unsigned nof_sch_llrs = 0;
  unsigned harq_ack_offset = 0;  ///< HARQ-ACK / CSI Part 1 streams in the launch's downloaded UCI region.
  unsigned csi1_offset     = 0;
  std::array<uint32_t, 14> harq_ack_counts{};  ///< UCI LLRs per OFDM symbol.
  std::array<uint32_t, 14> csi1_counts{};
  int      tb_index     = -1;  ///< The TB's index in the launch's decoder plan (-1: decoded in the CSI Part 2 phase).
  // CSI Part 2 (pusch_processor_impl.cpp:55-101): the UL-SCH bit count depends on CSI Part 1, decoded on the host
  // during the replay, so the UL-SCH is demultiplexed and decoded by a second, per-PDU launch from there
  // (pusch_launcher::decode_deferred) with what the first launch left in HBM (the codeword LLRs).
  bool                               csi2 = false;
  ulsch_configuration                ulsch_cfg;   ///< UL-SCH information input (CSI Part 2 bits 0)
  srsgpu_ulsch_demux_config          demux_cfg{}; ///< the first launch's demultiplexing (job-relative offsets)
  srsgpu_pusch_tb_config             tb_cfg{};    ///< the TB's decoding, CB / TB / LLR / HARQ offsets 0
  std::vector<srsgpu_harq_copy_job>  copies;      ///< HARQ arena copies (batch offsets from 0)
  std::vector<uint8_t>               flags;       ///< HARQ context: CB CRC flags
  std::vector<std::vector<uint8_t>>  msgs;        ///< messages of the CBs that passed before (empty otherwise)
};

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

/// The demultiplexer stage of the replay. The GPU demultiplexed the codeword already: the UL-SCH stream went to the
/// GPU decoder, the HARQ-ACK / CSI Part 1 streams came back. The replay demodulator calls on_symbol(l) for every OFDM
/// symbol with data after its provisional statistics, and this feeds the UCI decoder buffers the LLRs the reference's
/// demultiplexer hands them while it demultiplexes symbol l, ending each field in the symbol that completes it
/// (ulsch_demultiplex_impl.cpp:474-576), so UCI is decoded and notified at the reference's point of the codeword.
class replay_demux : public ulsch_demultiplex, private pusch_codeword_buffer
{
public:
  const int8_t*   harq_ack_llrs   = nullptr;
  const int8_t*   csi1_llrs       = nullptr;
  const uint32_t* harq_ack_counts = nullptr;
  const uint32_t* csi1_counts     = nullptr;
  /// CSI Part 2 PDUs: the second launch, given the CSI Part 2 size (0 bits: none) and the symbol it starts at; it
  /// returns the CSI Part 2 stream and its per-symbol counts and settles the replay decoder's results.
  std::function<void(unsigned bits, unsigned enc_bits, unsigned first_symbol, const int8_t*& llrs,
                     const uint32_t*& counts)>
      second_phase;

  void set_csi_part2(pusch_decoder_buffer& buffer, unsigned bits, unsigned enc_bits) override
  {
    // Called by the reference's CSI Part 1 feedback while the symbol completing CSI Part 1 is demultiplexed
    // (pusch_processor_impl.cpp:72-100): CSI Part 2 occupies REs of that symbol and the later ones.
    if (!second_phase) {
      throw std::logic_error("pusch_slot_batch: CSI Part 2 without a second phase");
    }
    second_phase(bits, enc_bits, current_symbol, csi2_llrs, csi2_counts);
    second_done = true;
    csi_part2   = &buffer;
    csi2_pos    = 0;
    csi2_total  = enc_bits;
  }

  pusch_codeword_buffer& demultiplex(pusch_decoder_buffer& sch_data_,
                                     pusch_decoder_buffer& harq_ack_,
                                     pusch_decoder_buffer& csi_part1_,
                                     const configuration&  config) override
  {
    sch_data  = &sch_data_;
    harq_ack  = config.nof_harq_ack_bits != 0 ? &harq_ack_ : nullptr;
    csi_part1 = config.nof_csi_part1_bits != 0 ? &csi_part1_ : nullptr;
    csi_part2 = nullptr;
    harq_pos = csi1_pos = csi2_pos = 0;
    harq_total                     = config.nof_enc_harq_ack_bits;
    csi1_total                     = config.nof_enc_csi_part1_bits;
    second_done                    = false;
    return *this;
  }

  /// The symbol's UCI in the reference's order (ulsch_demultiplex_impl.cpp:474-576): HARQ-ACK, CSI Part 1 (whose end
  /// may configure CSI Part 2 for this very symbol), CSI Part 2.
  void on_symbol(unsigned l)
  {
    current_symbol = l;
    feed(harq_ack, harq_ack_llrs, harq_ack_counts, harq_pos, harq_total, l);
    feed(csi_part1, csi1_llrs, csi1_counts, csi1_pos, csi1_total, l);
    feed(csi_part2, csi2_llrs, csi2_counts, csi2_pos, csi2_total, l);
  }

private:
  static void feed(pusch_decoder_buffer*& field,
                   const int8_t*          llrs,
                   const uint32_t*        counts,
                   unsigned&              pos,
                   unsigned               total,
                   unsigned               l)
  {
    if (field == nullptr || counts == nullptr || counts[l] == 0) {
      return;
    }
    field->on_new_softbits(
        span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llrs + pos), counts[l]));
    pos += counts[l];
    if (pos == total) {
      field->on_end_softbits();
      field = nullptr;
    }
  }

  span<log_likelihood_ratio> get_next_block_view(unsigned /*block_size*/) override
  {
    throw std::logic_error("pusch_slot_batch: replay demultiplexer fed LLRs");
  }
  void on_new_block(span<const log_likelihood_ratio> /*data*/, const bit_buffer& /*seq*/) override
  {
    throw std::logic_error("pusch_slot_batch: replay demultiplexer fed LLRs");
  }
  void on_end_codeword() override
  {
    // ulsch_demultiplex_impl::on_end_codeword (:321): every UCI field has ended by now.
    if (harq_ack != nullptr || csi_part1 != nullptr || csi_part2 != nullptr) {
      throw std::logic_error("pusch_slot_batch: UCI field not complete at the end of the codeword");
    }
    // A CSI Part 2 PDU whose CSI Part 1 did not configure CSI Part 2 (invalid, or zero CSI Part 2 bits): the UL-SCH
    // takes the REs CSI Part 2 would have had (the UL-SCH information without CSI Part 2, pusch_processor_impl.cpp:180).
    if (second_phase && !second_done) {
      const int8_t*   llrs   = nullptr;
      const uint32_t* counts = nullptr;
      second_phase(0, 0, 0, llrs, counts);
    }
    sch_data->on_end_softbits();
    sch_data = nullptr;
  }

  pusch_decoder_buffer* sch_data  = nullptr;
  pusch_decoder_buffer* harq_ack  = nullptr;
  pusch_decoder_buffer* csi_part1 = nullptr;
  pusch_decoder_buffer* csi_part2 = nullptr;
  const int8_t*         csi2_llrs   = nullptr;
  const uint32_t*       csi2_counts = nullptr;
  unsigned              harq_pos = 0, csi1_pos = 0, csi2_pos = 0, harq_total = 0, csi1_total = 0, csi2_total = 0;
  unsigned              current_symbol = 0;
  bool                  second_done    = false;
};

/// The demodulator stage of the replay: the demodulator's notifications in pusch_demodulator_impl's order
/// (pusch_demodulator_impl.cpp:272-443) - per OFDM symbol with data its provisional statistics, during which the
/// reference's demultiplexer processes the symbol (replay_demux::on_symbol), then the end statistics and the end of the
/// codeword. No LLR is touched: the GPU decoded the UL-SCH already (replay_decoder).
class replay_demodulator : public pusch_demodulator
{
public:
  pusch_demodulator_options opts;
  replay_demux*             demux  = nullptr;
  const float*              stats  = nullptr;
  unsigned                  nof_rb = 0;

  void demodulate(pusch_codeword_buffer&      codeword_buffer,
                  pusch_demodulator_notifier& notifier,
                  const resource_grid_reader& /*grid*/,
                  const channel_estimate& /*estimates*/,
                  const configuration& config) override
  {
    const unsigned dmrs_re_per_prb =
        config.nof_cdm_groups_without_data * (config.dmrs_config_type == dmrs_type::TYPE1 ? 6 : 4);
    for (unsigned l = config.start_symbol_index; l != config.start_symbol_index + config.nof_symbols; ++l) {
      const unsigned nof_re_symbol = nof_rb * (config.dmrs_symb_pos.test(l) ? NRE - dmrs_re_per_prb : NRE);
      if (nof_re_symbol == 0) {
        continue;
      }
      notifier.on_provisional_stats(l, demod_stats_of(stats + 2 * l, opts));
      demux->on_symbol(l);
    }
    notifier.on_end_stats(demod_stats_of(stats + 2 * 14, opts));
    codeword_buffer.on_end_codeword();
  }
};

/// The decoder stage of the replay: the TB was decoded on the GPU; on_end_softbits() settles the rx buffer like
/// pusch_decoder_impl::join_and_notify (pusch_decoder_impl.cpp:386-440) and notifies the result.
class replay_decoder : public pusch_decoder, private pusch_decoder_buffer
{
public:
  const uint8_t* cb_flags = nullptr;  ///< CB CRC flags after the decode (launch-wide array, first of the TB).
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
  span<log_likelihood_ratio> get_next_block_view(unsigned /*block_size*/) override
  {
    throw std::logic_error("pusch_slot_batch: replay decoder fed LLRs");
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

  span<uint8_t>           transport_block;
  unique_rx_buffer        rm;
  pusch_decoder_notifier* notifier = nullptr;
  std::vector<unsigned>   cb_stats;
};

/// A reference pusch_processor_impl over the replay stages (one per thread that replays: the processor's dependency
/// pool binds its instances to threads, concurrent_thread_local_object_pool.h:67-96).
struct replay_processor {
  replay_estimator*                est   = nullptr;
  replay_demodulator*              demod = nullptr;
  replay_demux*                    demux = nullptr;
  replay_decoder*                  dec   = nullptr;
  std::unique_ptr<pusch_processor> proc;
};

} // namespace

// ---------------------------------------------------------------------------------------------------------------------
// Jobs and the GPU service
// ---------------------------------------------------------------------------------------------------------------------

namespace {

/// The descriptors of one job, built by the thread that submits it (pusch_slot_batch::build_layout), with offsets
/// relative to the job: a launch concatenates its jobs' layouts, and a recurring sequence of job keys finds its plans
/// and graph cached (pusch_gpu_service::launch).
struct job_layout {
  std::vector<pusch_chest_desc>          chests;
  std::vector<pusch_demod_desc>          demods;
  std::vector<srsgpu_pusch_tb_config>    tbs;
  std::vector<srsgpu_ulsch_demux_config> demuxes;
  std::vector<srsgpu_harq_copy_job>      copies;  ///< HARQ arena copies; batch offsets relative to the job's HARQ region
  std::vector<uint8_t>                   flags;   ///< HARQ context: CB CRC flags (1: passed in an earlier transmission)
  std::vector<std::pair<unsigned, std::vector<uint8_t>>> msgs;  ///< (job CB, message bytes) of those CBs
  std::vector<std::pair<size_t, unsigned>> dc_zero_local;  ///< DC zeroings: estimate byte offset (the job's grid slot
                                                           ///< included), rows (pusch_processor_impl.cpp:222-240)
  std::vector<uint8_t>                   key;
  uint8_t  layout    = SRSGPU_CE_COMPACT;
  unsigned n         = 0;
  unsigned llr_total = 0, cb_total = 0, tb_total = 0, harq_total = 0, uci_total = 0;
};

/// One slot of one batch (uplink processor): its batchable PDUs, its grid (already uploading to its HBM grid slot),
/// its layout and its completion.
struct pusch_job {
  pusch_slot_batch*        batch = nullptr;
  unsigned                 batch_id  = 0;
  std::vector<pusch_entry> entries;
  job_layout               lay;
  uint32_t                 slot_key  = 0;  ///< Slot number (system slot) the job belongs to.
  unsigned                 slot_in_frame = 0;
  unsigned                 grid_slot = 0;  ///< The batch's grid index in the service's grid class.
  unsigned                 P         = 0;
  unsigned                 grid_prb  = 0;
  hipEvent_t               uploaded  = nullptr;  ///< DMA upload of the grid (multi-device shards), else nullptr
  const void*              grid_src  = nullptr;  ///< The grid in mapped host memory, copied in by the launch
  uint32_t*                grid_dst  = nullptr;  ///< ... into the batch's HBM grid slot
  size_t                   grid_bytes = 0;
  const pusch_harq_arena*  harq      = nullptr;  ///< The HARQ arena the layout addresses.
  clock_type::time_point   arrival;
};

} // namespace

/// A launch's plans and captured graph, cached by the sequence of its jobs' layout keys.
struct launch_plan {
  srsgpu_pusch_chest_plan*       chest         = nullptr;
  srsgpu_pusch_demodulator_plan* demod         = nullptr;
  srsgpu_ulsch_demux_plan*       demux         = nullptr;
  srsgpu_pusch_decoder_plan*     dec           = nullptr;
  hipGraphExec_t                 graph         = nullptr;
  uint64_t                       graph_buffers = 0;  ///< pusch_launcher::buffer_generation the graph was captured with
  bool                           graph_download = false;
  std::vector<std::array<uint32_t, 14>> harq_ack_counts, csi1_counts;  ///< per demultiplexed transmission
  std::vector<int8_t*>           arenas;     ///< HARQ arenas of the launch's sectors (the copies' arena table)
  std::vector<uint32_t>          job_arena;  ///< per job: its arena's index in `arenas`
  unsigned                       nof_copies = 0;
  std::vector<std::pair<size_t, unsigned>> dc_zero;  ///< estimate byte offset and rows of each DC zeroing
  size_t   arena_o = 0, ptr_o = 0, flag_o = 0, iter_o = 0, tbok_o = 0, nv_o = 0, m_o = 0, st_o = 0, uci_o = 0, tb_o = 0,
           end_o = 0;
  std::vector<uint16_t> dmrs_rows;  ///< Per job: the union of its PDUs' DM-RS symbol masks (rows the estimator reads).
  unsigned nof_dmrs_spans = 0, nof_data_spans = 0;  ///< Split grid copy: one span per (port, symbol) row.
  bool     graph_split    = false;                 ///< The captured graph copies the grids itself (split).
  const void* graph_spans = nullptr;               ///< ... from this span list.
  unsigned n = 0, cb_total = 0, llr_total = 0, harq_total = 0, max_grid = 0;

  static void destroy(launch_plan* p)
  {
    if (p->graph != nullptr) {
      (void)hipGraphExecDestroy(p->graph);
    }
    srsgpu_pusch_chest_plan_destroy(p->chest);
    srsgpu_pusch_demodulator_plan_destroy(p->demod);
    srsgpu_ulsch_demux_plan_destroy(p->demux);
    srsgpu_pusch_decoder_plan_destroy(p->dec);
    delete p;
  }
};

/// The device side of a launch on one GPU and stream: the launch plans (cached; plans hold mutable state - the
/// demodulator's statistics accumulators, the decoder's TB slices - so every launcher owns its own), staging and device
/// buffers, the captured graph, and the replay of the results through the reference's processor. Used by the GPU
/// service (one per launch set) and by the multi-GPU batch (one per shard device).
class pusch_launcher
{
  static constexpr const char* WHO = "pusch_launcher";

public:
  explicit pusch_launcher(srsgpu_context* ctx_) :
    ctx(ctx_), stream(ctx_, WHO), launches(launch_plan::destroy, SLOT_PLANS), io(WHO), msgs(WHO)
  {
    hip_check(hipEventCreateWithFlags(&done, hipEventDisableTiming), WHO, "event");
  }
  ~pusch_launcher()
  {
    (void)hipStreamSynchronize(stream.get());
    launches.clear();
    (void)hipEventDestroy(done);
    (void)hipFree(d_ce);
    (void)hipFree(d_llr);
    (void)hipFree(d_sch_b);
    (void)hipFree(d_uci_b);
  }

  /// Host-clock stamps of a launch (diagnostics).
  struct stamps {
    clock_type::time_point start, built, filled, launched;
    bool                   plan_created   = false;  ///< the launch plan was not cached (a new group layout)
    bool                   graph_captured = false;  ///< its graph was (re)captured
  };

  /// Launches `jobs` (one grid shape; their grids in d_grids, uploads signalled by the jobs' events): the launch plan,
  /// the HARQ context, the captured graph. download: the results come back to pinned memory (else they stay in the
  /// device result region for a transport to gather).
  stamps launch(const std::vector<std::unique_ptr<pusch_job>>& jobs, uint32_t* d_grids, bool download);

  /// Waits for the launch; fetches the kept CB messages when a failed TB has passed CBs (download mode).
  void wait(const std::vector<std::unique_ptr<pusch_job>>& jobs);

  /// Replays every PDU of `jobs` through the reference's processor from results at io_host (the staging image: result
  /// offsets of the launch plan) and msgs_host (the CB messages).
  void replay(const std::vector<std::unique_ptr<pusch_job>>& jobs, const uint8_t* io_host, const uint8_t* msgs_host);
  /// One job's replay. Jobs of distinct batches replay concurrently on different threads, except those with a CSI Part 2
  /// PDU (needs_second_phase), whose second launch uses this launcher's deferred-decode state: one thread at a time.
  void        replay_job(pusch_job& job, const uint8_t* io_host, const uint8_t* msgs_host);
  static bool needs_second_phase(const pusch_job& job);

  const launch_plan& current() const { return *plan; }
  /// The device result region [flag_o, end_o) and the CB messages of the current launch.
  const uint8_t* device_results() { return io.dev<uint8_t>(plan->flag_o); }
  size_t         results_bytes() const { return plan->end_o - plan->flag_o; }
  const uint8_t* device_msgs() { return msgs.dev<uint8_t>(); }
  size_t         msgs_bytes() const { return static_cast<size_t>(plan->cb_total) * SRSGPU_CB_MSG_STRIDE; }
  const uint8_t* host_io() { return ioh<uint8_t>(0); }
  const uint8_t* host_msgs() { return msgs.host<uint8_t>(); }
  hipStream_t    get_stream() const { return stream.get(); }
  hipEvent_t     done_event() const { return done; }

private:
  launch_plan* create_plan(const std::vector<std::unique_ptr<pusch_job>>& jobs, unsigned P, unsigned grid_prb);

  /// The second launch of a CSI Part 2 PDU (from the replay, once CSI Part 1 is decoded): the codeword LLRs the first
  /// launch left in HBM demultiplexed again with the CSI Part 2 size (0: none) from first_symbol on, the UL-SCH decoded
  /// with the bit count that leaves (pusch_processor_impl.cpp:84-100), the HARQ arena around it; synchronous. Results
  /// in d_io / d_msgs at d_lay.
  void decode_deferred(const pusch_entry& e, const pusch_harq_arena& harq, unsigned bits, unsigned enc_bits,
                       unsigned first_symbol);

  struct deferred_plan {
    srsgpu_ulsch_demux_plan*   demux = nullptr;
    srsgpu_pusch_decoder_plan* dec   = nullptr;
    static void                destroy(deferred_plan* p)
    {
      srsgpu_ulsch_demux_plan_destroy(p->demux);
      srsgpu_pusch_decoder_plan_destroy(p->dec);
      delete p;
    }
  };
  struct deferred_layout {
    size_t arena_o = 0, ptr_o = 0, flag_o = 0, iter_o = 0, tbok_o = 0, csi2_o = 0, tb_o = 0, end_o = 0;
    std::array<uint32_t, 14> csi2_counts{};
  };
  plan_cache<deferred_plan> deferred_plans{deferred_plan::destroy, 16};
  staged_buffer             d_io{"pusch_launcher deferred"};
  staged_buffer             d_msgs{"pusch_launcher deferred"};
  int8_t*                   d_sch_b     = nullptr;
  size_t                    d_sch_b_cap = 0;
  int8_t*                   d_uci_b     = nullptr;
  size_t                    d_uci_b_cap = 0;
  deferred_layout           d_lay;
  std::vector<uint8_t>      d_decoded;

  template <typename T>
  static void reserve_device(T*& ptr, size_t& cap, size_t bytes, const char* what)
  {
    if (bytes <= cap) {
      return;
    }
    std::lock_guard<std::recursive_mutex> lock(hip_setup_mutex());
    (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    hip_check(hipMalloc(reinterpret_cast<void**>(&ptr), bytes), WHO, what);
    cap = bytes;
  }

  srsgpu_context*         ctx;
  owned_stream            stream;
  hipEvent_t              done = nullptr;
  plan_cache<launch_plan> launches;
  staged_buffer           io;    ///< Inputs and results (layout in launch_plan).

  template <typename T = uint8_t>
  T* ioh(size_t off)
  {
    return io.host<T>(off);
  }
  template <typename T = uint8_t>
  T* iod(size_t off)
  {
    return io.dev<T>(off);
  }
  staged_buffer           msgs;  ///< CB messages: HARQ context in, kept messages out.
  mapped_buffer           spans{"pusch_launcher grid spans"};  ///< the launch's rx-grid copies (srsgpu_copy_spans)
  uint32_t*               d_ce       = nullptr;
  size_t                  d_ce_cap   = 0;
  int8_t*                 d_llr      = nullptr;
  size_t                  d_llr_cap  = 0;
  uint64_t                buffer_generation = 1;  ///< Bumped when a buffer above moves (graphs capture pointers).
  // The launch in flight.
  launch_plan*            plan = nullptr;
  bool                    downloaded = true;
  std::vector<uint8_t>    decoded_flags;
  std::vector<const pusch_job*> plan_jobs;
};

class pusch_slot_batch
{
  static constexpr const char* WHO = "pusch_slot_batch";

public:
  pusch_slot_batch(const pusch_batch_configuration&     cfg_,
                   std::shared_ptr<pusch_harq_arena>    arena_,
                   std::shared_ptr<uci_decoder_factory> uci_factory_,
                   std::unique_ptr<pusch_processor>     fallback_,
                   std::shared_ptr<pusch_gpu_service>   service_);
  ~pusch_slot_batch();

  /// Unmaps the uplink processor's grid storage (grid_in_place) once every launch is done; the owner calls it before
  /// the grid goes away.
  void release_host_grid();

  /// The device address of the grid's rows of ports 0..P-1 when they are one [port][symbol][subcarrier] block in
  /// host memory (the reference's resource_grid_impl tensor), mapped for the launch's copy kernel to read in place:
  /// no per-slot memcpy into the batch's buffer. nullptr: another layout (the rows are copied).
  const void* grid_in_place(const resource_grid_reader& grid, unsigned P, size_t row);

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

  /// Runs the PDUs the batch does not cover on the fallback processor and hands the others to the GPU service.
  void run(std::vector<pusch_entry>& entries);

  /// The estimator / demodulator / demultiplexer / decoder configurations pusch_processor_impl derives from each PDU
  /// (pusch_processor_impl.cpp:150-337) as srsgpu descriptors, the HARQ context and the layout key of a job, on the
  /// submitting thread (the service's dispatcher only concatenates layouts).
  void build_layout(pusch_job& job, const pusch_harq_arena& harq) const;

  /// Service side: replays one entry of a finished launch (completion thread).
  replay_processor& replay_for_this_thread();
  /// Service side: the job ended (replayed or failed).
  void job_done();

  const pusch_batch_configuration   cfg;
  std::shared_ptr<pusch_harq_arena> arena;

private:
  /// PDUs the batch covers: SCH data with or without UCI on PUSCH (HARQ-ACK, CSI Part 1, CSI Part 2: the UL-SCH of a
  /// CSI Part 2 PDU is decoded in a second launch once the replay has decoded CSI Part 1), identity rx port list, up
  /// to four layers.
  static bool batchable(const pusch_entry& e)
  {
    const pusch_processor::pdu_t& pdu = e.pdu;
    if (!pdu.codeword.has_value() || pdu.nof_tx_layers == 0 || pdu.nof_tx_layers > 4 || pdu.rx_ports.empty() ||
        pdu.rx_ports.size() > 4 || pdu.cp != cyclic_prefix::NORMAL) {
      return false;
    }
    for (unsigned p = 0; p != pdu.rx_ports.size(); ++p) {
      if (pdu.rx_ports[p] != p) {
        return false;
      }
    }
    return true;
  }

  std::shared_ptr<pusch_gpu_service>   service;
  srsgpu_context*                      ctx;
  std::shared_ptr<uci_decoder_factory> uci_factory;
  std::unique_ptr<pusch_processor>     fallback;
  staged_buffer                        grid_buf;  ///< Pinned copy of the rx grid for the shards' DMA uploads.
  mapped_buffer                        grid_map{"pusch_slot_batch grid"};  ///< The rx grid, read in place by the launch
  /// The uplink processor's own grid storage, page-locked and mapped once (grid_in_place): base, bytes, device address.
  const uint8_t*                       host_grid      = nullptr;
  size_t                               host_grid_size = 0;
  const void*                          host_grid_dev  = nullptr;
  bool                                 host_grid_off  = false;  ///< registration failed once: copy from now on
  /// The grid's HBM twin (host_blocks::twin): the batch's grid slot, announced once the host grid is registered; the
  /// lower PHY sets a bit per symbol it demodulated into both, and a slot with all of them set copies nothing.
  bool                                 twin_announced = false;
  std::atomic<uint32_t>                twin_symbols{0};
  unsigned                             batch_id   = 0;
  int                                  grid_slot  = -1;
  unsigned                             grid_P     = 0;
  unsigned                             grid_prb   = 0;
  uint32_t*                            d_grid     = nullptr;
  std::mutex                           pending_mtx;
  std::vector<pusch_entry>             pending;
  std::mutex                           run_mtx;
  std::mutex                           done_mtx;
  std::condition_variable              done_cv;
  unsigned                             outstanding = 0;
  std::map<std::thread::id, replay_processor> replays;
  std::mutex                                  replays_mtx;

  /// Multi-GPU mode (cfg.devices): one shard per listed device.
  struct shard_device {
    int                               device = 0;
    std::shared_ptr<srsgpu_context>   ctx;
    std::shared_ptr<pusch_harq_arena> arena;
    std::unique_ptr<pusch_launcher>   launcher;
    std::unique_ptr<owned_stream>     upload;
    hipEvent_t                        uploaded = nullptr;
    uint32_t*                         d_grid   = nullptr;
    size_t                            grid_cap = 0;
  };
  void                                    run_multi(std::unique_ptr<pusch_job> job);
  void                                    multi_complete_loop();
  std::vector<shard_device>               shards;
  std::shared_ptr<pusch_result_transport> transport;
  std::unique_ptr<owned_stream>           root_stream;
  staged_buffer                           gathered{"pusch_slot_batch gather"};
  mapped_buffer                           shard_spans{"pusch_slot_batch shard spans"};  ///< grid copies per shard
  /// The slot in flight (one per batch: run waits for the previous): its shards' jobs and their result offsets in
  /// the gathered image, replayed by the completion thread once root_done has passed.
  std::vector<std::vector<std::unique_ptr<pusch_job>>> multi_jobs;
  std::vector<std::pair<size_t, size_t>>               multi_offsets;
  hipEvent_t                                           root_done = nullptr;
  std::thread                                          multi_completion;
  std::mutex                                           multi_mtx;
  std::condition_variable                              multi_cv;
  bool                                                 multi_pending = false;
  bool                                                 multi_stop    = false;
};

class pusch_gpu_service
{
  static constexpr const char* WHO = "pusch_gpu_service";

public:
  explicit pusch_gpu_service(const pusch_service_configuration& cfg_);
  ~pusch_gpu_service();

  srsgpu_context* context() const { return ctx.get(); }

  /// A batch's fixed HBM grid slot for grids of P ports x grid_prb PRBs: (index within the shape's arena, pointer).
  std::pair<unsigned, uint32_t*> register_grid(unsigned P, unsigned grid_prb);
  /// Returns a batch's grid slot (the batch is destroyed): uplink processors come and go with the factories that
  /// create them, while the device's service lives on.
  void     release_grid(unsigned P, unsigned grid_prb, unsigned index);
  unsigned new_batch_id() { return next_batch_id++; }

  void submit(std::unique_ptr<pusch_job> job);

private:
  struct grid_class {
    unsigned              P = 0, prb = 0, used = 0;
    uint32_t*             d_grids = nullptr;
    std::vector<unsigned> free;  ///< released slots below `used`
  };

  /// One launch in flight: a launcher (stream, staging, buffers, cached launch plans) and its jobs.
  struct launch_set {
    explicit launch_set(srsgpu_context* ctx) : L(ctx) {}
    pusch_launcher                          L;
    std::vector<std::unique_ptr<pusch_job>> jobs;
    clock_type::time_point                  t_launched;
    bool                                    busy = false;  ///< Guarded by the service's mutex.
  };

  void dispatch_loop();
  void complete_loop();
  void replay_loop();
  void replay_share(launch_set& set);
  void launch(launch_set& set);
  void finish(launch_set& set);
  void fail_jobs(launch_set& set, const char* what);

  const pusch_service_configuration cfg;
  std::shared_ptr<srsgpu_context>   ctx;
  std::atomic<unsigned>             next_batch_id{0};
  std::mutex                        grid_mtx;
  std::vector<grid_class>           grid_classes;
  std::vector<std::unique_ptr<launch_set>> sets;

  std::mutex                              mtx;
  std::condition_variable                 cv;       ///< New job, or stop.
  std::condition_variable                 free_cv;  ///< A launch set was released.
  std::condition_variable                 done_cv;  ///< A launch set was queued for completion.
  std::deque<std::unique_ptr<pusch_job>>  pending;
  std::deque<launch_set*>                 in_flight;
  bool                                    stop            = false;
  bool                                    dispatcher_done = false;
  std::thread                             dispatcher;
  std::thread                             completer;

  // Replay helpers (cfg.replay_threads - 1 of them; the completion thread replays too): a launch's jobs are shared
  // out through rp_next, one job at a time.
  std::vector<std::thread> replayers;
  std::mutex               rp_mtx;
  std::condition_variable  rp_cv;       ///< new work or stop
  std::condition_variable  rp_done_cv;  ///< a helper finished its share
  launch_set*              rp_set    = nullptr;
  std::atomic<size_t>      rp_next{0};
  uint64_t                 rp_gen    = 0;
  unsigned                 rp_busy   = 0;
  bool                     rp_stop   = false;

  // SRSGPU_BATCH_TIMING=1: mean host-clock time per launch of each phase (diagnostics).
  const bool timing = std::getenv("SRSGPU_BATCH_TIMING") != nullptr;
  double     phase_us[5]   = {};  ///< build + plans, fill, graph + launch, wait for GPU, replay
  uint64_t   timed_launches = 0;
  uint64_t   timed_slots    = 0;
  uint64_t   plans_created   = 0;  ///< launches whose group layout was not cached (new plans)
  uint64_t   graphs_captured = 0;  ///< launches that (re)captured their graph
  double     setup_us        = 0;  ///< dispatcher time of those launches
  std::array<uint64_t, 33> launch_sizes{};  ///< launches by slots per launch (32: 32 or more)
};

// ---------------------------------------------------------------------------------------------------------------------

pusch_gpu_service::pusch_gpu_service(const pusch_service_configuration& cfg_) :
  cfg(cfg_), ctx(shared_context(cfg_.device))
{
  if (cfg.nof_launch_sets == 0 || cfg.max_slots_per_launch == 0 || cfg.max_grids == 0) {
    throw std::invalid_argument(std::string(WHO) + ": invalid configuration");
  }
  device_scope dev(ctx.get(), WHO);
  for (unsigned i = 0; i != cfg.nof_launch_sets; ++i) {
    sets.push_back(std::make_unique<launch_set>(ctx.get()));
  }
  dispatcher = std::thread([this] { dispatch_loop(); });
  completer  = std::thread([this] { complete_loop(); });
  for (unsigned i = 1; i < cfg.replay_threads; ++i) {
    replayers.emplace_back([this] { replay_loop(); });
  }
}

pusch_gpu_service::~pusch_gpu_service()
{
  {
    std::lock_guard<std::mutex> lock(mtx);
    stop = true;
  }
  cv.notify_all();
  free_cv.notify_all();
  done_cv.notify_all();
  dispatcher.join();
  completer.join();
  {
    std::lock_guard<std::mutex> lock(rp_mtx);
    rp_stop = true;
  }
  rp_cv.notify_all();
  for (std::thread& t : replayers) {
    t.join();
  }
  if (timing && timed_launches > 0) {
    std::fprintf(stderr,
                 "pusch_gpu_service: %llu launches, %.2f slots per launch, us per launch: build %.1f, fill %.1f, "
                 "graph+launch %.1f, GPU wait %.1f, replay %.1f; new plans %llu, graph captures %llu (%.0f us of "
                 "dispatcher time)\n",
                 static_cast<unsigned long long>(timed_launches), static_cast<double>(timed_slots) / timed_launches,
                 phase_us[0] / timed_launches, phase_us[1] / timed_launches, phase_us[2] / timed_launches,
                 phase_us[3] / timed_launches, phase_us[4] / timed_launches,
                 static_cast<unsigned long long>(plans_created), static_cast<unsigned long long>(graphs_captured),
                 setup_us);
    std::fprintf(stderr, "pusch_gpu_service: launches by slots per launch:");
    for (size_t n = 1; n != launch_sizes.size(); ++n) {
      if (launch_sizes[n] != 0) {
        std::fprintf(stderr, " %zu:%llu", n, static_cast<unsigned long long>(launch_sizes[n]));
      }
    }
    std::fprintf(stderr, "\n");
  }
  std::lock_guard<std::recursive_mutex> lock(hip_setup_mutex());
  device_scope                          dev(ctx.get(), WHO);
  sets.clear();
  for (grid_class& g : grid_classes) {
    (void)hipFree(g.d_grids);
  }
}

std::pair<unsigned, uint32_t*> pusch_gpu_service::register_grid(unsigned P, unsigned grid_prb)
{
  std::lock_guard<std::mutex> lock(grid_mtx);
  grid_class*                 g = nullptr;
  for (grid_class& c : grid_classes) {
    if (c.P == P && c.prb == grid_prb) {
      g = &c;
    }
  }
  const size_t grid_bytes = static_cast<size_t>(P) * 14 * NRE * grid_prb * sizeof(uint32_t);
  if (g == nullptr) {
    grid_class c;
    c.P   = P;
    c.prb = grid_prb;
    {
      std::lock_guard<std::recursive_mutex> setup(hip_setup_mutex());
      device_scope                          dev(ctx.get(), WHO);
      hip_check(hipMalloc(reinterpret_cast<void**>(&c.d_grids), cfg.max_grids * grid_bytes), WHO, "grid arena");
    }
    grid_classes.push_back(c);
    g = &grid_classes.back();
  }
  unsigned index = 0;
  if (!g->free.empty()) {
    index = g->free.back();
    g->free.pop_back();
  } else {
    if (g->used == cfg.max_grids) {
      throw std::length_error(std::string(WHO) + ": more batches than max_grids for one grid shape");
    }
    index = g->used++;
  }
  return {index, g->d_grids + index * (grid_bytes / sizeof(uint32_t))};
}

void pusch_gpu_service::release_grid(unsigned P, unsigned grid_prb, unsigned index)
{
  std::lock_guard<std::mutex> lock(grid_mtx);
  for (grid_class& c : grid_classes) {
    if (c.P == P && c.prb == grid_prb) {
      c.free.push_back(index);
      return;
    }
  }
}

void pusch_gpu_service::submit(std::unique_ptr<pusch_job> job)
{
  job->arrival = clock_type::now();
  {
    std::lock_guard<std::mutex> lock(mtx);
    pending.push_back(std::move(job));
  }
  cv.notify_all();
}

void pusch_gpu_service::dispatch_loop()
{
  (void)hipSetDevice(srsgpu_context_device(ctx.get()));
  for (;;) {
    std::unique_lock<std::mutex> lock(mtx);
    cv.wait(lock, [&] { return stop || !pending.empty(); });
    if (pending.empty()) {
      dispatcher_done = true;  // stop, with every submitted slot launched
      lock.unlock();
      done_cv.notify_all();
      return;
    }
    // The slots of the oldest job's slot number and grid shape (one launch reads one grid arena).
    const pusch_job& front = *pending.front();
    auto             match = [&](const pusch_job& j) {
      return j.slot_key == front.slot_key && j.P == front.P && j.grid_prb == front.grid_prb;
    };
    size_t count = 0;
    for (const auto& j : pending) {
      count += match(*j) ? 1 : 0;
    }
    if (!stop && count < std::min(cfg.expected_slots_per_launch, cfg.max_slots_per_launch) &&
        cfg.gather_window_us > 0) {
      const auto deadline = front.arrival + std::chrono::microseconds(cfg.gather_window_us);
      if (clock_type::now() < deadline) {
        cv.wait_until(lock, deadline);
        continue;  // re-evaluate with what arrived
      }
    }
    std::vector<std::unique_ptr<pusch_job>> group;
    for (auto it = pending.begin(); it != pending.end() && group.size() < cfg.max_slots_per_launch;) {
      if (match(**it)) {
        group.push_back(std::move(*it));
        it = pending.erase(it);
      } else {
        ++it;
      }
    }
    // A canonical order, so that a recurring set of cells finds its cached plans and graph.
    std::sort(group.begin(), group.end(), [](const auto& a, const auto& b) { return a->batch_id < b->batch_id; });
    // The launch set of the slot's index within the frame: a recurring group of cells finds its launch plan cached in
    // one set instead of being planned once per set. The completion thread releases sets until the end.
    launch_set* set = sets[group.front()->slot_in_frame % sets.size()].get();
    free_cv.wait(lock, [&] { return !set->busy; });
    set->busy = true;
    lock.unlock();

    set->jobs = std::move(group);
    try {
      launch(*set);
    } catch (const std::exception& e) {
      fail_jobs(*set, e.what());
      std::lock_guard<std::mutex> relock(mtx);
      set->busy = false;
      continue;
    }
    {
      std::lock_guard<std::mutex> relock(mtx);
      in_flight.push_back(set);
    }
    done_cv.notify_all();
  }
}

void pusch_gpu_service::complete_loop()
{
  (void)hipSetDevice(srsgpu_context_device(ctx.get()));
  for (;;) {
    launch_set* set = nullptr;
    {
      std::unique_lock<std::mutex> lock(mtx);
      done_cv.wait(lock, [&] { return !in_flight.empty() || dispatcher_done; });
      if (in_flight.empty()) {
        return;  // the dispatcher has stopped and every launch is replayed
      }
      set = in_flight.front();
      in_flight.pop_front();
    }
    try {
      finish(*set);
    } catch (const std::exception& e) {
      fail_jobs(*set, e.what());
    }
    set->jobs.clear();
    {
      std::lock_guard<std::mutex> lock(mtx);
      set->busy = false;
    }
    free_cv.notify_all();
  }
}

/// Takes jobs of the shared launch one at a time and replays those without a second phase.
void pusch_gpu_service::replay_share(launch_set& set)
{
  for (size_t i = rp_next++; i < set.jobs.size(); i = rp_next++) {
    pusch_job& job = *set.jobs[i];
    if (!pusch_launcher::needs_second_phase(job)) {
      set.L.replay_job(job, set.L.host_io(), set.L.host_msgs());
    }
  }
}

void pusch_gpu_service::replay_loop()
{
  uint64_t seen = 0;
  for (;;) {
    launch_set* set = nullptr;
    {
      std::unique_lock<std::mutex> lock(rp_mtx);
      rp_cv.wait(lock, [&] { return rp_stop || rp_gen != seen; });
      if (rp_stop) {
        return;
      }
      seen = rp_gen;
      set  = rp_set;
    }
    try {
      replay_share(*set);
    } catch (const std::exception& e) {
      fail_jobs(*set, e.what());
    }
    {
      std::lock_guard<std::mutex> lock(rp_mtx);
      --rp_busy;
    }
    rp_done_cv.notify_all();
  }
}

void pusch_gpu_service::fail_jobs(launch_set& set, const char* what)
{
  // A GPU or configuration error leaves the slots' PUSCH results undeliverable: fatal, with its reason, as the
  // reference's own processors treat failures they cannot notify (error_handling.h report_fatal_error).
  report_fatal_error("pusch_slot_batch: {}", what);
  (void)set;
}

/// Concatenates the layouts of a launch's jobs into absolute descriptors and creates their plans (a cache miss).
launch_plan* pusch_launcher::create_plan(const std::vector<std::unique_ptr<pusch_job>>& jobs, unsigned P, unsigned grid_prb)
{
  std::vector<srsgpu_pusch_chest_config> chest_c;
  std::vector<srsgpu_pusch_demod_config> demod_c;
  std::vector<srsgpu_alloc_ext>          chest_x, demod_x;
  std::vector<srsgpu_pusch_tb_config>    tbs;
  std::vector<srsgpu_ulsch_demux_config> demuxes;
  auto                                   lp = std::make_unique<launch_plan>();
  unsigned llr_b = 0, cb_b = 0, tb_b = 0, harq_b = 0, uci_b = 0, copy_b = 0;
  for (const auto& job : jobs) {
    const job_layout& L = job->lay;
    for (const pusch_chest_desc& d : L.chests) {
      chest_c.push_back(d.c);
      chest_x.push_back(d.ext());
    }
    for (const pusch_demod_desc& d : L.demods) {
      demod_c.push_back(d.c);
      demod_c.back().llr_offset += llr_b;
      demod_x.push_back(d.ext());
    }
    for (srsgpu_pusch_tb_config t : L.tbs) {
      t.llr_offset += llr_b;
      t.harq_offset += harq_b;
      t.cb_offset += cb_b;
      t.tb_offset += tb_b;
      tbs.push_back(t);
    }
    for (srsgpu_ulsch_demux_config d : L.demuxes) {
      d.llr_offset += llr_b;
      d.sch_offset += llr_b;
      d.harq_offset += uci_b;
      d.csi1_offset += uci_b;
      demuxes.push_back(d);
    }
    for (const auto& z : L.dc_zero_local) {
      lp->dc_zero.push_back(z);
    }
    uint16_t rows = 0;
    for (const pusch_chest_desc& d : L.chests) {
      rows |= d.c.dmrs_symbol_mask;
    }
    lp->dmrs_rows.push_back(rows);
    lp->nof_dmrs_spans += P * static_cast<unsigned>(__builtin_popcount(rows & 0x3fffu));
    lp->nof_data_spans += P * (14u - static_cast<unsigned>(__builtin_popcount(rows & 0x3fffu)));
    int8_t*    arena = job->batch->arena->d_soft;
    const auto it    = std::find(lp->arenas.begin(), lp->arenas.end(), arena);
    lp->job_arena.push_back(static_cast<uint32_t>(it - lp->arenas.begin()));
    if (it == lp->arenas.end()) {
      lp->arenas.push_back(arena);
    }
    lp->max_grid = std::max(lp->max_grid, job->grid_slot + 1);
    llr_b += L.llr_total;
    cb_b += L.cb_total;
    tb_b += L.tb_total;
    harq_b += L.harq_total;
    uci_b += L.uci_total;
    copy_b += static_cast<unsigned>(L.copies.size());
    lp->n += L.n;
  }
  lp->nof_copies = copy_b;
  lp->cb_total   = cb_b;
  lp->llr_total  = llr_b;
  lp->harq_total = harq_b;
  const unsigned n = lp->n;
  srsgpu_check(srsgpu_pusch_chest_plan_create_ex(ctx, chest_c.data(), chest_x.data(), n, grid_prb, P, &lp->chest),
               WHO);
  srsgpu_check(
      srsgpu_pusch_demodulator_plan_create_ex(ctx, demod_c.data(), demod_x.data(), n, grid_prb, P, &lp->demod),
      WHO);
  if (!demuxes.empty()) {
    srsgpu_check(srsgpu_ulsch_demux_plan_create(ctx, demuxes.data(), demuxes.size(), &lp->demux), WHO);
    lp->harq_ack_counts.resize(demuxes.size());
    lp->csi1_counts.resize(demuxes.size());
    for (uint32_t k = 0; k != demuxes.size(); ++k) {
      srsgpu_check(srsgpu_ulsch_demux_plan_symbol_llrs(lp->demux, k, 2, lp->harq_ack_counts[k].data()), WHO);
      srsgpu_check(srsgpu_ulsch_demux_plan_symbol_llrs(lp->demux, k, 3, lp->csi1_counts[k].data()), WHO);
    }
  }
  if (!tbs.empty()) {
    srsgpu_check(srsgpu_pusch_decoder_plan_create(ctx, SRSGPU_LDPC_IMPL_SIMD, tbs.data(), tbs.size(), &lp->dec), WHO);
  }

  // Staging image: [copy jobs | arena table | HARQ buffer pointers | CB CRC flags] uploaded, [CB CRC flags | iterations |
  // TB CRC flags | nv | metrics | statistics | UCI streams | TBs] downloaded (the CRC flags are the HARQ context in and
  // the result out).
  auto align  = [](size_t x) { return (x + 63) / 64 * 64; };
  lp->arena_o = align(static_cast<size_t>(copy_b) * sizeof(srsgpu_harq_copy_job));
  lp->ptr_o   = align(lp->arena_o + lp->arenas.size() * sizeof(int8_t*));
  lp->flag_o  = align(lp->ptr_o + static_cast<size_t>(cb_b) * sizeof(int8_t*));
  lp->iter_o = align(lp->flag_o + cb_b);
  lp->tbok_o = align(lp->iter_o + static_cast<size_t>(cb_b) * sizeof(int32_t));
  lp->nv_o   = align(lp->tbok_o + n);
  lp->m_o    = align(lp->nv_o + 4 * n * sizeof(float));
  lp->st_o   = align(lp->m_o + 4 * n * SRSGPU_CHEST_METRICS * sizeof(float));
  lp->uci_o  = align(lp->st_o + n * SRSGPU_DEMOD_STATS * sizeof(float));
  lp->tb_o   = align(lp->uci_o + uci_b);
  lp->end_o  = lp->tb_o + std::max<unsigned>(tb_b, 16);
  return lp.release();
}

/// Launches jobs: the launch plan (cached by the sequence of the jobs' layout keys: a cell's grants repeat and the
/// service orders a launch's slots canonically), the HARQ context, the wait for the jobs' grid uploads and the
/// replay of the launch's captured graph.
pusch_launcher::stamps pusch_launcher::launch(const std::vector<std::unique_ptr<pusch_job>>& jobs, uint32_t* d_grids,
                                              bool download)
{
  stamps tm;
  tm.start = clock_type::now();
  const unsigned P        = jobs.front()->P;
  const unsigned grid_prb = jobs.front()->grid_prb;
  const size_t   row      = static_cast<size_t>(grid_prb) * NRE * sizeof(uint32_t);
  std::vector<uint8_t> key;
  key_append(key, P);
  key_append(key, grid_prb);
  for (const auto& job : jobs) {
    key_append(key, job->lay.key.size());
    key.insert(key.end(), job->lay.key.begin(), job->lay.key.end());
  }
  const uint64_t misses = launches.misses();
  launch_plan*   lp     = launches.get(key, [&] { return create_plan(jobs, P, grid_prb); });
  tm.plan_created       = launches.misses() != misses;
  plan                  = lp;
  downloaded      = download;
  // The staging image in HBM with an upload and a download node in the graph. (The image in mapped host memory, read
  // and written in place by the kernels, measured slower: 16-sector service 23.3-23.7k vs 42.7-45.0k one-PDU slots/s,
  // the decoder's and the statistics kernels' small scattered result stores cross PCIe one by one,
  // profiles/r5_io_mapped_ab.txt.)
  // Split grid copy: every job's grid is read from mapped host memory by the launch: a copy launch before the graph
  // moves the DM-RS symbol rows, and the channel estimator's launch (which reads only those) moves the data-symbol
  // rows on extra workgroups while it runs (one-PDU slot: grid copy 21 -> 7 us exposed). Shards whose grid came by
  // DMA copy nothing. (A fork onto a second stream inside the graph measured serialised and slower.)
  bool split = true;
  for (const auto& job : jobs) {
    split = split && job->grid_src != nullptr;
  }
  if (split) {
    spans.reserve((lp->nof_dmrs_spans + lp->nof_data_spans) * sizeof(srsgpu_copy_span));
  }

  // Buffers (grow-only; a move invalidates the captured graphs).
  {
    const void* before[4] = {io.host(), msgs.host(), d_ce, d_llr};
    io.reserve(lp->end_o);
    msgs.reserve(std::max<size_t>(static_cast<size_t>(lp->cb_total) * SRSGPU_CB_MSG_STRIDE, 64));
    reserve_device(d_ce, d_ce_cap, static_cast<size_t>(lp->max_grid) * 4 * P * 14 * row, "channel estimates");
    reserve_device(d_llr, d_llr_cap, std::max<size_t>(lp->llr_total, 64), "LLRs");
    const void* after[4] = {io.host(), msgs.host(), d_ce, d_llr};
    if (!std::equal(std::begin(before), std::end(before), std::begin(after))) {
      ++buffer_generation;
    }
  }
  hipStream_t s = stream.get();
  if (lp->graph == nullptr || lp->graph_buffers != buffer_generation || lp->graph_download != download ||
      lp->graph_split != split || (split && lp->graph_spans != spans.dev())) {
    std::lock_guard<std::recursive_mutex> setup_lock(hip_setup_mutex());
    if (lp->graph != nullptr) {
      (void)hipGraphExecDestroy(lp->graph);
      lp->graph = nullptr;
    }
    tm.graph_captured = true;
    lp->graph = capture_graph(s, WHO, [&] {
      io.upload(0, lp->iter_o, s);
      if (split) {
        // The estimator's launch also copies the data-symbol rows (extra workgroups), after the DM-RS rows it reads
        // were copied by the launch before the graph.
        srsgpu_check(srsgpu_pusch_chest_plan_execute_copy(
                         lp->chest, d_grids, d_ce, iod<float>(lp->nv_o), iod<float>(lp->m_o),
                         spans.dev<srsgpu_copy_span>() + lp->nof_dmrs_spans, lp->nof_data_spans, row, s),
                     WHO);
      } else {
        srsgpu_check(srsgpu_pusch_chest_plan_execute(lp->chest, d_grids, d_ce, iod<float>(lp->nv_o),
                                                     iod<float>(lp->m_o), s),
                     WHO);
      }
      // pusch_processor_impl.cpp:222-240: the DC subcarrier's estimate is zeroed for CP-OFDM transmissions over it.
      for (const auto& z : lp->dc_zero) {
        hip_check(hipMemset2DAsync(reinterpret_cast<uint8_t*>(d_ce) + z.first, row, 0, sizeof(uint32_t), z.second,
                                   s),
                  WHO, "DC");
      }
      srsgpu_check(srsgpu_pusch_demodulator_plan_execute_ex(lp->demod, d_grids, d_ce, iod<float>(lp->nv_o),
                                                            d_llr, iod<float>(lp->st_o), s),
                   WHO);
      if (lp->demux != nullptr) {
        int8_t* uci = iod<int8_t>(lp->uci_o);
        srsgpu_check(srsgpu_ulsch_demux_plan_execute(lp->demux, d_llr, d_llr, uci, uci, nullptr, s), WHO);
      }
      // The rate dematcher and the decoder work on the soft buffers in the rx-buffer arenas through the per-codeblock
      // pointer table (no copy into a batch HARQ buffer and back).
      if (lp->dec != nullptr) {
        srsgpu_check(srsgpu_pusch_decoder_plan_execute_arena(
                         lp->dec, d_llr, iod<int8_t*>(lp->ptr_o), iod<uint8_t>(lp->flag_o), msgs.dev<uint8_t>(),
                         iod<int32_t>(lp->iter_o), iod<uint8_t>(lp->tb_o), iod<uint8_t>(lp->tbok_o), s),
                     WHO);
      }
      if (download) {
        io.download(lp->flag_o, lp->end_o - lp->flag_o, s);
      }
    });
    lp->graph_buffers  = buffer_generation;
    lp->graph_download = download;
    lp->graph_split    = split;
    lp->graph_spans    = split ? spans.dev() : nullptr;
  }
  tm.built = clock_type::now();

  // Absolute offsets of the entries, the copy jobs and the HARQ context (flags; messages of CBs that passed before).
  decoded_flags.assign(lp->cb_total, 0);
  unsigned tx_b = 0, llr_b = 0, cb_b = 0, tb_b = 0, uci_b = 0, harq_b = 0, dmx_b = 0, tbi_b = 0;
  auto*    copies   = ioh<srsgpu_harq_copy_job>(0);
  bool     any_msgs = false;
  std::memcpy(ioh(lp->arena_o), lp->arenas.data(), lp->arenas.size() * sizeof(int8_t*));
  auto* harq_ptrs = ioh<int8_t*>(lp->ptr_o);
  for (size_t j = 0; j != jobs.size(); ++j) {
    const auto&       job = jobs[j];
    const job_layout& L   = job->lay;
    if (L.copies.size() != L.cb_total) {
      throw std::logic_error(std::string(WHO) + ": one HARQ copy per codeblock expected");
    }
    for (const srsgpu_harq_copy_job& c : L.copies) {
      *copies = c;
      copies->batch_offset += harq_b;
      copies->arena = lp->job_arena[j];
      // Codeblock cb_b + k of the plan (the job's copies are in codeblock order): its arena slot.
      *harq_ptrs++ = lp->arenas[lp->job_arena[j]] + static_cast<size_t>(c.slot) * HARQ_SLOT_BYTES;
      ++copies;
    }
    std::memcpy(ioh<uint8_t>(lp->flag_o + cb_b), L.flags.data(), L.cb_total);
    for (unsigned c = 0; c != L.cb_total; ++c) {
      decoded_flags[cb_b + c] = L.flags[c] != 0 ? 0 : 1;
    }
    for (const auto& m : L.msgs) {
      std::memcpy(msgs.host<uint8_t>(static_cast<size_t>(cb_b + m.first) * SRSGPU_CB_MSG_STRIDE), m.second.data(),
                  m.second.size());
      any_msgs = true;
    }
    for (pusch_entry& e : job->entries) {
      if (e.tb_index >= 0) {
        e.tb_index += static_cast<int>(tbi_b);
      }
      e.tx += tx_b;
      e.llr_offset += llr_b;
      e.sch_offset += llr_b;
      e.cb0 += cb_b;
      e.tb_offset += tb_b;
      e.harq0 += harq_b;
      e.harq_ack_offset += uci_b;
      e.csi1_offset += uci_b;
      if (e.demux_index >= 0) {
        e.demux_index += static_cast<int>(dmx_b);
        e.harq_ack_counts = lp->harq_ack_counts[static_cast<size_t>(e.demux_index)];
        e.csi1_counts     = lp->csi1_counts[static_cast<size_t>(e.demux_index)];
      }
    }
    tx_b += L.n;
    llr_b += L.llr_total;
    cb_b += L.cb_total;
    tb_b += L.tb_total;
    uci_b += L.uci_total;
    harq_b += L.harq_total;
    dmx_b += static_cast<unsigned>(L.demuxes.size());
    tbi_b += static_cast<unsigned>(L.tbs.size());
  }
  tm.filled = clock_type::now();

  // The grids: one launch copies every job's grid from mapped host memory into its HBM grid slot (zero-copy reads;
  // a DMA copy per slot ran the service at the DMA engines' ~29 GB/s); shards uploaded by DMA are waited for. The kept
  // messages only when a CB has passed before.
  if (split) {
    // The graph's copy nodes read this list: [DM-RS rows of every job | data rows of every job], one row per span.
    auto*    dm = spans.host<srsgpu_copy_span>();
    auto*    da = dm + lp->nof_dmrs_spans;
    unsigned nd = 0, na = 0;
    for (size_t j = 0; j != jobs.size(); ++j) {
      const auto* src = static_cast<const uint8_t*>(jobs[j]->grid_src);
      auto*       dst = reinterpret_cast<uint8_t*>(jobs[j]->grid_dst);
      for (unsigned r = 0; r != P * 14u; ++r) {
        const srsgpu_copy_span c{src + r * row, dst + r * row, row};
        if (((lp->dmrs_rows[j] >> (r % 14u)) & 1u) != 0) {
          dm[nd++] = c;
        } else {
          da[na++] = c;
        }
      }
    }
    if (nd != lp->nof_dmrs_spans || na != lp->nof_data_spans) {
      throw std::logic_error(std::string(WHO) + ": grid span count differs from the launch plan's");
    }
    if (nd > 0) {
      srsgpu_check(srsgpu_copy_spans(spans.dev<srsgpu_copy_span>(), nd, row, s), WHO);
    }
  } else {
    std::vector<srsgpu_copy_span> sp;
    uint64_t                      max_bytes = 0;
    for (const auto& job : jobs) {
      if (job->grid_src != nullptr) {
        sp.push_back({job->grid_src, job->grid_dst, job->grid_bytes});
        max_bytes = std::max<uint64_t>(max_bytes, job->grid_bytes);
      } else if (job->uploaded != nullptr) {
        hip_check(hipStreamWaitEvent(s, job->uploaded, 0), WHO, "wait for the grid upload");
      }
    }
    if (!sp.empty()) {
      spans.reserve(sp.size() * sizeof(srsgpu_copy_span));
      std::memcpy(spans.host(), sp.data(), sp.size() * sizeof(srsgpu_copy_span));
      srsgpu_check(srsgpu_copy_spans(spans.dev<srsgpu_copy_span>(), static_cast<uint32_t>(sp.size()), max_bytes, s),
                   WHO);
    }
  }
  if (any_msgs) {
    hip_check(hipMemcpyAsync(msgs.dev(), msgs.host(), static_cast<size_t>(lp->cb_total) * SRSGPU_CB_MSG_STRIDE,
                             hipMemcpyHostToDevice, s),
              WHO, "messages upload");
  }
  hip_check(hipGraphLaunch(lp->graph, s), WHO, "graph launch");
  hip_check(hipEventRecord(done, s), WHO, "event");
  tm.launched = clock_type::now();
  return tm;
}

void pusch_launcher::decode_deferred(const pusch_entry&      e,
                                     const pusch_harq_arena& harq,
                                     unsigned                bits,
                                     unsigned                enc_bits,
                                     unsigned                first_symbol)
{
  // The UL-SCH information with the CSI Part 2 size (pusch_processor_impl.cpp:84-87).
  ulsch_configuration uc = e.ulsch_cfg;
  uc.nof_csi_part2_bits  = units::bits(bits);
  const ulsch_information info = get_ulsch_information(uc);
  if (info.nof_csi_part2_bits.value() != enc_bits) {
    throw std::logic_error(std::string(WHO) + ": CSI Part 2 size differs from the processor's");
  }
  const unsigned            nsch = info.nof_ul_sch_bits.value();
  auto                      a64  = [](size_t x) { return (x + 63) / 64 * 64; };
  srsgpu_ulsch_demux_config d    = e.demux_cfg;
  d.llr_offset                   = e.llr_offset;  // the codeword in the first launch's LLR buffer
  d.nof_csi_part2_bits           = bits;
  d.nof_enc_csi_part2_bits       = enc_bits;
  d.csi2_first_symbol            = static_cast<uint16_t>(enc_bits != 0 ? first_symbol : 0);
  d.sch_offset                   = 0;
  d.harq_offset                  = 0;
  d.csi1_offset                  = static_cast<uint32_t>(a64(d.nof_enc_harq_ack_bits));
  d.csi2_offset                  = 0;
  srsgpu_pusch_tb_config t       = e.tb_cfg;
  t.nof_ch_symbols               = nsch / t.modulation_order;
  t.llr_offset = t.harq_offset = t.cb_offset = t.tb_offset = 0;
  std::vector<uint8_t> key;
  key_append(key, d);
  key_append(key, t);
  deferred_plan* dp = deferred_plans.get(key, [&] {
    auto p = std::make_unique<deferred_plan>();
    srsgpu_check(srsgpu_ulsch_demux_plan_create(ctx, &d, 1, &p->demux), WHO);
    srsgpu_check(srsgpu_pusch_decoder_plan_create(ctx, SRSGPU_LDPC_IMPL_SIMD, &t, 1, &p->dec), WHO);
    return p.release();
  });
  srsgpu_check(srsgpu_ulsch_demux_plan_symbol_llrs(dp->demux, 0, 4, d_lay.csi2_counts.data()), WHO);

  // [copies | arena table | HARQ buffer pointers | CB flags] up, [CB flags | iterations | TB flag | CSI Part 2 | TB]
  // down.
  const unsigned n_cb = static_cast<unsigned>(e.copies.size());
  d_lay.arena_o       = a64(n_cb * sizeof(srsgpu_harq_copy_job));
  d_lay.ptr_o         = a64(d_lay.arena_o + sizeof(int8_t*));
  d_lay.flag_o        = a64(d_lay.ptr_o + n_cb * sizeof(int8_t*));
  d_lay.iter_o        = a64(d_lay.flag_o + n_cb);
  d_lay.tbok_o        = a64(d_lay.iter_o + n_cb * sizeof(int32_t));
  d_lay.csi2_o        = a64(d_lay.tbok_o + 1);
  d_lay.tb_o          = a64(d_lay.csi2_o + enc_bits);
  d_lay.end_o         = d_lay.tb_o + std::max<size_t>(e.data.size(), 16);
  d_io.reserve(d_lay.end_o);
  d_msgs.reserve(std::max<size_t>(static_cast<size_t>(n_cb) * SRSGPU_CB_MSG_STRIDE, 64));
  reserve_device(d_sch_b, d_sch_b_cap, std::max<size_t>(nsch, 64), "deferred UL-SCH");
  reserve_device(d_uci_b, d_uci_b_cap, d.csi1_offset + a64(d.nof_enc_csi_part1_bits) + 64, "deferred UCI");
  std::memcpy(d_io.host(0), e.copies.data(), n_cb * sizeof(srsgpu_harq_copy_job));
  int8_t* arena_base = harq.d_soft;
  std::memcpy(d_io.host(d_lay.arena_o), &arena_base, sizeof(arena_base));
  for (unsigned c = 0; c != n_cb; ++c) {
    int8_t* p = arena_base + static_cast<size_t>(e.copies[c].slot) * HARQ_SLOT_BYTES;
    std::memcpy(d_io.host(d_lay.ptr_o + c * sizeof(int8_t*)), &p, sizeof(p));
  }
  std::memcpy(d_io.host(d_lay.flag_o), e.flags.data(), n_cb);
  d_decoded.assign(n_cb, 0);
  bool any_msgs = false;
  for (unsigned c = 0; c != n_cb; ++c) {
    d_decoded[c] = e.flags[c] != 0 ? 0 : 1;
    if (!e.msgs[c].empty()) {
      std::memcpy(d_msgs.host<uint8_t>(static_cast<size_t>(c) * SRSGPU_CB_MSG_STRIDE), e.msgs[c].data(),
                  e.msgs[c].size());
      any_msgs = true;
    }
  }
  hipStream_t s = stream.get();
  d_io.upload(0, d_lay.iter_o, s);
  if (any_msgs) {
    d_msgs.upload(0, static_cast<size_t>(n_cb) * SRSGPU_CB_MSG_STRIDE, s);
  }
  srsgpu_check(srsgpu_ulsch_demux_plan_execute(dp->demux, d_llr, d_sch_b, d_uci_b, d_uci_b,
                                               d_io.dev<int8_t>(d_lay.csi2_o), s),
               WHO);
  srsgpu_check(srsgpu_pusch_decoder_plan_execute_arena(dp->dec, d_sch_b, d_io.dev<int8_t*>(d_lay.ptr_o),
                                                       d_io.dev<uint8_t>(d_lay.flag_o), d_msgs.dev<uint8_t>(),
                                                       d_io.dev<int32_t>(d_lay.iter_o), d_io.dev<uint8_t>(d_lay.tb_o),
                                                       d_io.dev<uint8_t>(d_lay.tbok_o), s),
               WHO);
  d_io.download(d_lay.flag_o, d_lay.end_o - d_lay.flag_o, s);
  d_msgs.download(0, static_cast<size_t>(n_cb) * SRSGPU_CB_MSG_STRIDE, s);
  hip_check(hipStreamSynchronize(s), WHO, "synchronise");
}

void pusch_launcher::wait(const std::vector<std::unique_ptr<pusch_job>>& jobs)
{
  hip_check(hipEventSynchronize(done), WHO, "synchronise");
  if (!downloaded) {
    return;
  }
  // Messages of the passed CBs of failed TBs are kept in the rx buffer for the retransmission.
  const launch_plan& lp        = *plan;
  bool               need_msgs = false;
  for (const auto& job : jobs) {
    for (const pusch_entry& e : job->entries) {
      if (e.tb_index >= 0 && *ioh<uint8_t>(lp.tbok_o + static_cast<unsigned>(e.tb_index)) == 0) {
        for (unsigned c = 0; c != e.nof_cbs && !need_msgs; ++c) {
          need_msgs = *ioh<uint8_t>(lp.flag_o + e.cb0 + c) != 0;
        }
      }
    }
  }
  if (need_msgs) {
    msgs.download(0, msgs_bytes(), stream.get());
    hip_check(hipStreamSynchronize(stream.get()), WHO, "synchronise");
  }
}

void pusch_launcher::replay(const std::vector<std::unique_ptr<pusch_job>>& jobs,
                            const uint8_t*                                 io_host,
                            const uint8_t*                                 msgs_host)
{
  for (const auto& job : jobs) {
    replay_job(*job, io_host, msgs_host);
  }
}

bool pusch_launcher::needs_second_phase(const pusch_job& job)
{
  for (const pusch_entry& e : job.entries) {
    if (e.csi2) {
      return true;
    }
  }
  return false;
}

void pusch_launcher::replay_job(pusch_job& job_ref, const uint8_t* io_host, const uint8_t* msgs_host)
{
  const launch_plan& lp  = *plan;
  pusch_job*         job = &job_ref;
  {
    replay_processor&                r    = job->batch->replay_for_this_thread();
    const pusch_batch_configuration& bcfg = job->batch->cfg;
    for (pusch_entry& e : job->entries) {
      const unsigned i         = e.tx;
      r.est->nv                = reinterpret_cast<const float*>(io_host + lp.nv_o + 4 * i * sizeof(float));
      r.est->m = reinterpret_cast<const float*>(io_host + lp.m_o + 4 * i * SRSGPU_CHEST_METRICS * sizeof(float));
      r.demod->stats = reinterpret_cast<const float*>(io_host + lp.st_o + i * SRSGPU_DEMOD_STATS * sizeof(float));
      r.demod->nof_rb          = e.nof_rb;
      r.demux->harq_ack_llrs   = reinterpret_cast<const int8_t*>(io_host + lp.uci_o + e.harq_ack_offset);
      r.demux->csi1_llrs       = reinterpret_cast<const int8_t*>(io_host + lp.uci_o + e.csi1_offset);
      r.demux->harq_ack_counts = e.demux_index >= 0 ? e.harq_ack_counts.data() : nullptr;
      r.demux->csi1_counts     = e.demux_index >= 0 ? e.csi1_counts.data() : nullptr;
      r.dec->cb_flags          = io_host + lp.flag_o + e.cb0;
      r.dec->cb_iters          = reinterpret_cast<const int32_t*>(io_host + lp.iter_o + e.cb0 * sizeof(int32_t));
      r.dec->tb                = io_host + lp.tb_o + e.tb_offset;
      r.dec->cb_msgs           = msgs_host + static_cast<size_t>(e.cb0) * SRSGPU_CB_MSG_STRIDE;
      r.dec->decoded           = decoded_flags.data() + e.cb0;
      r.dec->tb_ok             = e.tb_index >= 0 && io_host[lp.tbok_o + static_cast<unsigned>(e.tb_index)] != 0;
      r.dec->cb_KZ             = e.cb_KZ;
      r.dec->max_iter          = bcfg.nof_ldpc_iterations;
      if (e.csi2) {
        r.demux->second_phase = [this, &e, &r, job](unsigned bits, unsigned enc_bits, unsigned first,
                                                                const int8_t*& llrs, const uint32_t*& counts) {
          decode_deferred(e, *job->harq, bits, enc_bits, first);
          llrs            = d_io.host<int8_t>(d_lay.csi2_o);
          counts          = d_lay.csi2_counts.data();
          r.dec->cb_flags = d_io.host<uint8_t>(d_lay.flag_o);
          r.dec->cb_iters = d_io.host<int32_t>(d_lay.iter_o);
          r.dec->tb       = d_io.host<uint8_t>(d_lay.tb_o);
          r.dec->cb_msgs  = d_msgs.host<uint8_t>();
          r.dec->decoded  = d_decoded.data();
          r.dec->tb_ok    = *d_io.host<uint8_t>(d_lay.tbok_o) != 0;
        };
      } else {
        r.demux->second_phase = nullptr;
      }
      r.proc->process(e.data, std::move(e.rm), *e.notifier, *e.grid, e.pdu);
      r.demux->second_phase = nullptr;
    }
  }
}

/// Launches set.jobs on the set's launcher (the dispatcher thread).
void pusch_gpu_service::launch(launch_set& set)
{
  const unsigned P        = set.jobs.front()->P;
  const unsigned grid_prb = set.jobs.front()->grid_prb;
  uint32_t*      d_grids  = nullptr;
  {
    std::lock_guard<std::mutex> lock(grid_mtx);
    for (const grid_class& c : grid_classes) {
      if (c.P == P && c.prb == grid_prb) {
        d_grids = c.d_grids;
      }
    }
  }
  const pusch_launcher::stamps tm = set.L.launch(set.jobs, d_grids, true);
  set.t_launched                  = tm.launched;
  if (timing) {
    phase_us[0] += us_between(tm.start, tm.built);
    phase_us[1] += us_between(tm.built, tm.filled);
    phase_us[2] += us_between(tm.filled, tm.launched);
    plans_created += tm.plan_created ? 1 : 0;
    graphs_captured += tm.graph_captured ? 1 : 0;
    if (tm.plan_created || tm.graph_captured) {
      setup_us += us_between(tm.start, tm.launched);
    }
    ++launch_sizes[std::min<size_t>(set.jobs.size(), launch_sizes.size() - 1)];
  }
}

/// Waits for a launch and replays its PDUs through the reference's own processor, PDU by PDU (completion thread).
void pusch_gpu_service::finish(launch_set& set)
{
  set.L.wait(set.jobs);
  const auto t_gpu = clock_type::now();
  if (replayers.empty() || set.jobs.size() < 2) {
    set.L.replay(set.jobs, set.L.host_io(), set.L.host_msgs());
  } else {
    // The jobs without a second phase shared with the helpers, then the others on this thread.
    {
      std::lock_guard<std::mutex> lock(rp_mtx);
      rp_set = &set;
      rp_next.store(0);
      rp_busy = static_cast<unsigned>(replayers.size());
      ++rp_gen;
    }
    rp_cv.notify_all();
    replay_share(set);
    {
      std::unique_lock<std::mutex> lock(rp_mtx);
      rp_done_cv.wait(lock, [this] { return rp_busy == 0; });
      rp_set = nullptr;
    }
    for (const auto& job : set.jobs) {
      if (pusch_launcher::needs_second_phase(*job)) {
        set.L.replay_job(*job, set.L.host_io(), set.L.host_msgs());
      }
    }
  }
  const auto t_end = clock_type::now();
  if (timing) {
    phase_us[3] += us_between(set.t_launched, t_gpu);
    phase_us[4] += us_between(t_gpu, t_end);
    ++timed_launches;
    timed_slots += set.jobs.size();
  }
  for (const auto& job : set.jobs) {
    job->batch->job_done();
  }
}

std::shared_ptr<pusch_gpu_service> create_pusch_gpu_service(const pusch_service_configuration& config)
{
  return std::make_shared<pusch_gpu_service>(config);
}

// ---------------------------------------------------------------------------------------------------------------------
// PUSCH slot batch
// ---------------------------------------------------------------------------------------------------------------------

namespace {

std::shared_ptr<pusch_gpu_service> private_service(int device)
{
  pusch_service_configuration c;
  c.device          = device;
  c.nof_launch_sets = 2;
  c.max_grids       = 4;
  return std::make_shared<pusch_gpu_service>(c);
}

} // namespace

pusch_slot_batch::pusch_slot_batch(const pusch_batch_configuration&     cfg_,
                                   std::shared_ptr<pusch_harq_arena>    arena_,
                                   std::shared_ptr<uci_decoder_factory> uci_factory_,
                                   std::unique_ptr<pusch_processor>     fallback_,
                                   std::shared_ptr<pusch_gpu_service>   service_) :
  cfg(cfg_),
  arena(std::move(arena_)),
  service(service_ ? std::move(service_) : private_service(cfg_.device)),
  ctx(service->context()),
  uci_factory(std::move(uci_factory_)),
  fallback(std::move(fallback_)),
  grid_buf(WHO)
{
  if (!fallback || !uci_factory || !arena) {
    throw std::invalid_argument(std::string(WHO) + ": invalid dependencies");
  }
  if (srsgpu_context_device(arena->ctx.get()) != srsgpu_context_device(ctx)) {
    throw std::invalid_argument(std::string(WHO) + ": HARQ arena and service on different devices");
  }
  device_scope dev(ctx, WHO);
  batch_id = service->new_batch_id();
  if (!cfg.devices.empty()) {
    if (cfg.devices.front() != srsgpu_context_device(ctx)) {
      throw std::invalid_argument(std::string(WHO) + ": the root device (devices[0]) must hold the HARQ arena");
    }
    transport = cfg.transport ? cfg.transport : create_pusch_copy_transport();
    root_stream = std::make_unique<owned_stream>(ctx, WHO);
    for (size_t i = 0; i != cfg.devices.size(); ++i) {
      shard_device sh;
      sh.device = cfg.devices[i];
      sh.ctx    = shared_context(sh.device);
      // The root shard keeps the sector's arena; every other shard a device arena over the same codeblock ids.
      sh.arena    = i == 0 ? arena : create_pusch_harq_arena(sh.device, arena->max_cb_ids);
      device_scope sdev(sh.ctx.get(), WHO);
      sh.launcher = std::make_unique<pusch_launcher>(sh.ctx.get());
      sh.upload   = std::make_unique<owned_stream>(sh.ctx.get(), WHO);
      hip_check(hipEventCreateWithFlags(&sh.uploaded, hipEventDisableTiming), WHO, "event");
      if (sh.device != cfg.devices.front()) {
        // The shard's grid rows are copied from the root's grid by a kernel on the shard (peer reads over xGMI).
        const hipError_t pe = hipDeviceEnablePeerAccess(cfg.devices.front(), 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) {
          throw std::runtime_error(std::string(WHO) + ": no peer access from device " + std::to_string(sh.device) +
                                   " to the root device");
        }
        (void)hipGetLastError();
      }
      shards.push_back(std::move(sh));
    }
    hip_check(hipEventCreateWithFlags(&root_done, hipEventDisableTiming), WHO, "event");
    multi_completion = std::thread([this]() { multi_complete_loop(); });
  }
}

pusch_slot_batch::~pusch_slot_batch()
{
  release_host_grid();  // waits for every slot in flight
  if (multi_completion.joinable()) {
    {
      std::lock_guard<std::mutex> lock(multi_mtx);
      multi_stop = true;
    }
    multi_cv.notify_all();
    multi_completion.join();
    (void)hipEventDestroy(root_done);
  }
  if (grid_slot >= 0) {
    service->release_grid(grid_P, grid_prb, static_cast<unsigned>(grid_slot));
  }
  for (shard_device& sh : shards) {
    device_scope sdev(sh.ctx.get(), WHO);
    (void)hipStreamSynchronize(sh.upload->get());
    (void)hipEventDestroy(sh.uploaded);
    (void)hipFree(sh.d_grid);
  }
}

void pusch_slot_batch::release_host_grid()
{
  {
    std::unique_lock<std::mutex> lock(done_mtx);
    done_cv.wait(lock, [&] { return outstanding == 0; });
  }
  std::lock_guard<std::mutex> lock(run_mtx);
  if (host_grid != nullptr) {
    device_scope dev(ctx, WHO);
    host_blocks::remove_twin(host_grid);
    host_blocks::remove(host_grid);
    host_grid      = nullptr;
    host_grid_dev  = nullptr;
    twin_announced = false;
  }
}

const void* pusch_slot_batch::grid_in_place(const resource_grid_reader& grid, unsigned P, size_t row)
{
  if (host_grid_off) {
    return nullptr;
  }
  const auto* base = reinterpret_cast<const uint8_t*>(grid.get_view(0, 0).data());
  for (unsigned p = 0; p != P; ++p) {
    for (unsigned l = 0; l != 14; ++l) {
      if (reinterpret_cast<const uint8_t*>(grid.get_view(p, l).data()) != base + (p * 14 + l) * row) {
        return nullptr;
      }
    }
  }
  const size_t bytes = static_cast<size_t>(P) * 14 * row;
  if (host_grid == nullptr || host_grid != base || host_grid_size < bytes) {
    if (host_grid == nullptr) {
      if (void* d = host_blocks::find(base, bytes)) {
        return d;  // mapped by another component (which unmaps it)
      }
    }
    device_scope dev(ctx, WHO);
    if (host_grid != nullptr) {
      host_blocks::remove_twin(host_grid);
      host_blocks::remove(host_grid);
      host_grid      = nullptr;
      host_grid_dev  = nullptr;
      twin_announced = false;
    }
    const void* d = host_blocks::add(base, bytes);
    if (d == nullptr) {
      host_grid_off = true;
      return nullptr;
    }
    host_grid      = base;
    host_grid_size = bytes;
    host_grid_dev  = d;
  }
  return host_grid_dev;
}

replay_processor& pusch_slot_batch::replay_for_this_thread()
{
  std::lock_guard<std::mutex> lock(replays_mtx);
  auto                        it = replays.find(std::this_thread::get_id());
  if (it != replays.end()) {
    return it->second;
  }
  replay_processor r;
  auto             est   = std::make_unique<replay_estimator>();
  auto             demod = std::make_unique<replay_demodulator>();
  auto             demux = std::make_unique<replay_demux>();
  auto             dec   = std::make_unique<replay_decoder>();
  r.est                  = est.get();
  r.demod                = demod.get();
  r.demux                = demux.get();
  r.dec                  = dec.get();
  demod->opts            = cfg.demodulator;
  demod->demux           = demux.get();
  std::vector<std::unique_ptr<pusch_processor_impl::concurrent_dependencies>> deps;
  deps.push_back(std::make_unique<pusch_processor_impl::concurrent_dependencies>(
      std::move(est),
      std::move(demod),
      std::move(demux),
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

void pusch_slot_batch::job_done()
{
  {
    std::lock_guard<std::mutex> lock(done_mtx);
    --outstanding;
  }
  done_cv.notify_all();
}

void pusch_slot_batch::build_layout(pusch_job& job, const pusch_harq_arena& harq) const
{
  job_layout&    L        = job.lay;
  const unsigned grid_prb = job.grid_prb;
  const unsigned P        = job.P;
  const size_t   row      = static_cast<size_t>(grid_prb) * NRE * sizeof(uint32_t);
  // Estimates in the compact layout with the "average" time strategy (one row per allocation and rx port, the CFO
  // rotation of each symbol applied by the demodulator; the LLRs equal the per-symbol layout's bit for bit,
  // tests/test_pusch_chest_gpu.py): the estimator writes 1 / 14 of the words. "interpolate" needs every symbol.
  L.layout = cfg.estimator.td_strategy == SRSGPU_CHEST_TD_AVERAGE ? SRSGPU_CE_COMPACT : SRSGPU_CE_PER_SYMBOL;
  job.harq = &harq;
  key_append(L.key, L.layout);
  key_append(L.key, job.grid_slot);
  key_append(L.key, harq.d_soft);
  unsigned uci_total = 0;
  for (pusch_entry& e : job.entries) {
    const pusch_processor::pdu_t& pdu     = e.pdu;
    const crb_bitmap              rb_mask = pdu.freq_alloc.get_crb_mask(pdu.bwp_start_rb, pdu.bwp_size_rb);
    e.tx                                  = L.n++;
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
    L.chests.push_back(make_pusch_chest_desc(est, grid_prb, cfg.estimator, L.layout, WHO));
    L.chests.back().c.grid_index = job.grid_slot;
    L.chests.back().append_key(L.key);

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
    L.demods.push_back(make_pusch_demod_desc(dem, grid_prb, cfg.demodulator, L.layout, WHO));
    pusch_demod_desc& dd = L.demods.back();
    dd.c.grid_index      = job.grid_slot;
    dd.c.cfo_compensated = (L.layout == SRSGPU_CE_COMPACT && cfg.estimator.compensate_cfo) ? 1 : 0;
    dd.c.numerology      = static_cast<uint8_t>(pdu.slot.numerology());  // the symbol epochs of the rotation

    // Codeword LLRs: nof_rb REs per data symbol (minus the DM-RS REs) x layers x Qm.
    const unsigned dmrs_re = cdm_groups * (dmrs == dmrs_type::TYPE1 ? 6 : 4);
    unsigned       nre     = 0;
    for (unsigned l = pdu.start_symbol_index; l != pdu.start_symbol_index + pdu.nof_symbols; ++l) {
      nre += e.nof_rb * (pdu.dmrs_symbol_mask.test(l) ? NRE - dmrs_re : NRE);
    }
    e.nof_llrs      = nre * pdu.nof_tx_layers * dd.qm;
    e.llr_offset    = L.llr_total;
    dd.c.llr_offset = L.llr_total;
    L.llr_total += (e.nof_llrs + 63) / 64 * 64;
    dd.append_key(L.key);

    // pusch_processor_impl.cpp:222-240: the DC subcarrier's estimate is zeroed for CP-OFDM transmissions over it.
    const int dc = pdu.dc_position.has_value() ? static_cast<int>(*pdu.dc_position) : -1;
    key_append(L.key, dc);
    if (dc >= 0 && !tp && static_cast<unsigned>(dc) < grid_prb * NRE) {
      for (unsigned ly = 0; ly != pdu.nof_tx_layers; ++ly) {
        for (unsigned p = 0; p != pdu.rx_ports.size(); ++p) {
          const size_t off = (((static_cast<size_t>(job.grid_slot) * 4 + ly) * P + p) * 14 + pdu.start_symbol_index) *
                                 row +
                             static_cast<size_t>(dc) * sizeof(uint32_t);
          // Compact layout: the one row every symbol reads.
          L.dc_zero_local.push_back({off, L.layout == SRSGPU_CE_COMPACT ? 1u : static_cast<unsigned>(pdu.nof_symbols)});
        }
      }
    }

    // UCI on PUSCH (pusch_processor_impl.cpp:180-202, 244-262): the UL-SCH stream feeds the decoder; the HARQ-ACK and
    // CSI Part 1 streams come back for the replay.
    unsigned nof_sch_llrs = e.nof_llrs;
    e.sch_offset          = e.llr_offset;
    e.demux_index         = -1;
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
      d.harq_offset                 = uci_total;
      e.harq_ack_offset             = uci_total;
      uci_total += (d.nof_enc_harq_ack_bits + 63) / 64 * 64;
      d.csi1_offset = uci_total;
      e.csi1_offset = uci_total;
      uci_total += (d.nof_enc_csi_part1_bits + 63) / 64 * 64;
      L.demuxes.push_back(d);  // sch_offset set once the codeword region's size is known
      e.demux_index = static_cast<int>(L.demuxes.size()) - 1;
      nof_sch_llrs  = info.nof_ul_sch_bits.value();
      e.csi2        = !pdu.uci.csi_part2_size.entries.empty();
      e.ulsch_cfg   = uc;
      e.demux_cfg   = d;
    }
    e.nof_sch_llrs = nof_sch_llrs;

    // TB decoding (pusch_processor_impl.cpp:278-296) and the HARQ context from the rx buffer: CB CRC flags and the
    // messages of CBs that already passed (a new transmission's flags are reset, pusch_decoder_impl.cpp:133-136).
    const units::bits tb_bits = units::bytes(e.data.size()).to_bits();
    const auto        bg      = pdu.codeword->ldpc_base_graph;
    e.nof_cbs                 = ldpc::compute_nof_codeblocks(tb_bits, bg);
    ldpc_lengths(tb_bits, bg, e.cb_N, e.cb_KZ);
    e.cb0       = L.cb_total;
    e.tb_offset = L.tb_total;
    e.harq0     = L.harq_total;
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
    span<const bool> crcs = e.rm->get_codeblocks_crc();
    if (e.csi2) {
      // Decoded by the second launch (pusch_launcher::decode_deferred): its own buffers, offsets from 0.
      e.tb_index = -1;
      e.tb_cfg   = t;
      for (unsigned c = 0; c != e.nof_cbs; ++c) {
        const unsigned id = e.rm->get_absolute_codeblock_id(c);
        if (id >= harq.max_cb_ids) {
          throw std::out_of_range(std::string(WHO) + ": absolute codeblock id " + std::to_string(id) +
                                  " beyond the HARQ arena");
        }
        e.copies.push_back({id, c * e.cb_N, e.cb_N, 0});
        const bool ok = !e.new_data && crcs[c];
        e.flags.push_back(ok ? 1 : 0);
        std::vector<uint8_t> msg;
        if (ok) {
          const bit_buffer bits = e.rm->get_codeblock_data_bits(c, e.cb_KZ);
          msg.resize((e.cb_KZ + 7) / 8);
          for (unsigned b = 0; b != msg.size(); ++b) {
            msg[b] = bits.get_byte(b);
          }
        }
        e.msgs.push_back(std::move(msg));
      }
      continue;
    }
    t.llr_offset = e.llr_offset;
    t.harq_offset = e.harq0;
    t.cb_offset   = e.cb0;
    t.tb_offset   = e.tb_offset;
    e.tb_index    = static_cast<int>(L.tbs.size());
    L.tbs.push_back(t);
    for (unsigned c = 0; c != e.nof_cbs; ++c) {
      const unsigned id = e.rm->get_absolute_codeblock_id(c);
      if (id >= harq.max_cb_ids) {
        throw std::out_of_range(std::string(WHO) + ": absolute codeblock id " + std::to_string(id) +
                                " beyond the HARQ arena");
      }
      L.copies.push_back({id, e.harq0 + c * e.cb_N, e.cb_N, 0});
      const bool ok = !e.new_data && crcs[c];
      L.flags.push_back(ok ? 1 : 0);
      if (ok) {
        const bit_buffer     bits = e.rm->get_codeblock_data_bits(c, e.cb_KZ);
        std::vector<uint8_t> msg((e.cb_KZ + 7) / 8);
        for (unsigned b = 0; b != msg.size(); ++b) {
          msg[b] = bits.get_byte(b);
        }
        L.msgs.push_back({e.cb0 + c, std::move(msg)});
      }
    }
    L.cb_total += e.nof_cbs;
    L.tb_total += (static_cast<unsigned>(e.data.size()) + 15) / 16 * 16;
    L.harq_total += e.nof_cbs * e.cb_N;
  }
  // UL-SCH streams of the UCI transmissions after the codewords in the LLR buffer.
  for (pusch_entry& e : job.entries) {
    if (e.demux_index >= 0) {
      L.demuxes[static_cast<size_t>(e.demux_index)].sch_offset = L.llr_total;
      e.sch_offset                                              = L.llr_total;
      if (e.tb_index >= 0) {
        L.tbs[static_cast<size_t>(e.tb_index)].llr_offset = L.llr_total;
      }
      L.llr_total += (e.nof_sch_llrs + 63) / 64 * 64;
    }
  }
  L.uci_total = uci_total;
  for (const srsgpu_pusch_tb_config& t : L.tbs) {
    key_append(L.key, t);
  }
  for (const pusch_entry& e : job.entries) {
    key_append(L.key, e.tb_index);
  }
  for (const srsgpu_ulsch_demux_config& d : L.demuxes) {
    key_append(L.key, d);
  }
}

void pusch_slot_batch::run(std::vector<pusch_entry>& all)
{
  std::lock_guard<std::mutex> lock(run_mtx);
  device_scope                dev(ctx, WHO);

  // PDUs outside the batch's scope go through the fallback processor, one by one, as the reference would.
  auto job = std::make_unique<pusch_job>();
  for (pusch_entry& e : all) {
    if (batchable(e)) {
      job->entries.push_back(std::move(e));
    } else {
      fallback->process(e.data, std::move(e.rm), *e.notifier, *e.grid, e.pdu);
    }
  }
  if (job->entries.empty()) {
    return;
  }
  const resource_grid_reader& grid = *job->entries.front().grid;
  const unsigned              nsc  = grid.get_nof_subc();
  unsigned                    P    = 0;
  for (const pusch_entry& e : job->entries) {
    P = std::max<unsigned>(P, e.pdu.rx_ports.size());
  }
  // The grid buffers are reused slot after slot: the previous slot of this batch must be done with them (an uplink
  // processor hands its next slot out only then; a second PUSCH task within one slot waits here).
  {
    std::unique_lock<std::mutex> done_lock(done_mtx);
    done_cv.wait(done_lock, [&] { return outstanding == 0; });
  }
  if (!shards.empty()) {
    job->P        = P;
    job->grid_prb = nsc / NRE;
    run_multi(std::move(job));
    return;
  }
  if (grid_slot < 0 || grid_P != P || grid_prb != nsc / NRE) {
    if (grid_slot >= 0) {
      throw std::invalid_argument(std::string(WHO) + ": the resource grid shape of a batch changed");
    }
    const auto g = service->register_grid(P, nsc / NRE);
    grid_slot    = static_cast<int>(g.first);
    d_grid       = g.second;
    grid_P       = P;
    grid_prb     = nsc / NRE;
  }
  const size_t row    = static_cast<size_t>(nsc) * sizeof(uint32_t);
  const size_t gbytes = static_cast<size_t>(P) * 14 * row;
  // The rx grid (every symbol of ports 0..P-1, [port][symbol][subcarrier]) into mapped host memory; the launch copies
  // it into the batch's HBM grid slot (srsgpu_copy_spans, with the other slots' grids: zero-copy reads instead of a DMA
  // copy per slot, which ran the service at the DMA engines' ~29 GB/s, profiles/r5_grid_span_copy_ab.txt).
  // The uplink processor's grid read in place when its storage is one block; otherwise a copy.
  const void* grid_src = grid_in_place(grid, P, row);
  if (grid_src == nullptr) {
    grid_map.reserve(gbytes);
    for (unsigned p = 0; p != P; ++p) {
      for (unsigned l = 0; l != 14; ++l) {
        std::memcpy(grid_map.host((p * 14 + l) * row), grid.get_view(p, l).data(), row);
      }
    }
    grid_src = grid_map.dev();
  } else if (host_grid != nullptr && grid_src == host_grid_dev) {
    // du_low with the lower PHY on this GPU: the sector group demodulates every symbol into the grid and into its
    // HBM twin (this batch's grid slot); when it did for all 14 symbols of this slot, the slot copies nothing.
    if (!twin_announced) {
      host_blocks::set_twin(host_grid, {reinterpret_cast<uint8_t*>(d_grid), gbytes, &twin_symbols});
      twin_announced = true;
    }
    if (twin_symbols.exchange(0, std::memory_order_acq_rel) == (1u << 14) - 1u) {
      grid_src = nullptr;
      multi_transfers.twin_grids.fetch_add(1, std::memory_order_relaxed);
    }
  }

  job->batch     = this;
  job->batch_id  = batch_id;
  job->slot_key      = job->entries.front().pdu.slot.system_slot();
  job->slot_in_frame = job->entries.front().pdu.slot.slot_index();
  job->grid_slot = static_cast<unsigned>(grid_slot);
  job->P         = P;
  job->grid_prb  = grid_prb;
  job->uploaded   = nullptr;
  job->grid_src   = grid_src;
  job->grid_dst   = d_grid;
  job->grid_bytes = gbytes;
  build_layout(*job, *arena);
  {
    std::lock_guard<std::mutex> done_lock(done_mtx);
    ++outstanding;
  }
  service->submit(std::move(job));
  if (!cfg.asynchronous) {
    std::unique_lock<std::mutex> done_lock(done_mtx);
    done_cv.wait(done_lock, [&] { return outstanding == 0; });
  }
}

/// Multi-GPU slot (row b7): the UEs sharded over cfg.devices by RNTI, each shard's estimator, demodulator,
/// demultiplexer and decoder on its device (its own rx grid copy, HARQ arena and cached launch plans, results left in
/// HBM), the shards' result regions gathered to the root device by the transport, one download there and the replay
/// into the reference's processor on this thread - the slot's decoded TBs reach the notifier (the FAPI side,
/// phy_to_fapi_results_event_translator.cpp:145 through uplink_processor_impl.cpp:408) from the root.
void pusch_slot_batch::run_multi(std::unique_ptr<pusch_job> job)
{
  const unsigned D        = static_cast<unsigned>(shards.size());
  const unsigned P        = job->P;
  const unsigned grid_prb = job->grid_prb;
  const size_t   row      = static_cast<size_t>(grid_prb) * NRE * sizeof(uint32_t);
  const size_t   gbytes   = static_cast<size_t>(P) * 14 * row;
  const resource_grid_reader& grid = *job->entries.front().grid;
  // UE shards: RNTI mod D (a UE's HARQ soft bits stay on the device that decodes it); each shard's subcarrier bands
  // (its UEs' allocations, merged).
  std::vector<std::vector<std::unique_ptr<pusch_job>>> shard_jobs(D);
  std::vector<std::vector<std::pair<unsigned, unsigned>>> bands(D);
  for (pusch_entry& e : job->entries) {
    const unsigned s = static_cast<unsigned>(e.pdu.rnti) % D;
    if (shard_jobs[s].empty()) {
      auto sj         = std::make_unique<pusch_job>();
      sj->batch       = this;
      sj->batch_id    = batch_id;
      sj->slot_key    = job->slot_key;
      sj->grid_slot   = 0;
      sj->P           = P;
      sj->grid_prb    = grid_prb;
      sj->uploaded    = shards[s].uploaded;
      shard_jobs[s].push_back(std::move(sj));
    }
    const crb_bitmap mask = e.pdu.freq_alloc.get_crb_mask(e.pdu.bwp_start_rb, e.pdu.bwp_size_rb);
    if (mask.any()) {
      bands[s].emplace_back(static_cast<unsigned>(mask.find_lowest()) * NRE,
                            (static_cast<unsigned>(mask.find_highest()) + 1) * NRE);
    }
    shard_jobs[s].front()->entries.push_back(std::move(e));
  }
  for (auto& b : bands) {
    std::sort(b.begin(), b.end());
    std::vector<std::pair<unsigned, unsigned>> merged;
    for (const auto& r : b) {
      if (!merged.empty() && r.first <= merged.back().second) {
        merged.back().second = std::max(merged.back().second, r.second);
      } else {
        merged.push_back(r);
      }
    }
    b = std::move(merged);
  }
  {
    std::lock_guard<std::mutex> lock(done_mtx);
    ++outstanding;
  }
  // The grid goes to the root device once (its in-place mapped image or the batch's copy, read by a copy kernel);
  // every other shard receives only its bands' subcarriers of every port and symbol from the root's HBM copy.
  const void* src = grid_in_place(grid, P, row);
  if (src == nullptr) {
    grid_map.reserve(gbytes);
    for (unsigned p = 0; p != P; ++p) {
      for (unsigned l = 0; l != 14; ++l) {
        std::memcpy(grid_map.host((p * 14 + l) * row), grid.get_view(p, l).data(), row);
      }
    }
    src = grid_map.dev();
  }
  size_t nspans = 1;
  for (unsigned s = 1; s != D; ++s) {
    nspans += shard_jobs[s].empty() ? 0 : bands[s].size() * P * 14;
  }
  shard_spans.reserve(nspans * sizeof(srsgpu_copy_span));
  auto* spans = shard_spans.host<srsgpu_copy_span>();
  for (unsigned s = 0; s != D; ++s) {
    shard_device& sh = shards[s];
    device_scope  sdev(sh.ctx.get(), WHO);
    if (sh.grid_cap < gbytes) {
      std::lock_guard<std::recursive_mutex> setup(hip_setup_mutex());
      (void)hipFree(sh.d_grid);
      sh.d_grid   = nullptr;
      sh.grid_cap = 0;
      hip_check(hipMalloc(reinterpret_cast<void**>(&sh.d_grid), gbytes), WHO, "shard grid");
      sh.grid_cap = gbytes;
    }
  }
  {
    shard_device& root = shards[0];
    device_scope  rdev(root.ctx.get(), WHO);
    spans[0] = {src, root.d_grid, gbytes};
    srsgpu_check(srsgpu_copy_spans(shard_spans.dev<srsgpu_copy_span>(), 1, gbytes, root.upload->get()), WHO);
    hip_check(hipEventRecord(root.uploaded, root.upload->get()), WHO, "event");
    multi_transfers.host_uploads.fetch_add(1, std::memory_order_relaxed);
  }
  size_t next = 1;
  for (unsigned s = 1; s != D; ++s) {
    if (shard_jobs[s].empty()) {
      continue;
    }
    shard_device& sh = shards[s];
    device_scope  sdev(sh.ctx.get(), WHO);
    const size_t  first = next;
    uint64_t      most  = 0;
    for (const auto& b : bands[s]) {
      const size_t off = static_cast<size_t>(b.first) * sizeof(uint32_t);
      const size_t len = static_cast<size_t>(b.second - b.first) * sizeof(uint32_t);
      for (unsigned r = 0; r != P * 14; ++r) {
        spans[next++] = {reinterpret_cast<const uint8_t*>(shards[0].d_grid) + r * row + off,
                         reinterpret_cast<uint8_t*>(sh.d_grid) + r * row + off, len};
        multi_transfers.shard_bytes.fetch_add(len, std::memory_order_relaxed);
      }
      most = std::max<uint64_t>(most, len);
    }
    hip_check(hipStreamWaitEvent(sh.upload->get(), shards[0].uploaded, 0), WHO, "wait for the root grid");
    if (next > first) {
      srsgpu_check(srsgpu_copy_spans(shard_spans.dev<srsgpu_copy_span>(first * sizeof(srsgpu_copy_span)),
                                     static_cast<uint32_t>(next - first), most, sh.upload->get()),
                   WHO);
      multi_transfers.shard_copies.fetch_add(1, std::memory_order_relaxed);
    }
    hip_check(hipEventRecord(sh.uploaded, sh.upload->get()), WHO, "event");
  }
  // Each shard's layout and launch (results stay in its HBM), then the gather to the root and one download.
  std::vector<pusch_result_transport::part> parts;
  std::vector<std::pair<size_t, size_t>>    offsets(D);  // (results, messages) in the gathered image
  size_t                                    total = 0;
  auto                                      align = [](size_t x) { return (x + 255) / 256 * 256; };
  for (unsigned s = 0; s != D; ++s) {
    if (shard_jobs[s].empty()) {
      continue;
    }
    shard_device& sh = shards[s];
    device_scope  sdev(sh.ctx.get(), WHO);
    build_layout(*shard_jobs[s].front(), *sh.arena);
    sh.launcher->launch(shard_jobs[s], sh.d_grid, false);
    offsets[s] = {total, align(total + sh.launcher->results_bytes())};
    parts.push_back({s, sh.device, sh.launcher->device_results(), sh.launcher->results_bytes(),
                     sh.launcher->get_stream(), offsets[s].first});
    parts.push_back({s, sh.device, sh.launcher->device_msgs(), sh.launcher->msgs_bytes(), sh.launcher->get_stream(),
                     offsets[s].second});
    total = align(offsets[s].second + sh.launcher->msgs_bytes());
  }
  device_scope root(ctx, WHO);
  gathered.reserve(std::max<size_t>(total, 256));
  transport->gather(cfg.devices.front(), root_stream->get(), gathered.dev(), parts);
  gathered.download(0, total, root_stream->get());
  hip_check(hipEventRecord(root_done, root_stream->get()), WHO, "event");
  // The replay (notifications) on the completion thread once the download has landed; a synchronous batch waits.
  {
    std::lock_guard<std::mutex> lock(multi_mtx);
    multi_jobs    = std::move(shard_jobs);
    multi_offsets = std::move(offsets);
    multi_pending = true;
  }
  multi_cv.notify_all();
  if (!cfg.asynchronous) {
    std::unique_lock<std::mutex> done_lock(done_mtx);
    done_cv.wait(done_lock, [&] { return outstanding == 0; });
  }
}

void pusch_slot_batch::multi_complete_loop()
{
  for (;;) {
    std::vector<std::vector<std::unique_ptr<pusch_job>>> jobs;
    std::vector<std::pair<size_t, size_t>>               offsets;
    {
      std::unique_lock<std::mutex> lock(multi_mtx);
      multi_cv.wait(lock, [&] { return multi_pending || multi_stop; });
      if (!multi_pending) {
        return;
      }
      jobs          = std::move(multi_jobs);
      offsets       = std::move(multi_offsets);
      multi_pending = false;
    }
    device_scope root(ctx, WHO);
    try {
      hip_check(hipEventSynchronize(root_done), WHO, "synchronise");
      for (size_t s = 0; s != jobs.size(); ++s) {
        if (jobs[s].empty()) {
          continue;
        }
        pusch_launcher&    L  = *shards[s].launcher;
        const launch_plan& lp = L.current();
        L.replay(jobs[s], gathered.host<uint8_t>(offsets[s].first) - lp.flag_o,
                 gathered.host<uint8_t>(offsets[s].second));
      }
    } catch (const std::exception& e) {
      report_fatal_error("pusch_slot_batch: {}", e.what());
    }
    {
      std::lock_guard<std::mutex> lock(done_mtx);
      --outstanding;
    }
    done_cv.notify_all();
  }
}

pusch_multi_transfer_counters get_pusch_multi_transfer_counters()
{
  return {multi_transfers.host_uploads.load(), multi_transfers.shard_copies.load(),
          multi_transfers.shard_bytes.load(), multi_transfers.twin_grids.load()};
}

namespace {

class pusch_copy_transport : public pusch_result_transport
{
public:
  ~pusch_copy_transport() override
  {
    for (auto& e : events) {
      (void)hipEventDestroy(e.second);
    }
  }
  void gather(int root_device, void* root_stream, void* dst, const std::vector<part>& parts) override
  {
    auto* rs = static_cast<hipStream_t>(root_stream);
    for (const part& p : parts) {
      if (p.bytes == 0) {
        continue;
      }
      hip_check(hipSetDevice(p.device), "pusch_copy_transport", "device");
      hipEvent_t& ev = events[p.stream];
      if (ev == nullptr) {
        hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "pusch_copy_transport", "event");
      }
      hip_check(hipEventRecord(ev, static_cast<hipStream_t>(p.stream)), "pusch_copy_transport", "event");
      hip_check(hipSetDevice(root_device), "pusch_copy_transport", "device");
      hip_check(hipStreamWaitEvent(rs, ev, 0), "pusch_copy_transport", "wait");
      hip_check(hipMemcpyPeerAsync(static_cast<uint8_t*>(dst) + p.dst_offset, root_device, p.src, p.device, p.bytes, rs),
                "pusch_copy_transport", "peer copy");
    }
  }

private:
  std::map<void*, hipEvent_t> events;
};

class pusch_rccl_transport : public pusch_result_transport
{
public:
  explicit pusch_rccl_transport(const std::vector<int>& devices_) : devices(devices_)
  {
    if (devices.empty() || std::set<int>(devices.begin(), devices.end()).size() != devices.size()) {
      throw std::invalid_argument("pusch_rccl_transport: one communicator per distinct device");
    }
    comms.resize(devices.size());
    std::lock_guard<std::recursive_mutex> setup(hip_setup_mutex());
    rccl_check(ncclCommInitAll(comms.data(), static_cast<int>(devices.size()), devices.data()), "ncclCommInitAll");
  }
  ~pusch_rccl_transport() override
  {
    for (ncclComm_t c : comms) {
      (void)ncclCommDestroy(c);
    }
  }
  void gather(int root_device, void* root_stream, void* dst, const std::vector<part>& parts) override
  {
    if (root_device != devices.front()) {
      throw std::invalid_argument("pusch_rccl_transport: the root is rank 0");
    }
    rccl_check(ncclGroupStart(), "ncclGroupStart");
    for (const part& p : parts) {
      if (p.bytes == 0) {
        continue;
      }
      rccl_check(ncclSend(p.src, p.bytes, ncclUint8, 0, comms[p.rank], static_cast<hipStream_t>(p.stream)),
                 "ncclSend");
      rccl_check(ncclRecv(static_cast<uint8_t*>(dst) + p.dst_offset, p.bytes, ncclUint8, static_cast<int>(p.rank),
                          comms[0], static_cast<hipStream_t>(root_stream)),
                 "ncclRecv");
    }
    rccl_check(ncclGroupEnd(), "ncclGroupEnd");
  }

private:
  static void rccl_check(ncclResult_t r, const char* what)
  {
    if (r != ncclSuccess) {
      throw std::runtime_error(std::string("pusch_rccl_transport: ") + what + ": " + ncclGetErrorString(r));
    }
  }
  std::vector<int>        devices;
  std::vector<ncclComm_t> comms;
};

} // namespace

std::shared_ptr<pusch_result_transport> create_pusch_copy_transport()
{
  return std::make_shared<pusch_copy_transport>();
}

std::shared_ptr<pusch_result_transport> create_pusch_rccl_transport(const std::vector<int>& devices)
{
  return std::make_shared<pusch_rccl_transport>(devices);
}

std::shared_ptr<pusch_slot_batch> create_pusch_slot_batch(const pusch_batch_configuration& config,
                                                          std::shared_ptr<pusch_harq_arena> arena,
                                                          std::shared_ptr<ulsch_demultiplex_factory> /*demux*/,
                                                          std::shared_ptr<uci_decoder_factory> uci,
                                                          std::unique_ptr<pusch_processor>     fallback,
                                                          std::shared_ptr<pusch_gpu_service>   service)
{
  return std::make_shared<pusch_slot_batch>(config, std::move(arena), std::move(uci), std::move(fallback),
                                            std::move(service));
}

// ---------------------------------------------------------------------------------------------------------------------
// The reference-facing wrappers
// ---------------------------------------------------------------------------------------------------------------------

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
  uplink_processor_batch_gpu(std::unique_ptr<uplink_processor>  inner_,
                             std::shared_ptr<pusch_slot_batch> batch_,
                             task_executor&                    executor_) :
    inner(std::move(inner_)), batch(std::move(batch_)), executor(executor_)
  {
    for (slot_processor& s : slots) {
      s.owner = this;
    }
  }

  // The inner processor owns the grid the batch reads in place: unmapped before it goes.
  ~uplink_processor_batch_gpu() override { batch->release_host_grid(); }

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

  std::unique_ptr<uplink_processor> inner;
  std::shared_ptr<pusch_slot_batch> batch;
  task_executor&                    executor;
  std::array<slot_processor, 16>    slots;
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

} // namespace gpu
} // namespace srsran
