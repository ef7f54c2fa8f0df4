// Slot-batched GPU processing behind the reference's upper-PHY slot processors (the declarations a srsRAN maintainer
// adds next to lib/phy/upper/upper_phy_factories.cpp).
//
// The reference's processors hand their channel processors one PDU at a time: uplink_processor_impl::process_pusch
// (uplink_processor_impl.cpp:191-247) runs pusch_processor::process per PDU on the PUSCH executor, and
// downlink_processor_single_executor_impl::process_pdsch (downlink_processor_single_executor_impl.cpp:96-135) runs
// pdsch_processor::process per PDU on its executor; the slot boundary is visible only to the processor
// (handle_rx_symbol after the last symbol of a PDU, finish_processing_pdus). On a GPU one PDU is far too small a
// launch and each would pay its own PCIe round trip, so the reference's processors stay in charge of their state
// machines, PDU repositories and notifications, and only the PUSCH / PDSCH work is gathered into one launch sequence
// per slot:
//
//  * UL: the reference's uplink_processor_impl is built with a pusch_processor that registers each PDU in a slot batch
//    (create_pusch_processor_batch_gpu) and an executor that runs the PUSCH task on the caller (pusch_inline_executor),
//    and is wrapped by create_uplink_processor_batch_gpu, whose handle_rx_symbol runs the reference's and then hands the
//    PDUs it registered to the PUSCH executor as one job: one upload of the grid, channel estimation, demodulation and
//    decoding of every PDU (HARQ soft bits kept in HBM across slots, one arena slot per absolute codeblock identifier of
//    the reference's rx buffer pool), one download. The results then go through the reference's own
//    pusch_processor_impl per PDU, fed the GPU results (channel-estimate metrics, LLRs + scrambling sequence +
//    post-equalisation statistics, decoded TB), so the CSI report, the UCI demultiplexing / decoding, the notifier
//    order and the rx buffer bookkeeping are the reference's. PDUs the batch does not cover (UCI only, non-identity
//    rx port lists, more than four layers or rx ports, extended CP) go to a caller-supplied pusch_processor.
//
//  * DL: the reference's downlink_processor_single_executor_impl is built with a pdsch_processor that runs the
//    reference's pdsch_processor_impl over recording encoder / modulator / DM-RS stages (create_pdsch_processor_batch_gpu)
//    and with pdsch_batch_executor, which runs the PDSCH task on the caller while create_downlink_processor_batch_gpu's
//    process_pdsch is inside it; at finish_processing_pdus the wrapper runs the slot's PDSCHs as one launch sequence
//    (TB CRC + LDPC encoding + rate matching, DM-RS, scrambling + modulation + layer mapping + precoding into one grid)
//    on the real executor, writes exactly the REs they map into the slot's grid and reports each PDSCH finished, after
//    which the reference's state machine sends the grid.
#pragma once

#include "signal_chain_gpu.h"
#include "srsran/phy/upper/channel_processors/pdsch/pdsch_processor.h"
#include "srsran/phy/upper/channel_processors/pusch/factories.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_processor.h"
#include "srsran/phy/upper/channel_processors/uci/factories.h"
#include "srsran/phy/upper/channel_state_information.h"
#include "srsran/phy/upper/downlink_processor.h"
#include "srsran/phy/upper/signal_processors/ptrs/ptrs_pdsch_generator.h"
#include "srsran/phy/upper/uplink_processor.h"
#include "srsran/phy/upper/upper_phy_factories.h"
#include "srsran/phy/upper/channel_processors/pdcch/factories.h"
#include "srsran/phy/upper/channel_processors/pucch/factories.h"
#include "srsran/phy/upper/channel_processors/ssb/factories.h"
#include "srsran/phy/upper/signal_processors/prs/factories.h"
#include "srsran/phy/upper/signal_processors/ptrs/ptrs_pdsch_generator_factory.h"
#include "srsran/phy/upper/signal_processors/signal_processor_factories.h"
#include "srsran/phy/upper/signal_processors/srs/srs_estimator_factory.h"
#include "srsran/support/executors/task_executor.h"

#include <memory>

namespace srsran {
namespace gpu {

class pusch_result_transport;

/// PUSCH slot batching parameters (the reference's pusch_processor_impl::configuration and the rx buffer pool size).
struct pusch_batch_configuration {
  int                                  device = 0;
  pusch_estimator_options              estimator;
  pusch_demodulator_options            demodulator;
  unsigned                             max_cb_ids          = 4096;  ///< rx buffer pool codeblocks (HARQ arena slots).
  unsigned                             nof_ldpc_iterations = 6;
  bool                                 ldpc_early_stop     = true;
  channel_state_information::sinr_type csi_sinr_calc_method = channel_state_information::sinr_type::post_equalization;
  /// false: the PUSCH task returns once the slot's results are notified (as the reference's processors do on their
  /// executor); true: it returns once the slot is handed to the GPU service, and the results are notified from the
  /// service's completion thread (the uplink processor keeps the grid and the slot until then, so a DU runs several
  /// uplink processors per sector, as du_low's processor pool does).
  bool asynchronous = false;
  /// Multi-GPU (row b7): the devices a slot's UEs are sharded over, the first one the root whose thread replays the
  /// results; empty: one device (`device`). A UE's shard is its RNTI modulo the number of devices, so its HARQ soft bits
  /// stay in the arena of the device that decodes its retransmissions. Each shard runs the estimator, demodulator,
  /// demultiplexer and decoder of its UEs on its own copy of the rx grid; `transport` gathers the results (TB bytes, CB
  /// / TB CRC flags, iterations, channel metrics, statistics, UCI streams, kept CB messages) to the root.
  std::vector<int>                        devices;
  std::shared_ptr<pusch_result_transport> transport;  ///< nullptr: create_pusch_copy_transport()
};

/// The per-GPU PUSCH service: one dispatcher that gathers the slots every cell's batches submit into one launch
/// sequence (cross-cell aggregation), several launch sets in flight on their own streams, and one completion thread
/// that replays the results into the reference's processors. Shared by every PUSCH batch of every sector on a GPU.
struct pusch_service_configuration {
  int      device                    = 0;
  unsigned nof_launch_sets           = 3;   ///< launches in flight (each with its own stream, staging and plans)
  unsigned max_slots_per_launch      = 16;  ///< slots (of any cells) gathered into one launch
  unsigned expected_slots_per_launch = 1;   ///< slots of one slot number to wait for before launching (the cells)
  unsigned gather_window_us          = 0;   ///< longest wait for them, from the first one's arrival
  unsigned max_grids                 = 64;  ///< batches (uplink processors) per grid shape on the device
  /// Threads replaying a launch's slots (the completion thread included). 1 by default: on the 16-CPU box with 16
  /// sector threads, 4 replay threads cut the 16-sector UL service from 39.4k to 33.5k one-PDU slots/s (15.1k from
  /// 39.0k with 16 UEs; profiles/r5_replay_threads_ab.txt): the helpers take the sectors' CPUs.
  unsigned replay_threads = 1;
};
class pusch_gpu_service;
std::shared_ptr<pusch_gpu_service> create_pusch_gpu_service(const pusch_service_configuration& config);

/// Moves a slot's PUSCH results from the GPUs that decoded its UEs to the device whose thread replays them into the
/// reference's processors and notifier (the FAPI side, row b7): every part lands at dst + dst_offset on the root device,
/// ordered on root_stream after the work already queued on the part's stream.
class pusch_result_transport
{
public:
  struct part {
    unsigned    rank;    ///< Index of the part's device in the transport's device list.
    int         device;
    const void* src;
    size_t      bytes;
    void*       stream;  ///< hipStream_t of the part's producer.
    size_t      dst_offset;
  };
  virtual ~pusch_result_transport() = default;
  virtual void gather(int root_device, void* root_stream, void* dst, const std::vector<part>& parts) = 0;
};
/// Device-to-device copies (hipMemcpyPeerAsync; any device list, devices may repeat).
/// Grid transfers of the multi-device UL batches, process-wide (row b7): host-to-device grid uploads (one per slot, to
/// the root device, whatever the number of devices), root-to-shard copy launches and the bytes they moved (each
/// shard receives only its UEs' subcarrier bands).
struct pusch_multi_transfer_counters {
  uint64_t host_uploads = 0;
  uint64_t shard_copies = 0;
  uint64_t shard_bytes  = 0;
  /// Single-device slots whose rx grid was already in HBM: the lower PHY's sector group demodulated every symbol into
  /// the uplink grid and its HBM twin (the batch's grid slot), so the slot read nothing back over PCIe.
  uint64_t twin_grids = 0;
};
pusch_multi_transfer_counters get_pusch_multi_transfer_counters();

std::shared_ptr<pusch_result_transport> create_pusch_copy_transport();
/// RCCL point-to-point over xGMI: one communicator per listed device in this process (ncclCommInitAll, devices distinct),
/// every part an ncclSend from its rank to rank 0 inside one group.
std::shared_ptr<pusch_result_transport> create_pusch_rccl_transport(const std::vector<int>& devices);

/// The HBM HARQ arena shared by every PUSCH batch of a sector (the rx buffer pool is shared too).
class pusch_harq_arena;
std::shared_ptr<pusch_harq_arena> create_pusch_harq_arena(int device, unsigned max_cb_ids);

/// A slot batch of PUSCH transmissions (one per uplink processor).
class pusch_slot_batch;

/// uci: factory of the reference's UCI decoder (host-side part of the result assembly); fallback: the processor for
/// PDUs the batch does not cover; service: the GPU service (nullptr: a private one on config.device). The demux factory
/// of earlier revisions is no longer used (the GPU demultiplexes; the replay feeds the UCI decoders its streams) and
/// is accepted for compatibility.
std::shared_ptr<pusch_slot_batch> create_pusch_slot_batch(const pusch_batch_configuration&           config,
                                                          std::shared_ptr<pusch_harq_arena>          arena,
                                                          std::shared_ptr<ulsch_demultiplex_factory> demux,
                                                          std::shared_ptr<uci_decoder_factory>       uci,
                                                          std::unique_ptr<pusch_processor>           fallback,
                                                          std::shared_ptr<pusch_gpu_service>         service = nullptr);

/// The pusch_processor given to the reference's uplink_processor_impl: process() registers the PDU in the batch.
std::unique_ptr<pusch_processor> create_pusch_processor_batch_gpu(std::shared_ptr<pusch_slot_batch> batch);

/// The PUSCH executor given to the reference's uplink_processor_impl: runs each task on the calling thread.
task_executor& pusch_inline_executor();

/// Wraps the reference's uplink_processor_impl (built with the two objects above): after each handle_rx_symbol the PDUs
/// it registered run as one GPU job on `executor`.
std::unique_ptr<uplink_processor> create_uplink_processor_batch_gpu(std::unique_ptr<uplink_processor>  inner,
                                                                    std::shared_ptr<pusch_slot_batch> batch,
                                                                    task_executor&                    executor);

/// PDSCH slot batching parameters.
struct pdsch_batch_configuration {
  int device = 0;
  /// Multi-GPU (the DL counterpart of row b7): the devices a slot's PDSCHs are sharded over, the first one the root;
  /// empty: one device (`device`). A PDSCH runs on the device of its RNTI modulo the number of devices; every shard maps
  /// its UEs into its own grid and the root merges the shards' subcarrier bands into its grid (peer reads over xGMI)
  /// before the slot's one download.
  std::vector<int> devices;
};

/// Grid transfers of the PDSCH slot batches, process-wide: device-to-host grid downloads (one per slot, from the root
/// device, whatever the number of devices), shard-to-root merges and the bytes they moved (each shard's bands only).
struct pdsch_multi_transfer_counters {
  uint64_t grid_downloads = 0;
  uint64_t shard_merges   = 0;
  uint64_t merge_bytes    = 0;
  uint64_t twin_grids     = 0;  ///< slots whose PDSCH REs stayed in the grid's HBM twin for the GPU PDxCH (no download)
};
pdsch_multi_transfer_counters get_pdsch_multi_transfer_counters();

/// A slot batch of PDSCH transmissions (one per downlink processor). ptrs: the reference's PT-RS generator (host);
/// fallback: the processor for PDUs the batch does not cover (two codewords).
class pdsch_slot_batch;
std::shared_ptr<pdsch_slot_batch> create_pdsch_slot_batch(const pdsch_batch_configuration&      config,
                                                          std::unique_ptr<ptrs_pdsch_generator> ptrs,
                                                          std::unique_ptr<pdsch_processor>      fallback);
std::shared_ptr<pdsch_slot_batch> create_pdsch_slot_batch(int                                   device,
                                                          std::unique_ptr<ptrs_pdsch_generator> ptrs,
                                                          std::unique_ptr<pdsch_processor>      fallback);

/// The pdsch_processor given to the reference's downlink processor: records each PDSCH into the batch.
std::unique_ptr<pdsch_processor> create_pdsch_processor_batch_gpu(std::shared_ptr<pdsch_slot_batch> batch);

/// The executor given to the reference's downlink processor: runs a task on the caller while the batching wrapper's
/// process_pdsch is in progress on this thread, forwards every other task to `real`.
class pdsch_batch_executor : public task_executor
{
public:
  explicit pdsch_batch_executor(task_executor& real_) : real(real_) {}
  [[nodiscard]] bool execute(unique_task task) override;
  [[nodiscard]] bool defer(unique_task task) override;

private:
  task_executor& real;
};

/// Wraps the reference's downlink_processor_single_executor_impl (built with the two objects above).
std::unique_ptr<downlink_processor_base> create_downlink_processor_batch_gpu(std::unique_ptr<downlink_processor_base> inner,
                                                                             std::shared_ptr<pdsch_slot_batch> batch,
                                                                             task_executor&                    executor);

/// The device's shared PUSCH service (one per GPU and process): the first call for a device creates it with `config`,
/// later calls for the same device return it while any batch still holds it (their `config` is then ignored).
std::shared_ptr<pusch_gpu_service> get_pusch_gpu_service(const pusch_service_configuration& config);

} // namespace gpu

// ---------------------------------------------------------------------------------------------------------------------
// Row b8: the slot-batched GPU processors behind the reference's factory interfaces (integration/
// upper_phy_factories_gpu.cpp). upper_phy_factories.cpp builds its slot processors only through
// uplink_processor_factory::create (upper_phy_factories.h:59-83) and downlink_processor_factory::create (:114-128), and
// its PUSCH / PDSCH processors through pusch_processor_factory / pdsch_processor_factory (pusch/factories.h:101,
// pdsch/factories.h): a maintainer selects the GPU by substituting these factories at upper_phy_factories.cpp:596
// (PUSCH processor), :680 (uplink processor), :1014 (PDSCH processor) and :1100 (downlink processor); see INTEGRATION.md.
// ---------------------------------------------------------------------------------------------------------------------

/// create_pusch_processor_factory_sw's configuration (pusch/factories.h:109-120) with the estimator and demodulator on
/// the GPU: the options replace the two factories.
struct pusch_processor_factory_gpu_configuration {
  int                                           device = 0;
  gpu::pusch_estimator_options                  estimator;
  gpu::pusch_demodulator_options                demodulator;
  std::shared_ptr<ulsch_demultiplex_factory>    demux_factory;
  std::shared_ptr<pusch_decoder_factory>        decoder_factory;  ///< e.g. create_pusch_decoder_factory_hw over the GPU HAL
  std::shared_ptr<uci_decoder_factory>          uci_dec_factory;
  channel_estimate::channel_estimate_dimensions ch_estimate_dimensions;
  unsigned                                      dec_nof_iterations         = 10;
  bool                                          dec_enable_early_stop      = true;
  unsigned                                      max_nof_concurrent_threads = 1;
  channel_state_information::sinr_type csi_sinr_calc_method = channel_state_information::sinr_type::channel_estimator;
};

/// The replacement of create_pusch_processor_factory_sw (upper_phy_factories.cpp:596): the reference's
/// pusch_processor_impl over the GPU DM-RS estimator and demodulator (row b3); validator: the reference's, with the
/// configured channel-estimate dimensions.
std::shared_ptr<pusch_processor_factory>
create_pusch_processor_factory_gpu(const pusch_processor_factory_gpu_configuration& config);

/// The replacement of create_pdsch_processor_factory_sw (upper_phy_factories.cpp:1014): the reference's
/// pdsch_processor_impl over the given encoder (e.g. create_pdsch_encoder_factory_hw over the GPU HAL) and the GPU
/// modulator and DM-RS processor.
std::shared_ptr<pdsch_processor_factory>
create_pdsch_processor_factory_gpu(int                                           device,
                                   std::shared_ptr<pdsch_encoder_factory>        encoder_factory,
                                   std::shared_ptr<ptrs_pdsch_generator_factory> ptrs_factory);

/// The uplink_processor_base_factory arguments (upper_phy_factories.cpp:52-70, :672-686) plus the GPU slot batch.
struct uplink_processor_factory_gpu_configuration {
  std::shared_ptr<pucch_processor_factory> pucch_factory;
  std::shared_ptr<prach_detector_factory>  prach_factory;
  std::shared_ptr<srs_estimator_factory>   srs_factory;
  std::shared_ptr<resource_grid_factory>   grid_factory;
  /// The PUSCH processors for the PDUs a slot batch does not cover (UCI only, more than four layers or rx ports,
  /// non-identity rx port lists, extended CP); its validator is the factory's PUSCH validator.
  std::shared_ptr<pusch_processor_factory> pusch_factory;
  /// The reference's UCI decoder factory (host part of the result replay).
  std::shared_ptr<uci_decoder_factory> uci_dec_factory;
  /// upper_phy_config's executors (upper_phy_factories.cpp:672-675); the PUSCH executor runs the slot batches' jobs.
  task_executor* pucch_executor = nullptr;
  task_executor* pusch_executor = nullptr;
  task_executor* srs_executor   = nullptr;
  task_executor* prach_executor = nullptr;
  /// The slot batches (device, estimator / demodulator options, HARQ arena size = the rx buffer pool's codeblocks,
  /// iterations, synchronous / asynchronous, multi-GPU shards).
  gpu::pusch_batch_configuration batch;
  /// The GPU service the batches submit to; nullptr: gpu::get_pusch_gpu_service(service_config) - one per device,
  /// shared by every uplink processor of every factory on that device (the cross-sector aggregation).
  std::shared_ptr<gpu::pusch_gpu_service> service;
  gpu::pusch_service_configuration        service_config;
};

/// The replacement of uplink_processor_base_factory (upper_phy_factories.cpp:680): create() builds the reference's
/// uplink_processor_impl over a GPU slot batch and wraps it so that each slot's PUSCH PDUs run as one GPU job. Uplink
/// processors created with the same rx_buffer_pool (one sector, as create_ul_processor_pool builds them) share one HBM
/// HARQ arena. create_pdu_validator() returns the reference's uplink_processor_validator_impl over the channel
/// factories' validators.
std::shared_ptr<uplink_processor_factory>
create_uplink_processor_factory_gpu(const uplink_processor_factory_gpu_configuration& config);

/// The downlink_processor_single_executor_factory arguments (upper_phy_factories.cpp:153-170, :1100) plus the GPU
/// device and the PT-RS generator the PDSCH slot batch maps on the host.
struct downlink_processor_factory_gpu_configuration {
  int                                           device = 0;
  std::vector<int>                              devices;  ///< multi-GPU PDSCH shards (gpu::pdsch_batch_configuration)
  std::shared_ptr<pdcch_processor_factory>      pdcch_factory;
  /// The PDSCH processors for the PDUs a slot batch does not cover (two codewords); its validator is the factory's.
  std::shared_ptr<pdsch_processor_factory>      pdsch_factory;
  std::shared_ptr<ssb_processor_factory>        ssb_factory;
  std::shared_ptr<nzp_csi_rs_generator_factory> nzp_csi_rs_factory;
  std::shared_ptr<prs_generator_factory>        prs_factory;
  std::shared_ptr<ptrs_pdsch_generator_factory> ptrs_factory;
};

/// The replacement of downlink_processor_single_executor_factory (upper_phy_factories.cpp:1100): create() builds the
/// reference's downlink_processor_single_executor_impl over a GPU PDSCH slot batch on `config.executor`, wrapped so that
/// the slot's PDSCHs run as one GPU launch at finish_processing_pdus.
std::shared_ptr<downlink_processor_factory>
create_downlink_processor_factory_gpu(const downlink_processor_factory_gpu_configuration& config);

} // namespace srsran
